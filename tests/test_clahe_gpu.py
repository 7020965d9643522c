"""GPU parity of the preprocessing step (CLAHE + histogram check, libgvx.so via
the C ABI) against the CPU restatement (oracle/clahe.c): equalised images are
required to be BIT-EXACT (integer histograms/LUTs, fp32 interpolation without
FMA on both sides), histogram means equal to the last bit."""
import numpy as np
import pytest

from gvx import synth

pytestmark = pytest.mark.gpu


def _img(w, h, seed):
    return synth.make_image(w, h, np.random.default_rng(seed))


def _same(a, b, what):
    if not np.array_equal(a, b):
        d = np.argwhere(a != b)
        raise AssertionError(f"{what}: {len(d)} mismatches, first at {d[:5].tolist()}: "
                             f"gpu={a[tuple(d[0])]} oracle={b[tuple(d[0])]}")


@pytest.mark.parametrize("w,h,tiles,clip", [
    (1280, 560, (21, 21), 3.0),    # the reference: both sides padded (61 x 27 tiles)
    (1920, 1200, (21, 21), 3.0),
    (210, 147, (21, 21), 3.0),     # divisible: no border
    (215, 147, (21, 21), 3.0),     # width only indivisible: a whole extra tile row
    (100, 100, (8, 8), 40.0),
    (96, 64, (6, 4), 0.0),         # no clipping
    (47, 33, (5, 3), 1.0),
    (161, 71, (64, 1), 3.0),       # widest grid
])
def test_clahe_bit_exact(ctx, orc, gvx_mod, w, h, tiles, clip):
    img = _img(w, h, w * 7 + h)
    p = gvx_mod.ClaheParams.default(clip_limit=clip, tiles_x=tiles[0], tiles_y=tiles[1])
    out, m = ctx.clahe(img, p, hist_mean=True)
    _same(out, orc.clahe(img, clip, tiles), "clahe")
    assert m == orc.hist_mean(img)


def test_clahe_constant_and_extremes(ctx, orc, gvx_mod):
    for v in (0, 255):
        img = np.full((140, 320), v, np.uint8)
        _same(ctx.clahe(img), orc.clahe(img), f"constant {v}")
    img = (np.indices((140, 320)).sum(0) % 2 * 255).astype(np.uint8)  # checkerboard of 0/255
    _same(ctx.clahe(img), orc.clahe(img), "checkerboard")


def test_clahe_batch_dev_strided_and_in_place(ctx, orc, gvx_mod):
    import torch
    w, h, n, pitch = 333, 97, 5, 340        # odd width: byte path; rows 340 bytes apart
    imgs = [_img(w, h, 100 + i) for i in range(n)]
    host = np.zeros((n, h, pitch), np.uint8)
    for i in range(n):
        host[i, :, :w] = imgs[i]
    src = torch.from_numpy(host).cuda()
    dst = torch.zeros((n, h, w), dtype=torch.uint8, device="cuda")
    means = torch.zeros(n, dtype=torch.float64, device="cuda")
    __import__("torch").cuda.synchronize()  # torch fills on its stream; gvx launches on its own
    ctx.clahe_batch_dev(n, w, h, src.data_ptr(), dst.data_ptr(), d_hist_mean=means.data_ptr(),
                        src_img_stride=h * pitch, src_stride=pitch)
    ctx.sync()
    out, mv = dst.cpu().numpy(), means.cpu().numpy()
    for i in range(n):
        _same(out[i], orc.clahe(imgs[i]), f"image {i}")
        assert mv[i] == orc.hist_mean(imgs[i])
    # in place (the reference's clahe_->apply(image, image)), aligned dword path
    w2, h2 = 1280, 560
    b = [_img(w2, h2, 7 + i) for i in range(3)]
    t = torch.from_numpy(np.stack(b)).cuda()
    ctx.clahe_batch_dev(3, w2, h2, t.data_ptr(), t.data_ptr())
    ctx.sync()
    tt = t.cpu().numpy()
    for i in range(3):
        _same(tt[i], orc.clahe(b[i]), f"in-place image {i}")


def test_frame_preprocess_feeds_pyramid(ctx, orc, gvx_mod):
    """Tracking::preprocessing then the frame's pyramid: level 0 is the CLAHE
    output and every level is the oracle pyramid of it."""
    img = _img(1280, 560, 42)
    eq, m = ctx.frame_preprocess(11, img, hist_mean=True)
    ref = orc.clahe(img)
    _same(eq, ref, "equalised frame")
    assert m == orc.hist_mean(img)
    for l, r in enumerate(orc.build_pyramid(ref, 3)):
        _same(ctx.frame_level(11, l), r, f"level {l}")
    ctx.frame_drop(11)


@pytest.mark.parametrize("w,h", [(1280, 560), (333, 149), (200, 70)])
def test_frame_preprocess_into_slot_with_rings(ctx, orc, gvx_mod, w, h):
    """gvx_frame_preprocess_dev without a CLAHE output buffer equalises straight
    into the frame's padded level-0 slot, ring included, and builds the levels
    from it: every level with its 32-pixel REFLECT_101 ring is the oracle's.  The
    indexed entry (frame *d_index of an HBM-resident sequence) gives the same."""
    import torch
    rng = np.random.default_rng(w + 3 * h)
    seq = np.stack([synth.make_image(w, h, rng) for _ in range(3)])
    d_seq = torch.from_numpy(seq).cuda()
    ref = orc.clahe(seq[2])
    levels = [np.pad(r, 32, mode="reflect") for r in orc.build_pyramid(ref, 3)]
    p = gvx_mod.KltParams.default(max_level=3)
    ctx.frame_preprocess_dev(12, d_seq[2].data_ptr(), w, h, params=p)
    idx = torch.tensor([2], dtype=torch.int32, device="cuda")
    ctx.frame_preprocess_indexed_dev(13, d_seq.data_ptr(), w * h, idx.data_ptr(), 3, w, h, params=p)
    # an index past the sequence is clamped to its last frame (never read past it)
    idx_past = torch.tensor([7], dtype=torch.int32, device="cuda")
    ctx.frame_preprocess_indexed_dev(14, d_seq.data_ptr(), w * h, idx_past.data_ptr(), 3, w, h, params=p)
    ctx.sync()
    for fid in (12, 13, 14):
        for l, r in enumerate(levels):
            _same(ctx.frame_level_padded(fid, l, 32), r, f"frame {fid} padded level {l}")
        ctx.frame_drop(fid)


def test_clahe_rejects_bad_grids(ctx, gvx_mod):
    img = _img(64, 40, 1)
    for p in (gvx_mod.ClaheParams.default(tiles_x=0), gvx_mod.ClaheParams.default(tiles_y=65),
              gvx_mod.ClaheParams.default(tiles_x=65), gvx_mod.ClaheParams.default(tiles_x=21, tiles_y=41)):
        with pytest.raises(gvx_mod.GvxError):
            ctx.clahe(img, p)


# ---- BGR8 frames (Tracking::preprocessing's cv::cvtColor(COLOR_BGR2GRAY),
# tracking.cc:111-113, folded into the CLAHE histogram pass) ----

def _bgr(w, h, seed):
    rng = np.random.default_rng(seed)
    return np.stack([synth.make_image(w, h, rng) for _ in range(3)], axis=-1)


@pytest.mark.parametrize("w,h", [(1280, 560), (333, 149), (210, 147), (47, 33)])
def test_clahe_bgr_bit_exact(ctx, orc, gvx_mod, w, h):
    """BGR8 in, the CLAHE of its gray conversion out (8-byte path at widths that
    are multiples of 8, the byte path otherwise), the histogram check of the gray
    frame: bit-exact against oracle bgr2gray + clahe."""
    bgr = _bgr(w, h, w + h)
    gray = orc.bgr2gray(bgr)
    out, m = ctx.clahe(bgr, hist_mean=True)
    _same(out, orc.clahe(gray), "clahe of the gray frame")
    assert m == orc.hist_mean(gray)


def test_bgr_extremes(ctx, orc, gvx_mod):
    """Pure channels and white: the fixed-point weights themselves."""
    for col in ((255, 0, 0), (0, 255, 0), (0, 0, 255), (255, 255, 255), (1, 2, 3)):
        bgr = np.zeros((64, 96, 3), np.uint8)
        bgr[:, 48:] = col
        _same(ctx.clahe(bgr), orc.clahe(orc.bgr2gray(bgr)), f"colour {col}")


def test_clahe_batch_dev_bgr(ctx, orc, gvx_mod):
    import torch
    w, h, n = 1280, 560, 3
    imgs = [_bgr(w, h, 50 + i) for i in range(n)]
    src = torch.from_numpy(np.stack(imgs)).cuda()
    dst = torch.zeros((n, h, w), dtype=torch.uint8, device="cuda")
    means = torch.zeros(n, dtype=torch.float64, device="cuda")
    __import__("torch").cuda.synchronize()  # torch fills on its stream; gvx launches on its own
    p = gvx_mod.ClaheParams.default(channels=3)
    ctx.clahe_batch_dev(n, w, h, src.data_ptr(), dst.data_ptr(), params=p, d_hist_mean=means.data_ptr(),
                        src_img_stride=3 * w * h, src_stride=3 * w)
    ctx.sync()
    out, mv = dst.cpu().numpy(), means.cpu().numpy()
    for i in range(n):
        g = orc.bgr2gray(imgs[i])
        _same(out[i], orc.clahe(g), f"image {i}")
        assert mv[i] == orc.hist_mean(g)


def test_frame_preprocess_bgr_feeds_pyramid(ctx, orc, gvx_mod):
    """A BGR8 frame through the whole preprocessing into the frame cache (host
    entry and the HBM-resident indexed entry): every pyramid level is the
    oracle's pyramid of clahe(bgr2gray(frame))."""
    import torch
    w, h = 1280, 560
    seq = np.stack([_bgr(w, h, 70 + i) for i in range(2)])
    ref = orc.clahe(orc.bgr2gray(seq[1]))
    eq, m = ctx.frame_preprocess(15, seq[1], hist_mean=True)
    _same(eq, ref, "equalised frame")
    assert m == orc.hist_mean(orc.bgr2gray(seq[1]))
    d_seq = torch.from_numpy(seq).cuda()
    idx = torch.tensor([1], dtype=torch.int32, device="cuda")
    ctx.frame_preprocess_indexed_dev(16, d_seq.data_ptr(), 3 * w * h, idx.data_ptr(), 2, w, h, stride=3 * w,
                                     clahe=gvx_mod.ClaheParams.default(channels=3),
                                     params=gvx_mod.KltParams.default(max_level=3))
    ctx.sync()
    for l, r in enumerate(orc.build_pyramid(ref, 3)):
        _same(ctx.frame_level(15, l), r, f"level {l}")
        _same(ctx.frame_level_padded(16, l, 32), np.pad(r, 32, mode="reflect"), f"indexed padded level {l}")
    ctx.frame_drop(15)
    ctx.frame_drop(16)


def test_bad_channels_refused(ctx, gvx_mod):
    import torch
    buf = torch.zeros(3 * 64 * 40, dtype=torch.uint8, device="cuda")
    ctx.clahe_batch_dev(1, 64, 40, buf.data_ptr(), buf.data_ptr())  # MONO8: fine
    with pytest.raises(gvx_mod.GvxError):
        ctx.clahe_batch_dev(1, 64, 40, buf.data_ptr(), buf.data_ptr(), params=gvx_mod.ClaheParams.default(channels=2))
    with pytest.raises(gvx_mod.GvxError):  # BGR8 rows need 3 w bytes
        ctx.clahe_batch_dev(1, 64, 40, buf.data_ptr(), buf.data_ptr(), params=gvx_mod.ClaheParams.default(channels=3),
                            src_stride=64)
    ctx.sync()

"""GPU parity of the fused one-pass CLAHE (clahe.hip fused_kernel), the form
batches of >= 8 frames take, against the CPU restatement (oracle/clahe.c):
bit-exact images and histogram means, at the segment counts the batch size
selects (1 segment per image at 256 frames, up to one band per workgroup at
8), mono and BGR8, 8-byte and byte paths, strided sources, and the
two-kernel form at the same inputs (in place, or too tall a tile for the
register ring) for comparison."""
import numpy as np
import pytest

from gvx import synth

pytestmark = pytest.mark.gpu


def _img(w, h, seed):
    return synth.make_image(w, h, np.random.default_rng(seed))


def _bgr(w, h, seed):
    rng = np.random.default_rng(seed)
    return np.stack([synth.make_image(w, h, rng) for _ in range(3)], axis=-1)


def _same(a, b, what):
    if not np.array_equal(a, b):
        d = np.argwhere(a != b)
        raise AssertionError(f"{what}: {len(d)} mismatches, first at {d[:5].tolist()}: "
                             f"gpu={a[tuple(d[0])]} oracle={b[tuple(d[0])]}")


def _run(ctx, gvx_mod, frames, w, h, params=None, pitch=None, chan=1):
    """n frames (distinct sources cycled) through gvx_clahe_batch_dev."""
    import torch
    n = len(frames)
    pitch = pitch or chan * w
    host = np.zeros((n, h, pitch), np.uint8)
    for i, f in enumerate(frames):
        host[i, :, :chan * w] = f.reshape(h, chan * w)
    src = torch.from_numpy(host).cuda()
    dst = torch.zeros((n, h, w), dtype=torch.uint8, device="cuda")
    means = torch.zeros(n, dtype=torch.float64, device="cuda")
    __import__("torch").cuda.synchronize()  # torch fills on its stream; gvx launches on its own
    ctx.clahe_batch_dev(n, w, h, src.data_ptr(), dst.data_ptr(), params=params, d_hist_mean=means.data_ptr(),
                        src_img_stride=h * pitch, src_stride=pitch)
    ctx.sync()
    return dst.cpu().numpy(), means.cpu().numpy()


@pytest.mark.parametrize("w,h,n,tiles,clip", [
    (1280, 560, 256, (21, 21), 3.0),   # the bench batch: one workgroup per image
    (1280, 560, 16, (21, 21), 3.0),    # 16 segments per image
    (1280, 560, 8, (21, 21), 3.0),     # 22 segments: one band each
    (640, 480, 12, (8, 8), 3.0),       # divisible grid, 5 row slots
    (333, 97, 9, (21, 21), 3.0),       # odd width: byte path for the last chunk
    (215, 147, 10, (21, 21), 0.0),     # no clipping, width pad only
    (161, 71, 8, (64, 1), 3.0),        # widest grid, one tile row
    (47, 33, 8, (5, 3), 1.0),
])
def test_fused_mono_bit_exact(ctx, orc, gvx_mod, w, h, n, tiles, clip):
    k = min(n, 4)
    imgs = [_img(w, h, 1000 + 13 * i + w) for i in range(k)]
    frames = [imgs[i % k] for i in range(n)]
    p = gvx_mod.ClaheParams.default(clip_limit=clip, tiles_x=tiles[0], tiles_y=tiles[1])
    out, mv = _run(ctx, gvx_mod, frames, w, h, params=p)
    want = [orc.clahe(im, clip, tiles) for im in imgs]
    means = [orc.hist_mean(im) for im in imgs]
    for i in range(n):
        _same(out[i], want[i % k], f"image {i}")
        assert mv[i] == means[i % k], f"hist mean {i}"


@pytest.mark.parametrize("w,h,n", [(1280, 560, 8), (1280, 560, 64), (333, 149, 8)])
def test_fused_bgr_bit_exact(ctx, orc, gvx_mod, w, h, n):
    k = min(n, 3)
    imgs = [_bgr(w, h, 77 + i) for i in range(k)]
    grays = [orc.bgr2gray(b) for b in imgs]
    frames = [imgs[i % k] for i in range(n)]
    out, mv = _run(ctx, gvx_mod, frames, w, h, params=gvx_mod.ClaheParams.default(channels=3), chan=3)
    for i in range(n):
        _same(out[i], orc.clahe(grays[i % k]), f"BGR image {i}")
        assert mv[i] == orc.hist_mean(grays[i % k])


def test_fused_strided_source(ctx, orc, gvx_mod):
    w, h, n = 1280, 560, 8
    imgs = [_img(w, h, 5 + i) for i in range(n)]
    out, mv = _run(ctx, gvx_mod, imgs, w, h, pitch=1344)
    for i in range(n):
        _same(out[i], orc.clahe(imgs[i]), f"image {i}")
        assert mv[i] == orc.hist_mean(imgs[i])


def test_fused_matches_two_kernel_form(ctx, orc, gvx_mod):
    """The same 8 frames in place (the two-kernel form: a fused seam would read
    rows another workgroup already wrote) and out of place (fused)."""
    import torch
    w, h, n = 1280, 560, 8
    imgs = np.stack([_img(w, h, 300 + i) for i in range(n)])
    out, _ = _run(ctx, gvx_mod, list(imgs), w, h)
    t = torch.from_numpy(imgs.copy()).cuda()
    ctx.clahe_batch_dev(n, w, h, t.data_ptr(), t.data_ptr())
    ctx.sync()
    _same(out, t.cpu().numpy(), "fused vs in-place two-kernel")
    for i in range(n):
        _same(out[i], orc.clahe(imgs[i]), f"image {i}")


def test_tall_tiles_take_two_kernel_form(ctx, orc, gvx_mod):
    """1920x1200: 58-row tiles need 15 row slots per thread, more than the
    register ring holds -- the batch still comes out bit-exact."""
    w, h, n = 1920, 1200, 8
    imgs = [_img(w, h, 900 + i) for i in range(2)]
    out, mv = _run(ctx, gvx_mod, [imgs[i % 2] for i in range(n)], w, h)
    want = [orc.clahe(im) for im in imgs]
    for i in range(n):
        _same(out[i], want[i % 2], f"image {i}")
        assert mv[i] == orc.hist_mean(imgs[i % 2])

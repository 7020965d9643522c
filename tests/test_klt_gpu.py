"""GPU parity of the KLT path (libgvx.so via the C ABI) against the CPU
restatement (oracle/): pyramid levels, calcOpticalFlowPyrLK outputs and the
fused fwd/bwd/FB/compaction are required to be BIT-EXACT (integer window sums,
IEEE fp32 solve without FMA on both sides); this is stricter than the 1e-4 px
flow tolerance of BASELINE.json's north_star."""
import numpy as np
import pytest

from gvx import synth

pytestmark = pytest.mark.gpu


def _assert_same(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    if not np.array_equal(a, b):
        diff = np.argwhere(a != b)
        raise AssertionError(f"{what}: {len(diff)} mismatches, first at {diff[:5].tolist()}: "
                             f"gpu={a[tuple(diff[0])]} oracle={b[tuple(diff[0])]}")


@pytest.mark.parametrize("w,h,L", [(160, 70, 3), (161, 71, 3), (1280, 560, 3), (1920, 1200, 4),
                                   (333, 97, 2)])
def test_pyramid_levels_bit_exact(ctx, orc, gvx_mod, w, h, L):
    img = synth.make_image(w, h, np.random.default_rng(w + h))
    p = gvx_mod.KltParams.default(max_level=L)
    ctx.frame_put(7, img, p)
    ref = orc.build_pyramid(img, L)
    for l, r in enumerate(ref):
        _assert_same(ctx.frame_level(7, l), r, f"level {l}")
    ctx.frame_drop(7)


@pytest.mark.parametrize("w,h,L", [(160, 70, 3), (161, 71, 3), (1280, 560, 3), (333, 97, 2), (130, 44, 1)])
def test_pyramid_rings_reflect101(ctx, orc, gvx_mod, w, h, L):
    """The padded levels LK reads: every level with its 32-pixel REFLECT_101 ring
    (numpy "reflect" = BORDER_REFLECT_101) around the oracle's level."""
    img = synth.make_image(w, h, np.random.default_rng(3 * w + h))
    p = gvx_mod.KltParams.default(max_level=L)
    ctx.frame_put(9, img, p)
    for l, r in enumerate(orc.build_pyramid(img, L)):
        _assert_same(ctx.frame_level_padded(9, l, 32), np.pad(r, 32, mode="reflect"), f"padded level {l}")
    ctx.frame_drop(9)


@pytest.mark.parametrize("w,h,n,L,seed", [(160, 70, 32, 3, 1), (320, 140, 64, 3, 2),
                                          (1280, 560, 150, 3, 20261015), (1920, 1200, 500, 4, 5)])
def test_calc_optical_flow_bit_exact(ctx, orc, gvx_mod, w, h, n, L, seed):
    I, J, prev, init, _ = synth.make_pair(w, h, n, seed)
    p = gvx_mod.KltParams.default(max_level=L)
    ctx.frame_put(1, I, p)
    ctx.frame_put(2, J, p)
    g_next, g_st, g_err = ctx.calc_optical_flow_pyr_lk(1, 2, prev, init, p)
    o_next, o_st, o_err = orc.calc_optical_flow_pyr_lk(I, J, prev, init, orc.KltParams.default(max_level=L))
    _assert_same(g_st, o_st, "status")
    _assert_same(g_next, o_next, "nextPts")
    _assert_same(g_err[o_st == 1], o_err[o_st == 1], "err")


@pytest.mark.parametrize("w,h,n,L,seed", [(320, 140, 80, 3, 3), (1280, 560, 150, 3, 20261015),
                                          (1920, 1200, 500, 4, 20261016)])
def test_track_fb_bit_exact(ctx, orc, gvx_mod, w, h, n, L, seed):
    I, J, prev, init, _ = synth.make_pair(w, h, n, seed)
    p = gvx_mod.KltParams.default(max_level=L)
    ctx.frame_put(1, I, p)
    ctx.frame_put(2, J, p)
    g = ctx.track_fb(1, 2, prev, init, w, h, params=p)
    o = orc.klt_fb(I, J, prev, init, w, h, params=orc.KltParams.default(max_level=L))
    for k in ("next", "back", "st_f", "st_b", "keep", "kept_idx"):
        _assert_same(g[k], o[k], k)


def test_batch_bit_exact(ctx, orc, gvx_mod):
    P, W, H, N = 6, 1280, 560, 150
    I, J, prev, init = synth.make_batch(P, W, H, N)
    g = ctx.klt_fb_batch(I, J, prev, init)
    for i in range(P):
        o = orc.klt_fb(I[i], J[i], prev[i], init[i], reuse_pyramids=True)
        _assert_same(g["next"][i], o["next"], f"pair {i} next")
        _assert_same(g["back"][i], o["back"], f"pair {i} back")
        flags = o["st_f"] | (o["st_b"] << 1) | (o["keep"] << 2)
        _assert_same(g["flags"][i], flags, f"pair {i} flags")
        assert g["n_kept"][i] == len(o["kept_idx"])
        _assert_same(g["kept"][i][:g["n_kept"][i]], o["kept_idx"], f"pair {i} kept")


def test_edge_points(ctx, orc, gvx_mod):
    """Points at / beyond the border, far outside, and on a flat patch."""
    I, J, _, _, _ = synth.make_pair(320, 140, 8, seed=9)
    I[40:80, 200:260] = 77
    J[40:80, 200:260] = 77
    prev = np.array([[0, 0], [319.9, 139.9], [-25, 10], [10, -25], [1000, 50], [230, 60], [5, 70],
                     [315, 5], [160.5, 70.25], [-21.0, -21.0], [330.0, 150.0]], np.float32)
    init = prev + np.float32(0.7)
    p = gvx_mod.KltParams.default()
    ctx.frame_put(1, I, p)
    ctx.frame_put(2, J, p)
    g_next, g_st, g_err = ctx.calc_optical_flow_pyr_lk(1, 2, prev, init, p)
    o_next, o_st, o_err = orc.calc_optical_flow_pyr_lk(I, J, prev, init)
    _assert_same(g_st, o_st, "status")
    _assert_same(g_next, o_next, "next")
    g = ctx.track_fb(1, 2, prev, init, 320, 140)
    o = orc.klt_fb(I, J, prev, init)
    for k in ("next", "back", "st_f", "st_b", "keep", "kept_idx"):
        _assert_same(g[k], o[k], k)


def test_empty_and_single(ctx, orc, gvx_mod):
    I, J, prev, init, _ = synth.make_pair(160, 70, 1, seed=10)
    ctx.frame_put(1, I)
    ctx.frame_put(2, J)
    r = ctx.track_fb(1, 2, prev[:0], init[:0], 160, 70)
    assert r["kept_idx"].size == 0
    g = ctx.track_fb(1, 2, prev, init, 160, 70)
    o = orc.klt_fb(I, J, prev, init)
    for k in ("next", "back", "keep", "kept_idx"):
        _assert_same(g[k], o[k], k)


def test_missing_frame_raises(ctx, gvx_mod):
    with pytest.raises(gvx_mod.GvxError):
        ctx.calc_optical_flow_pyr_lk(12345, 54321, np.zeros((1, 2), np.float32))


def test_large_batch_invariants(ctx, gvx_mod):
    """Size-independent properties at the config-3 scale (1920x1200, 500 feat,
    4-level): determinism across two runs and compaction consistency."""
    P, W, H, N = 32, 1920, 1200, 500
    I, J, prev, init = synth.make_batch(P, W, H, N, distinct=4)
    p = gvx_mod.KltParams.default(max_level=4)
    a = ctx.klt_fb_batch(I, J, prev, init, params=p)
    b = ctx.klt_fb_batch(I, J, prev, init, params=p)
    for k in a:
        _assert_same(a[k], b[k], k)
    for i in range(P):
        keep = np.nonzero(a["flags"][i] & 4)[0]
        assert a["n_kept"][i] == len(keep)
        _assert_same(a["kept"][i][:len(keep)], keep, "kept")
    # tiled pairs are identical inputs -> identical outputs
    _assert_same(a["next"][0], a["next"][4], "tiling")


def _border_points(w, h, n, rng):
    """Points hugging / crossing every border at level 0 (the in-place level-0
    read takes its REFLECT_101 gather path there) plus a few interior ones."""
    side = rng.integers(0, 4, n)
    t = rng.uniform(-30, 30, n)
    pts = np.empty((n, 2), np.float32)
    pts[:, 0] = np.where(side == 0, t, np.where(side == 1, w - 1 - t, rng.uniform(0, w, n)))
    pts[:, 1] = np.where(side == 2, t, np.where(side == 3, h - 1 - t, rng.uniform(0, h, n)))
    pts[:4] = [[0.5, 0.5], [w - 1.5, h - 1.5], [w / 2, h / 2], [3.25, h - 4.75]]
    return pts


@pytest.mark.parametrize("w,h,L", [(1280, 560, 3), (333, 149, 3), (324, 150, 2), (1000, 77, 1)])
def test_batch_border_and_odd_sizes(ctx, orc, gvx_mod, w, h, L):
    """Batched path with level 0 read in place: windows on the image border,
    widths that are not multiples of 16 (no 16-byte staging loads), odd level
    sizes, and 1- and 2-level pyramids (other fused-pyramid variants)."""
    P, N = 3, 96
    rng = np.random.default_rng(w * 7 + h)
    I = np.stack([synth.make_image(w, h, rng) for _ in range(P)])
    J = np.stack([np.roll(I[i], (1, -2), axis=(0, 1)) for i in range(P)])
    prev = np.stack([_border_points(w, h, N, rng) for _ in range(P)])
    init = (prev + rng.uniform(-1.5, 1.5, prev.shape)).astype(np.float32)
    p = gvx_mod.KltParams.default(max_level=L)
    g = ctx.klt_fb_batch(I, J, prev, init, params=p)
    for i in range(P):
        o = orc.klt_fb(I[i], J[i], prev[i], init[i], params=orc.KltParams.default(max_level=L),
                       reuse_pyramids=True)
        _assert_same(g["next"][i], o["next"], f"pair {i} next")
        _assert_same(g["back"][i], o["back"], f"pair {i} back")
        flags = o["st_f"] | (o["st_b"] << 1) | (o["keep"] << 2)
        _assert_same(g["flags"][i], flags, f"pair {i} flags")
        _assert_same(g["kept"][i][:g["n_kept"][i]], o["kept_idx"], f"pair {i} kept")


def test_frame_put_dev_matches_host_put(ctx, gvx_mod):
    """gvx_frame_put_dev (image already in HBM, any row stride) builds the same
    padded pyramid as gvx_frame_put."""
    import torch
    w, h, stride = 333, 150, 352
    img = synth.make_image(w, h, np.random.default_rng(5))
    buf = np.zeros((h, stride), np.uint8)
    buf[:, :w] = img
    d = torch.from_numpy(buf).cuda()
    p = gvx_mod.KltParams.default(max_level=3)
    ctx.frame_put(21, img, p)
    ctx.frame_put_dev(22, d.data_ptr(), w, h, stride, p)
    ctx.sync()
    for l in range(3):
        _assert_same(ctx.frame_level_padded(22, l, 32), ctx.frame_level_padded(21, l, 32), f"level {l}")
    ctx.frame_drop(21)
    ctx.frame_drop(22)


# gvx_set_klt_phases: each point group's whole chain in one wave (0, the
# default), or the batched LK as phases of 1, 2 or 3 levels
PHASES = [pytest.param(0, id="chain"), pytest.param(1, id="lpp1"), pytest.param(2, id="lpp2"),
          pytest.param(3, id="lpp3")]


@pytest.fixture
def phases(ctx, request):
    ctx.set_klt_phases(request.param, 64)  # small superchunks: several per launch, a ragged last one
    yield request.param
    ctx.set_klt_phases(0, 4096)


@pytest.mark.parametrize("phases", PHASES, indirect=True)
@pytest.mark.parametrize("n_pairs,n_pts", [(64, 149), (3, 2731), (30, 150)])
def test_batch_three_points_per_wave(ctx, orc, gvx_mod, n_pairs, n_pts, phases):
    """Launches of > 4096 points take the three-points-per-wave LK (the exact
    order); point counts that are not multiples of 3 leave one or two spare
    lane groups in each pair's last wave.  Border points included (the groups
    take turns on the wave's LDS tile).  Every way of cutting the chain into
    phases gives the oracle's bits."""
    w, h = 320, 140
    rng = np.random.default_rng(n_pairs + n_pts)
    I = np.stack([synth.make_image(w, h, rng) for _ in range(n_pairs)])
    J = np.stack([np.roll(I[i], (1, -1), axis=(0, 1)) for i in range(n_pairs)])
    prev = np.stack([np.concatenate([_border_points(w, h, 20, rng),
                                     rng.uniform([0, 0], [w, h], (n_pts - 20, 2)).astype(np.float32)])
                     for _ in range(n_pairs)])
    init = (prev + rng.uniform(-1.0, 1.0, prev.shape)).astype(np.float32)
    g = ctx.klt_fb_batch(I, J, prev, init)
    for i in range(0, n_pairs, max(1, n_pairs // 8)):
        o = orc.klt_fb(I[i], J[i], prev[i], init[i], reuse_pyramids=True)
        _assert_same(g["next"][i], o["next"], f"pair {i} next")
        _assert_same(g["back"][i], o["back"], f"pair {i} back")
        flags = o["st_f"] | (o["st_b"] << 1) | (o["keep"] << 2)
        _assert_same(g["flags"][i], flags, f"pair {i} flags")
        _assert_same(g["kept"][i][:g["n_kept"][i]], o["kept_idx"], f"pair {i} kept")


@pytest.mark.parametrize("phases", PHASES, indirect=True)
def test_single_call_three_points_per_wave_with_err(ctx, orc, gvx_mod, phases):
    """One pair with more than 4,096 points takes the three-point layout through
    gvx_calc_optical_flow_pyr_lk, whose level-0 error output is the layout's err
    path (the batch calls never ask for it): next, status and err bit-exact --
    also when the forward chain is cut into phases (mode 0: the last phase
    writes the status)."""
    W, H, N = 640, 480, 4500
    rng = np.random.default_rng(4500)
    I = synth.make_image(W, H, rng)
    J = np.roll(I, (2, -1), axis=(0, 1))
    prev = np.concatenate([_border_points(W, H, 300, rng),
                           rng.uniform([0, 0], [W, H], (N - 300, 2)).astype(np.float32)])
    init = (prev + rng.uniform(-1.5, 1.5, prev.shape)).astype(np.float32)
    p = gvx_mod.KltParams.default()
    ctx.frame_put(41, I, p)
    ctx.frame_put(42, J, p)
    g_next, g_st, g_err = ctx.calc_optical_flow_pyr_lk(41, 42, prev, init, p)
    o_next, o_st, o_err = orc.calc_optical_flow_pyr_lk(I, J, prev, init)
    _assert_same(g_st, o_st, "status")
    _assert_same(g_next, o_next, "next")
    _assert_same(g_err, o_err, "err")
    ctx.frame_drop(41)
    ctx.frame_drop(42)


def test_batch_three_points_per_wave_configs1(ctx, orc, gvx_mod):
    """configs[1] geometry (1280x560, 150 points, 3 levels) in a batch that takes
    the three-point layout, with border points at level 0 (read in place) in
    every pair: forward, backward, flags and kept indices bit-exact."""
    P, W, H, N = 30, 1280, 560, 150
    rng = np.random.default_rng(20261018)
    I = np.stack([synth.make_image(W, H, rng) for _ in range(P)])
    J = np.stack([np.roll(I[i], (2, -1), axis=(0, 1)) for i in range(P)])
    prev = np.stack([np.concatenate([_border_points(W, H, 30, rng),
                                     rng.uniform([0, 0], [W, H], (N - 30, 2)).astype(np.float32)])
                     for _ in range(P)])
    init = (prev + rng.uniform(-2.0, 2.0, prev.shape)).astype(np.float32)
    g = ctx.klt_fb_batch(I, J, prev, init)
    for i in (0, 13, P - 1):
        o = orc.klt_fb(I[i], J[i], prev[i], init[i], reuse_pyramids=True)
        _assert_same(g["next"][i], o["next"], f"pair {i} next")
        _assert_same(g["back"][i], o["back"], f"pair {i} back")
        flags = o["st_f"] | (o["st_b"] << 1) | (o["keep"] << 2)
        _assert_same(g["flags"][i], flags, f"pair {i} flags")
        _assert_same(g["kept"][i][:g["n_kept"][i]], o["kept_idx"], f"pair {i} kept")


def test_split_batch_entry_points_validate(ctx, gvx_mod):
    """gvx_klt_batch_pyramids_dev / gvx_klt_fb_batch_pyr_dev refuse what the one-call
    batch refuses (bad sizes, missing buffers) plus a missing pyramid buffer, and a
    zero-pair call is a no-op."""
    import torch
    dev = torch.device("cuda", 0)
    W, H = 64, 48
    img = torch.zeros((1, H, W), dtype=torch.uint8, device=dev)
    pyr = torch.zeros(2 * gvx_mod.pyramid_layout(W, H, 3)["bytes"], dtype=torch.uint8, device=dev)
    pts = torch.zeros((1, 4, 2), dtype=torch.float32, device=dev)
    flags = torch.zeros((1, 4), dtype=torch.uint8, device=dev)
    kept = torch.zeros((1, 4), dtype=torch.int32, device=dev)
    nk = torch.zeros((1,), dtype=torch.int32, device=dev)
    p = gvx_mod.KltParams.default(max_level=3)
    with pytest.raises(gvx_mod.GvxError):
        ctx.klt_batch_pyramids_dev(1, 16, H, img.data_ptr(), img.data_ptr(), 3, pyr.data_ptr())  # w <= win
    with pytest.raises(gvx_mod.GvxError):
        ctx.klt_batch_pyramids_dev(1, W, H, img.data_ptr(), img.data_ptr(), 3, 0)
    with pytest.raises(gvx_mod.GvxError):
        ctx.klt_fb_batch_pyr_dev(1, W, H, img.data_ptr(), img.data_ptr(), 0, 4, pts.data_ptr(), pts.data_ptr(),
                                 pts.data_ptr(), pts.data_ptr(), flags.data_ptr(), kept.data_ptr(), nk.data_ptr(),
                                 params=p)
    with pytest.raises(gvx_mod.GvxError):
        ctx.klt_fb_batch_pyr_dev(1, W, H, img.data_ptr(), img.data_ptr(), pyr.data_ptr(), 4, pts.data_ptr(),
                                 pts.data_ptr(), 0, pts.data_ptr(), flags.data_ptr(), kept.data_ptr(), nk.data_ptr(),
                                 params=p)
    ctx.klt_batch_pyramids_dev(0, W, H, 0, 0, 3, 0)
    ctx.klt_fb_batch_pyr_dev(0, W, H, img.data_ptr(), img.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0, 0, params=p)
    ctx.sync()


@pytest.mark.parametrize("phases", PHASES, indirect=True)
def test_three_point_wave_groups_leave_at_different_times(ctx, orc, gvx_mod, phases):
    """in the three-points-per-wave layout a group whose point stops
    early must not disturb the groups that go on iterating (the group sums rely
    on whole-group activity and on DPP reads of disabled lanes).  Every wave of
    this batch holds one point off the image at every level (it stops at the top
    level), one point that converges at once (J = I there, zero initial flow
    error) and one that needs many iterations (a 1.6 px error under a large
    iteration cap), in all three lane-group positions: next, back, flags and
    kept indices bit-exact against the oracle."""
    P, W, H, N = 40, 320, 140, 120  # 4,800 points: the three-point layout
    rng = np.random.default_rng(120)
    I = np.stack([synth.make_image(W, H, rng) for _ in range(P)])
    J = np.stack([np.roll(I[i], (3, -2), axis=(0, 1)) for i in range(P)])
    prev = rng.uniform([40, 40], [W - 40, H - 40], (P, N, 2)).astype(np.float32)
    init = prev + np.float32([-2.0, 3.0])  # the true shift
    for i in range(P):
        for k in range(N // 3):
            kind = (k + i) % 3  # which lane group holds which kind
            off, fast, slow = 3 * k + kind, 3 * k + (kind + 1) % 3, 3 * k + (kind + 2) % 3
            prev[i, off] = [-500.0, 60.0]  # off every level: stops at the top level
            init[i, off] = prev[i, off]
            init[i, fast] = prev[i, fast] + np.float32([-2.0, 3.0])
            init[i, slow] = prev[i, slow] + np.float32([-2.0, 3.0]) + rng.uniform(-1.6, 1.6, 2).astype(np.float32)
    p = gvx_mod.KltParams.default(max_level=3, max_iter=100)
    g = ctx.klt_fb_batch(I, J, prev, init, params=p)
    op = orc.KltParams.default(max_level=3, max_iter=100)
    for i in (0, 1, 2, P - 1):
        o = orc.klt_fb(I[i], J[i], prev[i], init[i], params=op, reuse_pyramids=True)
        _assert_same(g["next"][i], o["next"], f"pair {i} next")
        _assert_same(g["back"][i], o["back"], f"pair {i} back")
        flags = o["st_f"] | (o["st_b"] << 1) | (o["keep"] << 2)
        _assert_same(g["flags"][i], flags, f"pair {i} flags")
        _assert_same(g["kept"][i][:g["n_kept"][i]], o["kept_idx"], f"pair {i} kept")
        assert (flags[0::3] | flags[1::3] | flags[2::3]).any() and not o["st_f"].all()


@pytest.mark.parametrize("n_pairs,n_pts", [(1, 1), (3, 64), (5, 65), (2, 130), (27, 150)])
def test_fused_compaction_matches_two_launches(ctx, orc, gvx_mod, monkeypatch, n_pairs, n_pts):
    """One point per wave (n_pairs * n_pts <= 4096): the LK launch compacts by
    itself (klt.hip fused_compact).  Its kept_idx / n_kept must equal the
    compact_kernel launch's (a context made with GVX_FUSED_COMPACT=0) over
    repeated launches -- the keep words and arrival counts are left zero for the
    next one -- and, for the first pairs, the oracle's reduceVector."""
    monkeypatch.setenv("GVX_FUSED_COMPACT", "0")
    ref = gvx_mod.Context(0)
    monkeypatch.delenv("GVX_FUSED_COMPACT")
    try:
        for rep in range(3):
            I, J, prev, init = synth.make_batch(n_pairs, 320, 140, n_pts, seed=100 + 7 * rep + n_pts)
            g = ctx.klt_fb_batch(I, J, prev, init)
            r = ref.klt_fb_batch(I, J, prev, init)
            for k in g:
                if k != "kept":  # entries past n_kept are whatever the buffer held
                    _assert_same(g[k], r[k], f"rep {rep} {k}")
            for i in range(n_pairs):
                _assert_same(g["kept"][i][:g["n_kept"][i]], r["kept"][i][:r["n_kept"][i]], f"rep {rep} pair {i}")
            for i in range(min(n_pairs, 2)):
                o = orc.klt_fb(I[i], J[i], prev[i], init[i], reuse_pyramids=True)
                assert g["n_kept"][i] == len(o["kept_idx"])
                _assert_same(g["kept"][i][:g["n_kept"][i]], o["kept_idx"], f"rep {rep} pair {i} kept")
            assert int(np.sum(g["n_kept"])) > 0
    finally:
        ref.close()

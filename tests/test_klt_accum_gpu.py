"""GPU parity of LK's OpenCV fp32 window-sum orders (gvx_klt_params.accum,
include/gvx.h GVX_LK_ACCUM_*): the device's F32_SCALAR and F32_SIMD4 modes
against the CPU restatement in the same order (oracle/klt.c orc_set_lk_accum:
ORC_ACC_F32 = OpenCV 4.x's scalar loop, ORC_ACC_F32X4 = its CV_SIMD128 path),
BIT-EXACT in flow, status, err, FB flags and kept indices.  The reference calls
cv::calcOpticalFlowPyrLK at ic_gvins/ic_gvins/tracking/tracking.cc:385-393 and
:487-496; SURVEY.md Appendix A.3 holds the spec these orders restate."""
import numpy as np
import pytest

from gvx import synth

pytestmark = pytest.mark.gpu

MODES = [pytest.param(1, id="f32_scalar"), pytest.param(2, id="f32_simd4")]


def _assert_same(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    if not np.array_equal(a, b):
        diff = np.argwhere(a != b)
        raise AssertionError(f"{what}: {len(diff)} mismatches, first at {diff[:5].tolist()}: "
                             f"gpu={a[tuple(diff[0])]} oracle={b[tuple(diff[0])]}")


def _orc_mode(orc, mode):
    return orc.lk_accum({1: orc.ACC_F32, 2: orc.ACC_F32X4}[mode])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("w,h,n,L,seed", [(160, 70, 32, 3, 1), (1280, 560, 150, 3, 20261015),
                                          (1920, 1200, 500, 4, 5)])
def test_calc_optical_flow_f32_orders(ctx, orc, gvx_mod, mode, w, h, n, L, seed):
    I, J, prev, init, _ = synth.make_pair(w, h, n, seed)
    p = gvx_mod.KltParams.default(max_level=L, accum=mode)
    ctx.frame_put(1, I, p)
    ctx.frame_put(2, J, p)
    g_next, g_st, g_err = ctx.calc_optical_flow_pyr_lk(1, 2, prev, init, p)
    with _orc_mode(orc, mode):
        o_next, o_st, o_err = orc.calc_optical_flow_pyr_lk(I, J, prev, init, orc.KltParams.default(max_level=L))
    _assert_same(g_st, o_st, "status")
    _assert_same(g_next, o_next, "nextPts")
    _assert_same(g_err[o_st == 1], o_err[o_st == 1], "err")


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("w,h,n,L,seed", [(1280, 560, 150, 3, 20261015), (1920, 1200, 500, 4, 20261016)])
def test_track_fb_f32_orders(ctx, orc, gvx_mod, mode, w, h, n, L, seed):
    I, J, prev, init, _ = synth.make_pair(w, h, n, seed)
    p = gvx_mod.KltParams.default(max_level=L, accum=mode)
    ctx.frame_put(1, I, p)
    ctx.frame_put(2, J, p)
    g = ctx.track_fb(1, 2, prev, init, w, h, params=p)
    with _orc_mode(orc, mode):
        o = orc.klt_fb(I, J, prev, init, w, h, params=orc.KltParams.default(max_level=L))
    for k in ("next", "back", "st_f", "st_b", "keep", "kept_idx"):
        _assert_same(g[k], o[k], k)
    # the order really is different from the exact one on these inputs
    e = ctx.track_fb(1, 2, prev, init, w, h, params=gvx_mod.KltParams.default(max_level=L))
    assert not np.array_equal(e["next"], g["next"]) or not np.array_equal(e["back"], g["back"])


def _border_points(w, h, n, rng):
    side = rng.integers(0, 4, n)
    t = rng.uniform(-30, 30, n)
    pts = np.empty((n, 2), np.float32)
    pts[:, 0] = np.where(side == 0, t, np.where(side == 1, w - 1 - t, rng.uniform(0, w, n)))
    pts[:, 1] = np.where(side == 2, t, np.where(side == 3, h - 1 - t, rng.uniform(0, h, n)))
    pts[:4] = [[0.5, 0.5], [w - 1.5, h - 1.5], [w / 2, h / 2], [3.25, h - 4.75]]
    return pts


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("n_pairs,n_pts,w,h,L", [(64, 149, 320, 140, 3), (3, 96, 1280, 560, 3),
                                                 (3, 2731, 320, 140, 2)])
def test_batch_f32_orders(ctx, orc, gvx_mod, mode, n_pairs, n_pts, w, h, L):
    """Batched path (level 0 read in place, REFLECT_101 gathers at the border):
    one point per wave (3 x 96) and two per wave (> 4096 points, odd counts
    leave a spare lane group in a pair's last wave)."""
    rng = np.random.default_rng(n_pairs * 31 + n_pts + mode)
    I = np.stack([synth.make_image(w, h, rng) for _ in range(n_pairs)])
    J = np.stack([np.roll(I[i], (1, -2), axis=(0, 1)) for i in range(n_pairs)])
    prev = np.stack([np.concatenate([_border_points(w, h, 20, rng),
                                     rng.uniform([0, 0], [w, h], (n_pts - 20, 2)).astype(np.float32)])
                     for _ in range(n_pairs)])
    init = (prev + rng.uniform(-1.5, 1.5, prev.shape)).astype(np.float32)
    g = ctx.klt_fb_batch(I, J, prev, init, params=gvx_mod.KltParams.default(max_level=L, accum=mode))
    with _orc_mode(orc, mode):
        for i in range(0, n_pairs, max(1, n_pairs // 8)):
            o = orc.klt_fb(I[i], J[i], prev[i], init[i], params=orc.KltParams.default(max_level=L),
                           reuse_pyramids=True, nthreads=4)
            _assert_same(g["next"][i], o["next"], f"pair {i} next")
            _assert_same(g["back"][i], o["back"], f"pair {i} back")
            flags = o["st_f"] | (o["st_b"] << 1) | (o["keep"] << 2)
            _assert_same(g["flags"][i], flags, f"pair {i} flags")
            _assert_same(g["kept"][i][:g["n_kept"][i]], o["kept_idx"], f"pair {i} kept")


@pytest.mark.parametrize("mode", MODES)
def test_edge_points_f32_orders(ctx, orc, gvx_mod, mode):
    """Points at / beyond the border, far outside, and on a flat patch (the
    minEig gate sees the fp32 sums)."""
    I, J, _, _, _ = synth.make_pair(320, 140, 8, seed=9)
    I[40:80, 200:260] = 77
    J[40:80, 200:260] = 77
    prev = np.array([[0, 0], [319.9, 139.9], [-25, 10], [10, -25], [1000, 50], [230, 60], [5, 70],
                     [315, 5], [160.5, 70.25], [-21.0, -21.0], [330.0, 150.0]], np.float32)
    init = prev + np.float32(0.7)
    p = gvx_mod.KltParams.default(accum=mode)
    ctx.frame_put(1, I, p)
    ctx.frame_put(2, J, p)
    g = ctx.track_fb(1, 2, prev, init, 320, 140, params=p)
    with _orc_mode(orc, mode):
        o = orc.klt_fb(I, J, prev, init)
    for k in ("next", "back", "st_f", "st_b", "keep", "kept_idx"):
        _assert_same(g[k], o[k], k)


def test_unknown_accum_refused(ctx, gvx_mod):
    I, J, prev, init, _ = synth.make_pair(160, 70, 4, seed=2)
    ctx.frame_put(1, I)
    ctx.frame_put(2, J)
    with pytest.raises(gvx_mod.GvxError):
        ctx.calc_optical_flow_pyr_lk(1, 2, prev, init, gvx_mod.KltParams.default(accum=7))

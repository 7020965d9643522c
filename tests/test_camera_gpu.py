"""GPU parity of the per-point camera operations (libgvx.so via the C ABI)
against the CPU restatement (oracle/camera.c): float pixel outputs BIT-EXACT,
fp64 velocities / parallaxes equal to the last bit (same operation order, IEEE
division and square root on both sides, no FMA contraction)."""
import numpy as np
import pytest

import oracle as orc_mod

pytestmark = pytest.mark.gpu

CAMS = {
    # config/gvins.yaml:65-73 (KAIST), and a skewed 5-term camera
    "kaist": (787.1611861559479, 787.3928431375225, 664.4061078354368, 519.5129292754456, 0.0,
              -0.0917403092279957, 0.08134715036932794, 0.00017620136958692255, 0.00016737385248865412, 0.0,
              1278, 1022),
    "skew_k3": (610.5, 612.25, 640.3, 281.7, 0.35, -0.21, 0.04, -0.0011, 0.0007, 0.012, 1280, 560),
}


def _cams(gvx_mod, name):
    v = CAMS[name]
    return gvx_mod.Camera(*v), orc_mod.Camera(*v)


def _pts(n, seed, w, h, margin=0):
    rng = np.random.default_rng(seed)
    return np.c_[rng.uniform(-margin, w + margin, n), rng.uniform(-margin, h + margin, n)].astype(np.float32)


def _rot(seed, ang=0.05):
    rng = np.random.default_rng(seed)
    k = rng.normal(size=3)
    k /= np.linalg.norm(k)
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    a = rng.uniform(-ang, ang)
    return np.eye(3) + np.sin(a) * K + (1 - np.cos(a)) * K @ K


@pytest.mark.parametrize("name", list(CAMS))
@pytest.mark.parametrize("n", [0, 1, 150, 1000])
def test_point_ops_bit_exact(ctx, gvx_mod, name, n):
    gc, oc = _cams(gvx_mod, name)
    p = _pts(n, n + 1, gc.width, gc.height, margin=30)
    q = p + _pts(n, n + 2, 6, 6) - 3
    assert np.array_equal(ctx.undistort_points(gc, p), orc_mod.undistort_points(oc, p))
    assert np.array_equal(ctx.distort_points(gc, p), orc_mod.distort_points(oc, p))
    R = _rot(n)
    assert np.array_equal(ctx.predict_rotated(gc, R, p), orc_mod.predict_rotated(oc, R, p))
    assert np.array_equal(ctx.point_velocity(gc, p, q, 0.05), orc_mod.point_velocity(oc, p, q, 0.05))
    R0, R1 = _rot(n + 3, 0.5), _rot(n + 4, 0.5)
    assert np.array_equal(ctx.keypoint_parallax(gc, R0, R1, p, q), orc_mod.keypoint_parallax(oc, R0, R1, p, q))


@pytest.mark.parametrize("name", list(CAMS))
def test_project_points_bit_exact(ctx, gvx_mod, name):
    gc, oc = _cams(gvx_mod, name)
    rng = np.random.default_rng(9)
    R, t = _rot(11, 1.0), rng.normal(size=3) * 5
    pc = np.c_[rng.uniform(-8, 8, 400), rng.uniform(-4, 4, 400), rng.uniform(3, 60, 400)]
    pw = pc @ R.T + t
    assert np.array_equal(ctx.project_points(gc, R, t, pw), orc_mod.project_points(oc, R, t, pw))


def test_camera_ops_dev_match_host(ctx, gvx_mod):
    import ctypes as C
    import torch
    gc, _ = _cams(gvx_mod, "kaist")
    p = _pts(300, 5, gc.width, gc.height)
    dp = torch.from_numpy(p).cuda()
    out = torch.empty_like(dp)
    L = gvx_mod.lib()
    assert L.gvx_undistort_points_dev(ctx.handle, C.byref(gc), len(p), dp.data_ptr(), out.data_ptr()) == 0
    ctx.sync()
    assert np.array_equal(out.cpu().numpy(), ctx.undistort_points(gc, p))


def test_camera_rejects_bad_input(ctx, gvx_mod):
    bad = gvx_mod.Camera(0.0, 1.0, 0, 0, 0, 0, 0, 0, 0, 0, 10, 10)
    with pytest.raises(gvx_mod.GvxError):
        ctx.undistort_points(bad, np.zeros((3, 2), np.float32))

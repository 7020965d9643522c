"""The CPU restatement of the per-point camera operations around the KLT calls
(oracle/camera.c) against closed forms, round trips and an independent numpy
restatement.  OpenCV/Eigen are absent here, so it is "parity unpinned" against
cv::undistortPoints itself; the camera is the reference's own
(config/gvins.yaml:65-73)."""
import numpy as np
import pytest

import oracle as orc


def kaist_camera(skew=0.0, k3=0.0):
    """config/gvins.yaml:65-73 (4 distortion terms -> k3 = 0, camera.cc:62-64)."""
    return orc.Camera(787.1611861559479, 787.3928431375225, 664.4061078354368, 519.5129292754456, skew,
                      -0.0917403092279957, 0.08134715036932794, 0.00017620136958692255, 0.00016737385248865412,
                      k3, 1278, 1022)


def _pts(n, seed, w=1278, h=1022):
    rng = np.random.default_rng(seed)
    return np.c_[rng.uniform(0, w, n), rng.uniform(0, h, n)].astype(np.float32)


def _np_undistort(c, p):
    """numpy restatement of cvUndistortPointsInternal (COUNT 5, R = I, P = K)."""
    u, v = p[:, 0].astype(np.float64), p[:, 1].astype(np.float64)
    x = (u - c.cx) * (1.0 / c.fx)
    y = (v - c.cy) * (1.0 / c.fy)
    x0, y0 = x.copy(), y.copy()
    for _ in range(5):
        r2 = x * x + y * y
        icd = 1 / (1 + ((c.k3 * r2 + c.k2) * r2 + c.k1) * r2)
        dx = 2 * c.p1 * x * y + c.p2 * (r2 + 2 * x * x)
        dy = c.p1 * (r2 + 2 * y * y) + 2 * c.p2 * x * y
        x, y = (x0 - dx) * icd, (y0 - dy) * icd
    return np.c_[c.fx * x + c.skew * y + c.cx, c.fy * y + c.cy].astype(np.float32)


@pytest.mark.parametrize("skew,k3", [(0.0, 0.0), (0.7, 0.01)])
def test_undistort_matches_numpy(skew, k3):
    c = kaist_camera(skew, k3)
    p = _pts(500, 1)
    assert np.array_equal(orc.undistort_points(c, p), _np_undistort(c, p))


def test_distort_undistort_round_trip():
    """5 fixed-point steps invert the mild KAIST distortion to far below 1e-2 px
    inside the image."""
    c = kaist_camera()
    p = _pts(1000, 2)
    back = orc.undistort_points(c, orc.distort_points(c, p))
    assert np.abs(back - p).max() < 1e-2


def test_zero_distortion_is_identity():
    c = orc.Camera(500.0, 510.0, 320.0, 240.0, 0.0, 0, 0, 0, 0, 0, 640, 480)
    p = _pts(200, 3, 640, 480)
    assert np.abs(orc.undistort_points(c, p) - p).max() <= 1e-4
    assert np.abs(orc.distort_points(c, p) - p).max() <= 1e-4


def test_predict_rotated_identity_and_known_rotation():
    c = kaist_camera()
    p = _pts(300, 4)
    same = orc.predict_rotated(c, np.eye(3), p)
    assert np.abs(same - p).max() < 1e-2  # distort(undistort(p))
    # a pure yaw of a undistorted camera shifts the principal point by f*tan(a)
    c0 = orc.Camera(600.0, 600.0, 400.0, 300.0, 0.0, 0, 0, 0, 0, 0, 800, 600)
    a = 0.01
    R = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    q = orc.predict_rotated(c0, R, np.array([[400.0, 300.0]], np.float32))
    assert q[0, 0] == pytest.approx(400 + 600 * np.tan(a), abs=1e-3) and q[0, 1] == pytest.approx(300, abs=1e-4)


def test_project_points_known_answer():
    c0 = orc.Camera(600.0, 600.0, 400.0, 300.0, 0.0, 0, 0, 0, 0, 0, 800, 600)
    rng = np.random.default_rng(5)
    R = np.linalg.qr(rng.normal(size=(3, 3)))[0]
    R *= np.sign(np.linalg.det(R))
    t = rng.normal(size=3)
    pc = np.c_[rng.uniform(-2, 2, 50), rng.uniform(-1.5, 1.5, 50), rng.uniform(4, 30, 50)]
    pw = pc @ R.T + t  # pose.R * pc + pose.t (cam2world)
    got = orc.project_points(c0, R, t, pw)
    ref = np.c_[600 * pc[:, 0] / pc[:, 2] + 400, 600 * pc[:, 1] / pc[:, 2] + 300]
    assert np.abs(got - ref).max() < 1e-3


def test_velocity_and_parallax():
    c = kaist_camera()
    p = _pts(100, 6)
    assert np.all(orc.point_velocity(c, p, p, 0.05) == 0)
    q = p + np.array([2.0, -1.0], np.float32)
    v = orc.point_velocity(c, p, q, 0.1)
    d = q.astype(np.float64) - p.astype(np.float64)  # the float shift actually stored
    assert v[:, 0] == pytest.approx(d[:, 0] / c.fx / 0.1, rel=1e-12)
    assert v[:, 1] == pytest.approx(d[:, 1] / c.fy / 0.1, rel=1e-12)
    I3 = np.eye(3)
    assert np.all(orc.keypoint_parallax(c, I3, I3, p, p) == 0)
    par = orc.keypoint_parallax(c, I3, I3, p, q)
    f = (c.fx + c.fy) * 0.5
    assert par == pytest.approx(np.hypot(d[:, 0] / c.fx, d[:, 1] / c.fy) * f, rel=1e-9)

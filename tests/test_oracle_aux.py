"""The CPU restatement of the remaining window factors (oracle/aux_factors.c;
GnssFactor, ImuErrorFactor, ImuPosePriorFactor, ImuMixPriorFactor,
MarginalizationFactor) against closed forms and numeric Jacobians on the pose
manifold.  Ceres / Eigen are absent, so it is "parity unpinned" against the
reference binaries."""
import numpy as np
import pytest

import oracle as orc
from gvx import synth_ba


def _pose(rng):
    q = synth_ba.quat_from_rotvec(rng.normal(0, 0.5, 3))
    return np.concatenate([rng.normal(0, 5, 3), q / np.linalg.norm(q)])


def _plus(pose, d):
    """PoseParameterization::Plus: p + dp, q * q(dtheta) (right perturbation)."""
    q = synth_ba.quat_mul(pose[3:], synth_ba.quat_from_rotvec(d[3:6]))
    return np.concatenate([pose[:3] + d[:3], q / np.linalg.norm(q)])


def _numeric_pose_jac(f, pose, m, h=1e-6):
    J = np.zeros((m, 6))
    for k in range(6):
        d = np.zeros(6)
        d[k] = h
        J[:, k] = (f(_plus(pose, d)) - f(_plus(pose, -d))) / (2 * h)
    return J


def test_gnss_closed_form_and_jacobian():
    rng = np.random.default_rng(1)
    blh, std, lever = rng.normal(0, 5, 3), np.array([0.02, 0.03, 0.05]), np.array([0.1, -0.2, 0.3])
    c = np.concatenate([blh, std, lever])
    pose = _pose(rng)
    ident = pose.copy()
    ident[3:] = (0, 0, 0, 1)
    res, _ = orc.small_factor_eval(0, c, ident, [0])
    assert np.allclose(res[0], (1.0 / std) * (ident[:3] + lever - blh), rtol=1e-15, atol=0)
    res, jac = orc.small_factor_eval(0, c, pose, [0])
    J = jac[0].reshape(3, 7)
    f = lambda p: orc.small_factor_eval(0, c, p, [0], jacobians=False)[0][0]
    assert np.allclose(J[:, :6], _numeric_pose_jac(f, pose, 3), rtol=1e-6, atol=1e-4)
    assert np.all(J[:, 6] == 0)


def test_imu_error_closed_form():
    mix = np.arange(1.0, 10.0)
    res, jac = orc.small_factor_eval(1, None, mix, [0])
    gstd, astd = 7200 / 3600.0 * np.pi / 180.0, 2.0e4 * 1.0e-5
    assert np.array_equal(res[0], np.concatenate([mix[3:6] / gstd, mix[6:9] / astd]))
    J = jac[0].reshape(6, 9)
    assert np.array_equal(J[:3, 3:6], np.eye(3) / gstd) and np.array_equal(J[3:, 6:9], np.eye(3) / astd)
    assert np.count_nonzero(J) == 6


def test_pose_prior_zero_at_prior_and_jacobian():
    rng = np.random.default_rng(2)
    prior, std = _pose(rng), np.array([0.1, 0.1, 0.2, 0.01, 0.01, 0.02])
    c = np.concatenate([prior, std])
    res, jac = orc.small_factor_eval(2, c, prior, [0])
    assert np.abs(res).max() < 1e-12
    J = jac[0].reshape(6, 7)
    assert np.allclose(J[:3, :3], np.diag(1 / std[:3])) and np.allclose(J[3:, 3:6], -np.diag(1 / std[3:]))
    pose = _plus(prior, rng.normal(0, 0.05, 6))
    _, jac = orc.small_factor_eval(2, c, pose, [0])
    f = lambda p: orc.small_factor_eval(2, c, p, [0], jacobians=False)[0][0]
    assert np.allclose(jac[0].reshape(6, 7)[:, :6], _numeric_pose_jac(f, pose, 6), rtol=1e-5, atol=1e-3)


def test_mix_prior_closed_form():
    prior, std, mix = np.arange(9.0), np.linspace(0.1, 0.9, 9), np.arange(9.0) + 0.5
    res, jac = orc.small_factor_eval(3, np.concatenate([prior, std]), mix, [0])
    assert np.array_equal(res[0], (mix - prior) / std)
    assert np.array_equal(jac[0].reshape(9, 9), np.diag(1.0 / std))


def _marg_problem(rng, n_kf=9):
    """IC-GVINS-shaped remained blocks: pose[7] + mix[9] per keyframe, extrinsic pose[7], td[1]."""
    size = [7, 9] * n_kf + [7, 1]
    local = [6 if s == 7 else s for s in size]
    index = np.concatenate([[0], np.cumsum(local)[:-1]]).astype(np.int32)
    xoff = np.concatenate([[0], np.cumsum(size)[:-1]]).astype(np.int32)
    r = int(sum(local))
    x0 = np.concatenate([_pose(rng) if s == 7 else rng.normal(0, 1, s) for s in size])
    J0 = rng.normal(0, 1, (r, r))
    e0 = rng.normal(0, 1, r)
    return np.array(size, np.int32), index, xoff, x0, J0, e0


def test_marg_at_linearisation_point_and_linear_blocks():
    rng = np.random.default_rng(3)
    size, index, xoff, x0, J0, e0 = _marg_problem(rng)
    res, jac = orc.marg_factor_eval(size, index, xoff, x0, x0, J0, e0)
    assert np.allclose(res, e0, rtol=0, atol=1e-13)  # q0^-1 q0 is the identity to rounding
    # perturb one mix block only: e0 + J0[:, block] dx exactly as numpy (one column group)
    x = x0.copy()
    b = 3  # a mix block
    dx = rng.normal(0, 0.1, 9)
    x[xoff[b]:xoff[b] + 9] += dx
    res, _ = orc.marg_factor_eval(size, index, xoff, x0, x, J0, e0)
    dfull = np.zeros(J0.shape[0])
    dfull[index[b]:index[b] + 9] = x[xoff[b]:xoff[b] + 9] - x0[xoff[b]:xoff[b] + 9]
    assert np.allclose(res, e0 + J0 @ dfull, rtol=1e-13, atol=1e-13)
    # Jacobians: J0's columns, the pose blocks' 7th column zero
    r = J0.shape[0]
    for b in range(len(size)):
        Jb = jac[r * xoff[b]: r * (xoff[b] + size[b])].reshape(r, size[b])
        loc = 6 if size[b] == 7 else size[b]
        assert np.array_equal(Jb[:, :loc], J0[:, index[b]:index[b] + loc])
        assert not Jb[:, loc:].any()


def test_marg_quaternion_sign_invariance():
    rng = np.random.default_rng(4)
    size, index, xoff, x0, J0, e0 = _marg_problem(rng, n_kf=3)
    x = x0.copy()
    x[xoff[0]:xoff[0] + 7] = _plus(x0[xoff[0]:xoff[0] + 7], rng.normal(0, 0.05, 6))
    a, _ = orc.marg_factor_eval(size, index, xoff, x0, x, J0, e0, jacobians=False)
    x[xoff[0] + 3:xoff[0] + 7] *= -1  # the same rotation: dq.w < 0 branch
    b, _ = orc.marg_factor_eval(size, index, xoff, x0, x, J0, e0, jacobians=False)
    assert np.allclose(a, b, rtol=1e-14, atol=1e-14)

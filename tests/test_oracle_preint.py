"""CPU tests of the preintegration / factor restatement (oracle/preint.c,
oracle/factors.c): analytic known answers and numeric derivatives on the pose
manifold (PoseParameterization::Plus, factors/pose_parameterization.h:34-57).
The reference ships no fixtures for these classes."""
import numpy as np
import pytest

from gvx import synth_ba

NORMAL, EARTH = 0, 2


def _prm(orc):
    return orc.imu_params(*synth_ba.imu_params())


def _state(orc, s):
    return orc.make_state(float(s["time"]), s["p"], s["q"], s["v"], s["bg"], s["ba"])


def _quat_rot(q):
    return synth_ba.quat_to_rot(q)


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_constant_force_known_answer(orc, variant):
    """dtheta = 0, constant body acceleration a, q0 = I, zero biases:
    Dv = a T, Dp = a T^2 / 2, Dq = I; current state by trapezoid integration."""
    m, dt = 51, 0.005
    imu = np.zeros(m, orc.IMU_DTYPE)
    a = np.array([0.3, -0.2, 1.1])
    imu["time"] = np.arange(m) * dt
    imu["dt"] = dt
    imu["dvel"] = a * dt
    v0, p0 = np.array([1.0, 2.0, -0.5]), np.array([10.0, -3.0, 2.0])
    s0 = orc.make_state(0.0, p0, (0, 0, 0, 1), v0)
    seg = orc.PreintSeg(variant, _prm(orc), imu, s0)
    T = (m - 1) * dt
    d = seg.delta()
    np.testing.assert_allclose(d["v"], a * T, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(d["p"], 0.5 * a * T * T, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(d["q"], [0, 0, 0, 1], atol=1e-15)
    assert seg.s.delta_time == pytest.approx(T, rel=1e-14)
    if variant == NORMAL:
        g = np.array([0, 0, synth_ba.NORMAL_GRAVITY])
        c = seg.current()
        np.testing.assert_allclose(c["v"], v0 + (a + g) * T, rtol=1e-12)
        np.testing.assert_allclose(c["p"], p0 + v0 * T + 0.5 * (a + g) * T * T, rtol=1e-12)


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_constant_rate_rotation(orc, variant):
    m, dt = 101, 0.005
    w = np.array([0.1, -0.3, 0.2])
    imu = np.zeros(m, orc.IMU_DTYPE)
    imu["time"] = np.arange(m) * dt
    imu["dt"] = dt
    imu["dtheta"] = w * dt
    seg = orc.PreintSeg(variant, _prm(orc), imu, orc.make_state())
    T = (m - 1) * dt
    q = synth_ba.quat_from_rotvec(w * T)
    np.testing.assert_allclose(seg.delta()["q"], q, atol=1e-13)


def test_earth_with_zero_rate_equals_normal(orc):
    rng = np.random.default_rng(3)
    imu = synth_ba.make_imu_segment(rng, 80)
    s0 = _state(orc, synth_ba.random_state(rng))
    a = orc.PreintSeg(NORMAL, _prm(orc), imu, s0)
    b = orc.PreintSeg(EARTH, _prm(orc), imu, s0, iewn=(0, 0, 0))
    for k in ("p", "v", "q"):
        np.testing.assert_allclose(a.delta()[k], b.delta()[k], rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(a.current()[k], b.current()[k], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(a.jacobian, b.jacobian, rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(a.covariance, b.covariance, rtol=1e-9, atol=1e-22)


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_covariance_symmetric_psd_and_reintegration(orc, variant):
    rng = np.random.default_rng(4)
    imu = synth_ba.make_imu_segment(rng, 100)
    s0 = _state(orc, synth_ba.random_state(rng))
    iewn = orc.earth_iewn(np.zeros(3), np.asarray(s0.p[:]))
    seg = orc.PreintSeg(variant, _prm(orc), imu, s0, iewn)
    P = seg.covariance
    np.testing.assert_allclose(P, P.T, rtol=1e-9, atol=1e-20)
    assert np.linalg.eigvalsh(0.5 * (P + P.T)).min() > -1e-18
    J0, P0, d0 = seg.jacobian.copy(), P.copy(), seg.delta()
    seg.reintegrate(s0)
    assert np.array_equal(J0, seg.jacobian) and np.array_equal(P0, seg.covariance)
    for k in d0:
        assert np.array_equal(np.atleast_1d(d0[k]), np.atleast_1d(seg.delta()[k]))


def test_earth_iewn_quirk(orc):
    """Appendix C.1: station is never set -> origin (0,0,0): lat ~ north / RA."""
    w = 7.2921151467e-5
    i0 = orc.earth_iewn(np.zeros(3), np.zeros(3))
    np.testing.assert_allclose(i0, [w, 0, 0], atol=1e-20)
    i1 = orc.earth_iewn(np.zeros(3), np.array([6378137.0 * 0.1, 0, 0]))
    lat = i1[2] / -w
    assert 0.098 < np.arcsin(lat) < 0.101


def _bias_jacobian_check(orc, variant, which):
    """dDelta/dbias from the propagated jacobian_ vs finite differences."""
    rng = np.random.default_rng(5)
    imu = synth_ba.make_imu_segment(rng, 100)
    s0 = synth_ba.random_state(rng)
    base = orc.PreintSeg(variant, _prm(orc), imu, _state(orc, s0))
    J = base.jacobian
    col = 9 if which == "bg" else 12
    h = 1e-6 if which == "bg" else 1e-5
    for ax in range(3):
        s1 = s0.copy()
        s1[which] = s1[which] + np.eye(3)[ax] * h
        pert = orc.PreintSeg(variant, _prm(orc), imu, _state(orc, s1))
        dp = (pert.delta()["p"] - base.delta()["p"]) / h
        dv = (pert.delta()["v"] - base.delta()["v"]) / h
        # the reference propagates a first-order discrete error-state transition
        # (preintegration_*.cc updateJacobianAndCovariance): O(1/M) ~ 1-3 % at M=100
        jp, jv = J[0:3, col + ax], J[3:6, col + ax]
        assert np.abs(dp - jp).max() < 0.05 * np.abs(jp).max()
        assert np.abs(dv - jv).max() < 0.02 * np.abs(jv).max()


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
@pytest.mark.parametrize("which", ["bg", "ba"])
def test_bias_jacobian_numeric(orc, variant, which):
    _bias_jacobian_check(orc, variant, which)


def _preint_problem(orc, variant, seed=6, noise=0.0):
    rng = np.random.default_rng(seed)
    imu = synth_ba.make_imu_segment(rng, 100)
    s0 = synth_ba.random_state(rng)
    st0 = _state(orc, s0)
    iewn = orc.earth_iewn(np.zeros(3), s0["p"]) * (1.0 if variant == EARTH else 0.0)
    seg = orc.PreintSeg(variant, _prm(orc), imu, st0, iewn)
    c = seg.current()
    pose0 = np.r_[s0["p"], s0["q"]]
    mix0 = np.r_[s0["v"], s0["bg"], s0["ba"]]
    pose1 = np.r_[c["p"], c["q"]] + noise * rng.normal(size=7) * np.r_[np.ones(3), 0.01 * np.ones(4)]
    pose1[3:] /= np.linalg.norm(pose1[3:])
    mix1 = np.r_[c["v"], c["bg"], c["ba"]] + noise * rng.normal(size=9) * 1e-3
    return seg, pose0, mix0, pose1, mix1


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_preint_residual_zero_at_integrated_state(orc, variant):
    seg, p0, m0, p1, m1 = _preint_problem(orc, variant)
    r, _ = seg.evaluate(p0, m0, p1, m1, jacobians=False)
    # whitened residual of a self-consistent state pair is ~0 (the Earth variant's
    # evaluate() uses first-order Earth-rate corrections, so only ~1e-3 sigma)
    assert np.abs(r).max() < (1e-4 if variant == NORMAL else 1e-2)


def _num_jac_local(f, x, local_dim, plus):
    r0 = f(x)
    J = np.zeros((r0.size, local_dim))
    for k in range(local_dim):
        h = 1e-6
        d = np.zeros(local_dim)
        d[k] = h
        dm = -d
        J[:, k] = (f(plus(x, d)) - f(plus(x, dm))) / (2 * h)
    return J


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_preint_jacobians_numeric(orc, variant):
    seg, p0, m0, p1, m1 = _preint_problem(orc, variant, noise=1.0)
    blocks = [p0, m0, p1, m1]
    _, J = seg.evaluate(*blocks)
    for bi in range(4):
        def f(x, bi=bi):
            b = list(blocks)
            b[bi] = x
            return seg.evaluate(*b, jacobians=False)[0]
        if bi in (0, 2):
            Jn = _num_jac_local(f, blocks[bi], 6, orc.pose_plus)
            Ja = J[bi][:, :6]
            assert np.all(J[bi][:, 6] == 0)
        else:
            Jn = _num_jac_local(f, blocks[bi], 9, lambda x, d: x + d)
            Ja = J[bi]
        scale = np.abs(Ja).max()
        # analytic Jacobians of the reference are first-order (bias correction,
        # Earth-rate terms): compare at a relative 1e-3 of the block scale
        assert np.abs(Ja - Jn).max() < 1e-3 * scale + 1e-6, f"block {bi}"


def _reproj_case(orc, seed=7):
    prob = synth_ba.make_ba_problem(seed=seed, n_kf=3, n_lm=5)
    i = 3
    c = prob["consts"][i]
    o = prob["offs"][i]
    prm = prob["params"]
    blocks = [prm[o[0]:o[0] + 7], prm[o[1]:o[1] + 7], prm[o[2]:o[2] + 7], prm[o[3]:o[3] + 1],
              prm[o[4]:o[4] + 1]]
    rc = orc.reproj_const(c["pts0"], c["pts1"], c["vel0"], c["vel1"], c["td0"], c["td1"], c["std"])
    return rc, [b.copy() for b in blocks]


def test_reproj_residual_small_at_truth(orc):
    rc, b = _reproj_case(orc)
    r, _ = orc.reproj_eval(rc, *b, jacobians=False)
    assert np.abs(r).max() < 5.0   # 1-sigma pixel noise in units of std


def test_reproj_jacobians_numeric(orc):
    rc, b = _reproj_case(orc)
    b[4] = np.array([0.003])   # non-zero td so the td Jacobian is exercised
    _, J = orc.reproj_eval(rc, *b)
    for bi in range(5):
        def f(x, bi=bi):
            bb = list(b)
            bb[bi] = x
            return orc.reproj_eval(rc, *bb, jacobians=False)[0]
        if bi < 3:
            Jn = _num_jac_local(f, b[bi], 6, orc.pose_plus)
            Ja = J[bi][:, :6]
            assert np.all(J[bi][:, 6] == 0)
        else:
            Jn = _num_jac_local(f, b[bi], 1, lambda x, d: x + d)
            Ja = J[bi]
        scale = np.abs(Ja).max()
        assert np.abs(Ja - Jn).max() < 1e-5 * scale + 1e-6, f"block {bi}"


def test_pose_plus_normalises(orc):
    x = np.r_[1.0, 2.0, 3.0, 0.0, 0.0, 0.0, 1.0]
    y = orc.pose_plus(x, np.r_[0.1, 0.2, 0.3, 0.01, -0.02, 0.03])
    assert np.linalg.norm(y[3:]) == pytest.approx(1.0, abs=1e-15)
    np.testing.assert_allclose(y[:3], [1.1, 2.2, 3.3])


def test_factor_batches_match_single_evaluations(orc):
    """The threaded CPU-baseline batches (bench.py configs[3] cpu leg) return
    exactly the single-factor evaluations, for any thread count."""
    prob = synth_ba.make_ba_problem(n_kf=4, n_lm=12)
    cs, prm, offs = prob["consts"], prob["params"], prob["offs"]
    r1, j1 = orc.reproj_eval_batch(cs, prm, offs, nthreads=1)
    r4, j4 = orc.reproj_eval_batch(cs, prm, offs, nthreads=4)
    assert np.array_equal(r1, r4) and np.array_equal(j1, j4)
    for i in (0, 5, len(cs) - 1):
        c, o = cs[i], offs[i]
        rc = orc.reproj_const(c["pts0"], c["pts1"], c["vel0"], c["vel1"], c["td0"], c["td1"], c["std"])
        r, J = orc.reproj_eval(rc, prm[o[0]:o[0] + 7], prm[o[1]:o[1] + 7], prm[o[2]:o[2] + 7],
                               prm[o[3]:o[3] + 1], prm[o[4]:o[4] + 1])
        assert np.array_equal(r1[i], r)
        assert np.array_equal(j1[i], np.concatenate([b.ravel() for b in J]))
    rng = np.random.default_rng(3)
    segs, blocks, poffs = [], [], []
    for k in range(3):
        st = synth_ba.random_state(rng)
        s = orc.make_state(float(st["time"]), st["p"], st["q"], st["v"], st["bg"], st["ba"])
        segs.append(orc.PreintSeg(EARTH, orc.imu_params(*synth_ba.imu_params()),
                                  synth_ba.make_imu_segment(rng, 30), s, (7e-5, 0.0, -2e-5)))
        b = [np.r_[st["p"], st["q"]], np.r_[st["v"], st["bg"], st["ba"]],
             np.r_[st["p"] + 1.0, st["q"]], np.r_[st["v"], st["bg"], st["ba"]]]
        poffs.append([32 * k, 32 * k + 7, 32 * k + 16, 32 * k + 23])
        blocks += b
    pp = np.concatenate(blocks)
    pr, pj = orc.preint_factor_eval_batch(segs, pp, np.array(poffs), nthreads=2)
    for k in range(3):
        r, J = segs[k].evaluate(*blocks[4 * k:4 * k + 4])
        assert np.array_equal(pr[k], r)
        assert np.array_equal(pj[k], np.concatenate([b.ravel() for b in J]))

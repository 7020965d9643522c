"""GPU parity of IMU preintegration and the BA factor batches (libgvx.so via the
C ABI) against the CPU restatement (oracle/).

Tolerances (fp64): the reprojection factor uses no transcendental functions and
is required to be bit-exact.  Preintegration and the preintegration factor
evaluate sin/cos (rotvec2quaternion) with ROCm's ocml instead of glibc; every
other operation follows the oracle's order, so they are compared at a relative
1e-10 of each block's magnitude (SURVEY.md 8c parity contract)."""
import numpy as np
import pytest

from gvx import synth_ba

pytestmark = pytest.mark.gpu
NORMAL, EARTH = 0, 2
RTOL = 1e-10


def _close(g, o, what, rtol=RTOL):
    g, o = np.asarray(g, np.float64), np.asarray(o, np.float64)
    scale = max(np.abs(o).max(), 1e-300)
    err = np.abs(g - o).max()
    assert err <= rtol * scale, f"{what}: max |diff| {err:.3e} > {rtol:.0e} * {scale:.3e}"


def _segments(rng, ms):
    segs, states = [], []
    for m in ms:
        segs.append(synth_ba.make_imu_segment(rng, m))
        states.append(synth_ba.random_state(rng))
    return segs, np.array(states)


def _oracle_seg(orc, variant, imu, s, iewn):
    st = orc.make_state(float(s["time"]), s["p"], s["q"], s["v"], s["bg"], s["ba"])
    return orc.PreintSeg(variant, orc.imu_params(*synth_ba.imu_params()), imu, st, iewn)


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_preint_batch_parity(ctx, orc, gvx_mod, variant):
    rng = np.random.default_rng(21 + variant)
    ms = [2, 3, 20, 57, 100, 101, 100, 100]
    segs, states = _segments(rng, ms)
    iewn = np.array([orc.earth_iewn(np.zeros(3), s["p"]) for s in states])
    gstates = np.zeros(len(ms), gvx_mod.STATE_DTYPE)
    for k in ("time", "p", "q", "v", "bg", "ba"):
        gstates[k] = states[k]
    out, pn, pn_off = ctx.preint_integrate(variant, synth_ba.imu_params(), segs, gstates, iewn)
    for i, (imu, s) in enumerate(zip(segs, states)):
        o = _oracle_seg(orc, variant, imu, s, iewn[i])
        g = out[i]
        assert g["m"] == ms[i] and g["variant"] == variant
        # the two-phase form sums dt as a wave prefix sum (the reference adds in
        # sample order): rounding only, ~1e-16 on 100 samples
        assert g["delta_time"] == pytest.approx(o.s.delta_time, rel=1e-14)
        d, c = o.delta(), o.current()
        for k in ("p", "v", "q"):
            _close(g["delta"][k], d[k], f"seg {i} delta.{k}")
            _close(g["current"][k], c[k], f"seg {i} current.{k}")
        _close(g["jacobian"].reshape(15, 15), o.jacobian, f"seg {i} jacobian")
        _close(g["covariance"].reshape(15, 15), o.covariance, f"seg {i} covariance")
        if variant == EARTH and ms[i] > 1:
            _close(pn[pn_off[i]:pn_off[i] + ms[i] - 1], o.pn, f"seg {i} pn")


def test_reproj_bit_exact_config4(ctx, orc, gvx_mod):
    """Config 4 window: 10 keyframes x 200 landmarks = 1800 factors."""
    prob = synth_ba.make_ba_problem()
    cs, prm, offs = prob["consts"], prob["params"], prob["offs"]
    assert len(cs) == 1800
    gres, gjac = ctx.reproj_eval(cs.astype(gvx_mod.REPROJ_DTYPE), prm, offs)
    for i in range(0, len(cs), 7):
        c = cs[i]
        o = offs[i]
        rc = orc.reproj_const(c["pts0"], c["pts1"], c["vel0"], c["vel1"], c["td0"], c["td1"], c["std"])
        blocks = [prm[o[0]:o[0] + 7], prm[o[1]:o[1] + 7], prm[o[2]:o[2] + 7], prm[o[3]:o[3] + 1],
                  prm[o[4]:o[4] + 1]]
        r, J = orc.reproj_eval(rc, *blocks)
        assert np.array_equal(gres[i], r), f"factor {i} residual"
        oj = np.concatenate([J[0].ravel(), J[1].ravel(), J[2].ravel(), J[3].ravel(), J[4].ravel()])
        assert np.array_equal(gjac[i], oj), f"factor {i} jacobian"
    # residual-only call agrees with the full call
    r2, j2 = ctx.reproj_eval(cs.astype(gvx_mod.REPROJ_DTYPE), prm, offs, jacobians=False)
    assert j2 is None and np.array_equal(r2, gres)


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_preint_factor_parity(ctx, orc, gvx_mod, variant):
    rng = np.random.default_rng(31 + variant)
    n = 9
    segs, states = _segments(rng, [100] * n)
    iewn = np.array([orc.earth_iewn(np.zeros(3), s["p"]) for s in states])
    gstates = np.zeros(n, gvx_mod.STATE_DTYPE)
    for k in ("time", "p", "q", "v", "bg", "ba"):
        gstates[k] = states[k]
    out, pn, pn_off = ctx.preint_integrate(variant, synth_ba.imu_params(), segs, gstates, iewn)
    # parameter blocks near the integrated states (perturbed like an LM iterate)
    blocks, offs, oracle_blocks = [], [], []
    base = 0
    for i in range(n):
        s, c = states[i], out[i]["current"]
        p0 = np.r_[s["p"], s["q"]]
        m0 = np.r_[s["v"], s["bg"], s["ba"]] + rng.normal(0, 1e-4, 9)
        p1 = np.r_[c["p"] + rng.normal(0, 0.01, 3), c["q"]]
        m1 = np.r_[c["v"], c["bg"], c["ba"]] + rng.normal(0, 1e-4, 9)
        oracle_blocks.append((p0, m0, p1, m1))
        offs.append([base, base + 7, base + 16, base + 23])
        blocks += [p0, m0, p1, m1]
        base += 32
    params = np.concatenate(blocks)
    gres, gjac = ctx.preint_factor_eval(out, pn, pn_off, params, np.array(offs, np.int32))
    for i in range(n):
        o = _oracle_seg(orc, variant, segs[i], states[i], iewn[i])
        r, J = o.evaluate(*oracle_blocks[i])
        _close(gres[i], r, f"factor {i} residual", rtol=1e-9)
        oj = np.concatenate([J[0].ravel(), J[1].ravel(), J[2].ravel(), J[3].ravel()])
        for b, (lo, hi) in enumerate([(0, 105), (105, 240), (240, 345), (345, 480)]):
            _close(gjac[i][lo:hi], oj[lo:hi], f"factor {i} J{b}", rtol=1e-9)


def test_preint_invalid_variant(ctx, gvx_mod):
    with pytest.raises(gvx_mod.GvxError):
        ctx.preint_integrate(1, synth_ba.imu_params(), [synth_ba.make_imu_segment(np.random.default_rng(0), 5)],
                             np.zeros(1, gvx_mod.STATE_DTYPE))


def test_reproj_bad_offsets_rejected(ctx, gvx_mod):
    prob = synth_ba.make_ba_problem(n_kf=2, n_lm=3)
    offs = prob["offs"].copy()
    offs[0, 0] = 10 ** 6
    with pytest.raises(gvx_mod.GvxError):
        ctx.reproj_eval(prob["consts"].astype(gvx_mod.REPROJ_DTYPE), prob["params"], offs)


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_preint_two_phase_equals_one_phase(ctx, gvx_mod, variant):
    """launch_preint's two-launch form (the per-step terms with the quaternion
    chains as wave-wide prefix products, then the 16-lane covariance pass)
    against the single kernel (sequential chains, the reference's order),
    ragged segments included (the steps past a segment's m run an identity
    record): counts, sample times and biases equal; every float within 1e-12 of
    its block's magnitude (the chains' products and the delta_time sum are
    rounded differently, nothing else; both forms are held to the oracle at
    1e-10 by the tests above)."""
    rng = np.random.default_rng(5 + variant)
    ms = [1, 2, 3, 17, 64, 100, 101, 5, 100, 33, 65, 130]
    segs, states = _segments(rng, ms)
    iewn = np.array([[0.0, 4.1e-5, -5.7e-5]] * len(ms)) + rng.normal(0, 1e-6, (len(ms), 3))
    gstates = np.zeros(len(ms), gvx_mod.STATE_DTYPE)
    for k in ("time", "p", "q", "v", "bg", "ba"):
        gstates[k] = states[k]
    try:
        ctx.set_preint_path(gvx_mod.PREINT_PATH_ONEPHASE)
        o1, pn1, _ = ctx.preint_integrate(variant, synth_ba.imu_params(), segs, gstates, iewn)
    finally:
        ctx.set_preint_path(gvx_mod.PREINT_PATH_AUTO)
    o2, pn2, _ = ctx.preint_integrate(variant, synth_ba.imu_params(), segs, gstates, iewn)
    for name in ("variant", "m", "start_time", "end_time"):
        np.testing.assert_array_equal(o1[name], o2[name], err_msg=name)
    np.testing.assert_allclose(o1["delta_time"], o2["delta_time"], rtol=1e-14, err_msg="delta_time")

    full = np.array(ms) > 3  # P has full rank (sqrt_info exists) from m = 5 on

    def close(a, b, what, rows=None):
        a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
        a, b = a.reshape(len(ms), -1), b.reshape(len(ms), -1)
        if rows is not None:
            a, b = a[rows], b[rows]
        scale = np.maximum(np.abs(a).max(axis=1), 1e-300)
        err = np.abs(a - b).max(axis=1)
        assert np.all(err <= 1e-12 * scale), (what, (err / scale).max())

    for st in ("current", "delta"):
        np.testing.assert_array_equal(o1[st]["time"], o2[st]["time"])
        for f in ("p", "q", "v", "bg", "ba"):
            close(o1[st][f], o2[st][f], f"{st}.{f}")
    for f in ("jacobian", "covariance", "gravity", "iewn", "q0"):
        close(o1[f], o2[f], f)
    close(o1["sqrt_info"], o2["sqrt_info"], "sqrt_info", rows=full)
    if variant == EARTH:
        assert pn1.shape == pn2.shape
        assert np.array_equal(pn1[:, 0], pn2[:, 0])  # dt
        assert np.abs(pn1[:, 1:] - pn2[:, 1:]).max() <= 1e-12 * np.abs(pn1[:, 1:]).max()


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_preint_two_phase_identity_chains_bit_exact(ctx, gvx_mod, variant):
    """with the chain inputs at the identity -- zero gyro increments,
    zero gyro bias, iewn = 0 -- and dyadic sample times (256 Hz, so every
    delta_time partial sum is exact), the quaternion chains are the identity in
    both forms, and the two-launch form must agree with the single kernel bit
    for bit, on ragged segments (identity records past m) included."""
    rng = np.random.default_rng(77 + variant)
    ms = [1, 2, 5, 64, 100, 101, 33]
    segs, states = [], []
    for m in ms:
        imu = synth_ba.make_imu_segment(rng, m, rate=256.0)
        imu["dtheta"] = 0.0
        segs.append(imu)
        s = synth_ba.random_state(rng)
        s["bg"] = 0.0
        states.append(s)
    states = np.array(states)
    iewn = np.zeros((len(ms), 3))
    gstates = np.zeros(len(ms), gvx_mod.STATE_DTYPE)
    for k in ("time", "p", "q", "v", "bg", "ba"):
        gstates[k] = states[k]
    try:
        ctx.set_preint_path(gvx_mod.PREINT_PATH_ONEPHASE)
        o1, pn1, _ = ctx.preint_integrate(variant, synth_ba.imu_params(), segs, gstates, iewn)
    finally:
        ctx.set_preint_path(gvx_mod.PREINT_PATH_AUTO)
    o2, pn2, _ = ctx.preint_integrate(variant, synth_ba.imu_params(), segs, gstates, iewn)
    for name in ("variant", "m", "start_time", "end_time", "delta_time"):
        np.testing.assert_array_equal(o1[name], o2[name], err_msg=name)
    for st in ("current", "delta"):
        for f in ("time", "q", "bg", "ba"):
            np.testing.assert_array_equal(o1[st][f], o2[st][f], err_msg=f"{st}.{f}")
    if variant == EARTH:
        assert np.array_equal(pn1, pn2)

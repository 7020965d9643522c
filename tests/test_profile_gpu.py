"""Profiling on (gvx_profile): the timed kernels then launch through
hipExtLaunchKernel with start / stop events on their own dispatch (launch_timed,
csrc/gvx_internal.h) instead of hipLaunchKernelGGL.  The bench reports those
timings, so the launch path it times must compute the same bits as the plain
one: batch KLT (pyramid + LK + compaction), both BA factor kernels and a small
factor kind, each with profiling off and on."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _with_profile(ctx, on, fn):
    ctx.profile_reset()
    ctx.profile(on)
    try:
        out = fn()
        ctx.sync()
        fams = {f: ctx.profile_read(f) for f in ("pyramid", "klt", "compact", "reproj", "preint_factor",
                                                 "aux_factor")}
    finally:
        ctx.profile(False)
    return out, fams


@pytest.mark.parametrize("n_pts", [96, 1100])
def test_klt_batch_profiled_launch_bits(ctx, n_pts):
    """96 points a pair: one point per wave, the compaction inside the LK launch (no
    compact launch); 1,100: three points per wave, a compact_kernel launch."""
    from gvx import synth
    I, J, P, Q = synth.make_batch(4, 640, 280, n_pts, seed=synth.SEED, distinct=4)
    off, _ = _with_profile(ctx, False, lambda: ctx.klt_fb_batch(I, J, P, Q))
    on, fams = _with_profile(ctx, True, lambda: ctx.klt_fb_batch(I, J, P, Q))
    for k in off:
        if k == "kept":  # past n_kept: whatever the buffer held
            for i in range(len(off["n_kept"])):
                m = int(off["n_kept"][i])
                assert np.array_equal(np.asarray(off[k][i][:m]), np.asarray(on[k][i][:m])), k
            continue
        assert np.array_equal(np.asarray(off[k]), np.asarray(on[k])), k
    fused = 4 * n_pts <= 4096
    for f in ("pyramid", "klt") + (() if fused else ("compact",)):
        ms, n = fams[f]
        assert n >= 1 and ms > 0.0, (f, ms, n)
    if fused:
        assert fams["compact"][1] == 0


def test_factor_kernels_profiled_launch_bits(ctx, gvx_mod):
    from gvx import synth_ba
    prob = synth_ba.make_ba_problem()
    cs, prm, offs = prob["consts"][:300].astype(gvx_mod.REPROJ_DTYPE), prob["params"], prob["offs"][:300]
    r_off, _ = _with_profile(ctx, False, lambda: ctx.reproj_eval(cs, prm, offs))
    r_on, fams = _with_profile(ctx, True, lambda: ctx.reproj_eval(cs, prm, offs))
    for a, b in zip(r_off, r_on):
        assert np.array_equal(a, b)
    assert fams["reproj"][1] >= 1 and fams["reproj"][0] > 0.0

    rng = np.random.default_rng(7)
    n_kf = prob["poses"].shape[0]
    segs = [synth_ba.make_imu_segment(rng, 40, t0=0.5 * k) for k in range(n_kf - 1)]
    states = np.zeros(n_kf - 1, gvx_mod.STATE_DTYPE)
    for k in range(n_kf - 1):
        states[k]["time"] = 0.5 * k
        states[k]["p"] = prob["poses"][k, :3]
        states[k]["q"] = prob["poses"][k, 3:]
        states[k]["v"] = [5.0, 0.0, 0.0]
    iewn = np.array([gvx_mod.earth_iewn(np.zeros(3), st["p"]) for st in states])
    pre, pn, pn_off = ctx.preint_integrate(2, synth_ba.imu_params(), segs, states, iewn)
    mix = np.zeros((n_kf, 9))
    mix[:, 0] = 5.0
    params = np.concatenate([prm, mix.reshape(-1)])
    o_mix = prm.size
    poffs = np.array([[7 * k, o_mix + 9 * k, 7 * (k + 1), o_mix + 9 * (k + 1)] for k in range(n_kf - 1)], np.int32)
    p_off, _ = _with_profile(ctx, False, lambda: ctx.preint_factor_eval(pre, pn, pn_off, params, poffs))
    p_on, fams = _with_profile(ctx, True, lambda: ctx.preint_factor_eval(pre, pn, pn_off, params, poffs))
    for a, b in zip(p_off, p_on):
        assert np.array_equal(a, b)
    assert fams["preint_factor"][1] >= 1 and fams["preint_factor"][0] > 0.0


def test_small_factor_profiled_launch_bits(ctx, gvx_mod):
    kind = next(k for k, (_, _, nc) in gvx_mod.SMALL_FACTOR_DIMS.items() if nc == 0)
    _, P, _ = gvx_mod.SMALL_FACTOR_DIMS[kind]
    rng = np.random.default_rng(11)
    n = 200
    params = rng.normal(0, 1, P * (n + 3))
    offs = (rng.permutation(n + 3)[:n] * P).astype(np.int32)
    off, _ = _with_profile(ctx, False, lambda: ctx.small_factor_eval(kind, None, params, offs))
    on, fams = _with_profile(ctx, True, lambda: ctx.small_factor_eval(kind, None, params, offs))
    for a, b in zip(off, on):
        assert np.array_equal(a, b)
    assert fams["aux_factor"][1] >= 1 and fams["aux_factor"][0] > 0.0

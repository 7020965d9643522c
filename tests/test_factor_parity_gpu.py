"""fp64 factor parity at the survey's contract (preintegration
and factors within 1e-10 relative) with BOTH sides fed the SAME preintegration
result -- the oracle's (oracle/preint.c restating preintegration_earth.cc:205-303)
-- so integration error does not compound into the factor comparison:

* PreintegrationFactor::Evaluate (preintegration_factor.h:45-69 ->
  preintegration_earth.cc:37-164, preintegration_normal.cc:38-142): residual and
  the four Jacobian blocks at 1e-10 of each block's magnitude, both variants,
  ragged M;
* the whole configs[3] window (9 Earth preintegration + 1,800 reprojection
  factors, ic_gvins.cc:1207 / :1946-1971): reprojection bit-exact, preintegration
  at 1e-10;
* the replicated batch bench.py times (583 copies of the window: 5,247
  preintegration + 1,049,400 reprojection factors through
  gvx_factor_batch_eval_dev, the MFMA-whitened kernel), 1,000 sampled factors
  of each kind."""
import numpy as np
import pytest

from gvx import synth_ba

pytestmark = pytest.mark.gpu
NORMAL, EARTH = 0, 2
RTOL = 1e-10
BLOCKS = [(0, 105), (105, 240), (240, 345), (345, 480)]


def _close(g, o, what, rtol=RTOL):
    g, o = np.asarray(g, np.float64), np.asarray(o, np.float64)
    scale = max(np.abs(o).max(), 1e-300)
    err = np.abs(g - o).max()
    assert err <= rtol * scale, f"{what}: max |diff| {err:.3e} > {rtol:.0e} * {scale:.3e}"
    return err / scale


def _oracle_seg(orc, variant, imu, s, iewn):
    st = orc.make_state(float(s["time"]), s["p"], s["q"], s["v"], s["bg"], s["ba"])
    return orc.PreintSeg(variant, orc.imu_params(*synth_ba.imu_params()), imu, st, iewn)


def _records(ctx, gvx_mod, segs):
    """gvx_preint_result records (and the pn_ list) holding the oracle's
    preintegration; sqrt_info formed by the device from that covariance."""
    rec = np.zeros(len(segs), gvx_mod.PREINT_DTYPE)
    pns, off = [], []
    base = 0
    for i, o in enumerate(segs):
        s = o.s
        rec["variant"][i], rec["m"][i] = s.variant, s.m
        rec["delta_time"][i], rec["start_time"][i], rec["end_time"][i] = s.delta_time, s.start_time, s.end_time
        for name, st in (("current", o.current()), ("delta", o.delta())):
            for k in ("time", "p", "q", "v", "bg", "ba"):
                rec[name][k][i] = st[k]
        rec["gravity"][i] = np.array(s.gravity[:])
        rec["iewn"][i] = np.array(s.iewn[:])
        rec["q0"][i] = np.array(s.q0[:])
        rec["jacobian"][i] = o.jacobian.ravel()
        rec["covariance"][i] = o.covariance.ravel()
        pn = o.pn if s.m > 1 else np.zeros((0, 4))
        pns.append(pn)
        off.append(base)
        base += len(pn)
    rec = ctx.preint_sqrt_info(rec)
    pn = np.concatenate(pns) if base else np.zeros((1, 4))
    return rec, pn, np.array(off, np.int32)


def _blocks_near(rng, states, segs):
    blocks, offs, ob = [], [], []
    base = 0
    for s, o in zip(states, segs):
        c = o.current()
        p0 = np.r_[s["p"], s["q"]]
        m0 = np.r_[s["v"], s["bg"], s["ba"]] + rng.normal(0, 1e-4, 9)
        p1 = np.r_[c["p"] + rng.normal(0, 0.01, 3), c["q"]]
        m1 = np.r_[c["v"], c["bg"], c["ba"]] + rng.normal(0, 1e-4, 9)
        ob.append((p0, m0, p1, m1))
        offs.append([base, base + 7, base + 16, base + 23])
        blocks += [p0, m0, p1, m1]
        base += 32
    return np.concatenate(blocks), np.array(offs, np.int32), ob


def _check_factor(gres, gjac, o, blocks, what):
    r, J = o.evaluate(*blocks)
    worst = _close(gres, r, f"{what} residual")
    oj = np.concatenate([j.ravel() for j in J])
    for b, (lo, hi) in enumerate(BLOCKS):
        worst = max(worst, _close(gjac[lo:hi], oj[lo:hi], f"{what} J{b}"))
    return worst


@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_preint_factor_oracle_input(ctx, orc, gvx_mod, variant):
    rng = np.random.default_rng(41 + variant)
    ms = [100] * 9 + [5, 20, 57, 101]  # m <= 3: P is rank-deficient, no sqrt_info (nor in the reference)
    states = [synth_ba.random_state(rng) for _ in ms]
    imus = [synth_ba.make_imu_segment(rng, m) for m in ms]
    iewn = [orc.earth_iewn(np.zeros(3), s["p"]) for s in states]
    segs = [_oracle_seg(orc, variant, imu, s, w) for imu, s, w in zip(imus, states, iewn)]
    rec, pn, pn_off = _records(ctx, gvx_mod, segs)
    params, offs, ob = _blocks_near(rng, states, segs)
    gres, gjac = ctx.preint_factor_eval(rec, pn, pn_off, params, offs)
    for i, o in enumerate(segs):
        _check_factor(gres[i], gjac[i], o, ob[i], f"factor {i} (m={ms[i]})")
    # residual-only evaluation agrees with the full one
    r2, _ = ctx.preint_factor_eval(rec, pn, pn_off, params, offs, jacobians=False)
    assert np.array_equal(r2, gres)


def _window(orc, gvx_mod):
    """bench.py factor_leg's configs[3] window: poses, 9 Earth segments of M = 100
    between consecutive keyframes, the mix blocks, and both factor lists."""
    prob = synth_ba.make_ba_problem()
    n_kf = prob["poses"].shape[0]
    rng = np.random.default_rng(20261015)
    M = 100
    imus = [synth_ba.make_imu_segment(rng, M, t0=0.5 * k) for k in range(n_kf - 1)]
    states = np.zeros(n_kf - 1, gvx_mod.STATE_DTYPE)
    for k in range(n_kf - 1):
        states[k]["time"] = 0.5 * k
        states[k]["p"] = prob["poses"][k, :3]
        states[k]["q"] = prob["poses"][k, 3:]
        states[k]["v"] = [5.0, 0.0, 0.0]
    iewn = [orc.earth_iewn(np.zeros(3), st["p"]) for st in states]
    segs = [_oracle_seg(orc, EARTH, imu, s, w) for imu, s, w in zip(imus, states, iewn)]
    mix = np.zeros((n_kf, 9))
    mix[:, 0] = 5.0
    params = np.concatenate([prob["params"], mix.reshape(-1)])
    o_mix = prob["params"].size
    poffs = np.array([[7 * k, o_mix + 9 * k, 7 * (k + 1), o_mix + 9 * (k + 1)] for k in range(n_kf - 1)], np.int32)
    return prob, segs, params, poffs


def _oracle_reproj(orc, prm, c, o):
    rc = orc.reproj_const(c["pts0"], c["pts1"], c["vel0"], c["vel1"], c["td0"], c["td1"], c["std"])
    r, J = orc.reproj_eval(rc, prm[o[0]:o[0] + 7], prm[o[1]:o[1] + 7], prm[o[2]:o[2] + 7], prm[o[3]:o[3] + 1],
                           prm[o[4]:o[4] + 1])
    return r, np.concatenate([j.ravel() for j in J])


def _pblocks(params, o):
    return (params[o[0]:o[0] + 7], params[o[1]:o[1] + 9], params[o[2]:o[2] + 7], params[o[3]:o[3] + 9])


def test_configs3_window_parity(ctx, orc, gvx_mod):
    prob, segs, params, poffs = _window(orc, gvx_mod)
    rec, pn, pn_off = _records(ctx, gvx_mod, segs)
    gres, gjac = ctx.preint_factor_eval(rec, pn, pn_off, params, poffs)
    worst = 0.0
    for i, o in enumerate(segs):
        worst = max(worst, _check_factor(gres[i], gjac[i], o, _pblocks(params, poffs[i]), f"preint {i}"))
    cs, offs = prob["consts"], prob["offs"]
    assert len(cs) == 1800
    rres, rjac = ctx.reproj_eval(cs.astype(gvx_mod.REPROJ_DTYPE), params, offs)
    for i in range(len(cs)):
        r, oj = _oracle_reproj(orc, params, cs[i], offs[i])
        assert np.array_equal(rres[i], r), f"reprojection {i} residual"
        assert np.array_equal(rjac[i], oj), f"reprojection {i} jacobian"
    print(f"configs[3] window: worst preint factor relative error {worst:.3e}")


def test_bench_batch_sampled(ctx, orc, gvx_mod):
    """The factor batch bench.py times, built the same way (583 replicas of the
    window, shared parameter blocks), evaluated by gvx_factor_batch_eval_dev;
    1,000 sampled factors of each kind against the oracle."""
    import torch
    prob, segs, params, poffs = _window(orc, gvx_mod)
    rec, pn, pn_off = _records(ctx, gvx_mod, segs)
    n_rp = len(prob["consts"])
    reps = -(-(1 << 20) // n_rp)
    dev = torch.device("cuda", 0)

    def dev_t(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    d_consts = dev_t(np.tile(prob["consts"].astype(gvx_mod.REPROJ_DTYPE), reps).view(np.uint8))
    d_offs = dev_t(np.tile(prob["offs"], (reps, 1)))
    d_params = dev_t(params)
    n_r = n_rp * reps
    n_p = len(segs) * reps
    d_res = torch.empty((n_r, 2), dtype=torch.float64, device=dev)
    d_jac = torch.empty((n_r, 46), dtype=torch.float64, device=dev)
    d_pre = dev_t(np.tile(rec, reps).view(np.uint8))
    d_pn = dev_t(pn)
    d_pn_off = dev_t(np.tile(pn_off, reps))
    d_poffs = dev_t(np.tile(poffs, (reps, 1)))
    d_pres = torch.empty((n_p, 15), dtype=torch.float64, device=dev)
    d_pjac = torch.empty((n_p, 480), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ctx.factor_batch_eval_dev(n_r, d_consts.data_ptr(), d_offs.data_ptr(), d_res.data_ptr(), d_jac.data_ptr(),
                              n_p, d_pre.data_ptr(), d_pn.data_ptr(), d_pn_off.data_ptr(), d_poffs.data_ptr(),
                              d_pres.data_ptr(), d_pjac.data_ptr(), d_params.data_ptr())
    ctx.sync()
    assert n_p == 5247
    rng = np.random.default_rng(7)
    pres, pjac = d_pres.cpu().numpy(), d_pjac.cpu().numpy()
    oracle = {}
    worst = 0.0
    for i in rng.choice(n_p, 1000, replace=False):
        k = int(i) % len(segs)
        if k not in oracle:
            r, J = segs[k].evaluate(*_pblocks(params, poffs[k]))
            oracle[k] = (r, np.concatenate([j.ravel() for j in J]))
        r, oj = oracle[k]
        worst = max(worst, _close(pres[i], r, f"preint factor {i} residual"))
        for b, (lo, hi) in enumerate(BLOCKS):
            worst = max(worst, _close(pjac[i][lo:hi], oj[lo:hi], f"preint factor {i} J{b}"))
    rres, rjac = d_res.cpu().numpy(), d_jac.cpu().numpy()
    cs, offs = prob["consts"], prob["offs"]
    for i in rng.choice(n_r, 1000, replace=False):
        k = int(i) % n_rp
        r, oj = _oracle_reproj(orc, params, cs[k], offs[k])
        assert np.array_equal(rres[i], r), f"reprojection {i} residual"
        assert np.array_equal(rjac[i], oj), f"reprojection {i} jacobian"
    print(f"bench batch: worst sampled preint factor relative error {worst:.3e}")

"""Two-phase factor evaluation (gvx_factor_set_create / gvx_factors_prepare /
gvx_factor_read_*), the Ceres EvaluationCallback boundary of SURVEY.md 8b.

The set runs the same kernels as the batched entry points on the packed
parameter vector its prepare() gathers from the caller's blocks, so every
residual and Jacobian block it hands out must equal the batched call's output
bit for bit (the batched calls are themselves pinned to the oracle in
test_ba_gpu.py / test_golden.py)."""
import threading

import numpy as np
import pytest

from gvx import synth_ba

pytestmark = pytest.mark.gpu
EARTH = 2


def _window(ctx, gvx_mod, n_kf=6, n_lm=40, seed=7):
    """A sliding window as separate parameter blocks: poses[k] (7), ext (7),
    invdepth[j] (1), td (1), mix[k] (9) + Earth preintegration segments between
    consecutive keyframes."""
    prob = synth_ba.make_ba_problem(seed=seed, n_kf=n_kf, n_lm=n_lm)
    poses = [np.ascontiguousarray(p.copy()) for p in prob["poses"]]
    ext = prob["ext"].copy()
    inv = [np.array([d]) for d in prob["invdepth"]]
    td = np.zeros(1)
    mix = [np.r_[5.0, 0, 0, np.zeros(6)] for _ in range(n_kf)]
    blocks = poses + [ext] + inv + [td] + mix
    i_ext, i_inv, i_td, i_mix = n_kf, n_kf + 1, n_kf + 1 + n_lm, n_kf + 2 + n_lm
    # packed offsets of the same blocks (the batched API's convention)
    off = np.cumsum([0] + [b.size for b in blocks])[:-1]
    o = prob["offs"]
    # map the problem's packed pose / invdepth offsets back to blocks
    pose_of = {7 * k: k for k in range(n_kf)}
    inv_of = {7 * n_kf + 7 + j: j for j in range(n_lm)}
    r_blocks = np.array([[pose_of[a], pose_of[b], i_ext, i_inv + inv_of[d], i_td] for a, b, _, d, _ in o],
                        np.int32)
    rng = np.random.default_rng(seed)
    M = 40
    segs = [synth_ba.make_imu_segment(rng, M, t0=0.5 * k) for k in range(n_kf - 1)]
    states = np.zeros(n_kf - 1, gvx_mod.STATE_DTYPE)
    for k in range(n_kf - 1):
        states[k]["time"] = 0.5 * k
        states[k]["p"] = prob["poses"][k, :3]
        states[k]["q"] = prob["poses"][k, 3:]
        states[k]["v"] = [5.0, 0.0, 0.0]
    iewn = np.array([gvx_mod.earth_iewn(np.zeros(3), s["p"]) for s in states])
    pre, pn, pn_off = ctx.preint_integrate(EARTH, synth_ba.imu_params(), segs, states, iewn)
    p_blocks = np.array([[k, i_mix + k, k + 1, i_mix + k + 1] for k in range(n_kf - 1)], np.int32)
    return dict(blocks=blocks, off=off, consts=prob["consts"], r_blocks=r_blocks, pre=pre, pn=pn, pn_off=pn_off,
                p_blocks=p_blocks)


def _packed(w):
    return np.concatenate(w["blocks"])


def _batched(ctx, gvx_mod, w):
    params = _packed(w)
    off = w["off"]
    rres, rjac = ctx.reproj_eval(w["consts"].astype(gvx_mod.REPROJ_DTYPE), params, off[w["r_blocks"]])
    pres, pjac = ctx.preint_factor_eval(w["pre"], w["pn"], w["pn_off"], params, off[w["p_blocks"]])
    return rres, rjac, pres, pjac


def _check_set(fs, rres, rjac, pres, pjac):
    for i in range(fs.n_reproj):
        r, J = fs.read_reproj(i)
        assert np.array_equal(r, rres[i]), f"reproj {i} residual"
        assert np.array_equal(np.concatenate([j.ravel() for j in J]), rjac[i]), f"reproj {i} jacobians"
    for i in range(fs.n_preint):
        r, J = fs.read_preint(i)
        assert np.array_equal(r, pres[i]), f"preint {i} residual"
        assert np.array_equal(np.concatenate([j.ravel() for j in J]), pjac[i]), f"preint {i} jacobians"


def _make_set(ctx, gvx_mod, w):
    return gvx_mod.FactorSet(ctx, w["blocks"], w["consts"], w["r_blocks"], w["pre"], w["pn"], w["pn_off"],
                             w["p_blocks"])


def test_factor_set_matches_batched(ctx, gvx_mod):
    w = _window(ctx, gvx_mod)
    fs = _make_set(ctx, gvx_mod, w)
    fs.prepare(jacobians=True)
    _check_set(fs, *_batched(ctx, gvx_mod, w))
    fs.close()


def test_factor_set_rereads_blocks_in_place(ctx, gvx_mod):
    """A new evaluation point written into the caller's blocks (what Ceres does
    before PrepareForEvaluation) is picked up by the next prepare()."""
    w = _window(ctx, gvx_mod, seed=11)
    fs = _make_set(ctx, gvx_mod, w)
    fs.prepare()
    r0, _ = fs.read_reproj(3, jacobians=False)
    rng = np.random.default_rng(5)
    for b in w["blocks"]:
        b += rng.normal(0, 1e-3, b.size)  # in place: the set holds these arrays' addresses
    fs.prepare()
    _check_set(fs, *_batched(ctx, gvx_mod, w))
    assert not np.array_equal(fs.read_reproj(3, jacobians=False)[0], r0)
    fs.close()


def test_factor_set_null_blocks_and_residual_only(ctx, gvx_mod):
    w = _window(ctx, gvx_mod, n_kf=4, n_lm=10, seed=13)
    fs = _make_set(ctx, gvx_mod, w)
    fs.prepare(jacobians=True)
    r, J = fs.read_reproj(2)
    r2, J2 = fs.read_reproj(2, jacobians=[False, True, False, True, False])
    assert np.array_equal(r, r2) and J2[0] is None and J2[2] is None and J2[4] is None
    assert np.array_equal(J2[1], J[1]) and np.array_equal(J2[3], J[3])
    fs.prepare(jacobians=False)
    assert np.array_equal(fs.read_preint(1, jacobians=False)[0], fs.read_preint(1, jacobians=False)[0])
    with pytest.raises(gvx_mod.GvxError):
        fs.read_reproj(0)  # Jacobians after a residual-only prepare
    with pytest.raises(gvx_mod.GvxError):
        fs.read_reproj(fs.n_reproj, jacobians=False)
    fs.close()


def test_factor_set_concurrent_reads(ctx, gvx_mod):
    """Reads are reentrant (Ceres evaluates cost functions from 4 threads)."""
    w = _window(ctx, gvx_mod, seed=17)
    fs = _make_set(ctx, gvx_mod, w)
    fs.prepare()
    rres, rjac, _, _ = _batched(ctx, gvx_mod, w)
    errors = []

    def worker(t):
        for i in range(t, fs.n_reproj, 4):
            r, J = fs.read_reproj(i)
            if not (np.array_equal(r, rres[i]) and np.array_equal(np.concatenate([j.ravel() for j in J]), rjac[i])):
                errors.append(i)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    fs.close()


def test_factor_set_rejects_bad_block_sizes(ctx, gvx_mod):
    w = _window(ctx, gvx_mod, n_kf=3, n_lm=5, seed=19)
    rb = w["r_blocks"].copy()
    rb[0, 3] = 0  # a 7-double pose where the inverse depth (1) belongs
    with pytest.raises(gvx_mod.GvxError):
        gvx_mod.FactorSet(ctx, w["blocks"], w["consts"], rb)


def test_factor_batch_eval_dev_matches_batched(ctx, gvx_mod):
    """gvx_factor_batch_eval_dev (both kinds over one device parameter array, the
    configs[3] bench step) gives the separate batched calls' bits."""
    import torch
    w = _window(ctx, gvx_mod, seed=11)
    params = _packed(w)
    off = w["off"]
    roffs = off[w["r_blocks"]].astype(np.int32)
    poffs = off[w["p_blocks"]].astype(np.int32)
    dev = torch.device("cuda", 0)

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    consts = w["consts"].astype(gvx_mod.REPROJ_DTYPE)
    d_c, d_p, d_ro, d_po = t(consts.view(np.uint8)), t(params), t(roffs), t(poffs)
    d_pre, d_pn, d_pno = t(w["pre"].view(np.uint8)), t(w["pn"]), t(w["pn_off"].astype(np.int32))
    nr, npf = len(consts), len(w["pre"])
    d_rr = torch.empty((nr, 2), dtype=torch.float64, device=dev)
    d_rj = torch.empty((nr, 46), dtype=torch.float64, device=dev)
    d_pr = torch.empty((npf, 15), dtype=torch.float64, device=dev)
    d_pj = torch.empty((npf, 480), dtype=torch.float64, device=dev)
    ctx.factor_batch_eval_dev(nr, d_c.data_ptr(), d_ro.data_ptr(), d_rr.data_ptr(), d_rj.data_ptr(), npf,
                              d_pre.data_ptr(), d_pn.data_ptr(), d_pno.data_ptr(), d_po.data_ptr(), d_pr.data_ptr(),
                              d_pj.data_ptr(), d_p.data_ptr())
    ctx.sync()
    rres, rjac, pres, pjac = _batched(ctx, gvx_mod, w)
    assert np.array_equal(d_rr.cpu().numpy(), rres)
    assert np.array_equal(d_rj.cpu().numpy(), rjac)
    assert np.array_equal(d_pr.cpu().numpy(), pres)
    assert np.array_equal(d_pj.cpu().numpy(), pjac)


@pytest.mark.parametrize("n_kf,n_lm", [(6, 40), (10, 1500)])
def test_factor_set_d2h_mode_matches_mapped(ctx, gvx_mod, n_kf, n_lm):
    """the GVX_FACTORSET_D2H=1 fallback (device result buffer + one
    D2H copy per prepare, out_mode 0) gives the same bits as the default mapped
    host buffer the kernels write themselves (out_mode 1) -- on a small window
    and on one of 13,500 reprojection factors, whose launch exceeds one block per
    CU and takes the split kernels."""
    import os
    w = _window(ctx, gvx_mod, n_kf=n_kf, n_lm=n_lm, seed=17)
    ref = _batched(ctx, gvx_mod, w)
    fs = _make_set(ctx, gvx_mod, w)
    fs.prepare(jacobians=True)
    _check_set(fs, *ref)
    fs.close()
    os.environ["GVX_FACTORSET_D2H"] = "1"
    try:
        c2 = gvx_mod.Context(0)  # the switch is read once, at creation
    finally:
        del os.environ["GVX_FACTORSET_D2H"]
    try:
        fs2 = _make_set(c2, gvx_mod, w)
        fs2.prepare(jacobians=True)
        _check_set(fs2, *ref)
        fs2.prepare(jacobians=False)
        for i in range(0, fs2.n_reproj, 97):
            r, _ = fs2.read_reproj(i, jacobians=False)
            assert np.array_equal(r, ref[0][i])
        fs2.close()
    finally:
        c2.close()

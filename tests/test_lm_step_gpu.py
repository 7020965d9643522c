"""The LM step's DENSE_SCHUR reduced system on the device (gvx_schur_solve,
csrc/dense.hip): Ceres with linear_solver_type = DENSE_SCHUR
(ic_gvins/ic_gvins/ic_gvins.cc:1170-1180, Solve at :1217 and :1251) solves
(J^T J + diag(D^2)) delta = -J^T r by eliminating the landmarks' inverse depths
(the e-blocks) and factoring the dense reduced camera system S by Cholesky.

Ceres is not available here, so the check is the linear algebra
itself, from an independent dense assembly in numpy (synth_ba.dense_normal_
equations: the stacked Jacobian of every residual block): S against the Schur
complement of the dense normal matrix, delta against numpy.linalg.solve of the
full damped system.  The window's normal matrix has a condition number of 2e17
(inverse depths against the prior's strongest directions), so the forward error is
held to 1e-9 with LM damping and to 1e-4 without (numpy's own Cholesky-Schur
solve lands 6e-13 / 1.8e-6 from numpy.linalg.solve); the backward error -- the
relative residual of the full system -- to 1e-14 either way."""
import numpy as np
import pytest

from gvx import synth_ba

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def window(orc):
    ev = orc.FactorEvaluator()
    return {"configs[3] window (10 keyframes, 200 landmarks)": synth_ba.lm_problem(synth_ba.make_marg_problem(ev)),
            "prior over keyframes 0-8": synth_ba.lm_problem(synth_ba.make_marg_problem(ev, n_prior_kf=9)),
            "two keyframes": synth_ba.lm_problem(synth_ba.make_marg_problem(ev, seed=5, n_kf=2, n_lm=17))}


def _check(g, p, D, fwd):
    H, b = synth_ba.dense_normal_equations(p)
    if D is not None:
        H = H + np.diag(D * D)
    m = p["m"]
    Hee, Hef, Hff = H[:m, :m], H[:m, m:], H[m:, m:]
    S = Hff - Hef.T @ np.linalg.solve(Hee, Hef)
    assert list(g["info"]) == [0, 0]
    Sg = g["S"]
    assert np.abs(Sg - S).max() <= 1e-9 * np.abs(S).max(), np.abs(Sg - S).max() / np.abs(S).max()
    x = np.linalg.solve(H, b)
    d = g["delta"]
    # the full damped system's relative residual
    res = np.abs(H @ d - b).max() / (np.abs(H).max() * np.abs(d).max())
    assert res <= 1e-14, res
    assert np.abs(d - x).max() <= fwd * np.abs(x).max(), np.abs(d - x).max() / np.abs(x).max()


@pytest.mark.parametrize("name", ["configs[3] window (10 keyframes, 200 landmarks)", "prior over keyframes 0-8",
                                  "two keyframes"])
def test_schur_solve_matches_dense(ctx, window, name):
    p = window[name]
    H, _ = synth_ba.dense_normal_equations(p)
    # LM damping of the size Ceres applies: mu * diag(J^T J), mu = 1e-4
    D = np.sqrt(1e-4 * np.maximum(np.diag(H), 1e-6))
    _check(ctx.schur_solve(p, D), p, D, 1e-9)
    _check(ctx.schur_solve(p), p, None, 1e-4)  # undamped (Gauss-Newton)


def test_schur_solve_many_landmarks(ctx, orc):
    """A window with 700 landmarks: m = 700 inverse depths, above the dense
    Cholesky kernels' 512, taken by the diagonal-Hee path (one inverse depth per
    landmark, each reprojection factor touching one: Hee's factor is its square
    root) -- checked against the dense numpy solve like the windows above
    (the LM step refused windows of more than 512 landmarks)."""
    p = synth_ba.lm_problem(synth_ba.make_marg_problem(orc.FactorEvaluator(), seed=11, n_kf=10, n_lm=700))
    assert p["m"] == 700
    H, _ = synth_ba.dense_normal_equations(p)
    D = np.sqrt(1e-4 * np.maximum(np.diag(H), 1e-6))
    _check(ctx.schur_solve(p, D), p, D, 1e-9)


def test_schur_solve_dev_many_landmarks(ctx, orc):
    """The device-pointer entry on the diagonal-Hee path (m = 700 > 512, ADVICE
    r04): the same delta as the host entry, bit for bit."""
    import torch
    p = synth_ba.lm_problem(synth_ba.make_marg_problem(orc.FactorEvaluator(), seed=11, n_kf=10, n_lm=700))
    assert p["m"] == 700
    L = p["L"]
    H, _ = synth_ba.dense_normal_equations(p)
    D = np.sqrt(1e-4 * np.maximum(np.diag(H), 1e-6))
    g = ctx.schur_solve(p, D)
    dev = torch.device("cuda")
    d_data = torch.from_numpy(p["data"]).to(dev)
    d_D = torch.from_numpy(D).to(dev)
    d_delta = torch.zeros(L, dtype=torch.float64, device=dev)
    d_info = torch.full((2,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.schur_solve_dev(p, d_data.data_ptr(), d_delta.data_ptr(), d_D=d_D.data_ptr(), d_info=d_info.data_ptr())
    ctx.sync()
    assert np.array_equal(d_delta.cpu().numpy(), g["delta"])
    assert d_info.cpu().tolist() == [0, 0]


def test_schur_solve_dev_matches_host(ctx, window):
    import torch
    p = window["prior over keyframes 0-8"]
    L = p["L"]
    D = np.full(L, 1e-2)
    g = ctx.schur_solve(p, D)
    dev = torch.device("cuda")
    d_data = torch.from_numpy(p["data"]).to(dev)
    d_D = torch.from_numpy(D).to(dev)
    d_delta = torch.zeros(L, dtype=torch.float64, device=dev)
    d_info = torch.full((2,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.schur_solve_dev(p, d_data.data_ptr(), d_delta.data_ptr(), d_D=d_D.data_ptr(), d_info=d_info.data_ptr())
    ctx.sync()
    assert np.array_equal(d_delta.cpu().numpy(), g["delta"])
    assert d_info.cpu().tolist() == [0, 0]


def test_schur_solve_reports_indefinite(ctx, window):
    """An unobserved landmark without damping: Hee is singular, info[0] = 1."""
    p = window["two keyframes"]
    data = p["data"].copy()
    lm = [b for b, n in enumerate(p["names"]) if n.startswith("invdepth")][0]
    for f in range(len(p["nres"])):
        off = int(p["jac_off"][f])
        for b in p["blk"][p["blk_off"][f]:p["blk_off"][f + 1]]:
            n = int(p["nres"][f]) * int(p["size"][b])
            if b == lm:
                data[off:off + n] = 0.0
            off += n
    g = ctx.schur_solve(dict(p, data=data))
    assert g["info"][0] == 1 and g["info"][1] == 1  # S is never formed after a failed Hee
    assert g["ok"] is False
    assert np.isnan(g["delta"]).all()  # no stale step survives
    # the device entry reports the same through d_info and a NaN d_delta
    import torch
    L = int(p["L"]) if "L" in p else g["delta"].size
    d_data = torch.from_numpy(data).cuda()
    d_delta = torch.zeros(g["delta"].size, dtype=torch.float64, device="cuda")
    d_info = torch.zeros(2, dtype=torch.int32, device="cuda")
    ctx.schur_solve_dev(dict(p, data=data), d_data.data_ptr(), d_delta.data_ptr(), d_info=d_info.data_ptr())
    ctx.sync()
    assert d_info.cpu().tolist() == [1, 1] and torch.isnan(d_delta).all().item() and L == d_delta.numel()


def test_schur_solve_refuses_oversized_window_before_staging(ctx):
    """a window above GVX_SCHUR_MAX_L (16,384) parameters is refused
    with GVX_ERR_UNSUPPORTED by both entries before any list, pinned or device
    staging is sized -- an r x r staging of 2 GiB must not be attempted (which
    could surface as GVX_ERR_OOM instead)."""
    from gvx import _ptr
    L = 16384 + 1
    delta = np.zeros(1)
    info = np.zeros(2, np.int32)
    s = ctx._L.gvx_schur_solve(ctx._h, 0, None, None, None, None, None, _ptr(delta), 0, 0, None, None, 0, L,
                               None, _ptr(delta), None, _ptr(info))
    assert s == -6  # GVX_ERR_UNSUPPORTED
    s = ctx._L.gvx_schur_solve_dev(ctx._h, 0, None, None, None, None, None, 1, 0, 0, None, None, 0, L, None, 1,
                                   None, None)
    assert s == -6

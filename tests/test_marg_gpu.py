"""Device marginalisation (csrc/marg.hip through gvx_marginalize[_dev] and
gvx_sym_eigen) against the CPU restatement (oracle/marg.c).

With the EXACT solver both run Eigen's algorithms with the same operation order:
every sum is a sequential loop in the same order, no FMA contraction, IEEE
division and square root.  The device results are therefore required to be
bit-identical to the oracle's: H0/b0 (through Hp), Hp, bp, Hp's eigenvalues, J0
and e0, and the eigen-solver's eigenvectors themselves (signs included).

The FAST solver (the default; csrc/dense.hip: Cholesky where no eigenvalue is
dropped) is held to what the reference's result means: Hp and bp within the
rounding noise of the reference's own arithmetic (measured as the asymmetry of
its Hp: Hmm's condition number, 3e11 at configs[3], puts that near 5e-6 of |Hp|;
LAPACK's eigh lands 5.7e-6 away as well), J0^T J0 = Hp and J0^T e0 = -bp (the
prior ||e0 + J0 dx||^2 is the same function), and -- where Hmm is singular and the
eigen-solver runs -- Hp and bp bit-identical to the EXACT solver's."""
import numpy as np
import pytest

from gvx import synth_ba

pytestmark = pytest.mark.gpu


def _graded(rng, n, lo=-3, hi=4):
    A = rng.normal(size=(n, n))
    A = A @ A.T + np.diag(rng.uniform(0, 1, n))
    D = np.diag(10 ** rng.uniform(lo, hi, n))
    return D @ A @ D


def _same(g, o, what):
    g, o = np.asarray(g), np.asarray(o)
    if not np.array_equal(g, o, equal_nan=True):
        d = np.abs(g - o)
        i = np.unravel_index(np.argmax(d), d.shape)
        raise AssertionError(f"{what}: {np.count_nonzero(d)} of {d.size} differ, max |diff| {d.max():.3e} at {i} "
                             f"(scale {np.abs(o).max():.3e})")


@pytest.mark.parametrize("n", [1, 2, 3, 64, 150, 215, 512])
def test_sym_eigen_bit_exact(ctx, orc, n):
    rng = np.random.default_rng(100 + n)
    A = _graded(rng, n)
    A[np.triu_indices(n, 1)] = rng.normal(size=n * (n - 1) // 2)  # the upper triangle is never read
    w, V, info = ctx.sym_eigen(A)
    wo, Vo, io = orc.sym_eigen(A)
    assert info == io == 0
    _same(w, wo, "eigenvalues")
    _same(V, Vo, "eigenvectors")


def test_sym_eigen_degenerate(ctx, orc):
    rng = np.random.default_rng(7)
    Q, _ = np.linalg.qr(rng.normal(size=(30, 30)))
    A = Q @ np.diag(np.repeat([0.0, 1.0, 5.0], 10)) @ Q.T
    for M in (A, np.zeros((8, 8)), np.diag([3.0, -1.0, 2.0, 2.0])):
        w, V, _ = ctx.sym_eigen(M)
        wo, Vo, _ = orc.sym_eigen(M)
        _same(w, wo, "eigenvalues")
        _same(V, Vo, "eigenvectors")


@pytest.fixture(scope="module")
def problems(orc):
    ev = orc.FactorEvaluator()
    return {
        "prior over the whole window (r = 142)": synth_ba.make_marg_problem(ev),
        "prior over keyframes 0-8 (r = 133)": synth_ba.make_marg_problem(ev, n_prior_kf=9),
        "Huber on the reprojection blocks": synth_ba.make_marg_problem(ev, n_kf=5, n_lm=60, huber=0.5),
        "two keyframes": synth_ba.make_marg_problem(ev, seed=5, n_kf=2, n_lm=17),
    }


@pytest.fixture
def exact(ctx, gvx_mod):
    ctx.set_marg_solver(gvx_mod.MARG_SOLVER_EXACT)
    yield
    ctx.set_marg_solver(gvx_mod.MARG_SOLVER_FAST)


NAMES = ["prior over the whole window (r = 142)", "prior over keyframes 0-8 (r = 133)",
         "Huber on the reprojection blocks", "two keyframes"]


@pytest.mark.parametrize("name", NAMES)
def test_marginalize_bit_exact(ctx, orc, problems, name, exact):
    p = problems[name]
    g = ctx.marginalize(p)
    H0, b0 = orc.marg_construct(p)
    Hp, bp, info1 = orc.marg_schur(H0, b0, p["m"])
    J0, e0, ev, info2 = orc.marg_linearize(Hp, bp)
    assert list(g["info"]) == [info1, info2] == [0, 0]
    _same(g["Hp"], Hp, "Hp")
    _same(g["bp"], bp, "bp")
    _same(g["eval"], ev, "eigenvalues of Hp")
    _same(g["J0"], J0, "J0")
    _same(g["e0"], e0, "e0")
    if name.startswith("prior over the whole"):
        assert J0.shape == (142, 142)


def _asym(A):
    return np.abs(A - A.T).max() / np.abs(A).max()


@pytest.mark.parametrize("name", NAMES)
def test_marginalize_fast_solver(ctx, orc, gvx_mod, problems, name):
    """FAST (Cholesky) path: Hp / bp against the restatement within 10x the
    restatement's own rounding noise, J0^T J0 = Hp (lower triangle read, as
    Eigen's solver reads it) and J0^T e0 = -bp to 1e-10."""
    p = problems[name]
    g = ctx.marginalize(p)
    H0, b0 = orc.marg_construct(p)
    Hp, bp, _ = orc.marg_schur(H0, b0, p["m"])
    tol = max(1e-12, 10 * _asym(Hp))
    sHp = np.abs(Hp).max()
    assert np.abs(g["Hp"] - Hp).max() <= tol * sHp, (np.abs(g["Hp"] - Hp).max() / sHp, tol)
    assert np.abs(g["bp"] - bp).max() <= tol * np.abs(bp).max()
    assert np.isnan(g["eval"]).all() and list(g["info"]) == [0, 0]  # the Cholesky path ran for both steps
    J0, e0, Hg = g["J0"], g["e0"], g["Hp"]
    Hl = np.tril(Hg) + np.tril(Hg, -1).T
    assert np.abs(J0.T @ J0 - Hl).max() <= 1e-12 * np.abs(Hl).max()
    assert np.abs(J0.T @ e0 + g["bp"]).max() <= 1e-10 * np.abs(g["bp"]).max()
    assert np.allclose(np.triu(J0), J0)  # J0 = Lp^T


def _unobserved(p, block):
    """The problem with every Jacobian column of parameter block `block` zeroed:
    the block is unobserved, Hmm singular (an eigenvalue 0 <= EPS)."""
    data = p["data"].copy()
    size = p["size"]
    for f in range(len(p["nres"])):
        off = int(p["jac_off"][f])
        for b in p["blk"][p["blk_off"][f]:p["blk_off"][f + 1]]:
            n = int(p["nres"][f]) * int(size[b])
            if b == block:
                data[off:off + n] = 0.0
            off += n
    return dict(p, data=data)


def test_marginalize_fast_falls_back_on_singular_hmm(ctx, gvx_mod, problems):
    """An unobserved marginalized landmark: Hmm - EPS*I is not positive definite,
    so the FAST solver runs Eigen's eigen-solver for Hmm^-1 (dropping the zero
    eigenvalue, as the reference does): Hp and bp bit-identical to the EXACT
    solver's, then the Cholesky linearisation of that Hp."""
    p = problems["two keyframes"]
    m = p["m"]
    lm = [b for b in range(len(p["size"])) if p["size"][b] == 1 and p["index"][b] < m][0]
    q = _unobserved(p, lm)
    g = ctx.marginalize(q)
    ctx.set_marg_solver(gvx_mod.MARG_SOLVER_EXACT)
    try:
        x = ctx.marginalize(q)
    finally:
        ctx.set_marg_solver(gvx_mod.MARG_SOLVER_FAST)
    _same(g["Hp"], x["Hp"], "Hp")
    _same(g["bp"], x["bp"], "bp")
    J0, e0 = g["J0"], g["e0"]
    Hl = np.tril(x["Hp"]) + np.tril(x["Hp"], -1).T
    assert np.abs(J0.T @ J0 - Hl).max() <= 1e-12 * np.abs(Hl).max()
    assert np.abs(J0.T @ e0 + g["bp"]).max() <= 1e-10 * np.abs(g["bp"]).max()


@pytest.mark.parametrize("name", ["two keyframes", "prior over keyframes 0-8 (r = 133)"])
def test_marginalize_fast_falls_back_on_singular_hp(ctx, orc, problems, name):
    """A remaining block with every Jacobian column zeroed: Hmm stays positive
    definite (Cholesky Schur complement), but Hp has a zero eigenvalue, so
    Hp - EPS*I is not positive definite and the FAST solver linearises with
    Eigen's eigen-solver on the device (marg.hip: the gated sym_eigen +
    linearize_kernel instead of lin_chol / trsv).  The eigenvalues
    are then real numbers (NaN marks the Cholesky path), and J0 / e0 are
    bit-identical to the restatement's linearization of the same Hp / bp
    (marginalization_info.h:153-166)."""
    p = problems[name]
    m = p["m"]
    rem = [b for b in range(len(p["size"])) if p["index"][b] >= m]
    q = _unobserved(p, rem[-1])
    g = ctx.marginalize(q)
    assert list(g["info"]) == [0, 0]  # eigen-solver converged
    assert not np.isnan(g["eval"]).any()  # the eigen path produced the linearisation
    assert g["eval"].min() <= 1e-8 * max(1.0, g["eval"].max())  # the dropped direction
    J0, e0, ev, info2 = orc.marg_linearize(g["Hp"], g["bp"])
    assert info2 == 0
    _same(g["eval"], ev, "eigenvalues of Hp")
    _same(g["J0"], J0, "J0")
    _same(g["e0"], e0, "e0")
    # the healthy problem still takes the Cholesky path
    assert np.isnan(ctx.marginalize(p)["eval"]).all()


def test_marginalize_dev_matches_host(ctx, problems):
    import torch
    p = problems["prior over keyframes 0-8 (r = 133)"]
    g = ctx.marginalize(p)
    r = p["L"] - p["m"]
    dev = torch.device("cuda")
    d_data = torch.from_numpy(p["data"]).to(dev)
    out = {k: torch.zeros(n, dtype=torch.float64, device=dev)
           for k, n in (("J0", r * r), ("e0", r), ("Hp", r * r), ("bp", r), ("eval", r))}
    d_info = torch.full((2,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.marginalize_dev(p, d_data.data_ptr(), out["J0"].data_ptr(), out["e0"].data_ptr(), out["Hp"].data_ptr(),
                        out["bp"].data_ptr(), out["eval"].data_ptr(), d_info.data_ptr())
    ctx.sync()
    cm = lambda t: t.cpu().numpy().reshape(r, r).T
    _same(cm(out["J0"]), g["J0"], "J0")
    _same(cm(out["Hp"]), g["Hp"], "Hp")
    _same(out["e0"].cpu().numpy(), g["e0"], "e0")
    _same(out["bp"].cpu().numpy(), g["bp"], "bp")
    _same(out["eval"].cpu().numpy(), g["eval"], "eval")
    assert d_info.cpu().tolist() == [0, 0]


def test_marginalize_feeds_the_marginalization_factor(ctx, orc, problems):
    """The next window's MarginalizationFactor (marginalization_factor.h:54-110)
    evaluated on the device from the device J0 / e0 at the linearisation point
    reproduces e0 (dx = 0)."""
    p = problems["prior over keyframes 0-8 (r = 133)"]
    g = ctx.marginalize(p)
    m = p["m"]
    rem = [b for b in range(len(p["size"])) if p["index"][b] >= m]
    rem.sort(key=lambda b: p["index"][b])
    size = p["size"][rem]
    index = (p["index"][rem] - m).astype(np.int32)
    xoff = np.concatenate([[0], np.cumsum(size)[:-1]]).astype(np.int32)
    rng = np.random.default_rng(1)
    x0 = np.concatenate([synth_ba._pose_block_values(rng, 1)[0] if s == 7 else rng.normal(size=s) for s in size])
    res, _ = ctx.marg_factor_eval(size, index, xoff, x0, x0, g["J0"], g["e0"])
    # dx = 0 up to the rounding of q0^-1 q0 in the pose blocks
    np.testing.assert_allclose(res, g["e0"], rtol=0, atol=1e-14 * np.abs(g["J0"]).sum(1).max())


def test_marginalize_rejects_bad_problems(ctx, gvx_mod, problems):
    p = problems["two keyframes"]
    with pytest.raises(gvx_mod.GvxError):
        ctx.marginalize(dict(p, m=0))
    blk = p["blk"].copy()
    blk[3] = 10 ** 6
    with pytest.raises(gvx_mod.GvxError):
        ctx.marginalize(dict(p, blk=blk))
    with pytest.raises(gvx_mod.GvxError):
        ctx.marginalize(dict(p, m=513, L=513 + 10))
    with pytest.raises(gvx_mod.GvxError):
        ctx.sym_eigen(np.eye(513))

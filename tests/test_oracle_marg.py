"""The CPU restatement of MarginalizationInfo::marginalization() (oracle/marg.c)
pinned without Eigen: the eigen-solver against numpy/LAPACK (eigenvalues,
reconstruction, orthogonality, ascending order, lower triangle only), the
normal equations against a dense stacked Jacobian, the Schur complement and the
linearisation against their defining identities.

Eigen and Ceres are absent, so the restatement's own rounding is unpinned: the
known answers here are mathematical identities, held to tolerances that scale
with the conditioning where it matters (the configs[3] window's Hmm spans eleven
orders of magnitude)."""
import numpy as np
import pytest

from gvx import synth_ba


def _graded(rng, n, lo=-3, hi=4):
    A = rng.normal(size=(n, n))
    A = A @ A.T + np.diag(rng.uniform(0, 1, n))
    D = np.diag(10 ** rng.uniform(lo, hi, n))
    return D @ A @ D


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 150])
def test_sym_eigen_matches_lapack(orc, n):
    rng = np.random.default_rng(n)
    A = _graded(rng, n)
    w, V, info = orc.sym_eigen(A)
    assert info == 0
    assert np.all(np.diff(w) >= 0), "ascending (the selection sort)"
    scale = np.abs(A).max()
    np.testing.assert_allclose(w, np.linalg.eigvalsh(A), rtol=0, atol=1e-13 * scale)
    assert np.abs(V @ np.diag(w) @ V.T - A).max() <= 1e-13 * scale
    assert np.abs(V.T @ V - np.eye(n)).max() <= 1e-13


def test_sym_eigen_reads_lower_triangle_only(orc):
    rng = np.random.default_rng(5)
    A = _graded(rng, 40, 0, 2)
    B = np.tril(A) + np.triu(rng.normal(size=A.shape) * 1e6, 1)  # garbage above the diagonal
    w1, V1, _ = orc.sym_eigen(A)
    w2, V2, _ = orc.sym_eigen(B)
    assert np.array_equal(w1, w2) and np.array_equal(V1, V2)


def test_sym_eigen_special_cases(orc):
    w, V, info = orc.sym_eigen(np.zeros((4, 4)))
    assert info == 0 and np.array_equal(w, np.zeros(4)) and np.array_equal(V, np.eye(4))
    d = np.array([3.0, -1.0, 2.0, 2.0, 0.5])
    w, V, _ = orc.sym_eigen(np.diag(d))  # already tridiagonal and diagonal: only the sort acts
    assert np.array_equal(w, np.sort(d))
    assert np.array_equal(np.abs(V), np.eye(5)[:, np.argsort(d, kind="stable")])
    w, V, _ = orc.sym_eigen(np.array([[7.5]]))
    assert w[0] == 7.5 and V[0, 0] == 1.0
    # repeated eigenvalues: still an orthonormal basis of each eigenspace
    rng = np.random.default_rng(9)
    Q, _ = np.linalg.qr(rng.normal(size=(12, 12)))
    lam = np.repeat([1.0, 4.0, 9.0], 4)
    A = Q @ np.diag(lam) @ Q.T
    w, V, _ = orc.sym_eigen(A)
    np.testing.assert_allclose(w, lam, atol=1e-13)
    assert np.abs(V @ np.diag(w) @ V.T - A).max() <= 1e-13 * 9


@pytest.fixture(scope="module")
def window(orc):
    return synth_ba.make_marg_problem(orc.FactorEvaluator())


def _dense(p):
    """Stacked Jacobian over the local columns (pose: the first 6 of 7) and residuals."""
    L = p["L"]
    Js, es = [], []
    for f in range(len(p["nres"])):
        R = int(p["nres"][f])
        o = int(p["jac_off"][f])
        Jf = np.zeros((R, L))
        sr = 1.0
        e = p["data"][p["res_off"][f]:p["res_off"][f] + R]
        if p.get("loss") is not None and p["loss"][f] > 0:
            a, s = p["loss"][f], e @ e
            sr = np.sqrt(max(a / np.sqrt(s), np.finfo(float).tiny)) if s > a * a else 1.0
        for b in p["blk"][p["blk_off"][f]:p["blk_off"][f + 1]]:
            g = int(p["size"][b])
            loc = 6 if g == 7 else g
            J = p["data"][o:o + R * g].reshape(R, g)
            o += R * g
            Jf[:, p["index"][b]:p["index"][b] + loc] += sr * J[:, :loc]
        Js.append(Jf)
        es.append(sr * e)
    return np.vstack(Js), np.concatenate(es)


@pytest.mark.parametrize("huber", [None, 0.5])
def test_construct_equation_is_dense_normal_equations(orc, huber):
    p = synth_ba.make_marg_problem(orc.FactorEvaluator(), n_kf=4, n_lm=30, huber=huber)
    H0, b0 = orc.marg_construct(p)
    J, e = _dense(p)
    Hn, bn = J.T @ J, -J.T @ e
    assert np.array_equal(H0, H0.T), "constructEquation's transposed copy keeps H0 exactly symmetric"
    assert np.abs(H0 - Hn).max() <= 1e-13 * np.abs(Hn).max()
    assert np.abs(b0 - bn).max() <= 1e-13 * np.abs(bn).max()
    if huber is not None:
        H1, _ = orc.marg_construct(dict(p, loss=None))
        assert not np.array_equal(H0, H1), "the Huber corrector changes outlier blocks"


def test_window_structure(window):
    p = window
    assert p["m"] == 6 + 9 + 200 and p["L"] - p["m"] == 142
    assert len(p["nres"]) == 1 + 1 + 1 + 1800  # prior, GNSS, preintegration, reprojection
    assert p["nres"][0] == 157 and p["nres"][2] == 15 and p["nres"][3] == 2


def test_schur_complement_identities(orc, window):
    p = window
    m = p["m"]
    H0, b0 = orc.marg_construct(p)
    Hp, bp, info = orc.marg_schur(H0, b0, m)
    assert info == 0
    w, V = np.linalg.eigh(H0[:m, :m])
    assert w.min() > 1e-8, "this window's Hmm is positive definite: no eigenvalue is masked"
    Hi = np.linalg.inv(H0[:m, :m])
    Hn = H0[m:, m:] - H0[m:, :m] @ Hi @ H0[:m, m:]
    bn = b0[m:] - H0[m:, :m] @ Hi @ b0[:m]
    # Hmm's condition number (~3e11) bounds how closely two eigen-solvers can agree
    kappa = w.max() / w.min()
    tol = 1e-16 * kappa
    assert np.abs(Hp - Hn).max() <= tol * np.abs(Hn).max()
    assert np.abs(bp - bn).max() <= tol * np.abs(bn).max()
    # the exact identity the masked inverse must satisfy on a well-conditioned problem
    rng = np.random.default_rng(3)
    A = rng.normal(size=(40, 40))
    H = A @ A.T + 40 * np.eye(40)
    b = rng.normal(size=40)
    Hp2, bp2, _ = orc.marg_schur(H, b, 15)
    S = H[15:, 15:] - H[15:, :15] @ np.linalg.solve(H[:15, :15], H[:15, 15:])
    np.testing.assert_allclose(Hp2, S, rtol=0, atol=1e-12 * np.abs(S).max())
    np.testing.assert_allclose(bp2, b[15:] - H[15:, :15] @ np.linalg.solve(H[:15, :15], b[:15]), atol=1e-12)


def test_schur_masks_small_eigenvalues(orc):
    """Hmm with a null direction: the reference drops eigenvalues <= 1e-8 (a
    pseudo-inverse), it does not fail."""
    rng = np.random.default_rng(4)
    A = rng.normal(size=(12, 12))
    H = A @ A.T + 12 * np.eye(12)
    u = np.zeros(12)
    u[:4] = rng.normal(size=4)
    u /= np.linalg.norm(u)
    P = np.eye(12) - np.outer(u, u)
    H[:4, :4] = (P @ H @ P)[:4, :4]  # Hmm = P Hmm P: u is in its null space
    H[4:, :4] = (H[4:, :4] @ P[:4, :4])
    H[:4, 4:] = H[4:, :4].T
    b = rng.normal(size=12)
    Hp, bp, _ = orc.marg_schur(H, b, 4)
    w, V = np.linalg.eigh(H[:4, :4])
    d = np.where(w > 1e-8, 1 / w, 0.0)
    Hi = (V * d) @ V.T
    np.testing.assert_allclose(Hp, H[4:, 4:] - H[4:, :4] @ Hi @ H[:4, 4:], atol=1e-10)
    np.testing.assert_allclose(bp, b[4:] - H[4:, :4] @ Hi @ b[:4], atol=1e-10)


def test_linearization_identities(orc, window):
    p = window
    H0, b0 = orc.marg_construct(p)
    Hp, bp, _ = orc.marg_schur(H0, b0, p["m"])
    J0, e0, ev, info = orc.marg_linearize(Hp, bp)
    assert info == 0 and np.all(np.diff(ev) >= 0)
    Hl = np.tril(Hp) + np.tril(Hp, -1).T  # the solver reads the lower triangle
    keep = ev > 1e-8
    assert keep.all()
    # J0^T J0 = Hp and J0^T e0 = -bp on the kept spectrum
    assert np.abs(J0.T @ J0 - Hl).max() <= 1e-13 * np.abs(Hl).max()
    assert np.abs(J0.T @ e0 + bp).max() <= 1e-12 * np.abs(bp).max()
    # e0^T e0 = bp^T Hp^-1 bp (independent of eigenvector signs)
    np.testing.assert_allclose(e0 @ e0, bp @ np.linalg.solve(Hl, bp), rtol=1e-9)


def test_linearization_drops_null_directions(orc):
    rng = np.random.default_rng(6)
    A = rng.normal(size=(10, 7))
    Hp = A @ A.T  # rank 7
    bp = Hp @ rng.normal(size=10)
    J0, e0, ev, _ = orc.marg_linearize(Hp, bp)
    assert np.all(J0[:3] == 0.0) and np.all(e0[:3] == 0.0), "rows of the dropped eigenvalues are zero"
    assert np.abs(J0.T @ J0 - Hp).max() <= 1e-12 * np.abs(Hp).max()
    assert np.abs(J0.T @ e0 + bp).max() <= 1e-11 * np.abs(bp).max()

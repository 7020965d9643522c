"""The remaining window factors on the device (csrc/aux_factors.hip through
gvx_small_factor_eval / gvx_marg_factor_eval) against the CPU restatement
(oracle/aux_factors.c).  Both evaluate the same expressions in the same order
without FMA contraction; the bound is the factor contract's fp64 tolerance
(1e-12 relative), the Jacobian copies of the marginalisation factor are exact."""
import numpy as np
import pytest

from gvx import synth_ba

pytestmark = pytest.mark.gpu


def _pose(rng):
    q = synth_ba.quat_from_rotvec(rng.normal(0, 0.5, 3))
    return np.concatenate([rng.normal(0, 5, 3), q / np.linalg.norm(q)])


def _consts(rng, kind, n):
    if kind == 0:
        return np.concatenate([rng.normal(0, 5, (n, 3)), rng.uniform(0.01, 0.1, (n, 3)),
                               np.tile([0.1, -0.2, 0.3], (n, 1))], axis=1)
    if kind == 1:
        return None
    if kind == 2:
        return np.concatenate([np.array([_pose(rng) for _ in range(n)]), rng.uniform(0.01, 0.2, (n, 6))], axis=1)
    return np.concatenate([rng.normal(0, 1, (n, 9)), rng.uniform(0.01, 0.2, (n, 9))], axis=1)


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
@pytest.mark.parametrize("n", [1, 63, 1000])
def test_small_factors_match_oracle(ctx, gvx_mod, orc, kind, n):
    rng = np.random.default_rng(100 * kind + n)
    R, P, NC = gvx_mod.SMALL_FACTOR_DIMS[kind]
    blocks = [_pose(rng) if P == 7 else rng.normal(0, 1, 9) for _ in range(n + 3)]
    params = np.concatenate(blocks)
    offs = (rng.permutation(n + 3)[:n] * P).astype(np.int32)  # blocks shared / out of order
    c = _consts(rng, kind, n)
    res, jac = ctx.small_factor_eval(kind, c, params, offs)
    rref, jref = orc.small_factor_eval(kind, c, params, offs)
    np.testing.assert_allclose(res, rref, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(jac, jref, rtol=1e-12, atol=1e-14)
    r2, j2 = ctx.small_factor_eval(kind, c, params, offs, jacobians=False)
    assert j2 is None and np.array_equal(r2, res)


def test_small_factor_rejects_bad_blocks(ctx, gvx_mod):
    with pytest.raises(gvx_mod.GvxError):
        ctx.small_factor_eval(1, None, np.zeros(9), [1])  # block [1, 10) outside 9 values
    with pytest.raises(gvx_mod.GvxError):
        ctx.small_factor_eval(7, None, np.zeros(9), [0])


@pytest.mark.parametrize("n_kf", [1, 2, 4, 9, 40])
def test_marg_factor_matches_oracle(ctx, orc, n_kf):
    rng = np.random.default_rng(n_kf)
    size = [7, 9] * n_kf + [7, 1]
    local = [6 if s == 7 else s for s in size]
    index = np.concatenate([[0], np.cumsum(local)[:-1]]).astype(np.int32)
    xoff = np.concatenate([[0], np.cumsum(size)[:-1]]).astype(np.int32)
    r = int(sum(local))
    x0 = np.concatenate([_pose(rng) if s == 7 else rng.normal(0, 1, s) for s in size])
    x = x0 + rng.normal(0, 0.01, x0.size)
    for b, s in enumerate(size):
        if s == 7:
            q = x[xoff[b] + 3:xoff[b] + 7]
            x[xoff[b] + 3:xoff[b] + 7] = q / np.linalg.norm(q) * (-1 if b % 4 == 0 else 1)
    J0, e0 = rng.normal(0, 1, (r, r)), rng.normal(0, 1, r)
    res, jac = ctx.marg_factor_eval(size, index, xoff, x0, x, J0, e0)
    rref, jref = orc.marg_factor_eval(size, index, xoff, x0, x, J0, e0)
    scale = np.abs(J0).sum(1) * 0.1 + np.abs(e0)
    assert np.all(np.abs(res - rref) <= 1e-13 * scale)
    assert np.array_equal(jac, jref)

"""Device cv::findFundamentalMat(FM_RANSAC) (csrc/fmat.hip through
gvx_find_fundamental_ransac[_dev]) against the CPU restatement (oracle/fmat.c).

The device draws the same RNG stream, solves the same 7-point problems with the
same sequential fp64 arithmetic and replays RANSAC's bookkeeping in order, so
the inlier masks and results must be identical.  hypot / acos / cos / pow / log
come from ROCm's ocml instead of glibc, so the models are compared at a relative
1e-9, not bit for bit."""
import numpy as np
import pytest

from gvx import synth

pytestmark = pytest.mark.gpu


def _check(g, o):
    r, mask, F = g
    ro, masko, Fo, _ = o
    assert r == ro
    assert np.array_equal(mask, masko), f"{np.count_nonzero(mask != masko)} mask entries differ"
    if r == 1:
        np.testing.assert_allclose(F, Fo, rtol=0, atol=1e-9 * np.abs(Fo).max())


@pytest.mark.parametrize("n,frac,seed", [(15, 0.2, 1), (40, 0.25, 2), (150, 0.25, 3), (150, 0.5, 6), (500, 0.3, 4),
                                         (1000, 0.1, 8)])
def test_ransac_matches_oracle(ctx, orc, n, frac, seed):
    p1, p2, _ = synth.two_view_scene(n, outlier_frac=frac, noise_px=0.3, seed=seed)
    (g,) = ctx.find_fundamental_ransac([(p1, p2)])
    _check(g, orc.find_fundamental_ransac(p1, p2))


def test_ransac_batch_of_sequence_frames(ctx, orc):
    """Many frames' reference points in one launch (a batch replay), with the
    edge cases: < 15 points (not the RANSAC path), an all-collinear set, a clean
    scene, and a many-iteration set (50 % outliers)."""
    rng = np.random.default_rng(3)
    sets = []
    for k in range(40):
        n = int(rng.integers(15, 200))
        p1, p2, _ = synth.two_view_scene(n, outlier_frac=float(rng.uniform(0, 0.5)), seed=100 + k)
        sets.append((p1, p2))
    p1, p2, _ = synth.two_view_scene(10, seed=7)
    sets.append((p1, p2))
    line = np.c_[np.linspace(0, 100, 30), np.linspace(0, 50, 30)].astype(np.float32)
    sets.append((line, line + 1))
    p1, p2, _ = synth.two_view_scene(150, outlier_frac=0.0, noise_px=0.0, seed=9)
    sets.append((p1, p2))
    out = ctx.find_fundamental_ransac(sets)
    for (a, b), g in zip(sets, out):
        if len(a) < 15:
            assert g[0] == -1 and g[1].all()
            continue
        _check(g, orc.find_fundamental_ransac(a, b))
    assert out[-2][0] == 0 and out[-1][1].all()

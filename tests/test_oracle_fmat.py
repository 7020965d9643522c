"""The CPU restatement of cv::findFundamentalMat(FM_RANSAC) (oracle/fmat.c)
pinned without OpenCV: known answers of synthetic two-view scenes (exact
epipolar geometry, gross outliers), the constraints every 7-point model must
satisfy, solveCubic against numpy.roots, cv::RNG's multiply-with-carry recurrence
and RANSACUpdateNumIters' closed form.  OpenCV itself is absent, so the RNG
stream / SVD / iteration order are restated from recalled 4.x sources: parity
with OpenCV is unpinned."""
import numpy as np
import pytest

from gvx import synth


@pytest.mark.parametrize("n,seed", [(15, 1), (40, 2), (150, 3), (500, 4)])
def test_ransac_separates_outliers(orc, n, seed):
    p1, p2, inl = synth.two_view_scene(n, outlier_frac=0.25, noise_px=0.2, seed=seed)
    r, mask, F, iters = orc.find_fundamental_ransac(p1, p2)
    assert r == 1 and 1 <= iters <= 1000
    assert np.linalg.matrix_rank(F, tol=1e-9 * np.abs(F).max()) == 2
    # gross outliers (moved by >= a few px off their epipolar line) are rejected,
    # almost all true inliers (noise 0.2 px << threshold 1.5 px) are kept
    err = orc.fm_error(p1, p2, F)
    assert np.array_equal(mask.astype(bool), err <= np.float32(1.5 * 1.5))
    assert (mask.astype(bool) & inl).sum() >= 0.8 * inl.sum()
    far = ~inl & (err > 25)
    assert not (mask.astype(bool) & far).any()


def test_ransac_clean_scene_keeps_everything(orc):
    p1, p2, _ = synth.two_view_scene(150, outlier_frac=0.0, noise_px=0.0, seed=9)
    r, mask, F, iters = orc.find_fundamental_ransac(p1, p2)
    assert r == 1 and mask.all()
    assert iters <= 3, "all-inlier sample: RANSACUpdateNumIters drops to 1"


def test_ransac_is_deterministic_and_guarded(orc):
    p1, p2, _ = synth.two_view_scene(80, seed=5)
    a = orc.find_fundamental_ransac(p1, p2)
    b = orc.find_fundamental_ransac(p1, p2)
    assert a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert orc.find_fundamental_ransac(p1[:14], p2[:14])[0] == -1
    # every point on one line: no non-collinear subset within 10000 attempts
    line = np.c_[np.linspace(0, 100, 30), np.linspace(0, 50, 30)].astype(np.float32)
    r, mask, F, _ = orc.find_fundamental_ransac(line, line + 1)
    assert r == 0 and not mask.any()


def test_run7point_models(orc):
    p1, p2, _ = synth.two_view_scene(7, outlier_frac=0.0, noise_px=0.0, seed=11)
    Fs = orc.run7point(p1, p2)
    assert 1 <= len(Fs) <= 3
    h1, h2 = np.c_[p1, np.ones(7)], np.c_[p2, np.ones(7)]
    for F in Fs:
        assert F[2, 2] == pytest.approx(1.0)
        assert np.abs(np.einsum("ij,jk,ik->i", h2, F, h1)).max() <= 1e-9 * np.abs(F).max() * 1e3
        assert abs(np.linalg.det(F)) <= 1e-10 * np.abs(F).max() ** 3


@pytest.mark.parametrize("c", [[1, -6, 11, -6], [2, 0, -3, 1], [1, 0, 0, -8], [0, 1, -3, 2], [0, 0, 2, -4],
                               [1, 3, 3, 1.000001]])
def test_solve_cubic(orc, c):
    n, r = orc.solve_cubic(c)
    ref = np.roots(c)
    real = np.sort(ref[np.abs(ref.imag) < 1e-7].real)
    got = np.sort(r[:n])
    assert n == len(real) or (n == 1 and len(real) >= 1)
    for g in got:
        assert np.min(np.abs(real - g)) <= 1e-6 * max(1, np.abs(real).max())


def test_cv_rng_recurrence(orc):
    s = (1 << 64) - 1
    seq = orc.cvrng_sequence(s, 4)
    for v in seq:  # state = (uint64)(unsigned)state * 4164903690 + (state >> 32)
        s = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & ((1 << 64) - 1)
        assert v == s & 0xFFFFFFFF


def test_ransac_update_num_iters(orc):
    # log(1 - p) / log(1 - (1 - ep)^7), rounded to nearest
    for ep in (0.1, 0.3, 0.5):
        want = int(np.rint(np.log(0.01) / np.log(1 - (1 - ep) ** 7)))
        assert orc.ransac_update_num_iters(0.99, ep, 7, 1000) == min(want, 1000)
    assert orc.ransac_update_num_iters(0.99, 0.0, 7, 1000) == 0
    assert orc.ransac_update_num_iters(0.99, 0.95, 7, 1000) == 1000

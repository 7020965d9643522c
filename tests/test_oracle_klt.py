"""CPU tests of the KLT restatement (oracle/klt.c) against independent numpy
restatements and analytic known answers (the reference ships no fixtures for
this path: SURVEY.md 8c, parity vs. OpenCV unpinned)."""
import numpy as np
import pytest

from gvx import synth


def np_pyrdown(src: np.ndarray) -> np.ndarray:
    """Independent pyrDown: separable [1 4 6 4 1]/256, REFLECT_101, (s+128)>>8."""
    h, w = src.shape
    dh, dw = (h + 1) // 2, (w + 1) // 2
    p = np.pad(src.astype(np.int64), 2, mode="reflect")
    k = np.array([1, 4, 6, 4, 1], np.int64)
    rows = np.zeros((h + 4, dw), np.int64)
    for j in range(5):
        rows += k[j] * p[:, j:j + 2 * dw:2][:, :dw]
    out = np.zeros((dh, dw), np.int64)
    for i in range(5):
        out += k[i] * rows[i:i + 2 * dh:2][:dh]
    return ((out + 128) >> 8).astype(np.uint8)


def np_scharr(img: np.ndarray) -> np.ndarray:
    p = np.pad(img.astype(np.int32), 1, mode="reflect")
    t0 = (p[:-2] + p[2:]) * 3 + p[1:-1] * 10
    t1 = p[2:] - p[:-2]
    dx = t0[:, 2:] - t0[:, :-2]
    dy = (t1[:, 2:] + t1[:, :-2]) * 3 + t1[:, 1:-1] * 10
    return np.stack([dx, dy], -1).astype(np.int16)


@pytest.mark.parametrize("w,h", [(160, 70), (161, 71), (1280, 560), (333, 97)])
def test_pyramid_matches_numpy(orc, w, h):
    rng = np.random.default_rng(1)
    img = synth.make_image(w, h, rng)
    lv = orc.build_pyramid(img, max_level=4)
    assert np.array_equal(lv[0], img)
    for l in range(1, len(lv)):
        assert lv[l].shape == ((lv[l - 1].shape[0] + 1) // 2, (lv[l - 1].shape[1] + 1) // 2)
        assert np.array_equal(lv[l], np_pyrdown(lv[l - 1])), f"level {l}"


def test_pyramid_level_count_rule(orc):
    # buildOpticalFlowPyramid stops when the next level is <= winSize on a side
    img = np.zeros((100, 400), np.uint8)
    lv = orc.build_pyramid(img, max_level=6)
    # 400x100 -> 200x50 -> 100x25 -> (50x13 stops)
    assert [a.shape for a in lv] == [(100, 400), (50, 200), (25, 100)]


def test_pyramid_constant(orc):
    img = np.full((70, 160), 137, np.uint8)
    for a in orc.build_pyramid(img, 3):
        assert np.all(a == 137)


@pytest.mark.parametrize("w,h", [(64, 40), (1280, 560)])
def test_scharr_matches_numpy(orc, w, h):
    img = synth.make_image(w, h, np.random.default_rng(2))
    assert np.array_equal(orc.scharr(img), np_scharr(img))


def test_scharr_ramp(orc):
    x = np.arange(64, dtype=np.int32)
    img = np.tile((3 * x) % 256, (32, 1)).astype(np.uint8)[:, :60]
    d = orc.scharr(img)
    # interior of a ramp of slope 3: dx = 16*2*3 = 96, dy = 0
    assert np.all(d[1:-1, 1:-1, 0] == 96)
    assert np.all(d[..., 1] == 0)


def _shifted_pair(w, h, dx, dy, seed=3):
    rng = np.random.default_rng(seed)
    big = synth.make_image(w + 40, h + 40, rng)
    I = big[20:20 + h, 20:20 + w].copy()
    J = big[20 - dy:20 - dy + h, 20 - dx:20 - dx + w].copy()   # J(x) = I(x - d)
    return I, J


@pytest.mark.parametrize("dx,dy", [(3, -2), (-7, 5), (0, 0), (12, 9)])
def test_lk_integer_shift_known_answer(orc, dx, dy):
    I, J = _shifted_pair(320, 140, dx, dy)
    rng = np.random.default_rng(4)
    pts = synth.pick_points(I, 40, rng).astype(np.float32)
    pts = pts[(pts[:, 0] > 30) & (pts[:, 0] < 290) & (pts[:, 1] > 30) & (pts[:, 1] < 110)]
    # initial flow = true shift + U(-1.5, 1.5) px, like the INS-predicted flow
    init = pts + np.array([dx, dy], np.float32) + rng.uniform(-1.5, 1.5, pts.shape).astype(np.float32)
    nxt, st, err = orc.calc_optical_flow_pyr_lk(I, J, pts, init)
    ok = st == 1
    assert ok.mean() > 0.9
    flow = nxt[ok] - pts[ok]
    assert np.abs(flow[:, 0] - dx).max() < 0.05
    assert np.abs(flow[:, 1] - dy).max() < 0.05


def test_lk_identity_exact(orc):
    I, _ = _shifted_pair(160, 70, 0, 0)
    pts = np.array([[40.25, 30.5], [80.0, 35.0], [120.75, 40.125]], np.float32)
    nxt, st, err = orc.calc_optical_flow_pyr_lk(I, I, pts, pts.copy())
    assert np.all(st == 1)
    assert np.array_equal(nxt, pts)
    assert np.all(err == 0)


def test_lk_out_of_image_status(orc):
    I, J = _shifted_pair(160, 70, 1, 1)
    pts = np.array([[-40.0, 10.0], [10.0, 500.0], [80.0, 35.0]], np.float32)
    nxt, st, err = orc.calc_optical_flow_pyr_lk(I, J, pts, pts.copy())
    assert st[0] == 0 and st[1] == 0
    assert err[0] == 0 and err[1] == 0


def test_lk_flat_image_min_eig(orc):
    I = np.full((70, 160), 90, np.uint8)
    pts = np.array([[80.0, 35.0]], np.float32)
    nxt, st, err = orc.calc_optical_flow_pyr_lk(I, I, pts, pts.copy())
    assert st[0] == 0


def test_fb_pyramid_reuse_identical(orc):
    """Appendix C.7: reusing pyramids is bit-identical to the 4x rebuild."""
    I, J, prev, init, _ = synth.make_pair(320, 140, 60, seed=11)
    a = orc.klt_fb(I, J, prev, init, reuse_pyramids=False)
    b = orc.klt_fb(I, J, prev, init, reuse_pyramids=True)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_fb_threaded_identical(orc):
    I, J, prev, init, _ = synth.make_pair(320, 140, 60, seed=12)
    a = orc.klt_fb(I, J, prev, init, nthreads=1)
    b = orc.klt_fb(I, J, prev, init, nthreads=4)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_fb_semantics(orc):
    """keep == st_f & st_b & !border & FB<0.5; kept_idx is the ordered keep list."""
    I, J, prev, init, truth = synth.make_pair(320, 140, 80, seed=13)
    r = orc.klt_fb(I, J, prev, init)
    nx, bk = r["next"], r["back"]
    border = (nx[:, 0] < 5) | (nx[:, 1] < 5) | (nx[:, 0] > 320 - 5.0) | (nx[:, 1] > 140 - 5.0)
    d = (bk - prev).astype(np.float32).astype(np.float64)
    fbd = np.sqrt(d[:, 0] ** 2 + d[:, 1] ** 2)
    keep = (r["st_f"] == 1) & (r["st_b"] == 1) & ~border & (fbd < 0.5)
    assert np.array_equal(keep.astype(np.uint8), r["keep"])
    assert np.array_equal(np.nonzero(keep)[0], r["kept_idx"])
    # on a clean similarity warp most points track to within a pixel of truth
    good = r["keep"] == 1
    assert good.mean() > 0.8
    assert np.median(np.abs(nx[good] - truth[good])) < 0.5


def test_empty_points(orc):
    I, J, prev, init, _ = synth.make_pair(160, 70, 4, seed=14)
    r = orc.klt_fb(I, J, prev[:0], init[:0])
    assert r["kept_idx"].size == 0

"""CPU tests of the detection restatement (oracle/detect.c): independent numpy
restatements of cornerMinEigenVal and the FILLED circle raster, structural
properties of goodFeaturesToTrack and a sub-pixel known answer for cornerSubPix.
(No reference fixtures exist for this path: SURVEY.md 8c.)"""
import numpy as np
import pytest

from gvx import synth


def np_circle_mask(w, h, pts, r):
    mask = np.full((h, w), 255, np.uint8)
    for x, y in pts:
        cx, cy = int(np.rint(np.float32(x))), int(np.rint(np.float32(y)))
        err, dx, dy, plus, minus = 0, r, 0, 1, 2 * r - 1
        while dx >= dy:
            for yy, x1, x2 in ((cy - dy, cx - dx, cx + dx), (cy + dy, cx - dx, cx + dx),
                               (cy - dx, cx - dy, cx + dy), (cy + dx, cx - dy, cx + dy)):
                if 0 <= yy < h:
                    mask[yy, max(x1, 0):min(x2, w - 1) + 1] = 0
            dy += 1
            err += plus
            plus += 2
            m = -1 if err > 0 else 0
            err -= minus & m
            dx += m
            minus -= m & 2
    return mask


def np_min_eig(img, x0, y0, rw, rh):
    """numpy float32 restatement of cornerMinEigenVal (ROI, parent-read Sobel)."""
    f32 = np.float32
    H, W = img.shape
    sc = f32(1.0 / 3060.0)
    sc2 = f32(2.0 / 3060.0)
    ys = np.arange(y0 - 1, y0 + rh + 1)
    xs = np.arange(x0 - 1, x0 + rw + 1)
    refl = lambda p, n: np.where(p < 0, -p, np.where(p >= n, 2 * n - 2 - p, p))  # noqa: E731
    P = img[refl(ys, H)][:, refl(xs, W)].astype(f32)
    s0, s1, s2 = P[:, :-2], P[:, 1:-1], P[:, 2:]
    rdx = (f32(-1) * s0 + f32(0) * s1) + s2
    rdy = (sc * s0 + sc2 * s1) + sc * s2
    dx = (rdx[:-2] + rdx[2:]) * sc + rdx[1:-1] * sc2
    dy = rdy[2:] - rdy[:-2]
    cov = [dx * dx, dx * dy, dy * dy]
    out = []
    for c in cov:
        p = np.pad(c.astype(np.float64), 1, mode="reflect")
        rs = (p[:, :-2] + p[:, 1:-1]) + p[:, 2:]
        s = ((rs[:-2] + rs[1:-1]) + rs[2:])
        out.append(s.astype(f32))
    a = out[0] * f32(0.5)
    b = out[1]
    c = out[2] * f32(0.5)
    return ((a + c) - np.sqrt((a - c) * (a - c) + b * b)).astype(f32)


def test_circle_mask_matches_numpy(orc):
    rng = np.random.default_rng(1)
    pts = np.c_[rng.uniform(-30, 350, 20), rng.uniform(-30, 170, 20)].astype(np.float32)
    pts = np.r_[pts, [[100.5, 50.5], [101.5, 60.5]]].astype(np.float32)  # round-half-even centres
    assert np.array_equal(orc.mask_circles(320, 140, pts, 58), np_circle_mask(320, 140, pts, 58))


def test_circle_mask_area(orc):
    m = orc.mask_circles(400, 400, np.array([[200, 200]], np.float32), 58)
    area = (m == 0).sum()
    assert abs(area - np.pi * 58 ** 2) < 2 * np.pi * 58


@pytest.mark.parametrize("roi", [(0, 0, 208, 181), (213, 186, 208, 181), (1065, 372, 213, 186), (5, 3, 40, 30)])
def test_min_eig_matches_numpy(orc, roi):
    img = synth.make_image(1280, 560, np.random.default_rng(2))
    x0, y0, rw, rh = roi
    a = orc.corner_min_eigen_val(img, x0, y0, rw, rh)
    b = np_min_eig(img, x0, y0, rw, rh)
    assert np.array_equal(a, b)


def test_gftt_properties(orc):
    img = synth.make_image(1280, 560, np.random.default_rng(3))
    x0, y0, rw, rh = 213, 0, 208, 181
    mask = np.full((rh, rw), 255, np.uint8)
    mask[50:100, 50:120] = 0
    pts = orc.good_features_to_track(img, x0, y0, rw, rh, mask, 8, 0.01, 58)
    assert 1 <= len(pts) <= 8
    eig = orc.corner_min_eigen_val(img, x0, y0, rw, rh)
    vals = [eig[int(y), int(x)] for x, y in pts]
    assert all(vals[i] >= vals[i + 1] for i in range(len(vals) - 1))
    for i in range(len(pts)):
        x, y = pts[i]
        assert x == int(x) and y == int(y)
        assert 1 <= x <= rw - 2 and 1 <= y <= rh - 2
        assert mask[int(y), int(x)] != 0
        for j in range(i):
            assert ((pts[i] - pts[j]) ** 2).sum() >= 58 ** 2


def _corner_image(cx, cy, w=120, h=100):
    """Blurred quadrant corner at (cx, cy)."""
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float64)
    sx = 1 / (1 + np.exp(-(xs - cx) / 0.8))
    sy = 1 / (1 + np.exp(-(ys - cy) / 0.8))
    v = 40 + 170 * (sx * sy + (1 - sx) * (1 - sy))
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("cx,cy", [(50.3, 40.7), (61.8, 52.2)])
def test_corner_subpix_known_answer(orc, cx, cy):
    img = _corner_image(cx, cy)
    xy = np.array([[round(cx), round(cy)]], np.float32)
    orc.lib().orc_corner_subpix(img.ctypes.data, img.shape[1], 0, 0, img.shape[1], img.shape[0],
                                xy.ctypes.data, 1, 5, 20, 0.01)
    # pixel centres sit on integer coordinates: the corner is at (cx, cy)
    assert abs(xy[0, 0] - cx) < 0.15 and abs(xy[0, 1] - cy) < 0.15


def test_features_detection_block_semantics(orc):
    img = synth.make_image(1280, 560, np.random.default_rng(4))
    g = orc.block_grid(1280, 560)
    assert (g.block_cols, g.block_rows, g.col, g.row, g.max_block_features, g.min_pixel_distance) == \
        (6, 3, 213, 186, 8, 58)
    pts, blk = orc.features_detection(img)
    assert blk.sum() == len(pts) and np.all(blk <= 8)
    # existing features: blocks that already hold >= 8 features detect nothing
    existing = np.array([[100.0, 100.0]] * 8 + [[300.0, 300.0]] * 3, np.float32)
    pts2, blk2 = orc.features_detection(img, existing, existing, True, 11)
    assert blk2[0] == 0 and blk2[1 * 6 + 1] <= 5
    # new corners avoid the masked discs
    for x, y in pts2:
        for ex, ey in existing:
            assert (x - ex) ** 2 + (y - ey) ** 2 > 50 ** 2
    # early exit when enough features are tracked
    none, _ = orc.features_detection(img, None, None, True, 146)
    assert none is None

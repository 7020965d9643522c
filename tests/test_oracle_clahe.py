"""The CPU restatement of Tracking::preprocessing's CLAHE and histogram check
(oracle/clahe.c) against an independent numpy restatement of the same OpenCV
4.x rules and against closed-form known answers.

OpenCV is absent here and the reference holds no CLAHE fixtures, so the
restatement is "parity unpinned" against cv::CLAHE itself."""
import numpy as np
import pytest

import oracle as orc

F32 = np.float32


def _np_clahe(img, clip_limit=3.0, tiles=(21, 21)):
    """numpy restatement of CLAHE_Impl::apply (8-bit), written from the rules in
    oracle/clahe.c's header, not from its code."""
    h, w = img.shape
    tx, ty = tiles
    if w % tx == 0 and h % ty == 0:
        ext = img
    else:
        ext = np.pad(img, ((0, ty - h % ty), (0, tx - w % tx)), mode="reflect")  # numpy reflect = REFLECT_101
    th, tw = ext.shape[0] // ty, ext.shape[1] // tx
    total = tw * th
    scale = F32(255) / F32(total)
    clip = max(int(clip_limit * total / 256), 1) if clip_limit > 0 else 0
    luts = np.zeros((ty, tx, 256), np.uint8)
    for j in range(ty):
        for i in range(tx):
            hist = np.bincount(ext[j * th:(j + 1) * th, i * tw:(i + 1) * tw].ravel(), minlength=256).astype(np.int64)
            if clip > 0:
                clipped = int(np.maximum(hist - clip, 0).sum())
                hist = np.minimum(hist, clip) + clipped // 256
                residual = clipped % 256
                if residual:
                    step = max(256 // residual, 1)
                    idx = np.arange(0, 256, step)[:residual]
                    hist[idx] += 1
            cs = np.cumsum(hist).astype(F32)
            luts[j, i] = np.clip(np.rint(cs * scale), 0, 255).astype(np.uint8)
    ys = np.arange(h, dtype=F32) * (F32(1) / F32(th)) - F32(0.5)
    xs = np.arange(w, dtype=F32) * (F32(1) / F32(tw)) - F32(0.5)
    ty1 = np.floor(ys).astype(np.int64)
    tx1 = np.floor(xs).astype(np.int64)
    ya = (ys - ty1.astype(F32)).astype(F32)
    xa = (xs - tx1.astype(F32)).astype(F32)
    ya1, xa1 = F32(1) - ya, F32(1) - xa
    ty2 = np.minimum(ty1 + 1, ty - 1)
    tx2 = np.minimum(tx1 + 1, tx - 1)
    ty1, tx1 = np.maximum(ty1, 0), np.maximum(tx1, 0)
    v = img.astype(np.int64)
    Y1, Y2 = ty1[:, None], ty2[:, None]
    X1, X2 = tx1[None, :], tx2[None, :]
    l11 = luts[Y1, X1, v].astype(F32)
    l12 = luts[Y1, X2, v].astype(F32)
    l21 = luts[Y2, X1, v].astype(F32)
    l22 = luts[Y2, X2, v].astype(F32)
    XA, XA1, YA, YA1 = xa[None, :], xa1[None, :], ya[:, None], ya1[:, None]
    res = (l11 * XA1 + l12 * XA) * YA1 + (l21 * XA1 + l22 * XA) * YA
    return np.clip(np.rint(res), 0, 255).astype(np.uint8), luts.reshape(ty * tx, 256)


def _img(h, w, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (h // 4 + 2, w // 4 + 2)).astype(np.float64)
    up = np.kron(base, np.ones((4, 4)))[:h, :w]
    return np.clip(up * 0.6 + rng.normal(0, 12, (h, w)) + 30, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("h,w,tiles,clip", [
    (560, 1280, (21, 21), 3.0),   # the reference geometry: both sides padded (61 x 27 tiles)
    (147, 210, (21, 21), 3.0),    # divisible both ways: no border
    (147, 215, (21, 21), 3.0),    # only width indivisible: a whole extra tile of rows
    (100, 100, (8, 8), 40.0),
    (64, 96, (4, 6), 0.0),        # clip disabled
    (33, 47, (3, 5), 1.0),        # clip floor of 1
])
def test_clahe_matches_numpy(h, w, tiles, clip):
    img = _img(h, w, seed=h * 1000 + w)
    ref, ref_luts = _np_clahe(img, clip, tiles)
    assert np.array_equal(orc.clahe_luts(img, clip, tiles), ref_luts)
    assert np.array_equal(orc.clahe(img, clip, tiles), ref)


@pytest.mark.parametrize("v", [0, 17, 128, 255])
def test_clahe_constant_image(v):
    """Constant image: every tile has one bin of tw*th pixels.  With the clip at
    c, the bin keeps c, the rest spreads evenly, so lut[v] = round(cumsum * scale)
    is the same for all tiles and the output is that constant."""
    h, w = 56, 84
    img = np.full((h, w), v, np.uint8)
    tw, th = 84 // 21 + 1, 56 // 21 + 1    # both sides indivisible -> padded
    total = tw * th
    clip = max(int(3.0 * total / 256), 1)
    clipped = total - clip
    hist = np.full(256, clipped // 256)
    hist[v] += clip
    res = clipped % 256
    if res:
        hist[np.arange(0, 256, max(256 // res, 1))[:res]] += 1
    expect = int(np.rint(F32(hist[:v + 1].sum()) * (F32(255) / F32(total))))
    out = orc.clahe(img, 3.0, (21, 21))
    assert np.all(out == expect)
    # without clipping a constant image maps to 255 (the cumsum is total at v)
    assert np.all(orc.clahe(img, 0.0, (21, 21)) == 255)


def test_hist_mean_known_answer():
    img = np.zeros((10, 20), np.uint8)
    img[:5] = 128
    img[5:, :10] = 255
    # sum_k hist[k]*k/256 / N : (100*128 + 50*255)/256/200
    assert orc.hist_mean(img) == pytest.approx((100 * 128 + 50 * 255) / 256 / 200, rel=1e-15)
    h = np.bincount(_img(60, 70, 3).ravel(), minlength=256)
    m = sum(float(F32(h[k]) * F32(k)) / 256.0 for k in range(256)) / (60 * 70)
    assert orc.hist_mean(_img(60, 70, 3)) == m


def test_bgr2gray_known_answers(orc):
    """cv::cvtColor(COLOR_BGR2GRAY), 8-bit: (B*1868 + G*9617 + R*4899 + 8192) >> 14
    (OpenCV 4.x RGB2Gray<uchar>, yuv_shift 14; BGR channel order)."""
    rng = np.random.default_rng(3)
    bgr = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    b, g, r = (bgr[..., k].astype(np.int64) for k in range(3))
    assert np.array_equal(orc.bgr2gray(bgr), ((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14).astype(np.uint8))
    px = np.array([[[255, 255, 255], [0, 0, 0], [255, 0, 0], [0, 255, 0], [0, 0, 255]]], np.uint8)
    # white stays 255 (the weights sum to 2^14); pure B / G / R: 29, 150, 76
    assert orc.bgr2gray(px).tolist() == [[255, 0, 29, 150, 76]]

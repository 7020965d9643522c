"""GPU parity of block-grid detection (gvx_detect) against the CPU restatement
(oracle/detect.c): corner positions after cornerSubPix and per-block counts are
required to be bit-exact (selection is integer/ordering work; the fp32/fp64
arithmetic follows the oracle's order, including the sequential fp64 sums)."""
import numpy as np
import pytest

from gvx import synth

pytestmark = pytest.mark.gpu


def _check(ctx, orc, gvx_mod, img, count_xy=None, mask_xy=None, ismask=True, n_existing=0, **kw):
    gp = gvx_mod.DetectParams.default(**kw)
    op = orc.DetectParams.default(**kw)
    ctx.frame_put(5, img)
    g, gb = ctx.detect(5, count_xy, mask_xy, ismask, n_existing, gp)
    o, ob = orc.features_detection(img, count_xy, mask_xy, ismask, n_existing, op)
    if o is None:
        assert g is None
        return None
    assert np.array_equal(gb[:len(ob)], ob), f"block counts gpu={gb[:len(ob)]} oracle={ob}"
    if not np.array_equal(g, o):
        bad = np.argwhere(np.any(g != o, axis=1))[:5, 0]
        raise AssertionError(f"corners differ at {bad.tolist()}: gpu={g[bad].tolist()} oracle={o[bad].tolist()}")
    return g


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_detect_fresh_frame(ctx, orc, gvx_mod, seed):
    img = synth.make_image(1280, 560, np.random.default_rng(seed))
    g = _check(ctx, orc, gvx_mod, img, ismask=False)
    assert len(g) > 100


def test_detect_with_tracked_points(ctx, orc, gvx_mod):
    rng = np.random.default_rng(7)
    img = synth.make_image(1280, 560, rng)
    pts = np.c_[rng.uniform(0, 1280, 70), rng.uniform(0, 560, 70)].astype(np.float32)
    pts[:3] = [[1279.6, 100.0], [10.5, 559.5], [400.5, 200.5]]  # out-of-grid index, half-way rounding
    _check(ctx, orc, gvx_mod, img, pts, pts, True, 70)


def test_detect_1920x1200_500(ctx, orc, gvx_mod):
    img = synth.make_image(1920, 1200, np.random.default_rng(9))
    _check(ctx, orc, gvx_mod, img, ismask=False, max_features=500)


def test_detect_small_and_flat(ctx, orc, gvx_mod):
    img = synth.make_image(320, 140, np.random.default_rng(11))
    img[:, :160] = 90  # flat half: no candidates there
    _check(ctx, orc, gvx_mod, img, ismask=False, max_features=40)


def test_detect_early_exit(ctx, orc, gvx_mod):
    img = synth.make_image(320, 140, np.random.default_rng(12))
    assert _check(ctx, orc, gvx_mod, img, n_existing=146) is None

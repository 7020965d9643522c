"""GPU parity of the batched pyramid pass (gvx_build_pyramids_dev, the pass
gvx_klt_fb_batch runs before LK) against the CPU restatement of OpenCV's
buildOpticalFlowPyramid (oracle.build_pyramid): every level >= 1 with its whole
32-pixel REFLECT_101 ring, BIT-EXACT.  Level 0 is read in place when w % 4 == 0
(edge strips gather the reflected columns; the ring is written by the streaming
pass itself), copied to a padded slot otherwise; levels smaller than 66 pixels get
their ring from the separate ring kernel."""
import numpy as np
import pytest

from gvx import synth

pytestmark = pytest.mark.gpu

PAD = 32


def _build(ctx, imgs, L, stride=None):
    import torch
    n, h, w = imgs.shape
    stride = stride or w
    buf = np.zeros((n, h, stride), np.uint8)
    buf[:, :, :w] = imgs
    d_img = torch.from_numpy(buf).cuda()
    lay = ctx.pyramid_layout(w, h, L)
    d_out = torch.zeros(n * lay["bytes"], dtype=torch.uint8, device="cuda")
    # torch's upload and fill run on torch's stream, the pass on the context's own:
    # they must be done first (a 300 MB fill still running overwrote the pass's rows)
    torch.cuda.synchronize()
    ctx.build_pyramids_dev(n, w, h, d_img.data_ptr(), h * stride, stride, L, d_out.data_ptr())
    ctx.sync()
    return lay, d_out.cpu().numpy().reshape(n, lay["bytes"])


def _level(lay, pyr, l):
    rows, pitch = int(lay["h"][l]) + 2 * PAD, int(lay["pitch"][l])
    o = int(lay["off"][l])
    return pyr[o:o + rows * pitch].reshape(rows, pitch)[:, :int(lay["w"][l]) + 2 * PAD]


@pytest.mark.parametrize("w,h,L,stride", [
    (1280, 560, 3, None),    # configs[1]: three strips, in-place level 0
    (1920, 1200, 4, None),   # configs[2]: a second pass (level 4 from padded level 3)
    (640, 480, 3, None),     # widths that are multiples of 8: right edge r = 1
    (324, 150, 2, None),     # w % 8 == 4: right edge r = 2, one strip, two levels
    (1000, 77, 1, None),     # one level, band taller than the level
    (488, 200, 3, None),     # a last strip with fewer than 33 level-1 columns
    (200, 100, 3, None),     # levels below 66 px: rings from ring_kernel
    (333, 149, 3, None),     # w % 4 != 0: padded level-0 copy path
    (320, 140, 3, 352),      # row stride > w (in place)
])
def test_batched_pyramid_bit_exact(ctx, orc, w, h, L, stride):
    rng = np.random.default_rng(w * 31 + h)
    imgs = np.stack([synth.make_image(w, h, rng) for _ in range(3)])
    imgs[1] = rng.integers(0, 256, (h, w), dtype=np.uint8)  # full-range noise at every border
    lay, pyr = _build(ctx, imgs, L, stride)
    for i in range(imgs.shape[0]):
        ref = orc.build_pyramid(imgs[i], L)
        assert len(ref) == lay["nlev"]
        for l in range(1, lay["nlev"]):
            got = _level(lay, pyr[i], l)
            want = np.pad(ref[l], PAD, mode="reflect")
            if not np.array_equal(got, want):
                bad = np.argwhere(got != want)
                raise AssertionError(f"image {i} level {l}: {len(bad)} mismatches, first (padded row, col) "
                                     f"{bad[:6].tolist()}")


def test_batched_pyramid_matches_frame_cache(ctx, gvx_mod):
    """The in-place batched pass and the frame cache's padded-copy pass give the
    same levels (two border paths, one result)."""
    w, h, L = 1280, 560, 3
    img = synth.make_image(w, h, np.random.default_rng(77))
    lay, pyr = _build(ctx, img[None], L)
    ctx.frame_put(31, img, gvx_mod.KltParams.default(max_level=L))
    for l in range(1, L + 1):
        np.testing.assert_array_equal(_level(lay, pyr[0], l), ctx.frame_level_padded(31, l, PAD))
    ctx.frame_drop(31)


@pytest.mark.parametrize("w,h,L,stride", [
    (1280, 560, 3, None),    # configs[1]: side bands by side_kernel at every level
    (1920, 1200, 4, None),   # configs[2]: and a second pass
    (324, 150, 2, None),     # level-1 width % 4 == 2: ring_kernel's generic sides mode
    (488, 200, 3, None),     # side_kernel, generic sides, and a whole ring (level 3 < 66 rows)
    (200, 100, 3, None),     # whole rings from ring_kernel
    (320, 140, 3, 352),      # row stride > w
])
def test_batched_pyramid_large_launch_bit_exact(ctx, orc, w, h, L, stride):
    """Launches of at least 16 waves per CU leave the side bands to side_kernel /
    ring_kernel (pyramid.hip stream_sides).  Enough images for that mode, three
    distinct ones tiled; the first three and the last are checked, rings included."""
    w1, h1 = (w + 1) // 2, (h + 1) // 2
    units = -(-w1 // 240) * -(-h1 // 72)  # strips x bands per image (pyramid.hip STREAM_BAND 72)
    n = max(3, -(-16 * 256 * 5 // 4 // units))  # 1.25x the large-launch threshold at 256 CUs
    rng = np.random.default_rng(w * 17 + h)
    base = np.stack([synth.make_image(w, h, rng) for _ in range(3)])
    base[1] = rng.integers(0, 256, (h, w), dtype=np.uint8)
    imgs = base[np.arange(n) % 3]
    lay, pyr = _build(ctx, imgs, L, stride)
    refs = [orc.build_pyramid(base[i], L) for i in range(3)]
    for i in (0, 1, 2, n - 1):
        ref = refs[i % 3]
        for l in range(1, lay["nlev"]):
            got = _level(lay, pyr[i], l)
            want = np.pad(ref[l], PAD, mode="reflect")
            if not np.array_equal(got, want):
                bad = np.argwhere(got != want)
                raise AssertionError(f"{n} images, image {i} level {l}: {len(bad)} mismatches, first (padded row, "
                                     f"col) {bad[:6].tolist()}")

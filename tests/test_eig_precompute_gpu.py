"""gvx_frame_eig_dev: the detection's eigenvalue map computed ahead of the
tracking call (the pipelined replay puts it on the preprocessing branch).
The corners of a detection that reads the precomputed map are bit-identical to
one that computes it in line, and a map computed for an earlier image of the
same frame slot is never used (the slot's write count invalidates it).  The
sequence tests hold both forms against the oracle frame by frame."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, N, L = 1280, 560, 150, 3


def _detect(ctx, gvx_mod, fid, pts_xy):
    """Detection on cached frame fid with the given tracked points (no LK):
    -> (track list, corners, n_corners)."""
    import torch
    dev = torch.device("cuda", 0)
    kp = gvx_mod.KltParams.default(max_level=L)
    dp = gvx_mod.DetectParams.default(max_features=N)
    pts = torch.zeros((N, 2), dtype=torch.float32, device=dev)
    pts[:len(pts_xy)] = torch.from_numpy(pts_xy)
    vel = torch.zeros_like(pts)
    init = pts.clone()
    n = torch.tensor([len(pts_xy)], dtype=torch.int32, device=dev)
    corners = torch.zeros((64 * 64, 2), dtype=torch.float32, device=dev)
    nc = torch.zeros(1, dtype=torch.int32, device=dev)
    __import__("torch").cuda.synchronize()  # torch fills on its stream; gvx launches on its own
    ctx.track_frame_dev(fid, fid, False, pts.data_ptr(), vel.data_ptr(), init.data_ptr(), n.data_ptr(), N, W, H,
                        klt=kp, detect=dp, d_corners=corners.data_ptr(), d_n_corners=nc.data_ptr())
    ctx.sync()
    k = int(n.cpu()[0])
    m = int(nc.cpu()[0])
    return pts.cpu().numpy()[:k], corners.cpu().numpy()[:max(m, 0)], m


def test_precomputed_map_matches_inline(ctx, gvx_mod):
    import torch
    from gvx import synth
    dev = torch.device("cuda", 0)
    frames, _ = synth.make_sequence(W, H, 3, dev, seed=synth.SEED + 5)
    kp = gvx_mod.KltParams.default(max_level=L)
    dp = gvx_mod.DetectParams.default(max_features=N)
    rng = np.random.default_rng(3)
    pts = np.stack([rng.uniform(5, W - 5, 40), rng.uniform(5, H - 5, 40)], 1).astype(np.float32)
    for t in range(3):
        ctx.frame_preprocess_dev(70, frames[t].data_ptr(), W, H, params=kp)
        want = _detect(ctx, gvx_mod, 70, pts)   # eigenvalues in line
        ctx.frame_preprocess_dev(71, frames[t].data_ptr(), W, H, params=kp)
        ctx.frame_eig_dev(71, detect=dp)
        got = _detect(ctx, gvx_mod, 71, pts)    # the precomputed map
        assert want[2] > 0, "the detection ran"
        assert got[2] == want[2]
        assert np.array_equal(got[1], want[1]), f"frame {t}: corners"
        assert np.array_equal(got[0], want[0]), f"frame {t}: track list"


def test_stale_map_not_used(ctx, gvx_mod):
    import torch
    from gvx import synth
    dev = torch.device("cuda", 0)
    frames, _ = synth.make_sequence(W, H, 40, dev, seed=synth.SEED + 6)
    kp = gvx_mod.KltParams.default(max_level=L)
    dp = gvx_mod.DetectParams.default(max_features=N)
    pts = np.zeros((0, 2), np.float32)
    ctx.frame_preprocess_dev(72, frames[39].data_ptr(), W, H, params=kp)
    want = _detect(ctx, gvx_mod, 72, pts)
    # slot 73: the map of frame 0, then frame 39 written over it
    ctx.frame_preprocess_dev(73, frames[0].data_ptr(), W, H, params=kp)
    ctx.frame_eig_dev(73, detect=dp)
    ctx.frame_preprocess_dev(73, frames[39].data_ptr(), W, H, params=kp)
    got = _detect(ctx, gvx_mod, 73, pts)
    assert got[2] == want[2] and np.array_equal(got[1], want[1])

"""hipGraph capture of one frame pair (gvx_capture_begin / gvx_capture_end /
gvx_graph_launch): replaying the captured initial-flow copy
+ pyramid + LK + compaction gives the eager call's outputs bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_graph_replay_matches_eager(ctx, gvx_mod):
    import torch
    from gvx import synth
    W, H, N = 1280, 560, 150
    I, J, P, Q = synth.make_batch(1, W, H, N, seed=synth.SEED, distinct=1)
    dev = torch.device("cuda", 0)
    dI, dJ, dP, dQ = (torch.from_numpy(a).to(dev) for a in (I, J, P, Q))

    def outputs():
        o = dict(N=torch.empty_like(dQ), B=torch.empty_like(dQ),
                 F=torch.zeros((1, N), dtype=torch.uint8, device=dev),
                 K=torch.full((1, N), -7, dtype=torch.int32, device=dev),
                 NK=torch.full((1,), -7, dtype=torch.int32, device=dev))
        torch.cuda.synchronize()  # torch fills on its stream; gvx launches on its own
        return o

    eager, replay = outputs(), outputs()
    params = gvx_mod.KltParams.default()

    def enqueue(o):
        ctx.copy_dev(o["N"].data_ptr(), dQ.data_ptr(), dQ.numel() * dQ.element_size())
        ctx.klt_fb_batch_dev(1, W, H, dI.data_ptr(), dJ.data_ptr(), N, dP.data_ptr(), o["N"].data_ptr(),
                             o["B"].data_ptr(), o["F"].data_ptr(), o["K"].data_ptr(), o["NK"].data_ptr(),
                             params=params)

    torch.cuda.synchronize()
    enqueue(eager)  # uncaptured first call: sizes the scratch buffers
    ctx.sync()
    ctx.capture_begin()
    enqueue(replay)
    g = ctx.capture_end()
    ctx.sync()
    assert int(replay["NK"].cpu()[0]) == -7  # capturing runs nothing
    for _ in range(3):
        g.launch()
    ctx.sync()
    assert int(eager["NK"].cpu()[0]) > 0
    for k in eager:
        assert torch.equal(eager[k], replay[k]), k
    g.destroy()


def test_capture_refused_while_profiling(ctx, gvx_mod):
    ctx.profile(True)
    try:
        with pytest.raises(gvx_mod.GvxError):
            ctx.capture_begin()
    finally:
        ctx.profile(False)


def test_stale_graph_refused(gvx_mod):
    """A graph holds raw pointers into the context's scratch: once a larger call
    reallocates the batch pyramids, replaying it must be refused (not read freed
    memory).  A private context: the session one's scratch may already be larger
    than `big` needs."""
    import torch
    from gvx import synth
    ctx = gvx_mod.Context(0)
    W, H, N = 320, 140, 16
    dev = torch.device("cuda", 0)
    params = gvx_mod.KltParams.default()

    def bufs(n):
        I, J, P, Q = synth.make_batch(n, W, H, N, seed=synth.SEED, distinct=1)
        d = {k: torch.from_numpy(a).to(dev) for k, a in zip("IJPQ", (I, J, P, Q))}
        d.update(N=d["Q"].clone(), B=torch.empty_like(d["Q"]), F=torch.zeros((n, N), dtype=torch.uint8, device=dev),
                 K=torch.zeros((n, N), dtype=torch.int32, device=dev), NK=torch.zeros((n,), dtype=torch.int32, device=dev))
        torch.cuda.synchronize()  # torch fills on its stream; gvx launches on its own
        return d

    def enqueue(d, n):
        ctx.klt_fb_batch_dev(n, W, H, d["I"].data_ptr(), d["J"].data_ptr(), N, d["P"].data_ptr(), d["N"].data_ptr(),
                             d["B"].data_ptr(), d["F"].data_ptr(), d["K"].data_ptr(), d["NK"].data_ptr(),
                             params=params)

    small, big = bufs(1), bufs(64)
    enqueue(small, 1)
    ctx.sync()
    ctx.capture_begin()
    enqueue(small, 1)
    g = ctx.capture_end()
    g.launch()
    ctx.sync()
    enqueue(big, 64)  # grows the batch pyramid scratch: the graph's pointers are freed
    ctx.sync()
    with pytest.raises(gvx_mod.GvxError):
        g.launch()
    g.destroy()
    ctx.close()


def test_branch_order_and_misuse(gvx_mod):
    """gvx_branch_begin / _end / _join: the branch sees everything enqueued before
    it, the context stream after gvx_branch_join sees the branch's writes, index
    advance is a device-side += , and misuse is refused (nested branches, ending
    without a branch, capturing with a branch open).  A private context."""
    import torch
    ctx = gvx_mod.Context(0)
    dev = torch.device("cuda", 0)
    n = 1 << 20
    src = torch.arange(n, dtype=torch.int32, device=dev)
    a, b, c = (torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(3))
    idx = torch.full((1,), 5, dtype=torch.int32, device=dev)
    nb = n * 4
    try:
        torch.cuda.synchronize()
        with pytest.raises(gvx_mod.GvxError):
            ctx.branch_end()  # no branch open
        for _ in range(3):
            ctx.copy_dev(a.data_ptr(), src.data_ptr(), nb)        # context stream
            ctx.branch_begin()
            with pytest.raises(gvx_mod.GvxError):
                ctx.branch_begin()                                 # one branch at a time
            ctx.copy_dev(b.data_ptr(), a.data_ptr(), nb)           # branch: after the first copy
            ctx.index_advance_dev(idx.data_ptr(), 2)
            ctx.branch_end()
            with pytest.raises(gvx_mod.GvxError):
                ctx.capture_begin()                                # an ended branch is still open
            ctx.branch_join()
            ctx.copy_dev(c.data_ptr(), b.data_ptr(), nb)           # after the join
            ctx.sync()
            assert torch.equal(c, src)
            a.zero_(), b.zero_(), c.zero_()
            torch.cuda.synchronize()
        assert int(idx.cpu()[0]) == 5 + 2 * 3
        # gvx_sync completes an ended branch: a capture may begin afterwards
        ctx.branch_begin()
        ctx.branch_end()
        ctx.sync()
        ctx.capture_begin()
        ctx.copy_dev(a.data_ptr(), src.data_ptr(), nb)
        g = ctx.capture_end()
        g.destroy()
    finally:
        ctx.close()


def test_capture_needing_scratch_growth_refused(gvx_mod):
    """a captured gvx_build_pyramids_dev with more strip / band units
    than any earlier uncaptured call needs its scratch to grow, which cannot
    happen inside a capture: the call fails (no kernel with a null scratch
    pointer is captured) and gvx_capture_end refuses the graph; the context is
    usable afterwards."""
    import torch
    from gvx import synth
    ctx = gvx_mod.Context(0)
    try:
        W, H, L = 320, 140, 3
        lay = gvx_mod.pyramid_layout(W, H, L)
        dev = torch.device("cuda", 0)
        imgs = torch.from_numpy(np.stack([synth.make_image(W, H, np.random.default_rng(i)) for i in range(64)])).to(dev)
        out = torch.empty(64 * lay["bytes"], dtype=torch.uint8, device=dev)
        ctx.build_pyramids_dev(1, W, H, imgs.data_ptr(), W * H, W, L, out.data_ptr())  # sizes for one image
        ctx.sync()
        ctx.capture_begin()
        with pytest.raises(gvx_mod.GvxError):
            ctx.build_pyramids_dev(64, W, H, imgs.data_ptr(), W * H, W, L, out.data_ptr())
        with pytest.raises(gvx_mod.GvxError):
            ctx.capture_end()
        # the same call uncaptured now works, and so does a capture of it
        ctx.build_pyramids_dev(64, W, H, imgs.data_ptr(), W * H, W, L, out.data_ptr())
        ctx.sync()
        g = ctx.capture(ctx.build_pyramids_dev, 64, W, H, imgs.data_ptr(), W * H, W, L, out.data_ptr())
        g.launch()
        ctx.sync()
        g.destroy()
    finally:
        ctx.close()


def test_capture_abort_after_failed_call(gvx_mod):
    """A call that raises inside Context.capture aborts the capture
    (gvx_capture_abort): the context is not left capturing."""
    import torch
    ctx = gvx_mod.Context(0)
    try:
        def bad():
            ctx.frame_drop(12345)  # refused during a capture
        with pytest.raises(gvx_mod.GvxError):
            ctx.capture(bad)
        ctx.capture_abort()  # no capture open: a no-op
        # the context works and can capture again
        buf = torch.zeros(1024, dtype=torch.uint8, device="cuda")
        src = torch.full((1024,), 9, dtype=torch.uint8, device="cuda")
        g = ctx.capture(ctx.copy_dev, buf.data_ptr(), src.data_ptr(), 1024)
        g.launch()
        ctx.sync()
        assert int(buf.sum().item()) == 9 * 1024
        g.destroy()
    finally:
        ctx.close()

"""hipGraph capture of one frame pair (gvx_capture_begin / gvx_capture_end /
gvx_graph_launch): replaying the captured initial-flow copy
+ pyramid + LK + compaction gives the eager call's outputs bit for bit."""
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
        return dict(N=torch.empty_like(dQ), B=torch.empty_like(dQ),
                    F=torch.zeros((1, N), dtype=torch.uint8, device=dev),
                    K=torch.full((1, N), -7, dtype=torch.int32, device=dev),
                    NK=torch.full((1,), -7, dtype=torch.int32, device=dev))

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

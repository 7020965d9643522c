"""Parity of the exact launch bench.py times (VERDICT r03 "missing" 1).

bench.py's step is one gvx_klt_fb_batch_init_dev over 256 synthetic pairs
(bench.KltWorkload: synth.make_batch(256, ..., seed=synth.SEED, distinct=16),
the predictions in their own buffer, tracked points to a separate one).  At
38,400 / 128,000 points per launch that is the batched LK instance (klt.hip:
more than 4,096 points -> three points per wave in the exact order, two in the
fp32 orders) on the configs' own geometry.
Here the same object runs the same launch and sampled pairs are compared
BIT-EXACT with the restatement (oracle.klt_fb, pyramids built once per image,
as the batched path does) in the three window-sum orders: next, back, flags
(bit0 forward status, bit1 backward status, bit2 keep), n_kept and kept_idx.
Every one of the 256 pairs is also checked against the distinct pair it tiles
(same input, same output), so no launch position goes unchecked.
Reference call: ic_gvins/ic_gvins/tracking/tracking.cc:385-408."""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu

MODES = [pytest.param(0, id="exact"), pytest.param(1, id="f32_scalar"), pytest.param(2, id="f32_simd4")]
# configs[1] / configs[2] at the bench's batch size; 8 distinct pairs sampled at
# launch positions spread over the batch (pair i tiles distinct pair i % 16)
CONFIGS = [pytest.param(1280, 560, 150, 3, id="configs1_1280x560_n150_L3"),
           pytest.param(1920, 1200, 500, 4, id="configs2_1920x1200_n500_L4")]
SAMPLE = [0, 17, 34, 51, 100, 133, 202, 255]

_WL = {}


def _workload(w, h, n):
    import torch
    key = (w, h, n)
    if key not in _WL:
        _WL.clear()  # one configuration resident at a time
        _WL[key] = bench.KltWorkload(256, w, h, n, torch.device("cuda", 0))
    return _WL[key]


def _assert_same(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    if not np.array_equal(a, b):
        diff = np.argwhere(a != b)
        raise AssertionError(f"{what}: {len(diff)} mismatches, first at {diff[:5].tolist()}: "
                             f"gpu={a[tuple(diff[0])]} oracle={b[tuple(diff[0])]}")


@pytest.mark.parametrize("w,h,n,L", CONFIGS)
@pytest.mark.parametrize("mode", MODES)
def test_bench_launch_bit_exact(ctx, orc, gvx_mod, w, h, n, L, mode):
    wl = _workload(w, h, n)
    assert wl.n_pairs * n > 4096  # the batched (three / two points per wave) instance
    wl.N.fill_(np.nan)
    wl.NK.fill_(-1)
    __import__("torch").cuda.synchronize()  # torch fills on its stream; gvx launches on its own
    wl.step(ctx, gvx_mod.KltParams.default(max_level=L, accum=mode))
    ctx.sync()
    nxt, back = wl.N.cpu().numpy(), wl.B.cpu().numpy()
    flags, kept, nk = wl.F.cpu().numpy(), wl.K.cpu().numpy(), wl.NK.cpu().numpy()
    # the inputs are left as they were (the initial flow has its own buffer)
    I, J, P, Q = wl.host
    assert np.array_equal(wl.Q.cpu().numpy(), Q)
    # every launch position equals the distinct pair it tiles
    rep = np.arange(wl.n_pairs) % 16
    for name, a in (("next", nxt), ("back", back), ("flags", flags), ("n_kept", nk)):
        _assert_same(a, a[rep], f"tiling {name}")
    orc_mode = {0: orc.ACC_EXACT, 1: orc.ACC_F32, 2: orc.ACC_F32X4}[mode]
    with orc.lk_accum(orc_mode):
        for i in SAMPLE:
            o = orc.klt_fb(I[i], J[i], P[i], Q[i], params=orc.KltParams.default(max_level=L),
                           reuse_pyramids=True, nthreads=8)
            _assert_same(nxt[i], o["next"], f"pair {i} next")
            _assert_same(back[i], o["back"], f"pair {i} back")
            _assert_same(flags[i], o["st_f"] | (o["st_b"] << 1) | (o["keep"] << 2), f"pair {i} flags")
            assert nk[i] == len(o["kept_idx"]), f"pair {i} n_kept {nk[i]} vs {len(o['kept_idx'])}"
            _assert_same(kept[i][:nk[i]], o["kept_idx"], f"pair {i} kept_idx")
            assert nk[i] > 0.9 * n  # the synthetic pairs track


@pytest.mark.parametrize("w,h,n,L", CONFIGS[:1])
def test_bench_pipelined_run_equals_step(ctx, gvx_mod, w, h, n, L):
    """The headline's software-pipelined steps (bench.KltWorkload.run: batch t+1's
    pyramid pass on a side branch beside batch t's LK, gvx_klt_batch_pyramids_dev +
    gvx_klt_fb_batch_pyr_dev, two pyramid slots) give the bits of the single
    launch checked against the oracle above, after every one of k steps."""
    import torch
    wl = _workload(w, h, n)
    p = gvx_mod.KltParams.default(max_level=L)
    wl.step(ctx, p)
    ctx.sync()
    ref = [t.cpu().numpy() for t in (wl.N, wl.B, wl.F, wl.K, wl.NK)]
    seen = []

    def check():
        ctx.sync()
        got = [t.cpu().numpy() for t in (wl.N, wl.B, wl.F, wl.K, wl.NK)]
        for name, a, b in zip(("next", "back", "flags", "kept_idx", "n_kept"), got, ref):
            _assert_same(a, b, f"pipelined step {len(seen)} {name}")
        seen.append(1)
        for t in (wl.N, wl.B):
            t.fill_(np.nan)
        wl.NK.fill_(-1)
        torch.cuda.synchronize()  # the fills (torch's stream) land before the next LK (the context's)

    wl.run(ctx, p, 5, True, check)
    assert len(seen) == 5
    lay = gvx_mod.pyramid_layout(w, h, L)
    assert wl._pyr[0].numel() == 2 * wl.n_pairs * lay["bytes"]


@pytest.mark.parametrize("w,h,n,L", CONFIGS)
def test_bench_launch_phases_same_bits(ctx, gvx_mod, w, h, n, L):
    """The bench's launch with each point group's chain in one wave (the
    default) or cut into phases of 1, 2, 3 or 4 levels, dispatched in
    superchunks of 8 up to all groups (gvx_set_klt_phases): every output of all
    256 pairs identical (the default is pinned to the oracle above)."""
    wl = _workload(w, h, n)
    p = gvx_mod.KltParams.default(max_level=L)
    outs = {}
    try:
        for lpp, sc in ((0, 4096), (1, 0), (2, 0), (3, 0), (1, 8), (2, 1000), (4, 100000), (0, 4096)):
            ctx.set_klt_phases(lpp, sc)
            wl.N.fill_(np.nan)
            wl.B.fill_(np.nan)
            wl.F.fill_(255)
            wl.K.fill_(-1)
            wl.NK.fill_(-1)
            __import__("torch").cuda.synchronize()  # torch fills on its stream; gvx launches on its own
            wl.step(ctx, p)
            ctx.sync()
            got = [a.cpu().numpy() for a in (wl.N, wl.B, wl.F, wl.K, wl.NK)]
            if (lpp, sc) in outs:  # a repeated launch: the hand-off tags were left at 0
                for name, a, b in zip(("next", "back", "flags", "kept", "n_kept"), got, outs[(lpp, sc)]):
                    _assert_same(a, b, f"lpp {lpp} repeat {name}")
            outs[(lpp, sc)] = got
    finally:
        ctx.set_klt_phases(0, 4096)
    for key, o in outs.items():
        for name, a, b in zip(("next", "back", "flags", "kept", "n_kept"), o, outs[(0, 4096)]):
            _assert_same(a, b, f"lpp/superchunk {key} {name}")


@pytest.mark.parametrize("n_ctx", [2, 3])
def test_bench_multi_context_run_equals_step(ctx, gvx_mod, n_ctx):
    """The headline's default run (bench.KltWorkload.run with further contexts:
    step t on context t % n_ctx, each with its own stream, pyramid scratch and
    output buffers, no waits between the streams) gives, on every context's
    outputs, the bits of the single launch checked against the oracle above."""
    import torch
    wl = _workload(1280, 560, 150)
    p = gvx_mod.KltParams.default(max_level=3)
    wl.step(ctx, p)
    ctx.sync()
    ref = [t.cpu().numpy() for t in (wl.N, wl.B, wl.F, wl.K, wl.NK)]
    more = tuple(gvx_mod.Context(0) for _ in range(n_ctx - 1))
    try:
        outs = [dict(N=wl.N, B=wl.B, F=wl.F, K=wl.K, NK=wl.NK)] + [wl._outs(i) for i in range(1, n_ctx)]
        for o in outs:
            for k in ("N", "B"):
                o[k].fill_(np.nan)
            o["NK"].fill_(-1)
        torch.cuda.synchronize()
        wl.run(ctx, p, 2 * n_ctx + 1, False, more=more)
        for c in (ctx,) + more:
            c.sync()
        for i, o in enumerate(outs):
            got = [o[k].cpu().numpy() for k in ("N", "B", "F", "K", "NK")]
            for name, a, b in zip(("next", "back", "flags", "n_kept"), got[:3] + got[4:], ref[:3] + ref[4:]):
                _assert_same(a, b, f"context {i} {name}")
            for q in range(wl.n_pairs):  # kept_idx is defined up to n_kept
                _assert_same(got[3][q][:ref[4][q]], ref[3][q][:ref[4][q]], f"context {i} pair {q} kept_idx")
    finally:
        for c in more:
            c.close()

"""Host logic of bench.KltWorkload.run (CPU, no device calls): the software-
pipelined configs[1] steps enqueue exactly k pyramid passes and k LK passes, each
LK on the slot its batch's pyramids went to, every pyramid pass on a side branch
that is ended before the LK it overlaps and joined before the next LK reads it, and
never a build into the slot the LK in flight reads.  The eager form enqueues k
one-call steps."""
import torch

import bench


class _Ctx:
    def __init__(self):
        self.calls = []

    def __getattr__(self, name):
        def rec(*a, **kw):
            self.calls.append((name, a))
        return rec


class _Params:
    max_level = 3


def _workload():
    # 2 tiny pairs on the CPU: run() only enqueues (the context is a recorder)
    return bench.KltWorkload(2, 64, 48, 4, torch.device("cpu"), distinct=2)


def test_pipelined_run_order():
    wl = _workload()
    for k in (1, 2, 5):
        ctx = _Ctx()
        steps = []
        wl.run(ctx, _Params(), k, True, lambda: steps.append(len(ctx.calls)))
        names = [c[0] for c in ctx.calls]
        assert names.count("klt_batch_pyramids_dev") == k
        assert names.count("klt_fb_batch_pyr_dev") == k
        assert len(steps) == k
        slots = {0: wl._pyr[0].data_ptr(), 1: wl._pyr[1].data_ptr()}
        built, open_branch, in_branch = {}, False, False
        t = 0
        for name, a in ctx.calls:
            if name == "branch_begin":
                assert not open_branch and not in_branch
                in_branch = True
            elif name == "branch_end":
                assert in_branch
                in_branch, open_branch = False, True
            elif name == "branch_join":
                assert open_branch
                open_branch = False
            elif name == "klt_batch_pyramids_dev":
                # the first build runs on the context stream; later ones on the branch
                assert in_branch == (len(built) > 0)
                built[len(built)] = a[-1]
            elif name == "klt_fb_batch_pyr_dev":
                assert not in_branch
                assert a[5] == slots[t & 1] == built[t]  # this batch's slot
                if t + 1 < k:
                    assert open_branch  # batch t+1's build runs beside it
                t += 1
        assert t == k and not open_branch and not in_branch
        # consecutive builds alternate slots (a build never targets the slot read by
        # the LK enqueued just before it on the other stream)
        assert all(built[i] == slots[i & 1] for i in built)


def test_eager_run_is_one_call_per_step():
    wl = _workload()
    ctx = _Ctx()
    wl.run(ctx, _Params(), 4, False)
    assert [c[0] for c in ctx.calls] == ["klt_fb_batch_init_dev"] * 4


def test_multi_context_run_round_robin():
    """--streams N: step t runs on context t % N, the first context into the
    workload's own buffers and every other one into buffers of its own."""
    wl = _workload()
    ctxs = [_Ctx(), _Ctx(), _Ctx()]
    steps = []
    wl.run(ctxs[0], _Params(), 7, True, lambda: steps.append(1), more=tuple(ctxs[1:]))
    assert len(steps) == 7
    assert [len(c.calls) for c in ctxs] == [3, 2, 2]
    for c in ctxs:
        assert all(name == "klt_fb_batch_init_dev" for name, _ in c.calls)
    # output pointers (N, B, F, K, NK: args 8..12): one set per context
    sets = [{tuple(a[8:13]) for _, a in c.calls} for c in ctxs]
    assert all(len(s) == 1 for s in sets)
    assert len(set.union(*sets)) == 3
    assert sets[0] == {(wl.N.data_ptr(), wl.B.data_ptr(), wl.F.data_ptr(), wl.K.data_ptr(), wl.NK.data_ptr())}

#!/usr/bin/env python3
"""bench.py -- KLT frames/s on MI355X (BASELINE.json metric, configs[1]).

A step = one pass of the KLT hot path over one batch of synthetic frame pairs
resident in HBM: for every pair build both image pyramids, forward LK with the
initial flow, backward LK, FB/border status and reduceVector compaction
(SURVEY.md 8d "frame-pair" unit; tracking/tracking.cc:380-408 of the reference).
Workload (configs[1]): 1280x560 mono, 150 features, maxLevel 3, 21x21 window.
value = frame pairs processed by all ranks / max-over-ranks wall time.

Multi-GPU: one process per GPU (torch.distributed.run), pairs sharded by rank
with no data-path collective (weak scaling).  --gather adds the offline
batch-replay exchange (configs[4]): per-step results (n_kept per pair) are
all-gathered over RCCL inside the timed region.

roofline.achieved = SURVEY.md 8d algorithmic bytes x pairs / device time of the
pipeline's kernels (HIP events on the context stream, timed region only);
roofline.traffic = PMC HBM bytes per step from profiles/pmc_traffic.json
(tools/pmc.sh + tools/traffic.py) when it was measured on this workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs P] [--gather]
    python bench.py --mock [--backend gloo]   # launcher / aggregation logic without a GPU
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ic-gvins_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def rank_setup(args):
    """One process per GPU: (dist | None, device, world, rank, local).

    A process group is opened at world > 1, and at world 1 with --dist (under
    torch.distributed.run), so the RCCL code path -- device-tensor all_gather,
    gather and all_reduce -- runs on a one-GPU box (tests/test_bench_rccl_gpu.py).

    nccl (RCCL over xGMI, the default) needs one GPU per rank.  gloo is the
    rehearsal backend: ranks may share a GPU (local rank mod the device count),
    so the real per-rank path (context, kernels, collectives, max over ranks)
    runs at world_size 2 on a one-GPU box (tests/test_bench_dist_gpu.py)."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = args.backend or "nccl"
    ndev = torch.cuda.device_count()  # counting devices does not initialise the GPU
    if world > 1 and backend == "gloo" and ndev > 0:
        local = local % ndev
    elif local >= max(ndev, 1):
        sys.exit(f"bench.py: local rank {local} but {ndev} GPU(s); {backend} needs one GPU per rank")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1 or args.dist:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group(backend, device_id=dev)
        else:
            dist.init_process_group(backend)
    return dist, dev, world, rank, local


def coll_device(dist, dev):
    """Where a collective's tensors live: the GPU for RCCL, host memory for gloo."""
    import torch
    if dist and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return dev


def algorithmic_bytes(w, h, levels, n):
    """B = 2*A0 + 4*Ap + 16*(A0 + Ap) + 58*N per frame pair."""
    a0 = w * h
    ap = 0
    sw, sh = w, h
    for _ in range(levels):
        sw, sh = (sw + 1) // 2, (sh + 1) // 2
        ap += sw * sh
    return 2 * a0 + 4 * ap + 16 * (a0 + ap) + 58 * n


def min_bytes(w, h, levels, n):
    """The bytes this design must move per frame pair: read I and
    J once, write and read both pyramids' levels >= 1, the point I/O --
    B_min = 2*A0 + 4*Ap + 58*N (SURVEY 8d's B without the Scharr planes, which
    this build forms in registers and never stores)."""
    return algorithmic_bytes(w, h, levels, n) - 16 * (w * h + pyramid_area(w, h, levels))


def pyramid_area(w, h, levels):
    ap = 0
    for _ in range(levels):
        w, h = (w + 1) // 2, (h + 1) // 2
        ap += w * h
    return ap


def cpu_baseline(w, h, n, level, budget_s=12.0, threads=1, reuse=False, clahe=False, pair_workers=0):
    """Oracle (C restatement) on the reference's 4-call pattern (each
    calcOpticalFlowPyrLK rebuilds both pyramids; LK points split over `threads`
    like OpenCV's parallel_for_), bounded sample of about budget_s seconds.
    pair_workers > 0: independent frame pairs on that many host threads at once
    (one thread each; the oracle's ctypes calls release the GIL) -- the batch
    throughput a CPU system would get from separate sequences."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # test-infrastructure import: cpu_baseline leg only
    from gvx import synth
    pairs = [synth.make_pair(w, h, n, synth.SEED + 1000 + i) for i in range(4)]
    p = orc.KltParams.default(max_level=level)
    half = n // 2  # Tracking::trackMappoint / trackReferencePoint point sets

    def frame(I, J, P, Q):
        if clahe:
            orc.clahe(J)  # Tracking::preprocessing of the new frame (tracking.cc:139)
        if reuse:
            # baseline (b): the same LK work with each image's pyramid built once
            orc.klt_fb(I, J, P, Q, params=p, reuse_pyramids=True, nthreads=threads)
            return
        # tracking.cc:385/390 (map points, fwd + bwd) and :487/493 (reference
        # points): four calcOpticalFlowPyrLK calls, each rebuilding both pyramids
        orc.klt_fb(I, J, P[:half], Q[:half], params=p, reuse_pyramids=False, nthreads=threads)
        orc.klt_fb(I, J, P[half:], Q[half:], params=p, reuse_pyramids=False, nthreads=threads)

    frame(*pairs[0][:4])  # warm
    if pair_workers > 0:
        from concurrent.futures import ThreadPoolExecutor
        t0 = time.perf_counter()

        def worker(wi):
            k = 0
            while time.perf_counter() - t0 < budget_s:
                I, J, P, Q, _ = pairs[(wi + k) % len(pairs)]
                frame(I, J, P, Q)
                k += 1
            return k

        with ThreadPoolExecutor(pair_workers) as ex:
            done = sum(ex.map(worker, range(pair_workers)))
        dt = time.perf_counter() - t0
        threads = pair_workers
    else:
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s:
            I, J, P, Q, _ = pairs[done % len(pairs)]
            frame(I, J, P, Q)
            done += 1
        dt = time.perf_counter() - t0
    what = ("fwd + bwd LK of all points, each pyramid built once (baseline b)" if reuse else
            f"({half} map + {n - half} reference points), 4 LK calls each rebuilding both pyramids "
            f"(tracking.cc:385,390,487,493)")
    if pair_workers > 0:
        what += f"; {pair_workers} pairs at a time, one host thread each"
    if clahe:
        what += " + CLAHE of the new frame (1 thread)"
    return {"value": done / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{done} frame pairs {w}x{h}/{n} feat {what}, {threads} thread(s), {dt:.1f} s"}


def cpu_factor_baseline(prob, segs, states, iewn, params, poffs, threads, budget_s=3.0):
    """Oracle factor evaluation of one sliding window (every reprojection and
    preintegration factor, residuals + Jacobians) on `threads` host threads,
    bounded to about budget_s seconds -> factor evals/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # test-infrastructure import: cpu_baseline leg only
    from gvx import synth_ba
    prm = orc.imu_params(*synth_ba.imu_params())
    osegs = [orc.PreintSeg(2, prm, segs[k], orc.make_state(float(st["time"]), st["p"], st["q"], st["v"],
                                                           st["bg"], st["ba"]), iewn[k])
             for k, st in enumerate(states)]
    n = len(prob["consts"]) + len(osegs)
    orc.reproj_eval_batch(prob["consts"], params, prob["offs"], nthreads=threads)  # warm
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        orc.reproj_eval_batch(prob["consts"], params, prob["offs"], nthreads=threads)
        orc.preint_factor_eval_batch(osegs, params, poffs, nthreads=threads)
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done * n / dt, "unit": "factor evals/s", "cores": threads, "kind": "port",
            "sample": f"{done} windows x {n} factors ({len(prob['consts'])} reprojection + {len(osegs)} Earth "
                      f"preintegration, M=100, residuals + Jacobians), {threads} thread(s), {dt:.1f} s"}


def cpu_preint_baseline(segs, states, iewn, threads, budget_s=2.0):
    """Oracle preintegration (orc_preint_integrate: the reference's
    integrationProcess + updateJacobianAndCovariance per sample, Eigen's dense
    15 x 15 products restated in C) of configs[3]'s Earth segments, one segment
    per call, independent segments on `threads` host threads at once (the
    ctypes calls release the GIL), bounded to about budget_s seconds ->
    preintegration steps/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # test-infrastructure import: cpu_baseline leg only
    from concurrent.futures import ThreadPoolExecutor
    from gvx import synth_ba
    prm = orc.imu_params(*synth_ba.imu_params())
    st = [orc.make_state(float(s["time"]), s["p"], s["q"], s["v"], s["bg"], s["ba"]) for s in states]
    orc.PreintSeg(2, prm, segs[0], st[0], iewn[0])  # warm
    t0 = time.perf_counter()

    def worker(wi):
        n = 0
        k = wi
        while time.perf_counter() - t0 < budget_s:
            j = k % len(segs)
            orc.PreintSeg(2, prm, segs[j], st[j], iewn[j])
            n += len(segs[j]) - 1
            k += 1
        return n

    with ThreadPoolExecutor(threads) as ex:
        steps = sum(ex.map(worker, range(threads)))
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "preintegration steps/s", "cores": threads, "kind": "port",
            "sample": f"{steps} IMU steps of Earth segments (M = {len(segs[0])}) through orc_preint_integrate, "
                      f"one segment per call, {threads} thread(s), {dt:.1f} s"}


def _record_for(pattern, workload):
    """The profiles/<pattern> JSON record measured on this workload, or None."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload:
            return d
    return None


def traffic_for(workload):
    """PMC HBM bytes per step measured on this workload (tools/traffic.py:
    profiles/pmc_traffic.json for configs[1], pmc_traffic_*.json for others)."""
    return _record_for("pmc_traffic*.json", workload)


def issue_for(workload):
    """LK's VALU-issue fraction on this workload (tools/issue.py: one PMC pass,
    profiles/pmc_issue.json), or None."""
    d = _record_for("pmc_issue*.json", workload)
    if d is None:
        return None
    return {k: d[k] for k in ("valu_busy", "resident_waves_per_simd", "max_waves_per_simd", "valu_insts_per_wave",
                              "clock_ghz", "source", "commit") if k in d}


def host_threads():
    """CPU share for the baseline: the affinity mask, capped at 16 (the GPU box's
    per-GPU CPU share; os.cpu_count() reports the whole machine there)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", "16"))))


ACCUM_MODES = {"exact": 0, "f32_scalar": 1, "f32_simd4": 2}  # include/gvx.h GVX_LK_ACCUM_*


class KltWorkload:
    """The timed KLT step's inputs and launch, shared with the parity test of
    this exact launch (tests/test_bench_batch_gpu.py): `n_pairs` synthetic pairs
    (`distinct` of them rendered, then tiled; seed synth.SEED + 100000 * rank)
    resident in HBM, and one gvx_klt_fb_batch_init_dev over them -- the pyramid
    pass, forward LK from the predictions in their own buffer, backward LK, FB
    and compaction (tracking.cc:385-408)."""

    def __init__(self, n_pairs, w, h, n, dev, rank=0, distinct=16):
        import torch
        from gvx import synth
        self.n_pairs, self.w, self.h, self.n = n_pairs, w, h, n
        self.host = synth.make_batch(n_pairs, w, h, n, seed=synth.SEED + 100000 * rank, distinct=distinct)
        self.I, self.J, self.P, self.Q = (torch.from_numpy(a).to(dev) for a in self.host)
        self.N = torch.empty_like(self.Q)  # tracked points (next)
        self.B = torch.empty_like(self.Q)  # backward points
        self.F = torch.empty((n_pairs, n), dtype=torch.uint8, device=dev)
        self.K = torch.empty((n_pairs, n), dtype=torch.int32, device=dev)
        self.NK = torch.empty((n_pairs,), dtype=torch.int32, device=dev)
        if self.I.is_cuda:
            torch.cuda.synchronize()

    def step(self, ctx, params):
        # initial flow (the predictions) read from Q, tracked points out to N
        ctx.klt_fb_batch_init_dev(self.n_pairs, self.w, self.h, self.I.data_ptr(), self.J.data_ptr(), self.n,
                                  self.P.data_ptr(), self.Q.data_ptr(), self.N.data_ptr(), self.B.data_ptr(),
                                  self.F.data_ptr(), self.K.data_ptr(), self.NK.data_ptr(), params=params)

    # ---- the same steps software-pipelined: batch t+1's pyramid pass on a side
    # branch beside batch t's LK (gvx_klt_batch_pyramids_dev / _pyr_dev, two
    # pyramid slots).  k steps run k pyramid passes and k LK passes, the first
    # pyramid pass alone and the last LK alone, so a timed run of k steps holds
    # all of its work and nothing of the steps around it.
    def _pyr_slots(self, ctx, max_level):
        import torch
        import gvx
        if getattr(self, "_pyr_level", None) != max_level:
            nb = 2 * self.n_pairs * gvx.pyramid_layout(self.w, self.h, max_level)["bytes"]
            self._pyr = [torch.empty(nb, dtype=torch.uint8, device=self.I.device) for _ in range(2)]
            self._pyr_level = max_level
        return self._pyr

    def build(self, ctx, params, slot):
        pyr = self._pyr_slots(ctx, params.max_level)
        ctx.klt_batch_pyramids_dev(self.n_pairs, self.w, self.h, self.I.data_ptr(), self.J.data_ptr(),
                                   params.max_level, pyr[slot].data_ptr())

    def track(self, ctx, params, slot):
        pyr = self._pyr_slots(ctx, params.max_level)
        ctx.klt_fb_batch_pyr_dev(self.n_pairs, self.w, self.h, self.I.data_ptr(), self.J.data_ptr(),
                                 pyr[slot].data_ptr(), self.n, self.P.data_ptr(), self.Q.data_ptr(),
                                 self.N.data_ptr(), self.B.data_ptr(), self.F.data_ptr(), self.K.data_ptr(),
                                 self.NK.data_ptr(), params=params)

    # ---- the same steps on two contexts (two streams, no cross-stream waits):
    # steps take turns on several contexts, each with its own output buffers, so
    # one stream's pyramid pass and another's LK share the GPU as they come
    def _outs(self, i):
        """Output buffers of context i >= 1 of a multi-context run (0: self's)."""
        import torch
        if not hasattr(self, "_ox"):
            self._ox = {}
        if i not in self._ox:
            self._ox[i] = dict(N=torch.empty_like(self.Q), B=torch.empty_like(self.Q), F=torch.empty_like(self.F),
                               K=torch.empty_like(self.K), NK=torch.empty_like(self.NK))
        return self._ox[i]

    def step_into(self, ctx, params, o):
        ctx.klt_fb_batch_init_dev(self.n_pairs, self.w, self.h, self.I.data_ptr(), self.J.data_ptr(), self.n,
                                  self.P.data_ptr(), self.Q.data_ptr(), o["N"].data_ptr(), o["B"].data_ptr(),
                                  o["F"].data_ptr(), o["K"].data_ptr(), o["NK"].data_ptr(), params=params)

    def run(self, ctx, params, k, pipelined, after_step=None, more=()):
        """k steps; after_step() (if any) is called after each step's LK is enqueued.
        more: further contexts -- step t then runs on context t % (1 + len(more)),
        each with its own output buffers and its own stream, with no waits between
        the streams (every step reads only the resident inputs)."""
        if more:
            ctxs = (ctx,) + tuple(more)
            for t in range(k):
                i = t % len(ctxs)
                if i:
                    self.step_into(ctxs[i], params, self._outs(i))
                else:
                    self.step(ctx, params)
                if after_step:
                    after_step()
            return
        if not pipelined:
            for _ in range(k):
                self.step(ctx, params)
                if after_step:
                    after_step()
            return
        if k <= 0:
            return
        self.build(ctx, params, 0)
        for t in range(k):
            if t + 1 < k:
                # the branch waits for everything before it, batch t-1's LK included,
                # which read the slot it is about to overwrite
                ctx.branch_begin()
                self.build(ctx, params, (t + 1) & 1)
                ctx.branch_end()
            self.track(ctx, params, t & 1)
            if t + 1 < k:
                ctx.branch_join()
            if after_step:
                after_step()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=30,
                    help="untimed steps; the clock ramps up over the first ~20 (about 16 ms of load)")
    ap.add_argument("--pairs", type=int, default=256, help="frame pairs per GPU per step")
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=560)
    ap.add_argument("--features", type=int, default=150)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--distinct", type=int, default=16, help="distinct synthetic pairs (tiled)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pre", action="store_true", help="skip the CLAHE preprocessing leg")
    ap.add_argument("--no-factors", action="store_true", help="skip the configs[3] factor leg of the default line")
    ap.add_argument("--no-sequence", action="store_true",
                    help="skip the configs[4] sequence leg of the default line (one sequence per GPU + the RCCL "
                         "gather of the tracks to rank 0)")
    ap.add_argument("--seq-frames", type=int, default=2000,
                    help="configs[4] leg of the default line: frames per sequence (per GPU)")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds per CPU baseline leg")
    ap.add_argument("--gather", action="store_true", help="batch-replay: all-gather results every step")
    ap.add_argument("--mock", action="store_true", help="no GPU: exercise launch/aggregation logic only")
    ap.add_argument("--config", type=int, default=2, choices=(1, 2, 3, 4, 5),
                    help="BASELINE.json config, 1-based as in SURVEY.md 8d: 2 = 1280x560/150 L3 on "
                         "1 MI355X (default, the metric; 1 is accepted as an alias), "
                         "3 = 1920x1200/500 L4 batch, 4 = sliding-window BA factor batch, "
                         "5 = sequence replay (one sequence per GPU, RCCL gather of the tracks)")
    ap.add_argument("--frames", type=int, default=2000, help="configs[4]: frames per sequence")
    ap.add_argument("--host-loop", action="store_true",
                    help="configs[4]: the per-frame loop with host round trips (SequenceTracker) instead of the "
                         "device-resident one-graph-per-frame loop")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="configs[4]: one graph per frame, frame t+1's CLAHE + pyramid after frame t's tracking "
                         "(default: beside it, a preprocessing graph on a side stream)")
    ap.add_argument("--frame-batch", type=int, default=16,
                    help="configs[4] pipelined: frames per preprocessing / tracking graph (the stream fork / join "
                         "and the graph launches once per K frames; 1 = a graph pair per frame)")
    ap.add_argument("--eig-branch", action="store_true",
                    help="configs[4] pipelined: the detection's eigenvalue map on the preprocessing branch")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default nccl, mock: gloo)")
    ap.add_argument("--dist", action="store_true",
                    help="open the process group even at world size 1 (run under torch.distributed.run): the "
                         "collectives of --gather / configs[4] / max-over-ranks then go through RCCL")
    ap.add_argument("--streams", type=int, default=3,
                    help="configs[1]/[2]: contexts (one stream each) the steps take turns on, with no waits between "
                         "the streams, so one step's pyramid pass and another's LK share the GPU as they come "
                         "(default 3); 1 = one context, its branch stream carrying batch t+1's pyramid pass beside "
                         "batch t's LK (or back to back with --no-overlap)")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false",
                    help="configs[1]/[2]: pyramid pass and LK back to back (default: batch t+1's pyramid pass on a "
                         "side stream beside batch t's LK -- each fills the other's drain, DESIGN.md 4 / 5)")
    ap.add_argument("--accum", default="exact", choices=tuple(ACCUM_MODES),
                    help="LK window-sum order (gvx_klt_params.accum): exact integer sums (default), or "
                         "OpenCV 4.x's fp32 scalar-loop / CV_SIMD128 orders")
    args = ap.parse_args()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return sys.exit(spawn_ranks(args.gpus))
    if world_env is not None and int(world_env) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}; launch one rank per GPU")
    if args.config == 1:
        args.config = 2  # configs[0] is the CPU-only reference case; its GPU twin is configs[1]
    if args.mock:
        return mock_main(args)
    if args.config == 5:
        return sequence_main(args)
    if args.config == 3:
        args.width, args.height, args.features, args.levels = 1920, 1200, 500, 4
    if args.config == 4:
        return factors_main(args)

    import torch
    import gvx

    dist, dev, world, rank, local = rank_setup(args)

    W, H, N, L, Pn = args.width, args.height, args.features, args.levels, args.pairs
    wl = KltWorkload(Pn, W, H, N, dev, rank=rank, distinct=args.distinct)
    I, J, P, Q = wl.host
    dI, dJ, dP, dQ, dNK = wl.I, wl.J, wl.P, wl.Q, wl.NK

    ctx = gvx.Context(local)
    params = gvx.KltParams.default(max_level=L, accum=ACCUM_MODES[args.accum])

    def step(p=params):
        wl.step(ctx, p)

    cdev = coll_device(dist, dev)
    gathered = [torch.empty(dNK.shape, dtype=dNK.dtype, device=cdev) for _ in range(world)] if dist else None

    def collect():
        if dist and args.gather:
            ctx.sync()
            dist.all_gather(gathered, dNK.to(cdev))  # offline batch replay: results to every rank

    # The side legs run first: LK device time of each window-sum order on the same
    # batch and the CLAHE preprocessing of the step's frames.  They are
    # measurements of their own (not part of `value`); running them before the
    # headline's W warm-up steps means the headline is timed at the shader clock
    # a running tracker sees, not during the clock's ramp from idle.
    t_side = time.perf_counter()
    legs = side_legs_before_headline(args)
    progress("side legs")
    accum_cost = accum_leg(ctx, step, gvx, L, steps=max(5, args.steps // 4)) if "lk_accum" in legs else None
    pre = preprocess_leg(ctx, dI, dJ, Pn, W, H, args.steps) if "preprocess" in legs else None
    pipelined = args.overlap
    more = tuple(gvx.Context(local) for _ in range(max(1, args.streams) - 1))
    progress("settle")
    if "settle" in legs:
        wl.run(ctx, params, SETTLE_STEPS, pipelined, more=more)
        for c in (ctx,) + more:
            c.sync()
    t_side = time.perf_counter() - t_side
    side_ranks = ranks_that_ran(accum_cost is not None, dist, dev)
    progress("warm-up and timed steps")
    wl.run(ctx, params, args.warmup, pipelined, collect, more=more)
    for c in more:
        c.sync()
    ctx.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    for c in (ctx,) + more:
        c.profile_reset()
        c.profile(True)
    # HIP events on the context stream around the K steps: the device span of the
    # whole run (the side branch joins back into this stream every step; the
    # other contexts' streams wait for ev0 and are waited for before ev1)
    cstream = torch.cuda.ExternalStream(ctx.stream(), device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(cstream)
    others = [torch.cuda.ExternalStream(c.stream(), device=dev) for c in more]
    for s_ in others:
        s_.wait_event(ev0)
    wl.run(ctx, params, args.steps, pipelined, collect, more=more)
    for s_ in others:
        e_ = torch.cuda.Event()
        e_.record(s_)
        cstream.wait_event(e_)
    ev1.record(cstream)
    for c in (ctx,) + more:
        c.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    fam = {f: ctx.profile_read(f) for f in ("pyramid", "klt", "compact")}
    ctx.profile(False)
    for c in more:
        fam = {f: tuple(a + b for a, b in zip(v, c.profile_read(f))) for f, v in fam.items()}
        c.profile(False)
        c.close()
    elapsed = max_over_ranks(elapsed, dist, dev)
    progress("single pair")
    single = single_pair_leg(ctx, dI, dJ, dP, dQ, W, H, N, params, reps=max(200, 5 * args.steps)) \
        if world == 1 and not args.no_pre else None
    pcie = None
    if world == 1 and not args.no_pre:
        # host-buffer rate (gvx_klt_fb_batch: images and points copied in and out per
        # call, PCIe-inclusive) -- reported beside `value`, never as it
        ctx.klt_fb_batch(I, J, P, Q, params=params)
        hs = max(3, args.steps // 8)
        t1 = time.perf_counter()
        for _ in range(hs):
            ctx.klt_fb_batch(I, J, P, Q, params=params)
        pcie = {"pairs_per_s": round(Pn * hs / (time.perf_counter() - t1), 1), "steps": hs,
                "what": "gvx_klt_fb_batch on host buffers (2 x %.0f MB image upload + points per step)"
                        % (I.nbytes / 1e6)}
    gather_ok = None
    if dist:
        if not args.gather:
            gathered = [torch.empty(dNK.shape, dtype=dNK.dtype, device=cdev) for _ in range(world)]
            dist.all_gather(gathered, dNK.to(cdev))  # results exchange, outside the timed region
        # the exchange delivered this rank's own results, and every rank's are sane
        gather_ok = bool(torch.equal(gathered[rank].cpu(), dNK.cpu())
                         and all(int(g.min()) > 0 for g in gathered))

    # the metric's second half (BASELINE.json: factor-Jacobian eval/s), timed in
    # the same run: configs[3]'s factor batch (its own line under "factors")
    progress("factors")
    factors = None if args.no_factors else factor_leg(args, ctx, dev, dist, world, rank,
                                                      steps=max(10, args.steps // 2), window_extras=False)
    # the north_star scaling workload, timed in the same run at every N: one
    # configs[4] sequence per GPU replayed on the device, then every rank's
    # per-frame tracks gathered to rank 0 over RCCL (its own line under "sequence")
    progress("sequence")
    seq = None if args.no_sequence else sequence_leg(args, ctx, dev, dist, world, rank, args.seq_frames)
    kept_frac = float(dNK.float().mean().item()) / N
    total_pairs = world * Pn * args.steps
    value = total_pairs / elapsed
    ms_step = elapsed / args.steps * 1e3
    B = algorithmic_bytes(W, H, L, N)
    Bmin = min_bytes(W, H, L, N)
    span_ms = ev0.elapsed_time(ev1) / args.steps  # device span per step (all kernels, overlap included)
    workload = f"klt_fb_batch {Pn}x{W}x{H} N{N} L{L}"
    tr = traffic_for(workload)
    # roofline.achieved / frac: the HBM bytes the step really moves (PMC traffic of
    # this workload, profiles/pmc_traffic.json) over the device span; without a
    # matching PMC record, B_min (the bytes this design must move) stands in
    gbs = (lambda nbytes: nbytes / (span_ms * 1e-3) / 1e9) if span_ms > 0 else (lambda nbytes: None)
    achieved = gbs(tr["bytes_per_step"]) if tr else gbs(Bmin * Pn)
    frac = (lambda v: round(v / HBM_PEAK_GBS, 4) if v else None)

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            nt = host_threads()
            # value: independent pairs on every host thread at once (the batch
            # throughput of the CPU share); beside it the reference's per-frame
            # pattern with its LK points split over the threads, the pyramid-reuse
            # variant (b) and one thread
            cpu = cpu_baseline(W, H, N, L, args.cpu_budget / 2, pair_workers=nt)
            pf = cpu_baseline(W, H, N, L, args.cpu_budget / 2, threads=nt)
            cpu["per_frame_parallel_value"] = pf["value"]
            cpu["per_frame_parallel_sample"] = pf["sample"]
            reuse = cpu_baseline(W, H, N, L, args.cpu_budget / 4, threads=nt, reuse=True)
            cpu["reuse_value"] = reuse["value"]
            cpu["reuse_sample"] = reuse["sample"]
            if nt > 1:
                one = cpu_baseline(W, H, N, L, args.cpu_budget / 4, threads=1)
                cpu["single_thread_value"] = one["value"]
                cpu["single_thread_sample"] = one["sample"]
        line = {
            "metric": f"KLT frames/sec @{W}x{H},{N} feat",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/i32 windows, f32 solve",
            "data": "synthetic (KAIST bags unavailable offline): band-limited noise + rectangles, "
                    "similarity warp, seed 20261015",
            "config": {"workload": f"configs[{args.config - 1}]: batch of {Pn} frame pairs/GPU, {W}x{H} mono, {N} feat, "
                                   f"maxLevel {L}, win 21, fwd+bwd LK + FB + compaction",
                       "pairs_per_gpu_per_step": Pn, "parallelism": f"pairs sharded over {world} GPU(s)"},
            "roofline": {"bound": "hbm",
                         "kernel": ("klt pipeline (pyramid pass + LK/FB + compaction) per step, steps taking turns "
                                    "on %d streams" % (1 + len(more)) if more else
                                    "klt pipeline per step: batch t+1's pyramid pass beside batch t's LK/FB + "
                                    "compaction" if pipelined else
                                    "klt pipeline (pyramid pass + LK/FB + compaction) per step"),
                         "device_span_ms_per_step": round(span_ms, 4),
                         "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": frac(achieved),
                         "achieved_basis": ("measured: PMC HBM bytes per step (traffic) / device span" if tr else
                                            "B_min per step / device span (no PMC record for this workload)"),
                         "traffic": round(tr["bytes_per_step"]) if tr else None,
                         "traffic_unit": "HBM bytes per step (PMC 2*FETCH_SIZE+WRITE_SIZE)",
                         "traffic_source": tr["source"] if tr else None,
                         "traffic_commit": tr.get("commit") if tr else None,
                         "min_bytes_per_pair": Bmin,
                         "frac_min": frac(gbs(Bmin * Pn)),
                         "min_convention": "B_min = 2*A0 + 4*Ap + 58*N: I and J read once, pyramid levels "
                                           "written and read, point I/O",
                         "effective_frac": frac(gbs(B * Pn)),
                         "effective_convention": ("SURVEY 8d's B, which counts int16x2 Scharr planes written and "
                                                  "read; this build never stores them, so effective_frac passes 1 "
                                                  "above 454 k pairs/s and is no roofline"),
                         "klt_issue": issue_for(workload),
                         "algorithmic_bytes_per_step": B * Pn, "algorithmic_bytes_per_pair": B,
                         "device_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in fam.items()},
                         "device_ms_note": ("each kernel's own start-stop events summed over its launches; with "
                                            "several streams the kernels overlap, so these add to more than the "
                                            "span" if more or pipelined else "back to back: they add to the span"),
                         "overlap": pipelined and not more, "streams": 1 + len(more)},
            "cpu_baseline": cpu,
            "kept_fraction": round(kept_frac, 4),
            "lk_accum": args.accum,
            "lk_accum_cost": accum_cost,
            "side_legs_before_headline_s": round(t_side, 3),
            "side_legs_before_headline_ranks": side_ranks,
            "side_legs_before_headline": legs,
            "settle_steps": SETTLE_STEPS if "settle" in legs else 0,
            "preprocess": pre,
            "single_pair": single,
            "host_buffers": pcie,
            "factors": factors,
            "sequence": sequence_summary(seq) if seq else None,
            "dist_backend": dist.get_backend() if dist else None,
            "gather_check": gather_ok,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()
    ctx.close()


def accum_leg(ctx, step, gvx, L, steps):
    """LK device ms per step in each window-sum order (gvx_klt_params.accum):
    the exact integer order and OpenCV 4.x's fp32 scalar / CV_SIMD128 orders,
    which the device reproduces bit-exactly (tests/test_klt_accum_gpu.py)."""
    out = {}
    for _ in range(20):  # the shader clock up from idle before the first timed mode
        step(gvx.KltParams.default(max_level=L))
    for name, mode in ACCUM_MODES.items():
        p = gvx.KltParams.default(max_level=L, accum=mode)
        for _ in range(3):
            step(p)
        ctx.sync()
        ctx.profile_reset()
        ctx.profile(True)
        for _ in range(steps):
            step(p)
        ctx.sync()
        out[name] = round(ctx.profile_read("klt")[0] / steps, 4)
        ctx.profile(False)
    out["unit"] = "LK device ms per step"
    out["steps"] = steps
    return out


def single_pair_leg(ctx, dI, dJ, dP, dQ, W, H, N, params, reps):
    """configs[1] as the live tracker runs it: ONE frame pair per launch (the
    pyramid pass, LK with FB, the compaction: three kernels), back to back on the
    context stream -- eager host calls against the same work captured
    once into a hipGraph and replayed.  Latency, not `value`."""
    import torch
    dev = dI.device
    I1, J1, P1, Q1 = dI[0:1], dJ[0:1], dP[0:1], dQ[0:1]
    outs = [dict(N=torch.empty_like(Q1), B=torch.empty_like(Q1),
                 F=torch.empty((1, N), dtype=torch.uint8, device=dev),
                 K=torch.empty((1, N), dtype=torch.int32, device=dev),
                 NK=torch.empty((1,), dtype=torch.int32, device=dev)) for _ in range(2)]

    def enqueue(o):
        ctx.klt_fb_batch_init_dev(1, W, H, I1.data_ptr(), J1.data_ptr(), N, P1.data_ptr(), Q1.data_ptr(),
                                  o["N"].data_ptr(), o["B"].data_ptr(), o["F"].data_ptr(), o["K"].data_ptr(),
                                  o["NK"].data_ptr(), params=params)

    torch.cuda.synchronize()
    for _ in range(20):
        enqueue(outs[0])
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        enqueue(outs[0])
    ctx.sync()
    eager = (time.perf_counter() - t0) / reps
    ctx.capture_begin()
    enqueue(outs[1])
    g = ctx.capture_end()
    for _ in range(20):
        ctx.graph_launch(g)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.graph_launch(g)
    ctx.sync()
    graph = (time.perf_counter() - t0) / reps
    # two instantiations of the same work launched alternately: back-to-back
    # launches of ONE graph exec serialise on the host in ROCm's runtime
    ctx.capture_begin()
    enqueue(outs[1])
    g2 = ctx.capture_end()
    for _ in range(20):
        ctx.graph_launch(g)
        ctx.graph_launch(g2)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps // 2):
        ctx.graph_launch(g)
        ctx.graph_launch(g2)
    ctx.sync()
    graph2 = (time.perf_counter() - t0) / (2 * (reps // 2))
    same = all(torch.equal(outs[0][k], outs[1][k]) for k in outs[0])
    g.destroy()
    g2.destroy()
    return {"what": "one frame pair per launch, back to back: pyramid pass + LK / FB + compaction (3 kernels)",
            "us_per_pair_eager": round(eager * 1e6, 2), "us_per_pair_graph": round(graph * 1e6, 2),
            "us_per_pair_two_graphs": round(graph2 * 1e6, 2),
            "pairs_per_s_graph": round(1.0 / graph, 1), "graph_matches_eager": same, "reps": reps}


def preprocess_leg(ctx, dI, dJ, Pn, W, H, steps):
    """Tracking::preprocessing (CLAHE, tracking.cc:139) over the step's 2*Pn
    frames resident in HBM, timed on its own (not part of `value`, whose
    frame-pair unit in SURVEY 8d starts after CLAHE).  Algorithmic bytes: each
    pixel read once and written once (2 B/px); the design reads it twice (LUT
    pass + apply pass)."""
    import torch
    out = torch.empty_like(dI)

    def run():
        ctx.clahe_batch_dev(Pn, W, H, dI.data_ptr(), out.data_ptr())
        ctx.clahe_batch_dev(Pn, W, H, dJ.data_ptr(), out.data_ptr())

    for _ in range(5):
        run()
    ctx.sync()
    ctx.profile_reset()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    ctx.sync()
    el = time.perf_counter() - t0
    ms, _ = ctx.profile_read("clahe")
    ctx.profile(False)
    imgs = 2 * Pn * steps
    gbs = 2.0 * W * H * imgs / (ms * 1e-3) / 1e9 if ms > 0 else None
    return {"what": "CLAHE createCLAHE(3.0, 21x21)->apply on the 2*pairs frames of a step (tracking.cc:139)",
            "images_per_s": round(imgs / el, 1), "device_ms_per_image": round(ms / imgs, 5),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1) if gbs else None, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None,
                         "algorithmic_bytes_per_image": 2 * W * H}}


def factors_main(args):
    """`--config 4`: the factor leg on its own, as the line's headline."""
    import gvx
    dist, dev, world, rank, local = rank_setup(args)
    ctx = gvx.Context(local)
    line = factor_leg(args, ctx, dev, dist, world, rank, args.steps, window_extras=True)
    if rank == 0:
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()
    ctx.close()


def factor_leg(args, ctx, dev, dist, world, rank, steps, window_extras=True):
    """configs[3]: sliding-window BA factor evaluation (10 keyframes x 200
    landmarks -> 1800 ReprojectionFactor + 9 Earth PreintegrationFactor with
    M = 100 IMU samples), replicated to >= 2^20 reprojection
    factors per launch (the window's parameter blocks are shared, read once per
    batch).  A step = one LM iteration's residual + Jacobian evaluation of the
    whole batch (reprojection + preintegration factors); preintegration steps/s
    (9 x replicas segments) are timed separately."""
    import torch
    import gvx
    from gvx import synth_ba

    prob = synth_ba.make_ba_problem()
    n_kf = prob["poses"].shape[0]
    n_rp = len(prob["consts"])
    reps = -(-(1 << 20) // n_rp)
    rng = np.random.default_rng(synth_ba.SEED if hasattr(synth_ba, "SEED") else 20261015)
    # Earth preintegration segments between consecutive keyframes
    M = 100
    segs = [synth_ba.make_imu_segment(rng, M, t0=0.5 * k) for k in range(n_kf - 1)]
    states = np.zeros(n_kf - 1, gvx.STATE_DTYPE)
    for k in range(n_kf - 1):
        states[k]["time"] = 0.5 * k
        states[k]["p"] = prob["poses"][k, :3]
        states[k]["q"] = prob["poses"][k, 3:]
        states[k]["v"] = [5.0, 0.0, 0.0]
    iewn = np.array([gvx.earth_iewn(np.zeros(3), st["p"]) for st in states])
    pre, pn, pn_off = ctx.preint_integrate(2, synth_ba.imu_params(), segs, states, iewn)
    # parameter array: poses | ext | invdepth | td | mix blocks (v, bg, ba) per keyframe
    mix = np.zeros((n_kf, 9))
    mix[:, 0] = 5.0
    params = np.concatenate([prob["params"], mix.reshape(-1)])
    o_mix = prob["params"].size
    poffs = np.array([[7 * k, o_mix + 9 * k, 7 * (k + 1), o_mix + 9 * (k + 1)] for k in range(n_kf - 1)], np.int32)

    def dev_t(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    d_consts = dev_t(np.tile(prob["consts"], reps).view(np.uint8))
    d_offs = dev_t(np.tile(prob["offs"], (reps, 1)))
    d_params = dev_t(params)
    n_r = n_rp * reps
    d_res = torch.empty((n_r, 2), dtype=torch.float64, device=dev)
    d_jac = torch.empty((n_r, 46), dtype=torch.float64, device=dev)
    n_p = (n_kf - 1) * reps
    d_pre = dev_t(np.tile(pre, reps).view(np.uint8))
    # every replica its own copy of the pn_ samples (the streamed bytes the
    # preintegration factor roofline counts)
    d_pn = dev_t(np.tile(pn, (reps, 1)))
    d_pn_off = dev_t(np.concatenate([pn_off + r * len(pn) for r in range(reps)]).astype(np.int32))
    d_poffs = dev_t(np.tile(poffs, (reps, 1)))
    d_pres = torch.empty((n_p, 15), dtype=torch.float64, device=dev)
    d_pjac = torch.empty((n_p, 480), dtype=torch.float64, device=dev)
    # preintegration batch: (n_kf-1) * reps segments of M samples
    S = (n_kf - 1) * reps
    imu_all = np.concatenate(segs * reps)
    seg_off = np.arange(S + 1, dtype=np.int32) * M
    d_imu = dev_t(imu_all.astype(gvx.IMU_DTYPE).view(np.uint8))
    d_seg_off = dev_t(seg_off)
    d_states = dev_t(np.tile(states, reps).view(np.uint8))
    d_iewn = dev_t(np.tile(iewn, (reps, 1)))
    d_out = torch.empty(S * gvx.PREINT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_pnall = torch.empty((S * (M - 1), 4), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    def step():
        # both factor kinds in one call (gvx_factor_batch_eval_dev)
        ctx.factor_batch_eval_dev(n_r, d_consts.data_ptr(), d_offs.data_ptr(), d_res.data_ptr(), d_jac.data_ptr(),
                                  n_p, d_pre.data_ptr(), d_pn.data_ptr(), d_pn_off.data_ptr(), d_poffs.data_ptr(),
                                  d_pres.data_ptr(), d_pjac.data_ptr(), d_params.data_ptr())

    def integ():
        ctx.preint_integrate_dev(2, synth_ba.imu_params(), S, d_imu.data_ptr(), d_seg_off.data_ptr(),
                                 d_states.data_ptr(), d_iewn.data_ptr(), d_out.data_ptr(), d_pnall.data_ptr())

    def timed(fn, k, warm=None, prof=True):
        # prof: per-family device times by events on every launch (off for the
        # ~35 us single-window calls, whose wall time the events would inflate)
        for _ in range(args.warmup if warm is None else warm):
            fn()
        ctx.sync()
        if dist:
            dist.barrier()
        ctx.profile_reset()
        ctx.profile(prof)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        ctx.sync()
        if dist:
            dist.barrier()
        el = max_over_ranks(time.perf_counter() - t0, dist, dev)
        fam = {f: ctx.profile_read(f) for f in ("reproj", "preint_factor", "preint")}
        ctx.profile(False)
        return el, fam

    el, fam = timed(step, steps)
    # the integrate call is ~0.3 ms: time enough launches that the shader clock
    # has ramped and the host-side bracket is a small part of the span
    k_i = max(40, steps)
    el_i, fam_i = timed(integ, k_i, warm=max(20, args.warmup))

    # one window at problem size (1800 + 9 factors, latency-bound): device-pointer
    # launches, and the two-phase FactorSet prepare (block gather, H2D, both
    # kernels, D2H) that a Ceres EvaluationCallback would call per LM iteration
    n_w = n_rp + (n_kf - 1)

    def window():
        ctx.factor_batch_eval_dev(n_rp, d_consts.data_ptr(), d_offs.data_ptr(), d_res.data_ptr(), d_jac.data_ptr(),
                                  n_kf - 1, d_pre.data_ptr(), d_pn.data_ptr(), d_pn_off.data_ptr(),
                                  d_poffs.data_ptr(), d_pres.data_ptr(), d_pjac.data_ptr(), d_params.data_ptr())

    # ~35 us calls: hundreds of them, after enough warm-up calls that the clocks
    # and the host path have settled (50 calls gave 40-46 us where 2,000 give 34)
    k_w = max(500, steps)
    el_w, _ = timed(window, k_w, warm=max(100, args.warmup), prof=False)
    # parameter blocks as views of the packed vector (the layout the offsets index)
    starts = sorted({int(v) for v in prob["offs"].ravel()} | {int(v) for v in poffs.ravel()})
    sizes = {}
    for o, sz in zip(prob["offs"].T, (7, 7, 7, 1, 1)):
        sizes.update({int(v): sz for v in o})
    for o, sz in zip(poffs.T, (7, 9, 7, 9)):
        sizes.update({int(v): sz for v in o})
    bidx = {st: i for i, st in enumerate(starts)}
    blocks = [params[st:st + sizes[st]] for st in starts]
    fset = gvx.FactorSet(ctx, blocks, prob["consts"].astype(gvx.REPROJ_DTYPE),
                         np.vectorize(bidx.get)(prob["offs"]).astype(np.int32), pre, pn, pn_off,
                         np.vectorize(bidx.get)(poffs).astype(np.int32))
    el_p, _ = timed(lambda: fset.prepare(True), k_w, warm=max(100, args.warmup), prof=False)
    fset.close()
    evals = world * (n_r + n_p) * steps
    value = evals / el
    rp_ms = fam["reproj"][0] / steps
    pf_ms = fam["preint_factor"][0] / steps
    B_pf = 8 * (16 + 225 + 225 + 4 * M + 7) + 8 * (15 + 15 * 32)  # SURVEY 8d, M = 100: 10,944 B
    B_rp = 15 * 8 + 5 * 4 + 48 * 8  # consts + offsets in, residual + 5 Jacobian blocks out
    B_rp_survey = 504  # SURVEY 8d's per-factor figure (its Jacobian count, no offsets)
    achieved = B_rp * n_r / (rp_ms * 1e-3) / 1e9 if rp_ms > 0 else None
    line = None
    if rank == 0:
        wf = window_factor_leg(ctx, dev, cpu=world == 1 and not args.no_cpu) if window_extras else None
        pf_achieved = B_pf * n_p / (pf_ms * 1e-3) / 1e9 if pf_ms > 0 else None
        line = {
            "metric": "BA factor-Jacobian evaluations/s (configs[3])",
            "value": round(value, 1), "unit": "factor evals/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(el / steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic sliding window (seed 20261015)",
            "config": {"workload": f"configs[3]: {n_kf} keyframes x 200 landmarks = {n_rp} ReprojectionFactor + "
                                   f"{n_kf - 1} Earth PreintegrationFactor (M={M}), x{reps} windows per launch",
                       "reproj_factors_per_step": n_r, "preint_factors_per_step": n_p},
            "roofline": {"bound": "hbm", "kernel": "reproj_kernel", "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None, "traffic": None,
                         "algorithmic_bytes_per_factor": B_rp,
                         "survey_bytes_per_factor": B_rp_survey,
                         "frac_at_survey_bytes": round(B_rp_survey * n_r / (rp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                         if rp_ms > 0 else None,
                         "device_ms_per_step": {k: round(v[0] / steps, 4) for k, v in fam.items()}},
            "preint_factor_roofline": {"bound": "hbm", "kernel": "preint_factor_kernel",
                                       "achieved": round(pf_achieved, 1) if pf_achieved else None,
                                       "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                       "frac": round(pf_achieved / HBM_PEAK_GBS, 4) if pf_achieved else None,
                                       "algorithmic_bytes_per_factor": B_pf,
                                       "pn_samples": "one copy per replica (streamed, not shared)"},
            "preint_steps_per_s": round(world * S * (M - 1) * k_i / el_i, 1),
            "preint_device_ms_per_launch": round(fam_i["preint"][0] / k_i, 4),
            "preint_cpu_baseline": None,
            "problem_size": {"window_factors": n_w,
                             "device_launch_evals_per_s": round(world * n_w * k_w / el_w, 1),
                             "factor_set_prepare_evals_per_s": round(world * n_w * k_w / el_p, 1),
                             "factor_set_prepare_ms": round(el_p / k_w * 1e3, 4)},
            "window_factors": wf,
            "cpu_baseline": None,
            "dist_backend": dist.get_backend() if dist else None,
        }
        if world == 1 and not args.no_cpu:
            ref = cpu_factor_baseline(prob, segs, states, iewn, params, poffs, threads=4)
            nt = host_threads()
            if nt != 4:
                allc = cpu_factor_baseline(prob, segs, states, iewn, params, poffs, threads=nt)
                ref["all_cores_value"] = allc["value"]
                ref["all_cores_sample"] = allc["sample"]
            line["cpu_baseline"] = ref
            # the integrate scan on the CPU (preintegration_earth.cc:205-303 per
            # addNewImu), the same 99-step Earth segments: the reference's
            # 4 threads and the box's CPU share
            pre_ref = cpu_preint_baseline(segs, states, iewn, threads=4)
            if nt != 4:
                pre_all = cpu_preint_baseline(segs, states, iewn, threads=nt)
                pre_ref["all_cores_value"] = pre_all["value"]
                pre_ref["all_cores_sample"] = pre_all["sample"]
            line["preint_cpu_baseline"] = pre_ref
    return line


def window_factor_leg(ctx, dev, reps=20, cpu=True):
    """SURVEY 8f rank 3, beside configs[3]: GnssFactor as a device batch (2^20
    factors per launch for a throughput figure; the live system has one per GNSS
    epoch), one MarginalizationFactor of an IC-GVINS-shaped window (9 keyframes'
    pose + mix, extrinsic, td: r = 142) through the host entry, PCIe included, and
    the device marginalisation of the configs[3] window (marg_leg).  Not part of
    `value`."""
    import torch
    import gvx
    rng = np.random.default_rng(7)
    n = 1 << 20
    poses = np.zeros((n, 7))
    poses[:, :3] = rng.normal(0, 5, (n, 3))
    q = rng.normal(0, 1, (n, 4))
    poses[:, 3:] = q / np.linalg.norm(q, axis=1, keepdims=True)
    consts = np.concatenate([rng.normal(0, 5, (n, 3)), rng.uniform(0.01, 0.1, (n, 3)),
                             np.tile([0.1, -0.2, 0.3], (n, 1))], 1)
    d_p = torch.from_numpy(poses.ravel()).to(dev)
    d_c = torch.from_numpy(consts.ravel()).to(dev)
    d_o = torch.arange(0, 7 * n, 7, dtype=torch.int32, device=dev)
    d_r = torch.empty(n * 3, dtype=torch.float64, device=dev)
    d_j = torch.empty(n * 21, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    def run():
        ctx.small_factor_eval_dev(gvx.FACTOR_GNSS, n, d_c.data_ptr(), d_p.data_ptr(), d_o.data_ptr(), d_r.data_ptr(),
                                  d_j.data_ptr())

    for _ in range(3):
        run()
    ctx.sync()
    ctx.profile_reset()
    ctx.profile(True)
    for _ in range(reps):
        run()
    ctx.sync()
    ms, _ = ctx.profile_read("aux_factor")
    ctx.profile(False)
    per = ms / reps
    bytes_per = (9 + 7 + 3 + 21) * 8 + 4  # constants, pose, residuals, Jacobian, offset
    size = [7, 9] * 9 + [7, 1]
    local = [6 if s == 7 else s for s in size]
    index = np.concatenate([[0], np.cumsum(local)[:-1]]).astype(np.int32)
    xoff = np.concatenate([[0], np.cumsum(size)[:-1]]).astype(np.int32)
    r = int(sum(local))
    x0 = rng.normal(0, 1, int(sum(size)))
    for b, s in enumerate(size):
        if s == 7:
            x0[xoff[b] + 3:xoff[b] + 7] = (0, 0, 0, 1)
    J0, e0 = rng.normal(0, 1, (r, r)), rng.normal(0, 1, r)
    ctx.marg_factor_eval(size, index, xoff, x0, x0, J0, e0)
    t0 = time.perf_counter()
    for _ in range(50):
        ctx.marg_factor_eval(size, index, xoff, x0, x0, J0, e0)
    marg_us = (time.perf_counter() - t0) / 50 * 1e6
    return {"gnss_factors_per_launch": n, "gnss_device_ms_per_launch": round(per, 4),
            "gnss_factor_evals_per_s": round(n / (per * 1e-3)),
            "gnss_roofline": {"bound": "hbm", "achieved": round(n * bytes_per / (per * 1e-3) / 1e9, 1),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "algorithmic_bytes_per_factor": bytes_per},
            "marg_factor_r": r, "marg_factor_host_call_us": round(marg_us, 1),
            "marginalization": marg_leg(ctx, dev, cpu=cpu),
            "lm_step": lm_step_leg(ctx, dev, cpu=cpu)}


def lm_step_leg(ctx, dev, reps=20, cpu=True):
    """One LM linear step of the configs[3] window as Ceres' DENSE_SCHUR takes it
    (ic_gvins.cc:1170-1180): the normal equations of the window's evaluated
    residual blocks (the marginalisation problem's blocks: prior, GNSS,
    preintegration, 1,800 reprojection factors), the 200 inverse depths
    eliminated, the 157 x 157 reduced camera system factored by Cholesky, the
    step back-substituted (gvx_schur_solve_dev).  The CPU baseline is numpy's
    dense solve of the same damped system (LAPACK, all host threads)."""
    import torch
    from gvx import synth_ba
    p = synth_ba.lm_problem(synth_ba.make_marg_problem(synth_ba.DeviceFactorEvaluator(ctx)))
    L = p["L"]
    d_data = torch.from_numpy(p["data"]).to(dev)
    H, b = synth_ba.dense_normal_equations(p)
    D = np.sqrt(1e-4 * np.maximum(np.diag(H), 1e-6))
    d_D = torch.from_numpy(D).to(dev)
    d_delta = torch.empty(L, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    def run():
        ctx.schur_solve_dev(p, d_data.data_ptr(), d_delta.data_ptr(), d_D=d_D.data_ptr())

    for _ in range(3):
        run()
    ctx.sync()
    ctx.profile_reset()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
        ctx.sync()
    wall = (time.perf_counter() - t0) / reps
    ms, k = ctx.profile_read("lm_step")
    ctx.profile(False)
    out = {"what": "LM linear step (DENSE_SCHUR) of the configs[3] window: J^T J + D, 200 inverse depths "
                   "eliminated, reduced camera system by Cholesky (gvx_schur_solve_dev)",
           "eliminated": p["m"], "reduced": L - p["m"], "residual_blocks": len(p["nres"]),
           "device_ms_per_call": round(ms / max(k, 1), 3), "call_ms": round(wall * 1e3, 3), "cpu_baseline": None}
    if cpu:
        Hd = H + np.diag(D * D)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 1.0 or n < 3:
            Hs, bs = synth_ba.dense_normal_equations(p)
            np.linalg.solve(Hs + np.diag(D * D), bs)
            n += 1
        el = (time.perf_counter() - t0) / n
        out["cpu_baseline"] = {"value": round(el * 1e3, 2), "unit": "ms per LM step", "cores": host_threads(),
                               "kind": "port", "sample": f"{n} steps: dense assembly of J^T J from the blocks + "
                                                         "numpy.linalg.solve of the 357 x 357 damped system"}
        del Hd
    return out


def marg_leg(ctx, dev, reps=10, cpu=True):
    """MarginalizationInfo::marginalization() of the configs[3] window when its
    oldest keyframe leaves (synth_ba.make_marg_problem: the previous prior, a GNSS
    factor, preintegration 0->1 and the 1,800 reprojection factors; m = 215
    marginalized, r = 142 remained), residual blocks evaluated on the device, then
    gvx_marginalize_dev: H0/b0, Hmm's eigen-decomposition, Hp/bp, Hp's
    eigen-decomposition, J0/e0.  Once per keyframe in the live system: a latency
    item, bound by the dependent fp64 Givens chain of the two eigen-solvers."""
    import torch
    from gvx import synth_ba
    p = synth_ba.make_marg_problem(synth_ba.DeviceFactorEvaluator(ctx))
    r = p["L"] - p["m"]
    d_data = torch.from_numpy(p["data"]).to(dev)
    d_J0 = torch.empty(r * r, dtype=torch.float64, device=dev)
    d_e0 = torch.empty(r, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    def run():
        ctx.marginalize_dev(p, d_data.data_ptr(), d_J0.data_ptr(), d_e0.data_ptr())

    for _ in range(2):
        run()
    ctx.sync()
    ctx.profile_reset()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
        ctx.sync()
    wall = (time.perf_counter() - t0) / reps
    ms, k = ctx.profile_read("marg")
    ctx.profile(False)
    out = {"what": "device marginalisation of the configs[3] window (constructEquation + schurElimination + "
                   "linearization, marginalization_info.h:153-230)",
           "marginalized": p["m"], "remained": r, "residual_blocks": len(p["nres"]),
           "device_ms_per_call": round(ms / max(k, 1), 3), "call_ms": round(wall * 1e3, 3),
           "solver": "FAST (Cholesky where no eigenvalue is dropped; gvx_set_marg_solver)",
           "bound": "latency (one-workgroup fp64 Cholesky factorisations and triangular solves)", "cpu_baseline": None}
    # the EXACT solver (Eigen's SelfAdjointEigenSolver, bit-exact vs the restatement) beside it
    import gvx
    ctx.set_marg_solver(gvx.MARG_SOLVER_EXACT)
    try:
        run()
        ctx.sync()
        ctx.profile_reset()
        ctx.profile(True)
        for _ in range(3):
            run()
        ctx.sync()
        ms_x, k_x = ctx.profile_read("marg")
        ctx.profile(False)
        out["exact_solver_device_ms_per_call"] = round(ms_x / max(k_x, 1), 3)
    finally:
        ctx.set_marg_solver(gvx.MARG_SOLVER_FAST)
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as orc  # test-infrastructure import: cpu_baseline leg only
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 3.0 or n < 2:
            H0, b0 = orc.marg_construct(p)
            Hp, bp, _ = orc.marg_schur(H0, b0, p["m"])
            orc.marg_linearize(Hp, bp)
            n += 1
        el = (time.perf_counter() - t0) / n
        out["cpu_baseline"] = {"value": round(el * 1e3, 2), "unit": "ms per marginalisation", "cores": 1,
                               "kind": "port", "sample": f"{n} marginalisations of the same problem (oracle/marg.c, "
                                                        "scalar C, Eigen's algorithms), 1 thread"}
    return out


def gather_tracks(tracks, counts, dist, dev):
    """configs[4]'s exchange: every rank's per-frame tracks ([F, N, 2] f32 and
    [F] counts) to rank 0 in one collective (RCCL gather over xGMI on the GPU
    box, gloo in the CPU test).  Returns the list of (tracks, counts) per rank
    on rank 0 (tensors where the collective left them: the caller copies them
    to the host after its timed region), None elsewhere."""
    import torch
    if not dist:
        return [(tracks, counts)]
    packed = torch.cat([tracks.reshape(-1).to(torch.float32), counts.to(torch.float32)]).to(dev)
    world, rank = dist.get_world_size(), dist.get_rank()
    bufs = [torch.empty_like(packed) for _ in range(world)] if rank == 0 else None
    dist.gather(packed, bufs, dst=0)
    if rank != 0:
        return None
    n = tracks.numel()
    return [(b[:n].reshape(tracks.shape), b[n:].to(torch.int32)) for b in bufs]


def records_digest(tracks, counts):
    """Order-sensitive digest of one rank's per-frame records (tracks [F, N, 2]
    f32 -- only the first counts[f] rows of frame f are defined -- and counts
    [F]): two float64 sums, exact for these magnitudes, weighted by position."""
    F, N = tracks.shape[:2]
    valid = np.arange(N)[None, :] < counts[:, None]
    t = np.where(valid[..., None], tracks.astype(np.float64), 0.0)
    wts = 1.0 + (np.arange(F * N * 2, dtype=np.float64) % 7919).reshape(F, N, 2)
    return (float((t * wts).sum()), int(counts.astype(np.int64) @ (1 + np.arange(F, dtype=np.int64))))


def all_digests(tracks, counts, dist, cdev):
    """records_digest of every rank, all-gathered (one small collective)."""
    import torch
    d = records_digest(tracks, counts)
    if not dist:
        return [d]
    mine = torch.tensor([d[0], float(d[1])], dtype=torch.float64, device=cdev)
    out = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(out, mine)
    return [(float(o[0]), int(o[1])) for o in (x.cpu() for x in out)]


def sequence_main(args):
    """`--config 5`: the configs[4] sequence replay on its own, as the line's
    headline (sequence_leg, with the per-family profile and the CPU baseline)."""
    import gvx
    dist, dev, world, rank, local = rank_setup(args)
    ctx = gvx.Context(local)
    line = sequence_leg(args, ctx, dev, dist, world, rank, args.frames, cpu=world == 1 and not args.no_cpu)
    if rank == 0:
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()
    ctx.close()


def sequence_summary(line):
    """The configs[4] fields the default line carries under "sequence" (the
    north_star scaling workload: one sequence per GPU and the RCCL gather of every
    rank's per-frame tracks to rank 0, timed inside the region)."""
    keep = ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "frames_per_rank", "tracks_per_frame_mean",
            "gathered_ranks", "gather_check", "gather_bytes_per_rank", "gather_ms", "all_digests", "dist_backend",
            "host_enqueue_ms_per_frame", "scaling")
    out = {k: line[k] for k in keep if k in line}
    out["metric"] = line["metric"]
    out["workload"] = line["config"]["workload"]
    out["device_ms_per_frame"] = line["roofline"]["device_ms_per_frame"]
    return out


def sequence_leg(args, ctx, dev, dist, world, rank, n_frames, cpu=False):
    """configs[4]: one synthetic sequence per GPU (a moving
    camera over a textured plane, frames rendered into HBM before the timed
    region; rank r's seed is synth.SEED + 7919 r).  Per frame, as Tracking::track
    does: CLAHE, the frame's pyramid once, forward + backward LK of the tracked
    points from the previous frame with a constant-velocity initial flow, FB +
    border + compaction, and block-grid detection topping the tracks up to N
    whenever they drop below it.  After the last frame every rank's per-frame
    tracks go to rank 0 in one RCCL gather (inside the timed region).  A step =
    one frame per GPU; value = frames of all ranks / max-over-ranks time.
    Returns the line on rank 0, None elsewhere."""
    import torch
    import gvx
    from gvx import synth
    W, H, N, L = args.width, args.height, args.features, args.levels
    F = max(n_frames, args.warmup + 2)
    frames, _ = synth.make_sequence(W, H, F, dev, seed=synth.SEED + 7919 * rank)
    torch.cuda.synchronize()
    from gvx.tracking import DeviceSequenceTracker, SequenceTracker
    kp = gvx.KltParams.default(max_level=L)
    dp = gvx.DetectParams.default(max_features=N)
    tracks = np.zeros((F, N, 2), np.float32)
    counts = np.zeros(F, np.int32)
    stats = {"detect_frames": 0}
    device_loop = not args.host_loop
    if device_loop:
        # the whole frame (pick frame t on the device, CLAHE + pyramid, LK fwd/bwd +
        # FB + compaction, detection top-up, record the track list) is one graph
        # launch: no host round trip, the host only enqueues
        # pipelined (default): frame t+1's CLAHE + pyramid in a graph on the context's
        # side stream beside frame t's tracking graph (the outputs are the same:
        # tests/test_sequence_gpu.py); --no-pipeline: one graph per frame
        tracker = DeviceSequenceTracker(ctx, W, H, N, klt=kp, detect=dp, graph=True, device=dev, frames=frames,
                                        pipeline=not args.no_pipeline, eig_branch=args.eig_branch,
                                        batch=args.frame_batch)

        def frame(t):
            tracker.step()
    else:
        tracker = SequenceTracker(ctx, W, H, N, klt=kp, detect=dp)

        def frame(t):
            pts = tracker.step(frames[t].data_ptr())
            if "corners" in tracker.last:
                stats["detect_frames"] += 1
            tracks[t, :pts.shape[0]] = pts
            counts[t] = pts.shape[0]

    # K-frame batches are enqueued whole at their first frame: round the warm-up
    # up to a batch boundary, so the timed frames are exactly the batches enqueued
    # inside the timed region
    K = tracker.batch if device_loop else 1
    warm = -(-args.warmup // K) * K
    if warm >= F:
        sys.exit(f"bench.py: --warmup {args.warmup} rounds to {warm} >= {F} frames (batch {K})")
    t = 0
    for _ in range(warm):
        frame(t)
        t += 1
    ctx.sync()
    if dist:
        dist.barrier()
    stats["detect_frames"] = 0
    ctx.profile_reset()
    # per-family device times need event brackets around each call: profile the
    # host loop's calls, and the device loop on a separate pass below
    ctx.profile(not device_loop)
    t0 = time.perf_counter()
    timed = 0
    while t < F:
        frame(t)
        t += 1
        timed += 1
    t_enq = time.perf_counter() - t0  # host time to enqueue the timed frames
    ctx.sync()
    t_g = time.perf_counter()
    if device_loop:
        # the records stay in HBM: RCCL gathers them device to device
        d_tracks, d_counts = tracker.rec_tracks, tracker.rec_counts
    else:
        d_tracks, d_counts = torch.from_numpy(tracks), torch.from_numpy(counts)
    gathered = gather_tracks(d_tracks, d_counts, dist, coll_device(dist, dev))
    torch.cuda.synchronize()
    t_g = time.perf_counter() - t_g
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if device_loop:
        tracker.close()
        tracks[:] = tracker.rec_tracks.cpu().numpy()  # for the line's statistics, after the timed region
        counts[:] = tracker.rec_counts.cpu().numpy()
    # every rank's digest of its own records (outside the timed region): rank 0
    # checks each gathered record set against its owner's digest
    digests = all_digests(tracks, counts, dist, coll_device(dist, dev))
    if gathered:
        gathered = [(t.cpu(), c.cpu()) for t, c in gathered]
    if device_loop:
        # device time per kernel family of the same per-frame work, eager with event
        # brackets (outside the timed region: a captured graph cannot hold them)
        prof = DeviceSequenceTracker(ctx, W, H, N, klt=kp, detect=dp, graph=False, device=dev, frames=frames,
                                     ids=(2, 3))
        for _ in range(min(F, warm + 2)):
            prof.step()
        ctx.sync()
        ctx.profile_reset()
        ctx.profile(True)
        k_prof = min(F - prof.t, 200)
        for _ in range(k_prof):
            prof.step()
        ctx.sync()
        fam = {f: ctx.profile_read(f) for f in ("clahe", "pyramid", "klt", "compact", "detect")}
        fam = {k: (v[0] * timed / k_prof, v[1]) for k, v in fam.items() if v[1] > 0}
        ctx.profile(False)
        prof.close()
    else:
        fam = {f: ctx.profile_read(f) for f in ("clahe", "pyramid", "klt", "compact", "detect")}
        fam = {k: v for k, v in fam.items() if v[1] > 0}
        ctx.profile(False)
    elapsed = max_over_ranks(elapsed, dist, dev)
    t_g = max_over_ranks(t_g, dist, dev)
    del frames
    if rank != 0:
        return None
    value = world * timed / elapsed
    dev_ms = sum(v[0] for v in fam.values()) / timed
    # the frame-pair unit with each frame read and its pyramid
    # built once per sequence frame instead of twice
    ap, sw, sh = 0, W, H
    for _ in range(L):
        sw, sh = (sw + 1) // 2, (sh + 1) // 2
        ap += sw * sh
    B = algorithmic_bytes(W, H, L, N) - W * H - 2 * ap + 2 * W * H  # + CLAHE: read + write the frame
    achieved = B / (dev_ms * 1e-3) / 1e9 if dev_ms > 0 else None
    cpu_line = None
    if cpu:
        cpu_line = cpu_baseline(W, H, N, L, args.cpu_budget / 2, threads=host_threads(), clahe=True)
        cpu_line["sample"] += " (per sequence frame, detection not included)"
    tr = counts[F - timed:]
    return {
        "metric": f"KLT sequence frames/sec @{W}x{H},{N} feat (configs[4])", "value": round(value, 2),
        "unit": "frames/s", "n_gpus": world, "steps": timed, "warmup": warm,
        "ms_per_step": round(elapsed / timed * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8/i32 windows, f32 solve",
        "data": "synthetic sequences (moving camera over a band-limited texture, seed 20261015 + 7919*rank)",
        "config": {"workload": f"configs[4]: one {F}-frame sequence per GPU, {W}x{H} mono, {N} feat, maxLevel "
                               f"{L}: per frame CLAHE + pyramid + fwd/bwd LK + FB + compaction + detection top-up; "
                               f"RCCL gather of all per-frame tracks to rank 0",
                   "loop": (("device-resident: one captured hipGraph launch per frame (gvx_track_frame_dev)"
                             if args.no_pipeline else
                             ("device-resident, pipelined: a graph tracking frames t..t+K-1 "
                              "(gvx_track_frame_dev + the track record, per frame) on the context stream beside a "
                              "graph preprocessing frames t+K..t+2K-1 on its side stream "
                              "(gvx_branch_begin/_end/_join), K = %d" % args.frame_batch))
                            if device_loop else "host loop: SequenceTracker, host round trips per frame"),
                   "frame_batch": args.frame_batch if device_loop and not args.no_pipeline else None,
                   "parallelism": f"sequences sharded over {world} GPU(s)"},
        "roofline": {"bound": "hbm", "kernel": "per-frame pipeline (latency-bound: one frame at a time)",
                     "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": None, "algorithmic_bytes_per_frame": B,
                     "device_ms_per_frame": {k: round(v[0] / timed, 4) for k, v in fam.items()}},
        "cpu_baseline": cpu_line,
        "frames_per_rank": F,
        "tracks_per_frame_mean": round(float(tr.mean()), 1),
        "detect_frames": stats["detect_frames"] if not device_loop else None,
        "host_overhead_frac": round(max(0.0, 1.0 - dev_ms / (elapsed / timed * 1e3)), 3) if dev_ms else None,
        "host_enqueue_ms_per_frame": round(t_enq / timed * 1e3, 4),
        "gathered_ranks": len(gathered) if gathered else 0,
        # the exchange: F x N x 2 f32 tracks + F counts per rank, one gather to rank 0
        "gather_bytes_per_rank": int(4 * (F * N * 2 + F)),
        "gather_ms": round(t_g * 1e3, 3),
        "all_digests": [[d[0], d[1]] for d in digests],
        "gather_check": bool(gathered and np.array_equal(gathered[0][0].numpy(), tracks)
                             and np.array_equal(gathered[0][1].numpy(), counts)
                             and all(int(c[F - timed:].min()) > 0 for _, c in gathered)
                             and all(records_digest(t.numpy(), c.numpy()) == d
                                     for (t, c), d in zip(gathered, digests))),
        "dist_backend": dist.get_backend() if dist else None,
    }


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N ranks (one process per
    GPU) through torch.distributed.run as CHILD processes, before this process
    touches the GPU, and return their exit status.  Rank 0 prints the line."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.run(cmd, env=env).returncode


def progress(what):
    """GVX_BENCH_TRACE=1: one stderr line per leg (where a run under a profiler stalls)."""
    if os.environ.get("GVX_BENCH_TRACE"):
        print(f"[bench {time.strftime('%H:%M:%S')}] {what}", file=sys.stderr, flush=True)


def side_legs_before_headline(args):
    """The side legs that run before the headline's W warm-up steps ramp the
    shader clock: with 3 warm-up steps alone LK reads 0.50-0.55 ms
    instead of 0.47.  The last, "settle", runs SETTLE_STEPS of the headline's own
    steps: the clock settles to the pyramid-beside-LK load over ~20 ms
    (profiles/r06_c1: pipelined steps 0.53 -> 0.47 ms over the first 20).  They
    run at EVERY world size -- through r05 the LK leg ran
    at N = 1 only, so the N > 1 points of the scaling curve were timed at a
    colder clock."""
    return [] if args.no_pre else ["lk_accum", "preprocess", "settle"]


SETTLE_STEPS = 40  # the headline's own (pipelined) steps, untimed, after the other side legs


def ranks_that_ran(flag, dist, dev=None):
    """How many ranks report `flag` true (an all-reduce; 1 or 0 without dist)."""
    if not dist:
        return int(bool(flag))
    import torch
    t = torch.tensor([int(bool(flag))], dtype=torch.int64, device=coll_device(dist, dev))
    dist.all_reduce(t)
    return int(t.item())


def max_over_ranks(elapsed, dist, dev=None):
    if not dist:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=coll_device(dist, dev))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def mock_main(args):
    """The launcher contract without a GPU: same rank handling, barrier-bracketed
    timing, max over ranks and rank-0 JSON line; a step is a fixed host sleep.
    With --config 5 the sequence replay's track gather runs too (gloo).
    Used by tests/test_bench_dist.py (gloo, world_size 2)."""
    import torch
    import torch.distributed as tdist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        tdist.init_process_group(args.backend or "gloo")
        dist = tdist
    step_s = 0.002 * (1 + rank)  # ranks deliberately unequal: the max must win
    legs = side_legs_before_headline(args)  # the same decision main() takes
    for _ in legs:
        time.sleep(step_s)
    side_ranks = ranks_that_ran(bool(legs), dist)
    for _ in range(args.warmup):
        time.sleep(step_s)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(step_s)
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dist)
    # the configs[4] exchange (gather_tracks + all_digests), as the default line's
    # "sequence" sub-object and --config 5 run it: each rank's records differ
    F, N = 6, 4
    tr = torch.full((F, N, 2), float(rank)) + torch.arange(F, dtype=torch.float32)[:, None, None]
    cn = torch.full((F,), 3 + rank, dtype=torch.int32)
    t1 = time.perf_counter()
    for _ in range(F):
        time.sleep(step_s / 4)
    g = gather_tracks(tr, cn, dist, torch.device("cpu"))
    seq_el = max_over_ranks(time.perf_counter() - t1, dist)
    digests = all_digests(tr.numpy(), cn.numpy(), dist, torch.device("cpu"))
    gathered_ok = None
    if rank == 0:
        gathered_ok = len(g) == world and all(
            bool((gt[:, :, 0] == r + torch.arange(F)[:, None]).all()) and bool((gc == 3 + r).all())
            and records_digest(gt.numpy(), gc.numpy()) == d for r, ((gt, gc), d) in enumerate(zip(g, digests)))
    if rank == 0:
        line = {"metric": "mock", "value": world * args.pairs * args.steps / elapsed, "unit": "frames/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
                "scaling": "weak", "elapsed_s": elapsed, "gathered_ok": gathered_ok,
                "side_legs_before_headline": legs, "side_legs_before_headline_ranks": side_ranks}
        if args.config != 5 and not args.no_sequence:
            line["sequence"] = {"metric": "mock sequence", "value": world * F / seq_el, "unit": "frames/s",
                                "n_gpus": world, "steps": F, "frames_per_rank": F, "gathered_ranks": len(g),
                                "gather_check": gathered_ok, "all_digests": [[d[0], d[1]] for d in digests],
                                "dist_backend": dist.get_backend() if dist else None, "scaling": "weak"}
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

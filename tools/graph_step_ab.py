#!/usr/bin/env python3
"""Wall time per configs[1] step (256 pairs: pyramid pass + LK/FB + compaction)
enqueued eagerly vs replayed from a captured hipGraph, interleaved rounds on one
box.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ic-gvins_amd")]
import torch  # noqa: E402
import gvx  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
wl = bench.KltWorkload(256, 1280, 560, 150, dev)
ctx = gvx.Context(0)
p = gvx.KltParams.default(max_level=3)
K = 40
for _ in range(60):  # shader clock up
    wl.step(ctx, p)
ctx.sync()
graphs = [ctx.capture(wl.step, ctx, p) for _ in range(2)]


def eager():
    for _ in range(K):
        wl.step(ctx, p)


def graph():
    for i in range(K):
        ctx.graph_launch(graphs[i & 1])


out = {"eager_ms": [], "graph_ms": []}
for _ in range(4):
    for name, fn in (("eager_ms", eager), ("graph_ms", graph)):
        fn()
        ctx.sync()
        t0 = time.perf_counter()
        fn()
        ctx.sync()
        out[name].append(round((time.perf_counter() - t0) / K * 1e3, 4))
for g in graphs:
    g.destroy()
ctx.close()
print(json.dumps(out))

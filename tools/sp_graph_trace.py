#!/usr/bin/env python3
"""Single frame pair (configs[1], one pair per launch: pyramid pass, LK + FB,
compaction) eager vs replayed as a captured hipGraph, for a rocprofv3
--kernel-trace run: 300 eager pairs, a 50 ms pause, 300 graph replays.
    rocprofv3 --kernel-trace --output-format csv -d DIR -- python3 tools/sp_graph_trace.py
    python3 tools/sp_graph_trace.py --analyse DIR
The analysis splits the trace at the pause and reports, per phase, the median
duration of each kernel and of the gaps between consecutive kernels."""
import csv
import glob
import os
import statistics
import re
import sys


def kname(n):
    """short kernel name: the identifier before the argument list"""
    m = re.search(r"([A-Za-z_][A-Za-z_0-9]*(<[^()]*>)?)\(", n)
    return m.group(1) if m else n[:40]
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ic-gvins_amd")]

if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
    ops = []
    for f in glob.glob(f"{sys.argv[2]}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"])))
    ops.sort()
    gaps = [b[0] - a[1] for a, b in zip(ops, ops[1:])]
    cut = max(range(len(gaps)), key=lambda i: gaps[i]) + 1  # the pause
    for name, ph in (("eager", ops[:cut]), ("graph", ops[cut:])):
        ph = ph[-600:]
        kinds = sorted({o[2] for o in ph})
        print(f"== {name}: {len(ph)} kernels")
        for k in kinds:
            d = [(o[1] - o[0]) / 1000 for o in ph if o[2] == k]
            print(f"  {k[:40]:40s} {statistics.median(d):7.2f} us (n {len(d)})")
        for a_k in kinds:
            g = [(b[0] - a[1]) / 1000 for a, b in zip(ph, ph[1:]) if a[2] == a_k]
            print(f"  gap after {a_k[:30]:30s} {statistics.median(g):7.2f} us")
        per = [(b[0] - a[0]) / 1000 for a, b in zip(ph, ph[1:]) if a[2] == ph[0][2] and False]
        starts = [o[0] for o in ph if o[2] == ph[-1][2]]
        print(f"  period per pair {statistics.median([(b - a) / 1000 for a, b in zip(starts, starts[1:])]):7.2f} us")
    sys.exit(0)

import torch  # noqa: E402
import gvx  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
ctx = gvx.Context(0)
wl = bench.KltWorkload(2, 1280, 560, 150, dev, distinct=2)
params = gvx.KltParams.default(max_level=3)
I1, J1, P1, Q1 = wl.I[0:1], wl.J[0:1], wl.P[0:1], wl.Q[0:1]
N1, B1, F1, K1, NK1 = wl.N[0:1], wl.B[0:1], wl.F[0:1], wl.K[0:1], wl.NK[0:1]


def enqueue():
    ctx.klt_fb_batch_init_dev(1, 1280, 560, I1.data_ptr(), J1.data_ptr(), 150, P1.data_ptr(), Q1.data_ptr(),
                              N1.data_ptr(), B1.data_ptr(), F1.data_ptr(), K1.data_ptr(), NK1.data_ptr(),
                              params=params)


for _ in range(100):
    enqueue()
ctx.sync()
t0 = time.perf_counter()
for _ in range(300):
    enqueue()
ctx.sync()
eager = (time.perf_counter() - t0) / 300
time.sleep(0.05)
ctx.capture_begin()
enqueue()
g = ctx.capture_end()
for _ in range(100):
    ctx.graph_launch(g)
ctx.sync()
t0 = time.perf_counter()
for _ in range(300):
    ctx.graph_launch(g)
ctx.sync()
graph = (time.perf_counter() - t0) / 300
g.destroy()
ctx.close()
print({"us_per_pair_eager": round(eager * 1e6, 2), "us_per_pair_graph": round(graph * 1e6, 2)})

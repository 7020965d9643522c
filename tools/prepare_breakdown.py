#!/usr/bin/env python3
"""Per-prepare breakdown from a rocprofv3 --kernel-trace --memory-copy-trace
run of tools/prepare_trace.py: the median duration of each copy / kernel and of
the gaps between consecutive operations of one prepare.
    python3 tools/prepare_breakdown.py <rocprofv3 output dir>"""
import csv
import glob
import statistics
import re
import sys


def kname(n):
    """short kernel name: the identifier before the argument list"""
    m = re.search(r"([A-Za-z_][A-Za-z_0-9]*(<[^()]*>)?)\(", n)
    return m.group(1) if m else n[:40]

root = sys.argv[1]
ops = []
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"])))
for f in glob.glob(f"{root}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r["Direction"]))
ops.sort()
# the last 100 prepares: H2D, kernels, D2H ... group from each H2D
idx = [i for i, o in enumerate(ops) if o[2].startswith("copy") and "HOST_TO_DEVICE" in o[2].upper()]
groups = []
for a, b in zip(idx, idx[1:] + [len(ops)]):
    groups.append(ops[a:b])
groups = [g for g in groups[-100:] if len(g) >= 3]
names = [o[2] for o in groups[0]]
print("ops per prepare:", names)
for j, n in enumerate(names):
    d = statistics.median((g[j][1] - g[j][0]) / 1000 for g in groups if len(g) == len(names))
    print(f"  {n:40s} {d:8.2f} us")
    if j + 1 < len(names):
        gap = statistics.median((g[j + 1][0] - g[j][1]) / 1000 for g in groups if len(g) == len(names))
        print(f"  {'gap':40s} {gap:8.2f} us")
span = statistics.median((g[-1][1] - g[0][0]) / 1000 for g in groups)
starts = [g[0][0] for g in groups]
per = statistics.median((b - a) / 1000 for a, b in zip(starts, starts[1:]))
print(f"  device span per prepare (first op start -> last op end) {span:.2f} us; prepare period {per:.2f} us")

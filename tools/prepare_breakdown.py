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
# the last 100 prepares: the op sequence repeats with period L (copies and
# kernels of one prepare: mapped results are a parameter upload and one kernel,
# the D2H form adds the result copy); L is the shortest period of the tail
names_all = [o[2] for o in ops]
L = next(L for L in range(1, 16) if all(names_all[-i] == names_all[-i - L] for i in range(1, 3 * L + 1)))
tail = ops[len(ops) - (len(ops) // L) * L:]
groups = [tail[k:k + L] for k in range(0, len(tail), L)][-100:]
names = [o[2] for o in groups[-1]]
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

#!/usr/bin/env python3
"""The headline's own kernels in a rocprofv3 --kernel-trace of `bench.py`: runs of
consecutive configs[1] steps (stream_kernel<3,*>, klt_kernel<2,0>, compact_kernel);
the headline is the run of exactly W + K steps (the accumulation leg's EXACT run
before it is longer; the CLAHE leg and the single-pair leg bound it), and its last
K steps are the timed ones.  Prints their average durations, to set beside the
line's HIP-event `device_ms_per_step`.
    python3 tools/headline_trace.py <kernel_trace.csv> [K [W]]"""
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
W = int(sys.argv[3]) if len(sys.argv) > 3 else 5


def kind(r):
    n = r["Kernel_Name"]
    if "stream_kernel<3" in n:
        return "pyramid"
    if "klt_kernel<2, 0>" in n:
        return "klt"
    if "compact_kernel" in n:
        return "compact"
    return None


runs, cur = [], []
i = 0
while i + 2 < len(rows):
    if [kind(rows[i + j]) for j in range(3)] == ["pyramid", "klt", "compact"]:
        cur.append(rows[i:i + 3])
        i += 3
        continue
    if cur:
        runs.append(cur)
    cur = []
    i += 1
if cur:
    runs.append(cur)
exact = [r for r in runs if len(r) == W + K]
best = exact[-1] if exact else [r for r in runs if len(r) >= K][-1]
timed = best[-K:]
out = {"run_steps": len(best), "timed_steps": len(timed)}
for j, name in enumerate(("pyramid", "klt", "compact")):
    d = [(int(s[j]["End_Timestamp"]) - int(s[j]["Start_Timestamp"])) / 1e6 for s in timed]
    out[name + "_ms"] = round(sum(d) / len(d), 4)
span = (int(timed[-1][2]["End_Timestamp"]) - int(timed[0][0]["Start_Timestamp"])) / 1e6
out["span_ms_per_step"] = round(span / len(timed), 4)
print(json.dumps(out))

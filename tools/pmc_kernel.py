#!/usr/bin/env python3
"""Per-dispatch PMC values of one kernel (largest grid) from a rocprofv3 --pmc
output directory, per wave, with the gfx950 quad-cycle correction for SQ_*CYCLES
/ SQ_WAIT_* / SQ_ACTIVE_INST_* (MI355X_MICROARCH.md).
    python3 tools/pmc_kernel.py <dir> <kernel-substring>"""
import collections
import csv
import glob
import gzip
import sys

root, name = sys.argv[1], sys.argv[2]
# rows of one pass (file) are summed per dispatch; a counter collected in
# several passes (SQ_WAVES, in every group) is averaged over them.  Through r05
# it was summed, which doubled SQ_WAVES and halved every per-wave figure.
raw = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{root}/**/*counter_collection.csv*", recursive=True):
    for r in csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)):
        if name not in r["Kernel_Name"]:
            continue
        key = (int(r["Grid_Size"]), r["Dispatch_Id"])
        raw[(key, r["Counter_Name"])][f] += float(r["Counter_Value"])
acc = collections.defaultdict(dict)
for (key, cn), by_pass in raw.items():
    acc[key][cn] = sum(by_pass.values()) / len(by_pass)
if not acc:
    sys.exit(f"no dispatch of {name}")
grid = max(k[0] for k in acc)
rows = [v for k, v in acc.items() if k[0] == grid]
avg = {c: sum(r.get(c, 0.0) for r in rows) / len(rows) for c in rows[0]}
waves = avg.get("SQ_WAVES", 0.0)
print(f"{name}: grid {grid}, {len(rows)} dispatches")
for c in sorted(avg):
    v = avg[c]
    scale = 4 if ("CYCLES" in c or c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE_INST")) and c != "SQ_BUSY_CYCLES" else 1
    per = f"  per wave {v * scale / waves:.4g}" if waves and c != "SQ_WAVES" else ""
    print(f"  {c:28s} {v:.4g}{per}")

#!/usr/bin/env python3
"""Median duration per kernel name (substring filter) of rocprofv3 kernel-trace
csv files under each directory given: python3 tools/trace_medians.py <filter> <dir>..."""
import collections
import csv
import glob
import re
import sys


def kname(n):
    """short kernel name: the identifier before the argument list"""
    m = re.search(r"([A-Za-z_][A-Za-z_0-9]*(<[^()]*>)?)\(", n)
    return m.group(1) if m else n[:40]

flt = sys.argv[1]
for root in sys.argv[2:]:
    d = collections.defaultdict(list)
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if flt in n:
                k = kname(n)
                d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print(root, " | ".join("%s %.1f us (n %d)" % (k, sorted(v)[len(v) // 2], len(v)) for k, v in sorted(d.items())))

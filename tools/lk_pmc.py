#!/usr/bin/env python3
"""The bench's configs[1] KLT step (bench.KltWorkload: 256 pairs, pyramid pass +
LK/FB + compaction) for PMC passes of klt_kernel: K steps at the given LK
iteration cap (default 30, the reference's criteria; 0 = the window
extractions and level set-up alone, so iterations = full - capped).
    python3 tools/lk_pmc.py [max_iter] [steps] [3 = configs[2] geometry]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ic-gvins_amd")]
import torch  # noqa: E402
import gvx  # noqa: E402
import bench  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 30
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
# geometry: configs[1] by default; "3" = configs[2] (1920x1200, 500 points, maxLevel 4)
W_, H_, N_, L_ = (1920, 1200, 500, 4) if len(sys.argv) > 3 and sys.argv[3] == "3" else (1280, 560, 150, 3)
dev = torch.device("cuda", 0)
ctx = gvx.Context(0)
wl = bench.KltWorkload(256, W_, H_, N_, dev)
p = gvx.KltParams.default(max_level=L_, max_iter=it)
for _ in range(k):
    wl.step(ctx, p)
ctx.sync()
ctx.close()
print("lk_pmc done", it, k)

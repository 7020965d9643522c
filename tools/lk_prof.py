#!/usr/bin/env python3
"""Per-level timestamps of the one-point-wave LK kernel on sequence frames
(GVX_LIB = a build of klt.hip with wall_clock64 stamps at each level's start,
after its extraction + 2x2 set-up, and after its iterations).  For the slowest
wave of each frame (the one the frame waits for) and on average: extraction and
iteration microseconds per level and direction, iteration counts.  Timing probe
only: not product code."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ic-gvins_amd"))
import torch  # noqa: E402
import gvx  # noqa: E402
from gvx import synth  # noqa: E402
from gvx.tracking import DeviceSequenceTracker  # noqa: E402

lib = ctypes.CDLL(os.environ["GVX_LIB"])
W, H, N, F, L = 1280, 560, 150, int(os.environ.get("FRAMES", "40")), 3
dev = torch.device("cuda", 0)
frames, _ = synth.make_sequence(W, H, F, dev, seed=synth.SEED)
ctx = gvx.Context(0)
trk = DeviceSequenceTracker(ctx, W, H, N, klt=gvx.KltParams.default(max_level=L),
                            detect=gvx.DetectParams.default(max_features=N), graph=False, device=dev, frames=frames)
buf = np.zeros((512, 2, 6, 4), np.uint64)
acc = []
for t in range(F):
    lib.gvx_dbg_lk_clear()
    trk.step()
    ctx.sync()
    lib.gvx_dbg_lk_times(buf.ctypes.data_as(ctypes.c_void_p))
    if t < 3:
        continue
    b = buf.astype(np.int64)
    live = np.nonzero(b[:, 1, 5, 0])[0]
    if len(live) == 0:
        continue
    k0 = b[live, 0, 5, 0].min()
    end = b[live, 1, 5, 0]
    slow = live[np.argmax(end)]
    row = {"frame": t, "waves": int(len(live)), "kernel_us": float((end.max() - k0) * 0.01),
           "slowest_wave_us": float((b[slow, 1, 5, 0] - b[slow, 0, 5, 0]) * 0.01),
           "start_spread_us": float((b[live, 0, 5, 0].max() - k0) * 0.01)}
    per = {}
    for d in range(2):
        for lv in range(L, -1, -1):
            s0, s1, s2, it = b[slow, d, lv]
            if s0 == 0 or s1 == 0:
                continue
            per[f"{'fb'[d]}{lv}"] = [round((s1 - s0) * 0.01, 2), round((s2 - s1) * 0.01, 2), int(it)]
    row["slowest_extract_iter_us_iters"] = per
    # mean over waves of extraction / iteration time per level-direction
    ex = (b[live, :, :4, 1] - b[live, :, :4, 0]) * 0.01
    itt = (b[live, :, :4, 2] - b[live, :, :4, 1]) * 0.01
    ok = (b[live, :, :4, 1] > 0) & (b[live, :, :4, 0] > 0)
    row["mean_extract_us"] = round(float(ex[ok].mean()), 2)
    row["mean_iter_block_us"] = round(float(itt[ok].mean()), 2)
    row["mean_iters"] = round(float(b[live, :, :4, 3][ok].mean()), 2)
    acc.append(row)
    print(json.dumps(row))
trk.close()
ctx.close()

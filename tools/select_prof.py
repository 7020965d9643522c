#!/usr/bin/env python3
"""Phase times of the tracking path's selection kernel on detection frames
(GVX_LIB = a build of tools/ r03 select-timestamp variant, which stamps
wall_clock64 at each phase of select_track_kernel into a device array).
Timing probe only: not product code."""
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
W, H, N, F = 1280, 560, 150, int(os.environ.get("FRAMES", "60"))
dev = torch.device("cuda", 0)
frames, _ = synth.make_sequence(W, H, F, dev, seed=synth.SEED)
ctx = gvx.Context(0)
trk = DeviceSequenceTracker(ctx, W, H, N, klt=gvx.KltParams.default(max_level=3),
                            detect=gvx.DetectParams.default(max_features=N), graph=False, device=dev, frames=frames)
buf = np.zeros((64, 8), np.uint64)
sub = np.zeros((64, 21, 4), np.uint64)
names = ["want", "filter", "-", "-", "greedy", "subpix"]
rows = []
for t in range(F):
    lib.gvx_dbg_select_clear()
    lib.gvx_dbg_sub_clear()
    trk.step()
    ctx.sync()
    lib.gvx_dbg_select_times(buf.ctypes.data_as(ctypes.c_void_p))
    det = [k for k in range(64) if buf[k, 6] != 0]
    lib.gvx_dbg_sub_times(sub.ctypes.data_as(ctypes.c_void_p))
    if not det or t == 0:
        continue
    ph = np.array([[(int(buf[k, i + 1]) - int(buf[k, i])) * 0.01 for i in range(6)] for k in det])
    tot = max(int(buf[k, 6]) for k in det) - min(int(buf[k, 0]) for k in det)
    nc = [int(buf[k, 7]) >> 32 for k in det]
    na = [int(buf[k, 7]) & 0xffffffff for k in det]
    rows.append({"frame": t, "blocks": len(det), "span_us": tot * 0.01,
                 "phase_max_us": dict(zip(names, np.round(ph.max(0), 2).tolist())),
                 "phase_mean_us": dict(zip(names, np.round(ph.mean(0), 2).tolist())),
                 "cand_max": max(nc), "acc_max": max(na)})
    # cornerSubPix iterations of the first corner of the first detecting block
    k0 = det[0]
    its = [i for i in range(20) if sub[k0, i, 0] != 0]
    if its:
        per = np.array([[(int(sub[k0, i, q + 1]) - int(sub[k0, i, q])) * 0.01 for q in range(3)] for i in its])
        tail = [(int(sub[k0, i + 1, 0]) - int(sub[k0, i, 3])) * 0.01 for i in its[:-1]]
        rows[-1]["subpix_iters"] = len(its)
        rows[-1]["subpix_us_patch_terms_sums"] = np.round(per.mean(0), 2).tolist()
        rows[-1]["subpix_us_solve"] = round(float(np.mean(tail)), 2) if tail else None
        rows[-1]["subpix_us_per_iter"] = round((int(sub[k0, its[-1], 3]) - int(sub[k0, its[0], 0])) * 0.01 / len(its), 2)
for r in rows:
    print(json.dumps(r))
trk.close()
ctx.close()

#!/usr/bin/env python3
"""Residency timeline of one configs[1] LK launch, or of
one pyramid pass (argument 4 = pyr: stream_kernel, 256-thread workgroups).

Needs the diagnostic build (every wave stamps s_memrealtime at start and end,
plus HW_ID / XCC_ID; klt.hip GVX_KLT_TRACE):
    EXTRA=-DGVX_KLT_TRACE bash tools/variant.sh klttrace
    GVX_LIB=ic-gvins_amd/gvx/variants/libgvx_klttrace.so python3 tools/lk_residency.py <outdir> [warm] [lpp|-] [klt|pyr]

Writes <outdir>/waves.csv (one row per wave: id, start_us, end_us, xcc, se, sh,
cu, simd, slot) and <outdir>/timeline.csv (1 us bins: resident waves per SIMD,
mean over the SIMDs the launch used, and its minimum / maximum over SIMDs), and
prints a summary: span, wave-duration quantiles, the time-averaged residency
against the 4 waves per SIMD the kernel's registers and LDS allow, and the tail
(from the last wave start to the launch end)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ic-gvins_amd")]
import torch  # noqa: E402
import gvx  # noqa: E402
import bench  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/lk_residency"
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 300
lpp = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3] != "-" else None  # gvx_set_klt_phases
kern = sys.argv[4] if len(sys.argv) > 4 else "klt"  # klt: the LK launch; pyr: the pyramid pass (stream_kernel)
os.makedirs(out, exist_ok=True)
dev = torch.device("cuda", 0)
ctx = gvx.Context(0)
wl = bench.KltWorkload(256, 1280, 560, 150, dev)
p = gvx.KltParams.default(max_level=3)
if lpp is not None:
    ctx.set_klt_phases(lpp)
lib = gvx.lib()
trace_set = lib.gvx_klt_trace_set if kern == "klt" else lib.gvx_pyr_trace_set
trace_set.argtypes = [ctypes.c_void_p]
trace_set.restype = ctypes.c_int
# launch grid: 8 XCDs x ceil(waves / 8) one-wave workgroups (klt.hip launch_klt_ppw),
# times up to 8 phases (klt_phase_kernel)
n_waves = 256 * 50
grid = 8 * ((n_waves + 7) // 8)
buf = torch.zeros(4 * (8 * grid + 64), dtype=torch.int64, device=dev)
# the clock ramps up under load: warm-up steps first (stamps off)
for _ in range(warm):
    wl.step(ctx, p)
ctx.sync()
runs = []
for rep in range(3):
    buf.zero_()
    assert trace_set(ctypes.c_void_p(buf.data_ptr())) == 0
    wl.step(ctx, p)
    ctx.sync()
    assert trace_set(None) == 0
    for _ in range(20):
        wl.step(ctx, p)
    ctx.sync()
    runs.append(buf.view(-1, 4).cpu().numpy().astype(np.uint64))
ctx.close()


def analyse(rec, tag, write):
    rec = rec[rec[:, 1] > 0]
    t0 = rec[:, 1].min()
    s = (rec[:, 1] - t0).astype(np.float64) / 100.0  # us (100 MHz)
    e = (rec[:, 2] - t0).astype(np.float64) / 100.0
    hw = rec[:, 3] & 0xffffffff
    xcc = (rec[:, 3] >> 32) & 0xf
    slot = hw & 0xf
    simd = (hw >> 4) & 0x3
    cu = (hw >> 8) & 0xf
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    simd_key = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
    keys, inv = np.unique(simd_key, return_inverse=True)
    dur = e - s
    busy = dur > 1.0  # idle waves of the padded grid leave at once
    span = e.max()
    nb = int(np.ceil(span))
    occ = np.zeros((len(keys), nb + 1))
    for i in np.nonzero(busy)[0]:
        a, b = s[i], e[i]
        ia, ib = int(a), int(b)
        if ia == ib:
            occ[inv[i], ia] += b - a
        else:
            occ[inv[i], ia] += ia + 1 - a
            occ[inv[i], ia + 1:ib] += 1
            occ[inv[i], ib] += b - ib
    mean_t = occ.mean(axis=0)
    if write:
        with open(os.path.join(out, "waves.csv"), "w") as f:
            f.write("id,start_us,end_us,xcc,se,sh,cu,simd,slot\n")
            for i in np.argsort(s):
                f.write(f"{int(rec[i, 0])},{s[i]:.2f},{e[i]:.2f},{int(xcc[i])},{int(se[i])},{int(sh[i])},"
                        f"{int(cu[i])},{int(simd[i])},{int(slot[i])}\n")
        with open(os.path.join(out, "timeline.csv"), "w") as f:
            f.write("t_us,resident_per_simd_mean,min,max\n")
            for t in range(nb + 1):
                f.write(f"{t},{mean_t[t]:.3f},{occ[:, t].min():.2f},{occ[:, t].max():.2f}\n")
    last_start = s[busy].max()
    d = dur[busy]
    res = {
        "tag": tag,
        "span_us": round(span, 2),
        "waves": int(busy.sum()),
        "simds": int(len(keys)),
        "cus": int(len(np.unique(simd_key // 4))),
        "wave_us_q": [round(float(np.quantile(d, q)), 2) for q in (0.0, 0.1, 0.5, 0.9, 1.0)],
        "wave_us_mean": round(float(d.mean()), 2),
        "resident_mean": round(float(occ.sum() / (len(keys) * span)), 3),
        "resident_max_slots": 4,
        "fill_frac": round(float(occ.sum() / (len(keys) * span * 4)), 3),
        "first_start_spread_us": round(float(np.quantile(s[busy], 0.25)), 2),
        "last_start_us": round(float(last_start), 2),
        "tail_us": round(float(span - last_start), 2),
        "resident_mean_before_last_start": round(float(mean_t[:int(last_start)].mean()), 3),
        "resident_mean_in_tail": round(float(mean_t[int(last_start):].mean()), 3),
        "ramp_us_to_3.5": next((t for t in range(nb) if mean_t[t] >= 3.5), None),
    }
    return res


import json  # noqa: E402
summ = [analyse(r, f"rep{i}", i == len(runs) - 1) for i, r in enumerate(runs)]
with open(os.path.join(out, "summary.json"), "w") as f:
    json.dump(summ, f, indent=1)
for r in summ:
    print(json.dumps(r))

#!/usr/bin/env python3
"""Clock probe of the covariance pass (variant library built with the CLOCK PROBE
stamps: s_memtime and s_memrealtime written by lane 0 of each segment at every
step, over the first two doubles of its pn_ samples).  Runs warm launches of the
configs[3] preintegration batch and prints, for a few segments, the shader cycles
and the wall ns per step and the implied shader clock.  Timing only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
sys.argv = sys.argv[:1]
import preint_loop as pl  # noqa: E402  (builds the batch and runs the cold/warm timing)

pn = pl.d_pn.cpu().numpy().reshape(pl.S, pl.M - 1, 4)
out = {}
for seg in (0, 1, pl.S // 2, pl.S - 1):
    cyc = pn[seg, :, 0]
    rt = pn[seg, :, 1]
    dc = (cyc[-1] - cyc[1]) / (len(cyc) - 2)
    dr = (rt[-1] - rt[1]) / (len(rt) - 2) * 10.0  # 100 MHz ticks -> ns
    out[str(seg)] = {"cycles_per_step": round(dc, 1), "ns_per_step": round(dr, 1),
                     "ghz": round(dc / dr, 3) if dr > 0 else None,
                     "start_us": round((rt[1] - pn[0, 1, 1]) / 100.0, 2)}
print(json.dumps(out))

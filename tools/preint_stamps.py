#!/usr/bin/env python3
"""Stamp probe of the covariance step (variant library built with the STAMP
PROBE: s_memtime at the step's start, after the G stores, after the K reads
landed, and at the end, written by lane 0 of each segment over its pn_
sample): median shader cycles of each phase per step, and of the gap from one
step's end to the next step's start (the record phase every STAMP_CK steps, default 6).  Each
stamp waits for the outstanding LDS operations, so phases include drains.
Run with GVX_LIB=.../libgvx_stamp.so; PREINT_REPS as preint_loop.py."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
sys.argv = sys.argv[:1]
import numpy as np  # noqa: E402
import preint_loop as pl  # noqa: E402

pn = pl.d_pn.cpu().numpy().reshape(pl.S, pl.M - 1, 4)
out = {}
for seg in (0, 1, pl.S // 2, pl.S - 1):
    t = pn[seg]
    ph = np.diff(t, axis=1)  # t1-t0, t2-t1, t3-t2
    gap = t[1:, 0] - t[:-1, 3]
    CK = int(os.environ.get("STAMP_CK", "6"))  # steps per record chunk
    chunk = gap[np.arange(len(gap)) % CK == CK - 1]  # the record phase between chunks
    plain = gap[np.arange(len(gap)) % CK != CK - 1]
    out[str(seg)] = {"start_to_stores": float(np.median(ph[:, 0])), "stores_to_K": float(np.median(ph[:, 1])),
                     "K_to_end": float(np.median(ph[:, 2])), "gap_in_chunk": float(np.median(plain)),
                     "gap_record_phase": float(np.median(chunk)),
                     "per_step": float((t[-1, 3] - t[0, 0]) / (len(t) - 1))}
print(json.dumps(out))

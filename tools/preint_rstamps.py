#!/usr/bin/env python3
"""Record-phase stamps (variant from tools/preint_rstamp_variant.py): median
shader cycles per chunk of the DMA wait, the record build and the DMA issue,
and of the chunk's steps (top of one chunk to the top of the next).
Run with GVX_LIB=.../libgvx_rstamp.so; PREINT_REPS as preint_loop.py."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
sys.argv = sys.argv[:1]
import numpy as np  # noqa: E402
import preint_loop as pl  # noqa: E402

CK = int(os.environ.get("STAMP_CK", "6"))
pn = pl.d_pn.cpu().numpy().reshape(pl.S, pl.M - 1, 4)
out = {}
for seg in (0, 1, pl.S // 2, pl.S - 1):
    t = pn[seg, ::CK]
    t = t[: (pl.M - 2) // CK + 1]
    ph = np.diff(t, axis=1)
    out[str(seg)] = {"wait": float(np.median(ph[:, 0])), "records": float(np.median(ph[:, 1])),
                     "dma_issue": float(np.median(ph[:, 2])),
                     "chunk": float(np.median(np.diff(t[:, 0]))), "chunks": int(len(t))}
print(json.dumps(out))

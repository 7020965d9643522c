#!/usr/bin/env python3
"""Save the configs[3] preintegration batch's results (after tools/preint_loop.py's
launches) to an .npy file, for a byte comparison of two library variants:
    GVX_LIB=... python3 tools/preint_dump.py out.npy"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
out = sys.argv[1]
sys.argv = sys.argv[:1]
import numpy as np  # noqa: E402
import preint_loop as pl  # noqa: E402

np.save(out, pl.d_out.cpu().numpy())

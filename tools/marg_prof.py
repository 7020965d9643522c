#!/usr/bin/env python3
"""Kernel-level profile target: the configs[3] window's device marginalisation
(FAST solver) and LM DENSE_SCHUR step, a few calls each (run under
rocprofv3 --kernel-trace --stats)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ic-gvins_amd"))
import torch  # noqa: E402
import gvx  # noqa: E402
from gvx import synth_ba  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.init()
ctx = gvx.Context(0)
ev = synth_ba.DeviceFactorEvaluator(ctx)
p = synth_ba.make_marg_problem(ev)
q = synth_ba.lm_problem(p)
r = p["L"] - p["m"]
d_data = torch.from_numpy(p["data"]).to(dev)
d_J0 = torch.empty(r * r, dtype=torch.float64, device=dev)
d_e0 = torch.empty(r, dtype=torch.float64, device=dev)
d_delta = torch.empty(q["L"], dtype=torch.float64, device=dev)
for _ in range(5):
    ctx.marginalize_dev(p, d_data.data_ptr(), d_J0.data_ptr(), d_e0.data_ptr())
    ctx.schur_solve_dev(q, d_data.data_ptr(), d_delta.data_ptr())
ctx.sync()
ctx.close()
print("ok")

"""Device marginalisation timing (GPU box): the configs[3] window's
MarginalizationInfo problem (synth_ba.make_marg_problem, factors evaluated on the
device), gvx_marginalize_dev device time per kernel family and wall time of the
host entry; one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ic-gvins_amd")]
import torch  # noqa: E402

torch.cuda.init()
import gvx  # noqa: E402
from gvx import synth_ba  # noqa: E402

ctx = gvx.Context(0)
p = synth_ba.make_marg_problem(synth_ba.DeviceFactorEvaluator(ctx))
r = p["L"] - p["m"]
dev = torch.device("cuda")
d_data = torch.from_numpy(p["data"]).to(dev)
J0 = torch.zeros(r * r, dtype=torch.float64, device=dev)
e0 = torch.zeros(r, dtype=torch.float64, device=dev)
torch.cuda.synchronize()
for _ in range(3):
    ctx.marginalize_dev(p, d_data.data_ptr(), J0.data_ptr(), e0.data_ptr())
ctx.sync()
reps = int(os.environ.get("REPS", "10"))
t = time.perf_counter()
for _ in range(reps):
    ctx.marginalize_dev(p, d_data.data_ptr(), J0.data_ptr(), e0.data_ptr())
ctx.sync()
dev_wall = (time.perf_counter() - t) / reps
ctx.profile(True)
ctx.profile_reset()
for _ in range(reps):
    ctx.marginalize_dev(p, d_data.data_ptr(), J0.data_ptr(), e0.data_ptr())
ctx.sync()
ms, n = ctx.profile_read("marg")
ctx.profile(False)
t = time.perf_counter()
for _ in range(reps):
    ctx.marginalize(p)
host_wall = (time.perf_counter() - t) / reps
print(json.dumps(dict(m=p["m"], r=r, factors=len(p["nres"]), dev_call_ms=dev_wall * 1e3,
                      device_ms=ms / max(n, 1), host_call_ms=host_wall * 1e3)))

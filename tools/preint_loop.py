#!/usr/bin/env python3
"""Preintegration launch time (configs[3]'s batch: 5,247 Earth segments x 100
samples) cold and warm: after an idle pause, a bench-like short run (3 untimed, 5
timed launches), then the same after ~0.5 s of back-to-back launches (the shader
clock ramped).  Per launch: wall ms, device ms of the preint family and of
sqrt_info.  Prints one JSON line.  GVX_LIB selects a variant library."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ic-gvins_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gvx  # noqa: E402
from gvx import synth_ba  # noqa: E402

dev = torch.device("cuda", 0)
ctx = gvx.Context(0)
prob = synth_ba.make_ba_problem()
n_kf = prob["poses"].shape[0]
reps = int(os.environ.get("PREINT_REPS", 0)) or -(-(1 << 20) // len(prob["consts"]))  # 583 (5,247 segments)
rng = np.random.default_rng(synth_ba.SEED if hasattr(synth_ba, "SEED") else 20261015)
M = 100
segs = [synth_ba.make_imu_segment(rng, M, t0=0.5 * k) for k in range(n_kf - 1)]
states = np.zeros(n_kf - 1, gvx.STATE_DTYPE)
for k in range(n_kf - 1):
    states[k]["time"] = 0.5 * k
    states[k]["p"] = prob["poses"][k, :3]
    states[k]["q"] = prob["poses"][k, 3:]
    states[k]["v"] = [5.0, 0.0, 0.0]
iewn = np.array([gvx.earth_iewn(np.zeros(3), st["p"]) for st in states])
S = (n_kf - 1) * reps


def dev_t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


d_imu = dev_t(np.concatenate(segs * reps).astype(gvx.IMU_DTYPE).view(np.uint8))
d_seg_off = dev_t(np.arange(S + 1, dtype=np.int32) * M)
d_states = dev_t(np.tile(states, reps).view(np.uint8))
d_iewn = dev_t(np.tile(iewn, (reps, 1)))
d_out = torch.empty(S * gvx.PREINT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
d_pn = torch.empty((S * (M - 1), 4), dtype=torch.float64, device=dev)
torch.cuda.synchronize()


def integ():
    ctx.preint_integrate_dev(2, synth_ba.imu_params(), S, d_imu.data_ptr(), d_seg_off.data_ptr(),
                             d_states.data_ptr(), d_iewn.data_ptr(), d_out.data_ptr(), d_pn.data_ptr())


def timed(warm, k):
    for _ in range(warm):
        integ()
    ctx.sync()
    ctx.profile_reset()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(k):
        integ()
    ctx.sync()
    el = time.perf_counter() - t0
    fam = {f: round(ctx.profile_read(f)[0] / k, 4) for f in ("preint", "sqrt_info")}
    ctx.profile(False)
    return {"wall_ms": round(el / k * 1e3, 4), "steps_per_s": round(S * (M - 1) * k / el, 1), **fam}


integ()
ctx.sync()
time.sleep(0.5)
cold = timed(3, 5)
warm = timed(1000, 200)
time.sleep(0.5)
cold2 = timed(3, 5)
ctx.close()
print(json.dumps({"segments": S, "cold": cold, "warm": warm, "cold_again": cold2}))

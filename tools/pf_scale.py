#!/usr/bin/env python3
"""Device time of preint_factor_kernel against the batch size (the bench's
configs[3] factor records, first n of the 5,247): separates the per-wave latency
(small n, the chip mostly idle) from the whole-batch load / compute / store
phases.  GVX_LIB selects a build.  Timing probe only."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ic-gvins_amd"))
import torch  # noqa: E402
import gvx  # noqa: E402
from gvx import synth_ba  # noqa: E402

ctx = gvx.Context(0)
dev = torch.device("cuda", 0)
prob = synth_ba.make_ba_problem()
n_kf = prob["poses"].shape[0]
reps = 583
rng = np.random.default_rng(20261015)
M = 100
segs = [synth_ba.make_imu_segment(rng, M, t0=0.5 * k) for k in range(n_kf - 1)]
states = np.zeros(n_kf - 1, gvx.STATE_DTYPE)
for k in range(n_kf - 1):
    states[k]["time"] = 0.5 * k
    states[k]["p"] = prob["poses"][k, :3]
    states[k]["q"] = prob["poses"][k, 3:]
    states[k]["v"] = [5.0, 0.0, 0.0]
iewn = np.array([gvx.earth_iewn(np.zeros(3), st["p"]) for st in states])
pre, pn, pn_off = ctx.preint_integrate(2, synth_ba.imu_params(), segs, states, iewn)
mix = np.zeros((n_kf, 9))
mix[:, 0] = 5.0
params = np.concatenate([prob["params"], mix.reshape(-1)])
o_mix = prob["params"].size
poffs = np.array([[7 * k, o_mix + 9 * k, 7 * (k + 1), o_mix + 9 * (k + 1)] for k in range(n_kf - 1)], np.int32)


def dev_t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


n_p = (n_kf - 1) * reps
d_pre = dev_t(np.tile(pre, reps).view(np.uint8))
d_pn = dev_t(pn)
d_pn_off = dev_t(np.tile(pn_off, reps))
d_poffs = dev_t(np.tile(poffs, (reps, 1)))
d_params = dev_t(params)
d_pres = torch.empty((n_p, 15), dtype=torch.float64, device=dev)
d_pjac = torch.empty((n_p, 480), dtype=torch.float64, device=dev)
for n in (4, 64, 256, 1024, 2048, 4096, n_p):
    f = lambda: ctx.preint_factor_eval_dev(n, d_pre.data_ptr(), d_pn.data_ptr(), d_pn_off.data_ptr(),
                                           d_params.data_ptr(), d_poffs.data_ptr(), d_pres.data_ptr(),
                                           d_pjac.data_ptr())
    for _ in range(10):
        f()
    ctx.sync()
    ctx.profile_reset()
    ctx.profile(True)
    for _ in range(50):
        f()
    ctx.sync()
    ms, cnt = ctx.profile_read("preint_factor")
    ctx.profile(False)
    us = ms / 50 * 1e3
    row = {"lib": os.environ.get("GVX_LIB", "tree"), "n": n, "us": round(us, 2),
           "frac": round(10944 * n / (us * 1e-6) / 8e12, 4)}
    if os.environ.get("GVX_LIB", "").endswith("pfprof.so"):
        import ctypes
        t = np.zeros(16, np.uint64)
        ctypes.CDLL(os.environ["GVX_LIB"]).gvx_dbg_pf_times(t.ctypes.data_as(ctypes.c_void_p))
        t = t.astype(np.int64)
        row["wave0_phase_us"] = dict(zip(["issue", "wait_loads", "pn_sum", "residual+rawjac_part1", "rawjac_part2",
                                          "whiten+store_issue", "store_drain"], np.round(np.diff(t[:8]) * 0.01, 2).tolist()))
    print(json.dumps(row))
# the bench's order: the 1,049,400-factor reprojection launch before each
# preintegration-factor launch (its 550 MB evicts the factor records from the
# L2 / MALL), timed on the same HIP events as the bench line
n_rp = len(prob["consts"])
n_r = n_rp * reps
d_consts = dev_t(np.tile(prob["consts"], reps).view(np.uint8))
d_offs = dev_t(np.tile(prob["offs"], (reps, 1)))
d_res = torch.empty((n_r, 2), dtype=torch.float64, device=dev)
d_jac = torch.empty((n_r, 46), dtype=torch.float64, device=dev)
f = lambda: ctx.factor_batch_eval_dev(n_r, d_consts.data_ptr(), d_offs.data_ptr(), d_res.data_ptr(), d_jac.data_ptr(),
                                      n_p, d_pre.data_ptr(), d_pn.data_ptr(), d_pn_off.data_ptr(), d_poffs.data_ptr(),
                                      d_pres.data_ptr(), d_pjac.data_ptr(), d_params.data_ptr())
for _ in range(10):
    f()
ctx.sync()
ctx.profile_reset()
ctx.profile(True)
for _ in range(50):
    f()
ctx.sync()
us = ctx.profile_read("preint_factor")[0] / 50 * 1e3
rus = ctx.profile_read("reproj")[0] / 50 * 1e3
ctx.profile(False)
print(json.dumps({"lib": os.environ.get("GVX_LIB", "tree"), "n": n_p, "after_reproj": True, "us": round(us, 2),
                  "frac": round(10944 * n_p / (us * 1e-6) / 8e12, 4), "reproj_us": round(rus, 2)}))
ctx.close()

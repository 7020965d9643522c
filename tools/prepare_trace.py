#!/usr/bin/env python3
"""gvx_factors_prepare at the reference's own problem size (one configs[3]
window: 1,800 reprojection + 9 Earth preintegration factors, M = 100), the way
a Ceres EvaluationCallback calls it once per LM iteration: K prepares back to
back.  Prints one JSON line: wall us per prepare.  Run it under
`rocprofv3 --kernel-trace --memory-copy-trace` for the breakdown (copies,
kernels, gaps; tools/prepare_breakdown.py)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ic-gvins_amd")]
import numpy as np  # noqa: E402
import gvx  # noqa: E402
from gvx import synth_ba  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ctx = gvx.Context(0)
prob = synth_ba.make_ba_problem()
n_kf = prob["poses"].shape[0]
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
starts = sorted({int(v) for v in prob["offs"].ravel()} | {int(v) for v in poffs.ravel()})
sizes = {}
for o, sz in zip(prob["offs"].T, (7, 7, 7, 1, 1)):
    sizes.update({int(v): sz for v in o})
for o, sz in zip(poffs.T, (7, 9, 7, 9)):
    sizes.update({int(v): sz for v in o})
bidx = {st: i for i, st in enumerate(starts)}
blocks = [params[st:st + sizes[st]] for st in starts]
fset = gvx.FactorSet(ctx, blocks, prob["consts"].astype(gvx.REPROJ_DTYPE),
                     np.vectorize(bidx.get)(prob["offs"]).astype(np.int32), pre, pn, pn_off,
                     np.vectorize(bidx.get)(poffs).astype(np.int32))
for _ in range(50):
    fset.prepare(True)
t0 = time.perf_counter()
for _ in range(K):
    fset.prepare(True)
el = (time.perf_counter() - t0) / K
fset.close()
ctx.close()
print(json.dumps({"factors": len(prob["consts"]) + n_kf - 1, "prepares": K, "us_per_prepare": round(el * 1e6, 2)}))

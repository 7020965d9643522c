"""Device findFundamentalMat(FM_RANSAC) timing (GPU box): one 150-point set per
launch (the live tracker's reference points) and batches of sets; one JSON line."""
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
from gvx import synth  # noqa: E402

ctx = gvx.Context(0)
dev = torch.device("cuda")
out = {}
for n_sets in (1, 64, 1024):
    sets = [synth.two_view_scene(150, outlier_frac=0.2, noise_px=0.3, seed=k)[:2] for k in range(min(n_sets, 64))]
    sets = (sets * (n_sets // len(sets) + 1))[:n_sets]
    off = np.zeros(n_sets + 1, np.int32)
    off[1:] = np.cumsum([len(a) for a, _ in sets])
    d_off = torch.from_numpy(off).to(dev)
    d_p1 = torch.from_numpy(np.concatenate([a for a, _ in sets])).to(dev)
    d_p2 = torch.from_numpy(np.concatenate([b for _, b in sets])).to(dev)
    d_mask = torch.empty(int(off[-1]), dtype=torch.uint8, device=dev)
    d_F = torch.empty(n_sets * 9, dtype=torch.float64, device=dev)
    d_res = torch.empty(n_sets, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def run():
        ctx.find_fundamental_ransac_dev(n_sets, d_off.data_ptr(), d_p1.data_ptr(), d_p2.data_ptr(), d_mask.data_ptr(),
                                        d_F.data_ptr(), d_res.data_ptr())

    for _ in range(3):
        run()
    ctx.sync()
    reps = 20
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    ctx.sync()
    wall = (time.perf_counter() - t0) / reps
    ms, k = ctx.profile_read("fmat")
    ctx.profile(False)
    out[n_sets] = {"device_ms": round(ms / k, 4), "wall_ms": round(wall * 1e3, 4),
                   "sets_per_s": round(n_sets / (ms / k * 1e-3))}
print(json.dumps({"fmat_150pts": out}))

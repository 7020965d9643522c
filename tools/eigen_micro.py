"""gvx_sym_eigen device time per n (GPU box), for the marginalisation row."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ic-gvins_amd")]
import gvx  # noqa: E402

ctx = gvx.Context(0)
out = {}
for n in [int(x) for x in os.environ.get("NS", "64,142,215,512").split(",")]:
    rng = np.random.default_rng(n)
    A = rng.normal(size=(n, n))
    A = A @ A.T
    D = np.diag(10 ** rng.uniform(-3, 4, n))
    A = D @ A @ D
    ctx.sym_eigen(A)
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(3):
        ctx.sym_eigen(A)
    ms, k = ctx.profile_read("eigen")
    ctx.profile(False)
    out[n] = round(ms / k, 4)
print(json.dumps({"eigen_device_ms": out}))

#!/usr/bin/env python3
"""Device time of gvx_clahe_batch_dev over the bench's 256 1280x560 frames
(context profile events), for A/B runs of libgvx variants (GVX_LIB).
--inplace: source = destination, which takes the two-kernel form."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ic-gvins_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gvx  # noqa: E402
from gvx import synth  # noqa: E402

n, w, h = 256, 1280, 560
rng = np.random.default_rng(5)
imgs = np.stack([synth.make_image(w, h, rng) for _ in range(16)])
src = torch.from_numpy(np.tile(imgs, (n // 16, 1, 1))).cuda()
inplace = "--inplace" in sys.argv
dst = src if inplace else torch.empty_like(src)
ctx = gvx.Context(0)
for _ in range(5):
    ctx.clahe_batch_dev(n, w, h, src.data_ptr(), dst.data_ptr())
ctx.sync()
ctx.profile_reset()
ctx.profile(True)
reps = 20
for _ in range(reps):
    ctx.clahe_batch_dev(n, w, h, src.data_ptr(), dst.data_ptr())
ctx.sync()
ms, _ = ctx.profile_read("clahe")
ctx.profile(False)
print(json.dumps({"lib": os.environ.get("GVX_LIB", "base"), "inplace": inplace, "ms_per_call": ms / reps,
                  "frac": 2.0 * w * h * n / (ms / reps * 1e-3) / 8e12}))
ctx.close()

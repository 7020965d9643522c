"""CLAHE kernel micro-benchmark (run on the GPU box, optionally under rocprofv3):
gvx_clahe_batch_dev over 512 images of 1280x560 for three contents -- the
bench's synthetic frames, uniform noise (few LDS histogram conflicts) and a
constant image (every histogram add hits one bin) -- printing device ms per
512-image batch per content.  Usage: python3 tools/clahe_micro.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ic-gvins_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gvx  # noqa: E402
from gvx import synth  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W, H, N = 1280, 560, 512
torch.cuda.init()
ctx = gvx.Context(0)
I, J, _, _ = synth.make_batch(N // 2, W, H, 150, seed=synth.SEED, distinct=8)
contents = {
    "synthetic": np.concatenate([I, J]),
    "noise": np.random.default_rng(1).integers(0, 256, (N, H, W), dtype=np.uint8),
    "constant": np.full((N, H, W), 117, np.uint8),
}
for name, imgs in contents.items():
    src = torch.from_numpy(imgs).cuda()
    dst = torch.empty_like(src)
    for _ in range(3):
        ctx.clahe_batch_dev(N, W, H, src.data_ptr(), dst.data_ptr())
    ctx.sync()
    ctx.profile_reset()
    ctx.profile(True)
    for _ in range(iters):
        ctx.clahe_batch_dev(N, W, H, src.data_ptr(), dst.data_ptr())
    ctx.sync()
    ms, n = ctx.profile_read("clahe")
    ctx.profile(False)
    print(f"{name:10s} {ms / n:.4f} ms per {N} images ({2.0 * W * H * N / (ms / n * 1e-3) / 1e9:.0f} GB/s algorithmic)",
          flush=True)
# single frames (the live tracker / sequence replay), 1280x560, synthetic content
src1 = torch.from_numpy(np.ascontiguousarray(I[0])).cuda()
dst1 = torch.empty_like(src1)
for _ in range(20):
    ctx.clahe_batch_dev(1, W, H, src1.data_ptr(), dst1.data_ptr())
ctx.sync()
ctx.profile_reset()
ctx.profile(True)
for _ in range(200):
    ctx.clahe_batch_dev(1, W, H, src1.data_ptr(), dst1.data_ptr())
ctx.sync()
ms, n = ctx.profile_read("clahe")
ctx.profile(False)
print(f"single     {1e3 * ms / n:.2f} us per frame ",
      flush=True)
ctx.close()

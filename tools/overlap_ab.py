#!/usr/bin/env python3
"""Does the next batch's pyramid pass overlap the current batch's LK?  Wall time per
configs[1] step (256 pairs) for: the step alone; the step followed by a second
512-image pyramid pass (sequential); the step with that pyramid pass on a side
branch beside it.  Interleaved rounds on one box; prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ic-gvins_amd")]
import torch  # noqa: E402
import gvx  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
W, H, L = 1280, 560, 3
wl = bench.KltWorkload(256, W, H, 150, dev)
ctx = gvx.Context(0)
p = gvx.KltParams.default(max_level=L)
lay = gvx.pyramid_layout(W, H, L)
imgs = torch.cat([wl.I, wl.J]).contiguous()
out = torch.empty(imgs.shape[0] * lay["bytes"], dtype=torch.uint8, device=dev)
K = 40


def pyr():
    ctx.build_pyramids_dev(imgs.shape[0], W, H, imgs.data_ptr(), W * H, W, L, out.data_ptr())


def alone():
    for _ in range(K):
        wl.step(ctx, p)


def seq():
    for _ in range(K):
        wl.step(ctx, p)
        pyr()


def overlap():
    for _ in range(K):
        ctx.branch_begin()
        pyr()
        ctx.branch_end()
        wl.step(ctx, p)
        ctx.branch_join()


def pyr_only():
    for _ in range(K):
        pyr()


for _ in range(30):
    wl.step(ctx, p)
    pyr()
ctx.sync()
res = {}
for _ in range(3):
    for name, fn in (("alone", alone), ("pyr_only", pyr_only), ("seq", seq), ("overlap", overlap)):
        fn()
        ctx.sync()
        t0 = time.perf_counter()
        fn()
        ctx.sync()
        res.setdefault(name, []).append(round((time.perf_counter() - t0) / K * 1e3, 4))
ctx.close()
print(json.dumps(res))

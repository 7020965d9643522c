"""LK cost model on the bench workload: device time of the LK launch as the
iteration cap varies (max_iter = 0 times the per-level window extraction and
solve set-up alone), the marginal cost of an iteration, and the pyramid time.
Diagnostics only (the results are not the tracker's)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ic-gvins_amd"))

import torch  # noqa: E402
import gvx  # noqa: E402
from gvx import synth  # noqa: E402

W, H, N, L, Pn = 1280, 560, 150, 3, 256
I, J, P, Q = synth.make_batch(Pn, W, H, N, distinct=16)
dev = torch.device("cuda", 0)
dI, dJ = torch.from_numpy(I).to(dev), torch.from_numpy(J).to(dev)
dP, dQ = torch.from_numpy(P).to(dev), torch.from_numpy(Q).to(dev)
dN, dB = torch.empty_like(dQ), torch.empty_like(dQ)
dF = torch.empty((Pn, N), dtype=torch.uint8, device=dev)
dK = torch.empty((Pn, N), dtype=torch.int32, device=dev)
dNK = torch.empty((Pn,), dtype=torch.int32, device=dev)
ctx = gvx.Context(0)
stream = torch.cuda.ExternalStream(ctx.stream(), device=dev)


def run(max_iter, reps=10):
    prm = gvx.KltParams.default(max_level=L, max_iter=max_iter)
    for k in range(reps + 2):
        if k == 2:
            ctx.sync()
            ctx.profile_reset()
            ctx.profile(True)
        with torch.cuda.stream(stream):
            dN.copy_(dQ)
        ctx.klt_fb_batch_dev(Pn, W, H, dI.data_ptr(), dJ.data_ptr(), N, dP.data_ptr(), dN.data_ptr(),
                             dB.data_ptr(), dF.data_ptr(), dK.data_ptr(), dNK.data_ptr(), params=prm)
    ctx.sync()
    out = {f: ctx.profile_read(f)[0] / reps for f in ("pyramid", "klt")}
    ctx.profile(False)
    return out


base = None
for it in (0, 1, 2, 4, 8, 30):
    r = run(it)
    base = base or r["klt"]
    print(f"max_iter {it:2d}: klt {r['klt']:.4f} ms  (+{r['klt'] - base:.4f})  pyramid {r['pyramid']:.4f} ms",
          flush=True)

if len(sys.argv) > 1 and sys.argv[1] == "--reps":
    for reps in (5, 10, 20, 40, 80):
        r = run(30, reps)
        print(f"reps {reps:3d}: klt {r['klt']:.4f} ms  pyramid {r['pyramid']:.4f} ms", flush=True)

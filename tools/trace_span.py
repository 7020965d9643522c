"""The headline's timed region in a rocprofv3 --kernel-trace of the driver's
command (bench.py --steps K --warmup W, default line): the batch launches of
stream_kernel (pyramid pass; since r06 followed by side_kernel / ring_kernel,
the side bands), klt_kernel<3, 0> (LK) and compact_kernel in order, the timed K steps being the K after the LK side leg (28 exact-order
steps), the settle leg (bench.SETTLE_STEPS) and the W warm-up steps.

Prints per step: the span from the first timed pyramid pass's start to the last
timed compaction's end, and each kernel's own duration (mean over the K steps),
to set beside the bench line's device_span_ms_per_step / device_ms_per_step.
    python3 tools/trace_span.py <kernel_trace.csv> [K] [W]"""
import csv
import gzip
import json
import sys

ACCUM_EXACT_STEPS = 20 + 3 + 5  # accum_leg at --steps 20: 20 warm steps, then 3 + steps // 4 per order
SETTLE = 40
path = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
W = int(sys.argv[3]) if len(sys.argv) > 3 else 5
acc = {"stream_kernel": [], "side_kernel": [], "ring_kernel": [], "klt_kernel<3, 0>": [], "compact_kernel": []}
rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
for r in rows:
    for k in acc:
        if k in r["Kernel_Name"]:
            acc[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"])))
batch = {}
for k, v in acc.items():
    if not v:
        batch[k] = []
        continue
    g = max(x[2] for x in v)  # the batch launch: the largest grid
    batch[k] = sorted(x for x in v if x[2] == g)
lk = batch["klt_kernel<3, 0>"]
# LK launches in order: accum leg's exact order, settle, warm-up, timed, then the host-buffer leg
t0i = ACCUM_EXACT_STEPS + SETTLE + W
timed_lk = lk[t0i:t0i + K]
lo, hi = timed_lk[0][0], timed_lk[-1][1]
# the timed pyramid passes: those that end before the last timed LK and start
# after the warm-up's last LK began
w_last = lk[t0i - 1][0]
pyr = [x for x in batch["stream_kernel"] if x[0] > w_last and x[1] <= hi]
pyr = pyr[-K:]
ring = [x for x in batch["ring_kernel"] if x[0] > w_last and x[1] <= hi][-K:] + \
    [x for x in batch["side_kernel"] if x[0] > w_last and x[1] <= hi][-K:]
cmp_ = [x for x in batch["compact_kernel"] if x[0] >= timed_lk[0][0]][:K]
start = min(pyr[0][0], lo)
end = max(hi, cmp_[-1][1])
out = {
    "steps": K,
    "span_ms_per_step": round((end - start) / K / 1e6, 4),
    "kernel_ms_mean": {"pyramid": round(sum(b - a for a, b, _ in pyr + ring) / K / 1e6, 4),
                       "klt": round(sum(b - a for a, b, _ in timed_lk) / K / 1e6, 4),
                       "compact": round(sum(b - a for a, b, _ in cmp_) / K / 1e6, 4)},
    "batch_launches_in_trace": {k: len(v) for k, v in batch.items()},
}
print(json.dumps(out))

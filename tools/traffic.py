"""HBM traffic per bench step from rocprofv3 PMC passes (tools/pmc.sh with a
"FETCH_SIZE" pass and a "WRITE_SIZE" pass over `bench.py`), corrected as
MI355X_MICROARCH.md "HBM" prescribes: bytes = 2 * FETCH_SIZE + WRITE_SIZE
(FETCH_SIZE reads half on gfx950; both counters in KiB).

Writes profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.
Usage: python3 tools/traffic.py gpurun_out/<tag> [--workload KEY]"""
import argparse
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(__file__))
from pmc_summary import load  # noqa: E402

# launches per bench step of the KLT pipeline: one 3-level streaming pass over
# the prev and next images together (levels and rings; before r02 an edge-band
# pass and a ring pass ran beside it, which are counted when present); one LK
# launch for fwd+bwd; one compaction.
PER_STEP = {"stream_kernel": 1, "klt_kernel": 1, "compact_kernel": 1}
OPTIONAL = {"edge_kernel": 1, "ring_kernel": 1, "side_kernel": 1}  # r06: the side bands of large launches
ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("--workload", default="klt_fb_batch 256x1280x560 N150 L3")
ap.add_argument("--pairs", type=int, default=256)
ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json"))
a = ap.parse_args()
# the batch launch of each kernel: the largest grid (a full default line also
# launches them per frame and per pair)
res = {}
for key, d in load(a.pmc_dir, by_grid=True).items():
    name, grid = key.rsplit("@", 1)
    if name not in res or int(grid) > res[name][0]:
        res[name] = (int(grid), d)
res = {k: v[1] for k, v in res.items()}
kern = {}
step = 0.0
for name, n in list(PER_STEP.items()) + [(k, v) for k, v in OPTIONAL.items() if k in res]:
    d = res.get(name)
    if d is None or "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
        sys.exit(f"{name}: FETCH_SIZE / WRITE_SIZE missing in {a.pmc_dir}")
    b = (2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
    kern[name] = {"bytes_per_launch": b, "fetch_kib": d["FETCH_SIZE"], "write_kib": d["WRITE_SIZE"],
                  "launches_per_step": n}
    step += n * b
# the measured code's commit: GVX_COMMIT (the GPU box has no .git), else git HEAD
commit = os.environ.get("GVX_COMMIT", "")
if not commit:
    try:
        commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                                cwd=os.path.dirname(os.path.abspath(__file__))).stdout.strip()
    except OSError:
        commit = ""
out = {"workload": a.workload, "pairs_per_step": a.pairs, "bytes_per_step": step, "commit": commit,
       "bytes_per_pair": step / a.pairs, "kernels": kern, "source": os.path.relpath(a.pmc_dir),
       "correction": "2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md HBM"}
json.dump(out, open(a.out, "w"), indent=1)
print(json.dumps(out, indent=1))

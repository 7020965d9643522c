"""LK's VALU-issue fraction from one rocprofv3 --pmc pass:
SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES and SQ_WAVES with
GRBM_GUI_ACTIVE (the real clock) and --kernel-trace durations, over the bench's
configs[1] launch (tools/lk_pmc.py).

Corrections (MI355X_MICROARCH.md): SQ_*_CYCLES / SQ_ACTIVE_INST_* count
quad-cycles (x4); GRBM_GUI_ACTIVE is summed over the 8 XCDs (/8).  A wave64 VALU
instruction occupies its SIMD for 4 cycles, so
    valu_busy      = 4 * SQ_ACTIVE_INST_VALU / (SIMDs * GRBM_GUI_ACTIVE / 8)
    resident_waves = 4 * SQ_WAVE_CYCLES      / (SIMDs * GRBM_GUI_ACTIVE / 8)
    clock_ghz      = GRBM_GUI_ACTIVE / 8 / kernel duration.
Counters from several passes are averaged per dispatch (pmc_summary.load).
Writes profiles/pmc_issue.json, which bench.py reports as roofline.klt_issue.
Usage: python3 tools/issue.py gpurun_out/<tag>/lkpmc [--kernel klt_kernel]"""
import argparse
import csv
import glob
import gzip
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(__file__))
from pmc_summary import load  # noqa: E402

SIMDS = 1024  # 256 CUs x 4
ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("--kernel", default="klt_kernel")
ap.add_argument("--workload", default="klt_fb_batch 256x1280x560 N150 L3")
ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_issue.json"))
a = ap.parse_args()
res = load(a.pmc_dir)
d = res.get(a.kernel)
need = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE")
if d is None or any(k not in d for k in need):
    sys.exit(f"{a.kernel}: need {need} in {a.pmc_dir}")
durs = []
for f in glob.glob(f"{a.pmc_dir}/**/*kernel_trace.csv*", recursive=True):
    for r in csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)):
        if a.kernel in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
cyc = d["GRBM_GUI_ACTIVE"] / 8.0
out = {
    "workload": a.workload, "kernel": a.kernel,
    "valu_busy": round(4 * d["SQ_ACTIVE_INST_VALU"] / (SIMDS * cyc), 4),
    "valu_insts_per_wave": round(d["SQ_INSTS_VALU"] / d["SQ_WAVES"], 1),
    "resident_waves_per_simd": round(4 * d["SQ_WAVE_CYCLES"] / (SIMDS * cyc), 3),
    "max_waves_per_simd": 4,
    "waves": d["SQ_WAVES"],
    "clock_ghz": round(cyc / (sum(durs) / len(durs)) / 1e9, 3) if durs else None,
    "kernel_us_under_pmc": round(sum(durs) / len(durs) * 1e6, 1) if durs else None,
    "source": os.path.relpath(a.pmc_dir),
    "commit": os.environ.get("GVX_COMMIT") or subprocess.run(
        ["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
        cwd=os.path.dirname(os.path.abspath(__file__))).stdout.strip(),
    "counters": {k: d[k] for k in sorted(d)},
}
json.dump(out, open(a.out, "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "counters"}, indent=1))

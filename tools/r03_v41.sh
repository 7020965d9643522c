#!/bin/bash
# PMC at HEAD (LK batched J-row loads): FETCH_SIZE and WRITE_SIZE passes (HBM traffic per step,
# tools/traffic.py) and one SQ pass (VALU per wave) over the configs[1] batch
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=r03_v41
bash $R/tools/pmc.sh $T "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
cd $R
python3 tools/pmc_summary.py gpurun_out/$T > gpurun_out/$T/pmc_summary.txt 2>&1 || true
grep -A12 -E "^(klt_kernel|stream_kernel|compact_kernel)" gpurun_out/$T/pmc_summary.txt || true
python3 tools/traffic.py gpurun_out/$T --out gpurun_out/$T/pmc_traffic.json
cat gpurun_out/$T/pmc_traffic.json

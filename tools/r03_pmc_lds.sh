#!/bin/bash
# PMC passes over a short default bench run (CLAHE + LK + factors): issue / wait
# cycles and LDS conflict counters per kernel.  Usage: bash tools/r03_pmc_lds.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --steps 20 > $O/bench.json 2> $O/bench.err
PMC_BENCH_ARGS="--steps 3 --warmup 1 --no-cpu" bash tools/pmc.sh $T \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
python3 tools/pmc_summary.py $O > $O/pmc_summary.txt 2>&1 || true
grep -A9 -E "^(fused_kernel|lut_kernel|apply_kernel|preint_factor_kernel)" $O/pmc_summary.txt || true

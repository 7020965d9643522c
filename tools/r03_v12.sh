#!/bin/bash
# CLAHE fused (branch-free loads) parity + timing; sequence replay kernel trace;
# preint factor PMC (configs[3] bench).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_clahe_fused_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python tools/clahe_ab.py | tee -a $O/clahe_ab.txt
bash tools/r03_seq_prof.sh $T
PMC_BENCH_ARGS="--config 4 --steps 3 --warmup 1 --no-cpu" bash tools/pmc.sh $T \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" \
  "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"

#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 pass, no
# tracing domains combined with --pmc).  Usage: tools/pmc_klt.sh <outdir-tag>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-pmc}
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/$T/p$i \
     -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/$T/p$i.log 2>&1
done

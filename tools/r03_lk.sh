#!/bin/bash
# LK no-spill check: LK / sequence parity, interleaved A/B against the r02
# kernel (variant "old"), and the FETCH_SIZE / WRITE_SIZE passes of the batch.
# Usage (through gpurun): bash tools/r03_lk.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_klt_gpu.py tests/test_klt_accum_gpu.py tests/test_sequence_gpu.py \
  -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
bash tools/ab.sh $T 3 old base
bash tools/pmc.sh $T FETCH_SIZE WRITE_SIZE
python3 tools/pmc_summary.py $O > $O/pmc_summary.txt 2>&1 || true
cat $O/pmc_summary.txt | head -40

#!/bin/bash
# Live-path detection restructure (select per block + merge, eig on the branch):
# tracking / detection / graph parity, configs[4] timing; factor + CLAHE timing.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_sequence_gpu.py tests/test_graph_gpu.py tests/test_detect_gpu.py \
  tests/test_factor_parity_gpu.py tests/test_ba_gpu.py tests/test_clahe_fused_gpu.py -x -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --config 5 --no-cpu > $O/bench_config5.json 2> $O/bench_config5.err
head -c 300 $O/bench_config5.json; echo
timeout -k 10 300 python -u bench.py --config 4 --no-cpu > $O/bench_config4.json 2> $O/bench_config4.err
grep -o '"preint_factor_roofline": {[^}]*}' $O/bench_config4.json
for r in 1 2; do timeout -k 10 120 python tools/clahe_ab.py | tee -a $O/clahe_ab.txt; done

#!/bin/bash
# Tracking-path detection (early-exit eig tiles, per-block select, merge) parity
# and configs[4] A/B: eig in the tracking graph vs on the preprocessing branch.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_sequence_gpu.py tests/test_eig_precompute_gpu.py tests/test_detect_gpu.py \
  tests/test_graph_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config 5 --no-cpu > $O/c5_base_$r.json 2> $O/c5_base_$r.err
  timeout -k 10 300 python -u bench.py --config 5 --no-cpu --eig-branch > $O/c5_eigb_$r.json 2> $O/c5_eigb_$r.err
  timeout -k 10 300 python -u bench.py --config 5 --no-cpu --no-pipeline > $O/c5_nopipe_$r.json 2> $O/c5_nopipe_$r.err
done
for f in $O/c5_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['device_ms_per_frame'])"; done
for r in 1 2; do timeout -k 10 120 python tools/clahe_ab.py --inplace | tee -a $O/clahe_ab.txt; timeout -k 10 120 python tools/clahe_ab.py | tee -a $O/clahe_ab.txt; done

#!/bin/bash
# Staged preint factor kernel: parity + configs[3] bench; CLAHE knockout A/B.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_factor_parity_gpu.py tests/test_ba_gpu.py -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --config 4 --no-cpu > $O/bench_config4.json 2> $O/bench_config4.err
grep -o '"preint_factor_roofline": {[^}]*}' $O/bench_config4.json
grep -o '"device_ms_per_step": {[^}]*}' $O/bench_config4.json
for r in 1 2; do
  for v in base koapply kogather kohist kolut; do
    if [ $v = base ]; then L=""; else L=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
    GVX_LIB=$L timeout -k 10 120 python tools/clahe_ab.py | tee -a $O/clahe_ab.txt
  done
done

#!/bin/bash
# CLAHE fused-kernel variants A/B (base / integer divisions through rcp / + packed blend) and parity
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v21
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_clahe_fused_gpu.py tests/test_clahe_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/clahe_tests.log 2>&1 || { tail -30 $O/clahe_tests.log; exit 1; }
tail -2 $O/clahe_tests.log
V=$R/ic-gvins_amd/gvx/variants
for r in 1 2 3; do
  GVX_LIB=$V/libgvx_clahebase.so timeout -k 10 120 python tools/clahe_ab.py | tee -a $O/clahe_ab.txt
  GVX_LIB=$V/libgvx_clahediv.so timeout -k 10 120 python tools/clahe_ab.py | tee -a $O/clahe_ab.txt
  timeout -k 10 120 python tools/clahe_ab.py | tee -a $O/clahe_ab.txt
done
timeout -k 10 200 python -u bench.py --config 5 --no-cpu > $O/c5.json 2> $O/c5.err
python3 -c "import json;d=json.load(open('$O/c5.json'));print('c5', d['value'], d['ms_per_step'], d['config']['frame_batch'])"

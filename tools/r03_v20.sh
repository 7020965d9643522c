#!/bin/bash
# K-frame batched sequence replay: parity (sequence + graph tests) and configs[4] A/B over K.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v20
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_sequence_gpu.py tests/test_graph_gpu.py -x -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for k in 1 4 8 16; do
    timeout -k 10 200 python -u bench.py --config 5 --no-cpu --frame-batch $k > $O/c5_k${k}_$r.json 2> $O/c5_k${k}_$r.err
    python3 -c "import json;d=json.load(open('$O/c5_k${k}_$r.json'));print('K=$k', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_frame'])"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_clahe_fused_gpu.py tests/test_clahe_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/clahe_tests.log 2>&1 || { tail -30 $O/clahe_tests.log; exit 1; }
tail -2 $O/clahe_tests.log
for r in 1 2 3; do
  GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_clahebase.so timeout -k 10 120 python tools/clahe_ab.py | tee -a $O/clahe_ab.txt
  timeout -k 10 120 python tools/clahe_ab.py | tee -a $O/clahe_ab.txt
done

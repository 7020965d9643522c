#!/bin/bash
# cornerSubPix: hoisted patch terms + pipelined sums; parity + phase stamps + configs[4]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v24
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_detect_gpu.py tests/test_sequence_gpu.py tests/test_eig_precompute_gpu.py -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_selprof.so timeout -k 10 200 python -u tools/select_prof.py > $O/select_prof.txt 2> $O/select_prof.err || { tail -20 $O/select_prof.err; exit 1; }
cut -c1-900 $O/select_prof.txt | head -6
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config 5 --no-cpu > $O/c5_$r.json 2> $O/c5_$r.err
  python3 -c "import json;d=json.load(open('$O/c5_$r.json'));print('c5', d['value'], d['ms_per_step'], d['roofline']['device_ms_per_frame'])"
done

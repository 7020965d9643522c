#!/bin/bash
# selection-kernel phase timestamps on detection frames (variant build), detection parity
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v22
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_detect_gpu.py tests/test_sequence_gpu.py tests/test_eig_precompute_gpu.py -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_selprof.so timeout -k 10 200 python -u tools/select_prof.py > $O/select_prof.txt 2> $O/select_prof.err || { tail -20 $O/select_prof.err; exit 1; }
cut -c1-900 $O/select_prof.txt | head -8
timeout -k 10 200 python -u bench.py --config 5 --no-cpu > $O/c5.json 2> $O/c5.err
python3 -c "import json;d=json.load(open('$O/c5.json'));print('c5', d['value'], d['ms_per_step'])"

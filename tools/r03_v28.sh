#!/bin/bash
# preint factor: stores from the MFMA accumulators; parity + phases + scaling
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v28
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_factor_parity_gpu.py tests/test_ba_gpu.py tests/test_factorset_gpu.py -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_pfprof.so timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_phase.txt 2> $O/pf_phase.err || { tail -20 $O/pf_phase.err; exit 1; }
cat $O/pf_phase.txt
timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_scale.txt 2> $O/pf_scale.err
cat $O/pf_scale.txt
timeout -k 10 300 python -u bench.py --config 4 --no-cpu > $O/c4.json 2> $O/c4.err
python3 -c "import json;d=json.load(open('$O/c4.json'));print('c4', d['value'], d['preint_factor_roofline'], d['roofline']['device_ms_per_step'])"

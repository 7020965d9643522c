#!/bin/bash
# tree = nt stores in reproj / preint factor / small factors; ntld = + streaming loads of the reproj constants
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v33
mkdir -p $O
cd $R
for r in 1 2; do
for v in tree ldsc; do
  L=""; [ $v != tree ] && L=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so
  GVX_LIB=$L timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_${v}_$r.txt 2> $O/pf_$v.err || { tail -20 $O/pf_$v.err; exit 1; }
  tail -2 $O/pf_${v}_$r.txt
done
done
timeout -k 10 300 python -u -m pytest tests/test_factor_parity_gpu.py tests/test_ba_gpu.py tests/test_factorset_gpu.py tests/test_aux_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --config 4 --no-cpu > $O/c4.json 2> $O/c4.err
python3 -c "import json;d=json.load(open('$O/c4.json'));print('c4', d['value'], d['roofline']['frac'], d['preint_factor_roofline']['frac'], d['window_factors']['gnss_roofline'])"

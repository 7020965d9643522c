#!/bin/bash
# preint factor on two waves per workgroup (w2) vs base: factor parity on the variant, pf_scale both
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=r03_v43
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_w2.so timeout -k 10 300 python -u -m pytest tests/test_factor_parity_gpu.py tests/test_ba_gpu.py tests/test_factorset_gpu.py tests/test_profile_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
for v in base w2; do
  GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_${v}_$r.txt 2> $O/pf_$v.err || { tail -20 $O/pf_$v.err; exit 1; }
  head -1 $O/pf_${v}_$r.txt | cut -c60-; tail -2 $O/pf_${v}_$r.txt | cut -c60-
done
done

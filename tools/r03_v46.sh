#!/bin/bash
# pyramid: prefetch 6 row pairs at 3 waves/SIMD (pf63) vs base; pyramid parity on the variant, batch A/B
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=r03_v46
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_pf63.so timeout -k 10 300 python -u -m pytest tests/test_pyramid_gpu.py tests/test_klt_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab.sh $T 3 base_p pf63 | tee $O/ab.txt

#!/bin/bash
# CLAHE: 480-thread workgroups with an 8-byte {ty1, ty2} table (80 KB of LDS: two images
# per CU, c2wg) vs base; CLAHE parity on the variant, A/B of the batch
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=r03_v47
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_c2wg.so timeout -k 10 300 python -u -m pytest tests/test_clahe_gpu.py tests/test_clahe_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for v in base_c c2wg; do
    GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 120 python -u tools/clahe_ab.py >> $O/ab.txt 2>> $O/ab.err
  done
done
cat $O/ab.txt

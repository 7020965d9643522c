#!/bin/bash
# preint factor: closed-form record row index (sqr) vs base; pf tests on the tree
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v34
mkdir -p $O
cd $R
for r in 1 2 3; do
for v in base sqr; do
  L=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so
  GVX_LIB=$L timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_${v}_$r.txt 2> $O/pf_$v.err || { tail -20 $O/pf_$v.err; exit 1; }
  head -1 $O/pf_${v}_$r.txt; tail -2 $O/pf_${v}_$r.txt
done
done

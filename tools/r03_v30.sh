#!/bin/bash
# preint factor: lanes per factor (16 tree / 8 / 32), warm and in the bench's order
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v30
mkdir -p $O
cd $R
for v in tree pfl8 pfl32; do
  L=""; [ $v != tree ] && L=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so
  GVX_LIB=$L timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_$v.txt 2> $O/pf_$v.err || { tail -20 $O/pf_$v.err; exit 1; }
  cat $O/pf_$v.txt
done

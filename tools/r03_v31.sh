#!/bin/bash
# nontemporal stores: reproj outputs (rpnt), + preint factor outputs (rpntpfnt); two rounds
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v31
mkdir -p $O
cd $R
for r in 1 2; do
for v in tree rpnt rpntpfnt; do
  L=""; [ $v != tree ] && L=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so
  GVX_LIB=$L timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_${v}_$r.txt 2> $O/pf_$v.err || { tail -20 $O/pf_$v.err; exit 1; }
  tail -2 $O/pf_${v}_$r.txt
done
done

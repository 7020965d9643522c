#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v27
mkdir -p $O
cd $R
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_pfprof.so timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_phase.txt 2> $O/pf_phase.err || { tail -20 $O/pf_phase.err; exit 1; }
cat $O/pf_phase.txt

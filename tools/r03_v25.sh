#!/bin/bash
# subpix change parity + select phases + configs[4]; then LK per-level stamps
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
bash $R/tools/r03_v24.sh; exit 0
O=$R/gpurun_out/r03_v25
mkdir -p $O
cd $R
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_lkprof.so timeout -k 10 200 python -u tools/lk_prof.py > $O/lk_prof.txt 2> $O/lk_prof.err || { tail -20 $O/lk_prof.err; exit 1; }
head -5 $O/lk_prof.txt | cut -c1-1200

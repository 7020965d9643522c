#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v27
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_scale.txt 2> $O/pf_scale.err || { tail -20 $O/pf_scale.err; exit 1; }
cat $O/pf_scale.txt

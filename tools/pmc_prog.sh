#!/bin/bash
# rocprofv3 --pmc passes (one counter group per run, nothing else traced) over a
# short program, then the per-kernel summary.
#   bash tools/pmc_prog.sh <tag> "<program and args>" "<ctr ..>" ["<ctr ..>" ...]
# (ENV=... in the environment of the call applies to the program)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1; PROG=$2; shift 2
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -- python3 $R/$PROG > $O/p$i.log 2>&1
done
cd $R
python3 tools/pmc_summary.py $O > $O/pmc_summary.txt 2>&1 || true

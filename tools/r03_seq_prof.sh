#!/bin/bash
# Kernel trace of the configs[4] sequence replay (a 400-frame sequence, no CPU
# leg) for the per-frame critical path.  Usage: bash tools/r03_seq_prof.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seqprof -- python3 $R/bench.py --config 5 \
  --frames 400 --warmup 30 --no-cpu > $O/seq.json 2> $O/seq.err
head -c 600 $O/seq.json

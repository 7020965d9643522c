#!/bin/bash
# One rocprofv3 --pmc pass per counter group over a short bench run (no trace
# domains combined with --pmc).  Usage: tools/pmc.sh <tag> "<ctr ctr ..>" ["<ctr ..>" ...]
# Summarise with: python3 tools/pmc_summary.py gpurun_out/<tag>
# PMC_BENCH_ARGS overrides the bench arguments (default: the whole default line but the
# CPU baselines, sequence leg included -- r06: its torch synthesis now synchronises every
# 64 frames, the backlog that made rocprofv3's counter collection abort the queue in r05_m1).
# tools/traffic.py takes each kernel's largest-grid (batch) dispatches.  --streams 1: the
# headline's three contexts wait on each other's events at the timed region's ends, and
# under counter collection (dispatches serialised by the tool) that run stalled past 300 s
# (r06_m1); a kernel's traffic does not depend on the stream it runs on.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
shift
mkdir -p $R/gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  GVX_BENCH_TRACE=1 timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/$T/p$i \
     -- python3 $R/bench.py ${PMC_BENCH_ARGS:---steps 3 --warmup 1 --no-cpu --streams 1} > $R/gpurun_out/$T/p$i.log 2>&1
done

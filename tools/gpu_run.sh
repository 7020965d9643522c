#!/bin/bash
# One GPU-box pass over chosen test files and bench configs (every step with its
# own time limit; the first failure ends the script).
#   bash tools/gpu_run.sh <tag> "<test files or -m gpu>" [config ...]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1; TESTS=$2
shift 2 || shift $#
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_config$c.json 2> $O/bench_config$c.err
  cat $O/bench_config$c.json
done

#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, a rocprofv3 kernel
# trace (+ --stats) of the same bench, and optionally other configs.
# Usage (through gpurun): bash tools/gpu_check.sh <tag> [tests|notests] [config ...]
# Every step has its own time limit; the first failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
TESTS=${2:-tests}
shift 2 || shift $#
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ "$TESTS" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -3 $O/gpu_tests.log
fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof \
  -- python3 $R/bench.py --steps 20 --no-cpu > $O/prof.log 2>&1
cd $R
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cut -c1-60 $O/kernel_stats.csv
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_config$c.json 2> $O/bench_config$c.err
  cat $O/bench_config$c.json
done

#!/bin/bash
# The round's measurement pass on one GPU box: the whole -m gpu suite, smoke(), the
# driver's bench command, its rocprofv3 kernel-trace summary, the configs[3..5]
# lines and the FETCH_SIZE / WRITE_SIZE passes behind roofline.traffic.  Every step
# has its own time limit and the first failure ends the script.
#   bash tools/measure.sh <tag>     (results under gpurun_out/<tag>)
# Afterwards, here: python3 tools/traffic.py gpurun_out/<tag>/pmc
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=${1:?tag}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cat $O/bench.json
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_config$c.json 2> $O/bench_config$c.err
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err)
bash tools/pmc.sh $T/pmc FETCH_SIZE WRITE_SIZE
echo measure done

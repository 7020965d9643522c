# r06 final measurement pass at HEAD:
#  1. the whole -m gpu suite and smoke();
#  2. the driver's bench command, and its rocprofv3 --kernel-trace --stats summary;
#  3. FETCH_SIZE / WRITE_SIZE passes over the full default line (CPU legs off;
#     tools/traffic.py -> profiles/pmc_traffic.json);
#  4. the LK issue pass (tools/lk_pmc.py; tools/issue.py -> profiles/pmc_issue.json);
#  5. the configs[2], configs[3] and configs[4] lines.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); f=d['factors']; print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['device_ms_per_step'], f['preint_steps_per_s'], d['sequence']['value'], d['single_pair']['us_per_pair_eager'], d['preprocess']['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
python3 $R/tools/trace_span.py $O/prof/*/*_kernel_trace.csv > $O/trace_span.json && cat $O/trace_span.json
cp $O/prof/*/*_kernel_stats.csv $O/kernel_stats.csv && gzip -9 $O/prof/*/*_kernel_trace.csv
echo "kernel trace done"
cd $R
( while sleep 45; do echo "pmc running $(date +%T)"; done ) & TICK=$!
rc=0
PMC_BENCH_ARGS="${TRAFFIC_ARGS:---steps 3 --warmup 1 --no-cpu --streams 1 --no-overlap --no-sequence}" bash tools/pmc.sh $T/pmc FETCH_SIZE WRITE_SIZE || rc=$?
if [ $rc -eq 0 ]; then
  bash tools/pmc_prog.sh $T/lkpmc "tools/lk_pmc.py 30 10" "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" || rc=$?
fi
kill $TICK
[ $rc -eq 0 ] || { echo "pmc failed rc=$rc"; tail -20 $O/pmc/p1.log; exit 1; }
python3 tools/traffic.py $O/pmc --out $O/pmc_traffic.json > /dev/null && python3 tools/issue.py $O/lkpmc --out $O/pmc_issue.json
python3 tools/pmc_kernel.py $O/lkpmc klt_kernel > $O/lkpmc_klt.txt 2>&1 || true
gzip -9 $O/pmc/*/*/*.csv $O/lkpmc/*/*/*.csv 2>/dev/null || true
du -sh $O
echo "pmc done"
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 20 --warmup 5 > $O/bench_config$c.json 2> $O/bench_config$c.err || { tail -20 $O/bench_config$c.err; exit 1; }
  tail -c 300 $O/bench_config$c.json; echo
done
if [ -n "$DIAG" ]; then
  # one counter pass over the whole default line (sequence leg included), with the
  # bench's leg progress on stderr: where a stall under counter collection sits
  ( while sleep 45; do echo "pmc full line running $(date +%T)"; done ) & TICK=$!
  rc=0
  PMC_BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --streams 1" bash tools/pmc.sh $T/pmcfull FETCH_SIZE || rc=$?
  kill $TICK
  grep "^\[bench" $O/pmcfull/p1.log || true
  echo "full-line pmc rc=$rc"
  gzip -9 $O/pmcfull/*/*/*.csv 2>/dev/null || true
fi

# configs[2] (1920x1200, 500 points, maxLevel 4, 256 pairs): FETCH / WRITE passes over
# the batch leg alone (one serial context) and the LK issue pass, reduced on the box
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
( while sleep 45; do echo "pmc running $(date +%T)"; done ) & TICK=$!
rc=0
PMC_BENCH_ARGS="--config 3 --steps 3 --warmup 1 --no-cpu --no-pre --no-factors --no-sequence --streams 1 --no-overlap" bash tools/pmc.sh $T/pmc FETCH_SIZE WRITE_SIZE || rc=$?
if [ $rc -eq 0 ]; then
  bash tools/pmc_prog.sh $T/lkpmc "tools/lk_pmc.py 30 5 3" "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" || rc=$?
fi
kill $TICK
[ $rc -eq 0 ] || { echo "pmc failed rc=$rc"; tail -20 $O/pmc/p1.log; exit 1; }
W="klt_fb_batch 256x1920x1200 N500 L4"
python3 tools/traffic.py $O/pmc --workload "$W" --out $O/pmc_traffic_configs2.json
python3 tools/issue.py $O/lkpmc --workload "$W" --out $O/pmc_issue_configs2.json
gzip -9 $O/pmc/*/*/*.csv $O/lkpmc/*/*/*.csv 2>/dev/null || true
timeout -k 10 400 python -u bench.py --config 3 --steps 20 --warmup 5 > $O/bench_config3.json 2> $O/bench_config3.err || { tail -20 $O/bench_config3.err; exit 1; }
tail -c 1500 $O/bench_config3.json

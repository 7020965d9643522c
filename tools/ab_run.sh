# r06: fused compaction in the one-point LK launch -- parity tests, then the
# single-pair leg with and without it (GVX_FUSED_COMPACT=0)
set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/${TAG:-fc1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_klt_gpu.py tests/test_graph_gpu.py tests/test_bench_batch_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for v in on off; do
    if [ $v = off ]; then export GVX_FUSED_COMPACT=0; else unset GVX_FUSED_COMPACT; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-factors --no-sequence > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('single_pair'))"
  done
done

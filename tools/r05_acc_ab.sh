# r05 fp32-order A/B: the KLT accumulation-order and bench-launch parity tests on
# the in-tree library, then the default line's lk_accum_cost for it and each variant
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/${1:?tag}; mkdir -p $O; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_klt_accum_gpu.py tests/test_bench_batch_gpu.py tests/test_klt_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
  GVX_LIB="$lib" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-factors --no-sequence > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -20 $O/bench_${v}_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['lk_accum_cost'], d['roofline']['device_ms_per_step']['klt'])"
done
done

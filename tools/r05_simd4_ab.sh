# r05 F32_SIMD4 A/B: the LK parity tests (all orders, the bench's batch launch),
# then the configs[1] leg in F32_SIMD4 and EXACT for the tree and variants
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/${1:?tag}; mkdir -p $O; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_klt_gpu.py tests/test_klt_accum_gpu.py tests/test_bench_batch_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
  for acc in f32_simd4 exact; do
    GVX_LIB="$lib" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --accum $acc --no-cpu --no-pre --no-factors --no-sequence > $O/bench_${v}_${acc}_$r.json 2> $O/bench_${v}_${acc}_$r.err || { tail -20 $O/bench_${v}_${acc}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${v}_${acc}_$r.json').read().strip().splitlines()[-1]); print('$v $acc', d['value'], d['roofline']['device_ms_per_step'])"
  done
done
done

# r05 CLAHE A/B: the fused-CLAHE parity tests on each variant library (GVX_LIB),
# then the default line's preprocess leg (CLAHE over the step's 512 frames) for
# the in-tree library and each variant, interleaved twice
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/${1:?tag}; mkdir -p $O; shift
for v in "$@"; do
  GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_clahe_fused_gpu.py tests/test_clahe_gpu.py > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
for r in 1 2; do
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
  GVX_LIB="$lib" timeout -k 10 200 python3 bench.py --steps 10 --warmup 5 --no-cpu --no-factors --no-sequence > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -20 $O/bench_${v}_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_${v}_$r.json').read().strip().splitlines()[-1]); p=d['preprocess']; print('$v', p['roofline']['frac'], p.get('value'), p['roofline'].get('achieved'))"
done
done

# r05: the default line's headline and single-pair legs for the in-tree library and
# each variant (factor and sequence legs off), after the KLT / bench parity tests
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/${1:?tag}; mkdir -p $O; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_klt_gpu.py tests/test_bench_batch_gpu.py tests/test_profile_gpu.py tests/test_klt_accum_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
  GVX_LIB="$lib" timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-factors --no-sequence > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -20 $O/bench_${v}_$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['device_ms_per_step'], d['single_pair']['us_per_pair_eager'], d['single_pair']['us_per_pair_graph'])"
done
done

set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v27; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_acc1.so timeout -k 10 600 python -u -m pytest tests/test_klt_accum_gpu.py tests/test_klt_gpu.py tests/test_bench_batch_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_acc1.log 2>&1 || { tail -30 $O/tests_acc1.log; exit 1; }
echo acc1 $(tail -1 $O/tests_acc1.log)
bash tools/ab_run.sh r04_v27/ab 3 "bench.py --no-cpu --steps 20 --warmup 5 --no-factors" "(d['lk_accum_cost']['exact'], d['lk_accum_cost']['f32_simd4'], d['roofline']['device_ms_per_step']['klt'])" base acc1

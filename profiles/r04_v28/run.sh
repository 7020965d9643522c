set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v28; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_solo.so timeout -k 10 600 python -u -m pytest tests/test_klt_gpu.py tests/test_klt_accum_gpu.py tests/test_bench_batch_gpu.py tests/test_sequence_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_solo.log 2>&1 || { tail -30 $O/tests_solo.log; exit 1; }
echo solo $(tail -1 $O/tests_solo.log)
bash tools/ab_run.sh r04_v28/ab 3 "bench.py --no-cpu --steps 20 --warmup 5 --no-factors --no-pre" "(d['ms_per_step'], d['roofline']['device_ms_per_step']['pyramid'], d['roofline']['device_ms_per_step']['klt'])" base solo

set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v26; mkdir -p $O
for v in ring5 ring4; do
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 600 python -u -m pytest tests/test_pyramid_gpu.py tests/test_klt_gpu.py tests/test_bench_batch_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
echo $v $(tail -1 $O/tests_$v.log)
done
bash tools/ab_run.sh r04_v26/ab 3 "bench.py --no-cpu --steps 20 --warmup 5 --no-factors --no-pre" "(d['ms_per_step'], d['roofline']['device_ms_per_step']['pyramid'], d['roofline']['device_ms_per_step']['klt'])" base ring4 ring5

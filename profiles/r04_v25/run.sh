set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v25; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pyramid_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_base_pyr.log 2>&1 || { tail -30 $O/tests_base_pyr.log; exit 1; }
echo base-pyr $(tail -1 $O/tests_base_pyr.log)
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_ring.so timeout -k 10 600 python -u -m pytest tests/test_pyramid_gpu.py tests/test_klt_gpu.py tests/test_bench_batch_gpu.py tests/test_clahe_fused_gpu.py tests/test_sequence_gpu.py tests/test_graph_gpu.py tests/test_detect_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_ring.log 2>&1 || { tail -30 $O/tests_ring.log; exit 1; }
echo ring $(tail -1 $O/tests_ring.log)
bash tools/ab_run.sh r04_v25/ab 3 "bench.py --no-cpu --steps 20 --warmup 5 --no-factors" "(d['ms_per_step'], d['roofline']['device_ms_per_step']['pyramid'], d['roofline']['device_ms_per_step']['klt'])" base ring

set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v13; mkdir -p $O
for v in ck16 chain8 chain16; do
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
tail -1 $O/tests_$v.log
done
bash tools/preint_prof.sh r04_v13/prof base ck16 chain8 chain16
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_occ6.so timeout -k 10 300 python -u -m pytest tests/test_bench_batch_gpu.py tests/test_klt_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_occ6.log 2>&1 || { tail -30 $O/tests_occ6.log; exit 1; }
tail -1 $O/tests_occ6.log
bash tools/ab_run.sh r04_v13/lk 3 "bench.py --no-cpu --no-pre --no-factors --steps 20 --warmup 5" "(d['roofline']['device_ms_per_step']['klt'], d['ms_per_step'])" base occ6

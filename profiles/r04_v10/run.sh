set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v10; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_u8wg2.so timeout -k 10 300 python -u -m pytest tests/test_clahe_fused_gpu.py tests/test_clahe_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for n in u8tab u8wg2; do
    L=$PWD/ic-gvins_amd/gvx/variants/libgvx_$n.so
    GVX_CLAHE_FUSED1=1 GVX_LIB=$L timeout -k 10 120 python tools/clahe_ab.py > $O/${n}_$r.json
    echo $n $(python3 -c "import json;print(round(json.load(open('$O/${n}_$r.json'))['ms_per_call'],4))")
  done
done
timeout -k 10 300 python -u -m pytest tests/test_lm_step_gpu.py tests/test_marg_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_lm.log 2>&1 || { tail -30 $O/tests_lm.log; exit 1; }
tail -2 $O/tests_lm.log

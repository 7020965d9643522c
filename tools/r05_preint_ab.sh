set -e
O=gpurun_out/r05_v2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ba_gpu.py tests/test_factor_parity_gpu.py tests/test_factorset_gpu.py tests/test_golden.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  GVX_LIB=ic-gvins_amd/gvx/variants/libgvx_r04base.so timeout -k 10 120 python tools/preint_loop.py > $O/loop_base_$r.json
  timeout -k 10 120 python tools/preint_loop.py > $O/loop_new_$r.json
done
cat $O/loop_*.json

set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v15; mkdir -p $O
for v in ws wsf wsf2; do
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_factor_parity_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
echo $v $(tail -1 $O/tests_$v.log)
done
bash tools/preint_prof.sh r04_v15/prof1 base ws wsf wsf2 && bash tools/preint_prof.sh r04_v15/prof2 base ws wsf wsf2

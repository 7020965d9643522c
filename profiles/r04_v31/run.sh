set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v31; mkdir -p $O
for v in pst pst6; do
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_factor_parity_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
echo $v $(tail -1 $O/tests_$v.log)
done
timeout -k 10 300 python3 tools/preint_dump.py $O/base.npy > $O/dump_base.log 2>&1
for v in pst pst6; do
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 300 python3 tools/preint_dump.py $O/$v.npy > $O/dump_$v.log 2>&1
python3 -c "import numpy as np; a=np.load('$O/base.npy'); b=np.load('$O/$v.npy'); print('$v bytes equal:', np.array_equal(a, b))"
done
rm -f $O/*.npy
bash tools/ab_run.sh r04_v31/ab 3 "tools/preint_loop.py" "(d['cold']['preint'], d['warm']['preint'], d['warm']['steps_per_s'])" base pst pst6

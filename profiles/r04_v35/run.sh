set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v35; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_sqf.so timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_factor_parity_gpu.py tests/test_factorset_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_sqf.log 2>&1 || { tail -30 $O/tests_sqf.log; exit 1; }
echo sqf $(tail -1 $O/tests_sqf.log)
timeout -k 10 300 python3 tools/preint_dump.py $O/base.npy > $O/dump_base.log 2>&1
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_sqf.so timeout -k 10 300 python3 tools/preint_dump.py $O/sqf.npy > $O/dump_sqf.log 2>&1
python3 -c "import numpy as np; a=np.load('$O/base.npy'); b=np.load('$O/sqf.npy'); print('sqf bytes equal:', np.array_equal(a, b))"
rm -f $O/*.npy
bash tools/ab_run.sh r04_v35/ab 3 "tools/preint_loop.py" "(d['cold']['wall_ms'], d['warm']['wall_ms'], d['warm']['steps_per_s'])" base sqf

set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v33; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_fuse.so timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_factor_parity_gpu.py tests/test_factorset_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_fuse.log 2>&1 || { tail -30 $O/tests_fuse.log; exit 1; }
echo fuse $(tail -1 $O/tests_fuse.log)
timeout -k 10 300 python3 tools/preint_dump.py $O/base.npy > $O/dump_base.log 2>&1
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_fuse.so timeout -k 10 300 python3 tools/preint_dump.py $O/fuse.npy > $O/dump_fuse.log 2>&1
python3 -c "import numpy as np; a=np.load('$O/base.npy'); b=np.load('$O/fuse.npy'); print('fuse bytes equal:', np.array_equal(a, b))"
rm -f $O/*.npy
bash tools/ab_run.sh r04_v33/ab 3 "tools/preint_loop.py" "(d['cold']['preint'], d['warm']['preint'], d['warm']['steps_per_s'])" base fuse

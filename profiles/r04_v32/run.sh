set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v32; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_rot16.so timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_rot16.log 2>&1 || { tail -30 $O/tests_rot16.log; exit 1; }
echo rot16 $(tail -1 $O/tests_rot16.log)
bash tools/ab_run.sh r04_v32/ab 3 "tools/preint_loop.py" "(d['cold']['preint'], d['warm']['preint'], d['warm']['steps_per_s'])" base rot16 rot32

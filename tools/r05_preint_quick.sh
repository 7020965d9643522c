# r05 preintegration quick check: parity tests, the clock probe, warm launches
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/${1:?tag}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ba_gpu.py tests/test_factor_parity_gpu.py tests/test_factorset_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
if [ -f ic-gvins_amd/gvx/variants/libgvx_clk.so ]; then
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_clk.so timeout -k 10 200 python3 tools/preint_clock.py > $O/clock.json 2> $O/clock.err || { tail -20 $O/clock.err; exit 1; }
tail -1 $O/clock.json
fi
for v in ${2:-}; do GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 100 python3 tools/preint_loop.py > $O/loop_$v.json; echo $v; cat $O/loop_$v.json; done
timeout -k 10 100 python3 tools/preint_loop.py > $O/loop.json; cat $O/loop.json

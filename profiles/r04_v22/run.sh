set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v22; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_factor_parity_gpu.py tests/test_marg_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo tests $(tail -1 $O/tests.log)
for r in 1 2; do for sp in 1 2 3 4 8; do
  GVX_PREINT_SPLIT=$sp timeout -k 10 200 python3 tools/preint_loop.py > $O/loop_${sp}_$r.json 2> $O/loop_${sp}_$r.err || { tail -20 $O/loop_${sp}_$r.err; exit 1; }
  echo split$sp $(python3 -c "import json;d=json.load(open('$O/loop_${sp}_$r.json'));print(d['cold'],d['warm'])")
done; done

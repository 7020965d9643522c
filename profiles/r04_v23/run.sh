set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v23; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_pre6.so timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_pre6.log 2>&1 || { tail -30 $O/tests_pre6.log; exit 1; }
echo pre6 $(tail -1 $O/tests_pre6.log)
bash tools/preint_prof.sh r04_v23/prof base pre5 pre6
for r in 1 2; do for v in base pre5 pre6; do
  if [ $v = base ]; then lib=""; else lib=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
  GVX_LIB="$lib" timeout -k 10 200 python3 tools/preint_loop.py > $O/loop_${v}_$r.json 2> $O/loop_${v}_$r.err || { tail -20 $O/loop_${v}_$r.err; exit 1; }
  echo $v $(python3 -c "import json;d=json.load(open('$O/loop_${v}_$r.json'));print(d['cold'],d['warm'])")
done; done

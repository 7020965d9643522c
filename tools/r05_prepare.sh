# gvx_factors_prepare at window size: wall per prepare (mapped host results vs
# the D2H form) and the rocprofv3 copy / kernel breakdown of the default form
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out/${1:?tag}; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_factorset_gpu.py > $O/factorset_tests.log 2>&1 || { tail -30 $O/factorset_tests.log; exit 1; }
tail -1 $O/factorset_tests.log
for r in 1 2; do
  timeout -k 10 60 python3 tools/prepare_trace.py 2000 > $O/prep_mapped_$r.json
  GVX_FACTORSET_D2H=1 timeout -k 10 60 python3 tools/prepare_trace.py 2000 > $O/prep_d2h_$r.json
done
tail -n1 $O/prep_*.json
cd /tmp && export TMPDIR=/tmp
for m in mapped d2h; do
  if [ $m = d2h ]; then export GVX_FACTORSET_D2H=1; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_$m -- python3 $R/tools/prepare_trace.py 300 > $O/tr_$m.json 2>&1
  python3 $R/tools/prepare_breakdown.py $O/tr_$m > $O/breakdown_$m.txt 2>&1 || true
  echo "== $m"; cat $O/breakdown_$m.txt
done

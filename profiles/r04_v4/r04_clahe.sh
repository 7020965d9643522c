# CLAHE: parity tests, then interleaved A/B of fused_kernel (GVX_CLAHE_FUSED1=1) vs fused2_kernel
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; T=${1:-r04_clahe}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_clahe_fused_gpu.py tests/test_clahe_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  GVX_CLAHE_FUSED1=1 timeout -k 10 120 python tools/clahe_ab.py > $O/f1_$r.json
  timeout -k 10 120 python tools/clahe_ab.py > $O/f2_$r.json
  cat $O/f1_$r.json $O/f2_$r.json
done

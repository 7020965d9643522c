set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_factor_parity_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    GVX_PREINT_COV8=$v timeout -k 10 200 python bench.py --config 4 --no-cpu --steps 20 --warmup 5 > $O/c4_cov8_${v}_$r.json 2> $O/c4.err
    python3 -c "import json;d=json.load(open('$O/c4_cov8_${v}_$r.json'));print('cov8=$v', d['preint_steps_per_s'], d['preint_device_ms_per_launch'])"
  done
done
bash tools/r04_clahe_skew.sh

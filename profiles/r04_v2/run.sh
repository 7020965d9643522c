set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_klt_gpu.py tests/test_klt_accum_gpu.py tests/test_bench_batch_gpu.py tests/test_sequence_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab.sh r04_v2 3 r03 base
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench_driver_cmd.json'));print(d['value'],d['roofline']['device_ms_per_step'],d['lk_accum_cost'])"

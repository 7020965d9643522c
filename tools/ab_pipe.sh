# A/B of the pipelined configs[4] replay (frame t+1 preprocessed in a graph branch) on one box,
# after the sequence parity tests:  bash tools/ab_pipe.sh
set -e
mkdir -p gpurun_out/pipe
timeout -k 10 300 python -u -m pytest tests/test_sequence_gpu.py tests/test_graph_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pipe/tests.log 2>&1 || { tail -30 gpurun_out/pipe/tests.log; exit 1; }
tail -3 gpurun_out/pipe/tests.log
for r in 1 2; do
  for v in pipe nopipe; do
    a=""; [ $v = nopipe ] && a="--no-pipeline"
    timeout -k 10 200 python bench.py --config 5 --no-cpu $a > gpurun_out/pipe/b_${v}_$r.json 2> gpurun_out/pipe/b_${v}_$r.err
    python3 -c "import json; d=json.loads(open('gpurun_out/pipe/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_frame'])"
  done
done

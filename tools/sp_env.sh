for v in unset 0 1; do
  if [ $v = unset ]; then E=""; else E="DEBUG_CLR_GRAPH_PACKET_CAPTURE=$v"; fi
  env $E timeout -k 10 200 python bench.py --no-cpu --no-factors --steps 10 --warmup 10 > gpurun_out/sp_$v.json 2>gpurun_out/sp_$v.err
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sp_$v.json').read().strip().splitlines()[-1]); print('$v', d['single_pair'])"
done

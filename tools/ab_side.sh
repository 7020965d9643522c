# factor batch with / without the side stream (GVX_NO_SIDE_STREAM) on the configs[3] leg, one box
set -e
mkdir -p gpurun_out/abside
for r in 1 2; do for v in 1 0; do
GVX_NO_SIDE_STREAM=$v timeout -k 10 200 python bench.py --config 4 --no-cpu --steps 40 --warmup 30 > gpurun_out/abside/s${v}_$r.json 2>/dev/null
python3 -c "import json; d=json.loads(open('gpurun_out/abside/s${v}_$r.json').read().strip().splitlines()[-1]); print('no_side=$v', round(d['value']/1e9,3), 'G/s', d['ms_per_step'], 'ms', d['roofline']['device_ms_per_step'], 'window', d['problem_size'])"
done; done

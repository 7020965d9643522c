set -e
mkdir -p gpurun_out/abcov
for r in 1 2; do for v in 16 8; do
GVX_PREINT_COV_LANES=$v timeout -k 10 200 python bench.py --config 4 --no-cpu --steps 40 --warmup 30 > gpurun_out/abcov/c${v}_$r.json 2>/dev/null
python3 -c "import json; d=json.loads(open('gpurun_out/abcov/c${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['preint_device_ms_per_launch'], d['preint_steps_per_s']/1e6)"
done; done

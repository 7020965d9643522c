# A/B of the covariance pass on the configs[3] preintegration leg, interleaved on
# one box: bash tools/ab_cov.sh <tag> <rounds> <VAR> <value>...
# (e.g. GVX_PREINT_COV_SPLIT 0 1, or GVX_PREINT_COV_LANES 8 16)
set -e
T=$1; ROUNDS=$2; VAR=$3; shift 3
mkdir -p gpurun_out/$T
for r in $(seq 1 $ROUNDS); do for v in "$@"; do
  env $VAR=$v timeout -k 10 200 python bench.py --config 4 --no-cpu --steps 40 --warmup 30 > gpurun_out/$T/c${v}_$r.json 2> gpurun_out/$T/c${v}_$r.err
  python3 -c "import json; d=json.loads(open('gpurun_out/$T/c${v}_$r.json').read().strip().splitlines()[-1]); print('$VAR=$v', d['preint_device_ms_per_launch'], round(d['preint_steps_per_s']/1e6, 1))"
done; done

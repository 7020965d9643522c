# configs[4] timing of environment settings: bash tools/ab_env5.sh <tag> <frames> "VAR=a" ...
set -e
T=$1; NF=$2; shift 2
mkdir -p gpurun_out/$T
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 300 python bench.py --config 5 --frames $NF --no-cpu > gpurun_out/$T/b_$i.json 2> gpurun_out/$T/b_$i.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/$T/b_$i.json')); print('$kv', d['value'], d['roofline']['device_ms_per_frame'])"
done

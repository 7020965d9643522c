# Interleaved timing of environment settings (one bench run per setting per round):
#   bash tools/ab_env.sh <tag> <rounds> "VAR=a" "VAR=b" ...
set -e
T=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out/$T
for r in $(seq 1 $ROUNDS); do
  i=0
  for kv in "$@"; do
    i=$((i+1))
    env $kv timeout -k 10 200 python bench.py --no-cpu --steps 40 --warmup 30 > gpurun_out/$T/b_${i}_$r.json 2> gpurun_out/$T/b_${i}_$r.err
  done
done
python3 - "$T" "$ROUNDS" "$@" <<'PY'
import json, sys
t, rounds, kvs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for i, kv in enumerate(kvs, 1):
    out = []
    for r in range(1, rounds + 1):
        d = json.load(open(f"gpurun_out/{t}/b_{i}_{r}.json"))
        out.append(f"{d['value']:.0f} {d['roofline']['device_ms_per_step']}")
    print(kv, " | ".join(out))
PY

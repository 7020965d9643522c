# preint one-phase vs two-phase on the configs[3] bench leg, interleaved on one box
#   bash tools/ab_preint.sh <tag> <rounds>
set -e
T=$1; ROUNDS=$2
mkdir -p gpurun_out/$T
for r in $(seq 1 $ROUNDS); do
  for v in 1 0; do
    GVX_PREINT_ONEPHASE=$v timeout -k 10 200 python bench.py --config 4 --no-cpu --steps 40 --warmup 30 > gpurun_out/$T/p${v}_$r.json 2> gpurun_out/$T/p${v}_$r.err
  done
done
python3 - "$T" "$ROUNDS" <<'PY'
import json, sys
t, rounds = sys.argv[1], int(sys.argv[2])
for v in ("1", "0"):
    xs = [json.loads(open(f"gpurun_out/{t}/p{v}_{r}.json").read().strip().splitlines()[-1]) for r in range(1, rounds + 1)]
    print("one-phase" if v == "1" else "two-phase",
          " | ".join(f"{x['preint_device_ms_per_launch']:.4f} ms {x['preint_steps_per_s'] / 1e6:.1f} M steps/s" for x in xs))
PY

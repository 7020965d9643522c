# A/B timing of libgvx variants (tools/variant.sh) on the configs[3] factor leg,
# interleaved on one box:  bash tools/ab_fac.sh <tag> <rounds> <name>...
# ("base" = the in-tree libgvx.so)
set -e
T=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out/$T
for r in $(seq 1 $ROUNDS); do
  for n in "$@"; do
    if [ "$n" = base ]; then L=""; else L=$PWD/ic-gvins_amd/gvx/variants/libgvx_$n.so; fi
    GVX_LIB=$L timeout -k 10 200 python bench.py --config 4 --no-cpu --steps 40 --warmup 30 > gpurun_out/$T/f_${n}_$r.json 2> gpurun_out/$T/f_${n}_$r.err
  done
done
python3 - "$T" "$ROUNDS" "$@" <<'PY'
import json, sys
t, rounds, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for n in names:
    v = [json.loads(open(f"gpurun_out/{t}/f_{n}_{r}.json").read().strip().splitlines()[-1]) for r in range(1, rounds + 1)]
    print(n, " | ".join(f"{x['value']/1e9:.3f} G/s reproj {x['roofline']['device_ms_per_step']['reproj']:.4f} "
                        f"pf {x['roofline']['device_ms_per_step']['preint_factor']:.4f}" for x in v))
PY

# A/B timing of libgvx variants (tools/variant.sh) on one box, interleaved:
#   bash tools/ab.sh <tag> <rounds> <name>...   ("base" = the in-tree libgvx.so)
# BENCH_ARGS (env): extra bench.py arguments, e.g. "--accum f32_simd4" or "--config 3".
set -e
T=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out/$T
for r in $(seq 1 $ROUNDS); do
  for n in "$@"; do
    if [ "$n" = base ]; then L=""; else L=$PWD/ic-gvins_amd/gvx/variants/libgvx_$n.so; fi
    GVX_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-pre --no-factors --steps 40 --warmup 30 $BENCH_ARGS \
      > gpurun_out/$T/b_${n}_$r.json 2> gpurun_out/$T/b_${n}_$r.err
  done
done
python3 - "$T" "$ROUNDS" "$@" <<'PY'
import json, sys
t, rounds, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for n in names:
    v = [json.load(open(f"gpurun_out/{t}/b_{n}_{r}.json"))["roofline"]["device_ms_per_step"] for r in range(1, rounds + 1)]
    print(n, " ".join(f"klt {x['klt']:.4f} pyr {x['pyramid']:.4f}" for x in v))
PY

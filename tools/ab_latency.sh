# A/B of libgvx variants (tools/variant.sh) on the latency configurations, on
# one box, interleaved: bench.py's single_pair leg (one frame pair per launch)
# and the configs[4] sequence replay.  Runs the GPU parity tests first.
#   bash tools/ab_latency.sh <tag> <rounds> <name>...   ("base" = the in-tree libgvx.so)
set -e
T=$1; ROUNDS=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
for r in $(seq 1 $ROUNDS); do
  for n in "$@"; do
    if [ "$n" = base ]; then L=""; else L=$PWD/ic-gvins_amd/gvx/variants/libgvx_$n.so; fi
    GVX_LIB=$L timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 10 > $O/b_${n}_$r.json 2> $O/b_${n}_$r.err
    GVX_LIB=$L timeout -k 10 200 python bench.py --config 5 --frames 800 --no-cpu > $O/s_${n}_$r.json 2> $O/s_${n}_$r.err
    python3 - "$O" "$n" "$r" <<'PY'
import json, sys
o, n, r = sys.argv[1:]
b = json.load(open(f"{o}/b_{n}_{r}.json"))
s = json.load(open(f"{o}/s_{n}_{r}.json"))
print(n, "single pair us", b["single_pair"]["us_per_pair_eager"], "| sequence fps", s["value"],
      s["roofline"]["device_ms_per_frame"])
PY
  done
done

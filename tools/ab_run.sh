#!/bin/bash
# Interleaved A/B timing of libgvx variants and environment settings on one GPU box.
#   bash tools/ab_run.sh <tag> <rounds> "<program + args>" "<python expr over d>" <variant>...
# <variant> = name[:VAR=val,VAR=val]: name "base" runs the in-tree libgvx.so, any other
# name ic-gvins_amd/gvx/variants/libgvx_<name>.so (tools/variant.sh builds them); the
# VAR=val pairs go to the program's environment.  <program + args> prints one JSON line
# (the last line is read); the expression is evaluated with it as d.  Examples:
#   bash tools/ab_run.sh lk 3 "bench.py --no-cpu --no-pre --no-factors" "d['roofline']['device_ms_per_step']" r03 base
#   bash tools/ab_run.sh clahe 3 "tools/clahe_ab.py" "d['ms_per_call']" base u8tab
#   bash tools/ab_run.sh cov 2 "bench.py --config 4 --no-cpu --steps 20" "d['preint_steps_per_s']" base:GVX_PREINT_COV8=1 base
# Every run has its own time limit; the first failing run ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
T=$1; ROUNDS=$2; PROG=$3; EXPR=$4; shift 4
O=gpurun_out/$T
mkdir -p "$O"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    name=${v%%:*}
    envs=""
    if [ "$v" != "$name" ]; then envs=$(echo "${v#*:}" | tr ',' ' '); fi
    if [ "$name" = base ]; then lib=""; else lib=$R/ic-gvins_amd/gvx/variants/libgvx_$name.so; fi
    tag=$(echo "$v" | tr ':=,/' '____')
    env GVX_LIB="$lib" $envs timeout -k 10 300 python3 $PROG > "$O/${tag}_$r.json" 2> "$O/${tag}_$r.err"
  done
done
python3 - "$O" "$ROUNDS" "$EXPR" "$@" <<'PY'
import json, sys
o, rounds, expr, variants = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4:]
for v in variants:
    tag = v.replace(":", "_").replace("=", "_").replace(",", "_").replace("/", "_")
    vals = []
    for r in range(1, rounds + 1):
        d = json.loads(open(f"{o}/{tag}_{r}.json").read().strip().splitlines()[-1])
        vals.append(str(eval(expr, {"d": d})))
    print(v, " | ".join(vals))
PY

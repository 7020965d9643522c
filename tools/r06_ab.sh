# r06 interleaved A/B of environment settings on the headline leg.
#   CFGS="name|VAR=a VAR2=b|--extra-args;name2|...|..." bash tools/r06_ab.sh <tag> [rounds]
# TESTS (optional): pytest files to run first.  RES (optional): "name|ENV|lpp|kern;..."
# residency runs (trace build) after the A/B.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; ROUNDS=${2:-2}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
IFS=';' read -ra LIST <<< "$CFGS"
for r in $(seq 1 $ROUNDS); do
  for c in "${LIST[@]}"; do
    IFS='|' read -r name envs args <<< "$c"
    env $envs timeout -k 10 200 python3 bench.py --steps ${STEPS:-40} --warmup 30 --no-cpu --no-factors --no-sequence $args > $O/b_${name}_$r.json 2> $O/b_${name}_$r.err || { tail -20 $O/b_${name}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${name}_$r.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['roofline']['device_span_ms_per_step'], d['roofline']['device_ms_per_step'])"
  done
done
if [ -n "$RES" ]; then
  IFS=';' read -ra RL <<< "$RES"
  for c in "${RL[@]}"; do
    IFS='|' read -r name envs lpp kern <<< "$c"
    env $envs GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_klttrace.so timeout -k 10 240 python3 -u tools/lk_residency.py $O/res_$name 300 $lpp $kern > $O/res_$name.log 2>&1 || { tail -20 $O/res_$name.log; exit 1; }
    echo "residency $name"; tail -1 $O/res_$name.log
  done
fi

# the driver's command, twice, and once back to back (--no-overlap)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for v in a b nov; do
  extra=""; [ $v = nov ] && extra="--no-overlap"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $extra > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['device_ms_per_step'], d['single_pair']['us_per_pair_eager'], d['sequence']['value'])"
done

# r05: the configs[2], configs[3] and configs[4] lines (bench.py --config 3 / 4 / 5)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu > $O/bench_config$c.json 2> $O/bench_config$c.err || { tail -20 $O/bench_config$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_config$c.json').read().strip().splitlines()[-1]); print('config $c', d['metric'], d['value'], d['unit'])"
done

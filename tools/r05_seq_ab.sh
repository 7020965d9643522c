# r05: configs[4] with and without the eigenvalue map on the preprocessing branch
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/${1:?tag}; mkdir -p $O
for r in 1 2; do
for v in default eig; do
  extra=""; [ "$v" = eig ] && extra="--eig-branch"
  timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 5 --no-cpu $extra > $O/seq_${v}_$r.json 2> $O/seq_${v}_$r.err || { tail -20 $O/seq_${v}_$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/seq_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d.get('device_ms_per_frame') or d.get('config',{}).get('device_ms_per_frame'))"
done
done

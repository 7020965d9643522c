set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_m7; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do timeout -k 10 300 python -u bench.py --config 4 > $O/bench_config4_$i.json 2> $O/bench_config4_$i.err; done
python3 -c "
import json
for i in (1, 2):
    d = json.loads(open('$O/bench_config4_%d.json' % i).read().strip().splitlines()[-1])
    print(d['metric'], d['value'], d.get('preint_steps_per_s'))
"

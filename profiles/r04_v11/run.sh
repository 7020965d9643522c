set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out/r04_v11; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_factor_parity_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --config 4 --no-cpu --steps 10 --warmup 3 > $O/c4.json 2> $O/c4.err
cd $R
python3 - <<'PY'
import csv,glob,json
f=glob.glob('gpurun_out/r04_v11/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r['Name']
    if 'preint' in n or 'sqrt_info' in n:
        print(n.split('::')[-1].split('(')[0][:28], r['Calls'], round(float(r['AverageNs'])/1000,1),'us')
d=json.loads(open('gpurun_out/r04_v11/c4.json').read().strip().splitlines()[-1])
print('steps/s', d['preint_steps_per_s'], d['preint_device_ms_per_launch'])
PY
timeout -k 10 120 python3 tools/graph_step_ab.py

# r05: the whole -m gpu suite, smoke() and the driver's bench command at HEAD
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); f=d['factors']; print('bench', d['value'], d['roofline']['frac'], d['roofline']['device_ms_per_step'], f['preint_steps_per_s'], f['problem_size']['factor_set_prepare_ms'], d['sequence']['value'], d['lk_accum_cost'], d['preprocess']['roofline']['frac'])"

# r06: KLT / pyramid / sequence GPU tests, then the driver's bench command (full
# default line) and its rocprofv3 --kernel-trace --stats summary.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_klt_gpu.py tests/test_bench_batch_gpu.py tests/test_pyramid_gpu.py tests/test_graph_gpu.py} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); f=d['factors']; print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['frac_min'], d['roofline']['device_ms_per_step'], d['single_pair'], d['sequence']['value'], d['preprocess']['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
echo prof done

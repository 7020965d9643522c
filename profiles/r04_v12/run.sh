set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v12; mkdir -p $O
timeout -k 10 200 python3 tools/overlap_ab.py > $O/overlap.json 2> $O/overlap.err || { tail -20 $O/overlap.err; exit 1; }
cat $O/overlap.json
timeout -k 10 300 python -u -m pytest tests/test_bench_batch_gpu.py -x -v --timeout 200 --timeout-method thread -k "pipelined or exact" > $O/tests_pipe.log 2>&1 || { tail -30 $O/tests_pipe.log; exit 1; }
tail -1 $O/tests_pipe.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_overlap_$r.json 2> $O/bench_overlap_$r.err
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-overlap > $O/bench_seq_$r.json 2> $O/bench_seq_$r.err
done
for f in $O/bench_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['device_ms_per_step'])"; done
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_pfma.so timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_run.sh r04_v12/cov 2 "bench.py --config 4 --no-cpu --steps 20" "(d['preint_steps_per_s'], d['preint_device_ms_per_launch'])" base pfma

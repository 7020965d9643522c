# r06 LK phases: parity of the phase kernel, interleaved A/B of levels per phase
# (GVX_KLT_LPP; 0 = the single-wave chain), residency timelines, then the PMC
# run of the default line with the sequence leg (the dispatch-backlog fix) last.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_klt_gpu.py tests/test_bench_batch_gpu.py tests/test_klt_accum_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for k in 0 1 2 4; do
    GVX_KLT_LPP=$k timeout -k 10 200 python3 bench.py --steps 40 --warmup 30 --no-cpu --no-factors --no-sequence > $O/b_${k}_$r.json 2> $O/b_${k}_$r.err || { tail -20 $O/b_${k}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${k}_$r.json').read().strip().splitlines()[-1]); print('lpp $k', d['value'], d['roofline']['device_ms_per_step'], d['lk_accum_cost']['exact'])"
  done
done
for k in 1 2 0; do
  GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_klttrace.so timeout -k 10 240 python3 -u tools/lk_residency.py $O/res_$k 300 $k > $O/res_$k.log 2>&1 || { tail -20 $O/res_$k.log; exit 1; }
  echo "residency lpp $k"; tail -1 $O/res_$k.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcseq -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-pre --no-factors > $O/pmcseq.log 2>&1 || { echo "pmc run with the sequence leg failed"; grep -v "^    @" $O/pmcseq.log | tail -30; exit 1; }
echo "pmc run with the sequence leg completed"; tail -1 $O/pmcseq.log | cut -c1-200

# r06 LK phases, round 3 (superchunks): parity, then interleaved A/B over
# (levels per phase, groups per superchunk), then residency of two settings.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_klt_gpu.py tests/test_bench_batch_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
CFGS=${CFGS:-"0:4096 1:2048 1:4096 1:8192 2:4096 2:8192 4:4096 4:8192"}
for r in 1 2; do
  for kv in $CFGS; do
    k=${kv%%:*}; s=${kv##*:}
    GVX_KLT_LPP=$k GVX_KLT_SUPER=$s timeout -k 10 200 python3 bench.py --steps 40 --warmup 30 --no-cpu --no-factors --no-sequence > $O/b_${k}_${s}_$r.json 2> $O/b_${k}_${s}_$r.err || { tail -20 $O/b_${k}_${s}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${k}_${s}_$r.json').read().strip().splitlines()[-1]); print('lpp $k super $s', d['value'], d['roofline']['device_ms_per_step'], d['lk_accum_cost']['exact'])"
  done
done
for kv in ${RES:-"1:4096 2:4096"}; do
  k=${kv%%:*}; s=${kv##*:}
  GVX_KLT_SUPER=$s GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_klttrace.so timeout -k 10 240 python3 -u tools/lk_residency.py $O/res_${k}_$s 300 $k > $O/res_${k}_$s.log 2>&1 || { tail -20 $O/res_${k}_$s.log; exit 1; }
  echo "residency lpp $k super $s"; tail -1 $O/res_${k}_$s.log
done

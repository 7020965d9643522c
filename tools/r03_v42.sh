#!/bin/bash
# LK one-point waves: next level's I rows prefetched while the level iterates (pre) vs base;
# LK / sequence parity on the variant, then sequence + single-pair legs interleaved
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=r03_v42
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_pre.so timeout -k 10 400 python -u -m pytest tests/test_klt_gpu.py tests/test_klt_accum_gpu.py tests/test_sequence_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in base pre; do
    L=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so
    GVX_LIB=$L timeout -k 10 200 python -u bench.py --config 5 --no-cpu > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err
    python3 -c "import json;d=json.load(open('$O/c5_${v}_$r.json'));print('c5 $v', d['value'], d['roofline']['device_ms_per_frame'])"
    GVX_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu --no-factors --steps 10 --warmup 10 > $O/sp_${v}_$r.json 2> $O/sp_${v}_$r.err
    python3 -c "import json;d=json.load(open('$O/sp_${v}_$r.json'));print('sp $v', d['single_pair']['us_per_pair_eager'], d['single_pair']['us_per_pair_graph'])"
  done
done

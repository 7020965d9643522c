#!/bin/bash
# LK: every unit's J rows in flight before the first is realigned (jl) vs base;
# batch (configs[1]) and sequence (configs[4]) legs, interleaved
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=r03_v39
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
bash tools/ab.sh $T 3 base jl
for r in 1 2; do
  for v in base jl; do
    L=""; [ $v != base ] && L=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so
    GVX_LIB=$L timeout -k 10 200 python -u bench.py --config 5 --no-cpu > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err
    python3 -c "import json;d=json.load(open('$O/c5_${v}_$r.json'));print('c5 $v', d['value'], d['roofline']['device_ms_per_frame'])"
  done
done

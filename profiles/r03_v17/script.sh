#!/bin/bash
# HEAD check (full -m gpu suite, default bench + rocprof, configs 3/4/5) and an
# A/B of the one-point-wave LK prefetch (GVX_LIB=variants/libgvx_base.so = the
# previous klt.hip) on the sequence replay and the single-pair leg.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
bash $R/tools/gpu_check.sh $T tests 3 4 5
O=$R/gpurun_out/$T
cd $R
for r in 1 2; do
  for v in base new; do
    L=""; [ $v = base ] && L=$R/ic-gvins_amd/gvx/variants/libgvx_base.so
    GVX_LIB=$L timeout -k 10 200 python -u bench.py --config 5 --no-cpu > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err
    python3 -c "import json;d=json.load(open('$O/c5_${v}_$r.json'));print('c5 $v', d['value'], d['ms_per_step'], d['roofline']['device_ms_per_frame'])"
    GVX_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu --no-factors --steps 10 --warmup 10 > $O/sp_${v}_$r.json 2> $O/sp_${v}_$r.err
    python3 -c "import json;d=json.load(open('$O/sp_${v}_$r.json'));print('sp $v', d['single_pair'])"
  done
done

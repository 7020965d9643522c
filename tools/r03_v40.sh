#!/bin/bash
# tree = LK batched J-row loads for PPW > 1 (jl2); full check, then the batch and
# sequence legs interleaved against the previous tree (variants/libgvx_base.so)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=r03_v40
O=$R/gpurun_out/$T
bash $R/tools/gpu_check.sh $T tests
cd $R
bash tools/ab.sh ${T}_ab 3 base_old jl2 > $O/ab.txt
cat $O/ab.txt
for r in 1 2; do
  for v in base_old tree; do
    L=""; [ $v != tree ] && L=$R/ic-gvins_amd/gvx/variants/libgvx_base.so
    GVX_LIB=$L timeout -k 10 200 python -u bench.py --config 5 --no-cpu > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err
    python3 -c "import json;d=json.load(open('$O/c5_${v}_$r.json'));print('c5 $v', d['value'], d['roofline']['device_ms_per_frame'])"
  done
done

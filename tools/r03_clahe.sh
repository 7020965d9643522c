#!/bin/bash
# CLAHE round: the v_cvt_pk_u8_f32 rounding probe, CLAHE parity, a default
# bench and its kernel trace.  Usage: bash tools/r03_clahe.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
hipcc -O2 --offload-arch=gfx950 -Wno-unused-value -Wno-unused-result tools/cvt_pk_u8_probe.hip -o /tmp/cvt_probe
timeout -k 10 60 /tmp/cvt_probe | tee $O/cvt_probe.txt
timeout -k 10 400 python -u -m pytest tests/test_clahe_fused_gpu.py tests/test_clahe_gpu.py -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 20 > $O/bench.json 2> $O/bench.err
grep -o '"preprocess": {[^}]*}[^}]*}' $O/bench.json

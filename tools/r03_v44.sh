#!/bin/bash
# LK two-point waves: the eight I-window rows of a lane's two units via buffer_load ... lds,
# one round trip per level (dma) vs base: LK parity on the variant, batch A/B
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=r03_v44
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_dma.so timeout -k 10 400 python -u -m pytest tests/test_klt_gpu.py tests/test_klt_accum_gpu.py tests/test_golden.py tests/test_graph_gpu.py tests/test_pyramid_gpu.py tests/test_profile_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab.sh $T 3 base_v dma | tee $O/ab.txt

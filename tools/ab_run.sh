# r06: side bands out of the pyramid pass (ring_kernel), side-specialised edge
# gathers -- parity tests, the pass alone, then the step against HEAD's pass
set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/${TAG:-sb1}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pyramid_gpu.py tests/test_klt_gpu.py tests/test_bench_batch_gpu.py tests/test_sequence_gpu.py tests/test_graph_gpu.py tests/test_detect_gpu.py tests/test_golden.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 60 ./tools/pyr_probe 40 q > $O/probe.txt 2>&1; head -4 $O/probe.txt
V=$PWD/ic-gvins_amd/gvx/variants
CFGS="head|GVX_LIB=$V/libgvx_head3.so|;tree||;head_nov|GVX_LIB=$V/libgvx_head3.so|--no-overlap --streams 1;tree_nov||--no-overlap --streams 1" bash tools/r06_ab.sh $TAG ${ROUNDS:-3}
for f in gpurun_out/$TAG/b_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d.get('single_pair',{}).get('us_per_pair_eager'), d.get('single_pair',{}).get('us_per_pair_graph'))"; done

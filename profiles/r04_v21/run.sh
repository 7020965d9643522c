set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v21; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_sq.so timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_factor_parity_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_sq.log 2>&1 || { tail -30 $O/tests_sq.log; exit 1; }
echo sq $(tail -1 $O/tests_sq.log)
timeout -k 10 200 python3 tools/preint_dump.py $O/base.npy > $O/dump_base.log 2>&1
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_sq.so timeout -k 10 200 python3 tools/preint_dump.py $O/sq.npy > $O/dump_sq.log 2>&1
python3 -c "import numpy as np;a=np.load('$O/base.npy');b=np.load('$O/sq.npy');print('bytes equal', a.tobytes()==b.tobytes(), a.shape)"
for r in 1 2; do for v in base sq; do
  if [ $v = base ]; then lib=""; else lib=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
  GVX_LIB="$lib" timeout -k 10 200 python3 tools/preint_loop.py > $O/loop_${v}_$r.json 2> $O/loop_${v}_$r.err || { tail -20 $O/loop_${v}_$r.err; exit 1; }
  echo $v $(python3 -c "import json;d=json.load(open('$O/loop_${v}_$r.json'));print(d['cold'],d['warm'])")
done; done
rm -f $O/*.npy

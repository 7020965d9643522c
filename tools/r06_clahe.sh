# r06 CLAHE: packed 16-bit tile histograms (1 / 2 copies)
# against the r05 layout -- parity, device time (tools/clahe_ab.py, interleaved)
# and one LDS PMC pass of fused_kernel per layout.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for v in pack1 pack2; do
  GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_clahe_fused_gpu.py > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v tests"; tail -1 $O/tests_$v.log
done
for r in 1 2 3; do
  for v in base pack1 pack2; do
    lib=""; [ $v != base ] && lib=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so
    GVX_LIB=$lib timeout -k 10 120 python3 tools/clahe_ab.py >> $O/ab_$v.jsonl 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    tail -1 $O/ab_$v.jsonl
  done
done
cd /tmp && export TMPDIR=/tmp
for v in base pack1 pack2; do
  lib=""; [ $v != base ] && lib=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so
  GVX_LIB=$lib timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_$v -- python3 $R/tools/clahe_ab.py > $O/pmc_$v.log 2>&1 || { tail -20 $O/pmc_$v.log; exit 1; }
  cd $R; python3 tools/pmc_kernel.py $O/pmc_$v fused_kernel > $O/pmc_$v.txt 2>&1 || true; cat $O/pmc_$v.txt; cd /tmp
done

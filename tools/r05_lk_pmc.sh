# PMC of klt_kernel at HEAD: instructions and cycles per
# wave with the full iteration cap and with max_iter = 0 (extraction only)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O
for it in 30 0; do
  bash tools/pmc_prog.sh $T/it$it "tools/lk_pmc.py $it 10" \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS" \
    "SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
  python3 tools/pmc_kernel.py $O/it$it klt_kernel > $O/klt_it$it.txt 2>&1 || true
  cat $O/klt_it$it.txt
done

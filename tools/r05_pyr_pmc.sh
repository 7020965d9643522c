# PMC of the pyramid pass (stream_kernel) in the configs[1] KLT step: where its
# wave cycles go after the 37-VALU row
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O
bash tools/pmc_prog.sh $T "tools/lk_pmc.py 30 10" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_SCA" \
  "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"
python3 tools/pmc_kernel.py $O stream_kernel > $O/stream_pmc.txt 2>&1 || true
cat $O/stream_pmc.txt

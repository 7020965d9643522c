set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
G2="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE"
GVX_CLAHE_FUSED1=1 bash tools/pmc_prog.sh r04_v4/f1 tools/clahe_ab.py "$G1" "$G2"
bash tools/pmc_prog.sh r04_v4/f2 tools/clahe_ab.py "$G1" "$G2"
grep -A18 -E "^fused" gpurun_out/r04_v4/f1/pmc_summary.txt gpurun_out/r04_v4/f2/pmc_summary.txt

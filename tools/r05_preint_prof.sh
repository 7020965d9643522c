# r05 preintegration diagnostics: clock probe of the covariance pass, per-kernel
# trace of the integrate leg, PMC of the covariance pass (one group per pass)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/${1:-r05_v3}; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_clk.so timeout -k 10 200 python3 tools/preint_clock.py > $O/clock.json 2> $O/clock.err || { tail -20 $O/clock.err; exit 1; }
cat $O/clock.json
bash tools/preint_prof.sh ${1:-r05_v3}/prof base r04base
cat $O/prof/*.txt 2>/dev/null | head -20 || true
bash tools/pmc_prog.sh ${1:-r05_v3}/pmc "tools/preint_loop.py" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS" "SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
for k in preint_cov16 preint_chain preint_pre; do python3 tools/pmc_kernel.py $O/pmc $k; done > $O/pmc/kernels.txt 2>&1 || true
cat $O/pmc/kernels.txt

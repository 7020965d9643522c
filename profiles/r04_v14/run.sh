set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v14; mkdir -p $O
for v in rsq rsqp dsadd dsph dsphf; do
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_factor_parity_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
echo $v $(tail -1 $O/tests_$v.log)
done
bash tools/preint_prof.sh r04_v14/prof base rsq rsqp dsadd dsph dsphf
bash tools/pmc_prog.sh r04_v14/pmc "bench.py --config 4 --no-cpu --steps 4 --warmup 1" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS" "SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
for k in preint_cov16 preint_chain preint_pre preint_rot; do python3 tools/pmc_kernel.py gpurun_out/r04_v14/pmc $k; done > gpurun_out/r04_v14/pmc/kernels.txt 2>&1 || true
cat gpurun_out/r04_v14/pmc/kernels.txt

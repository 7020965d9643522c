# r05 measurement pass after the tests: the driver's bench command, its
# rocprofv3 kernel-trace summary, FETCH/WRITE passes of the configs[1] batch and
# PMC of the preintegration kernels.  Each step has its own time limit.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); f=d['factors']; print('bench', d['value'], d['roofline']['frac'], d['roofline']['device_ms_per_step'], f['preint_steps_per_s'], f['problem_size'], d['lk_accum_cost'], d['preprocess']['roofline']['frac'])"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err)
echo prof done
bash tools/pmc.sh $T/pmc FETCH_SIZE WRITE_SIZE
echo pmc done
bash tools/pmc_prog.sh $T/ppmc "tools/preint_loop.py" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS" "SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"
for k in preint_cov16 preint_pre; do python3 tools/pmc_kernel.py $O/ppmc $k; done > $O/ppmc/kernels.txt 2>&1 || true
cat $O/ppmc/kernels.txt
echo final done

# r06 diagnostics:
#  1. LK residency timeline (diagnostic build with per-wave stamps);
#  2. LK PMC: SQ_WAVES in each pass with the instruction / cycle counters, and
#     GRBM_GUI_ACTIVE with the kernel trace for the real clock;
#  3. the r05_m1 queue abort, A/B: the full default line (CPU legs off) under
#     --pmc with profiled launches as recorded markers (GVX_PROF_MARKERS=1),
#     then as dispatch-attached events (the r05_m1 configuration) -- last,
#     because it may abort.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; T=${1:?tag}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
GVX_LIB=$R/ic-gvins_amd/gvx/variants/libgvx_klttrace.so timeout -k 10 240 python3 -u tools/lk_residency.py $O/res 300 > $O/res.log 2>&1 || { tail -20 $O/res.log; exit 1; }
cat $O/res.log | tail -3
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/lkpmc/p$i -- python3 $R/tools/lk_pmc.py 30 10 > $O/lkpmc_p$i.log 2>&1 || { tail -20 $O/lkpmc_p$i.log; exit 1; }
done
cd $R
python3 tools/pmc_kernel.py $O/lkpmc klt_kernel > $O/lkpmc/klt_it30.txt 2>&1 || true
cat $O/lkpmc/klt_it30.txt
cd /tmp
GVX_PROF_MARKERS=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/abort/markers -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-pre --no-factors > $O/abort_markers.log 2>&1 || { echo "markers run failed"; tail -30 $O/abort_markers.log; exit 1; }
echo "markers run completed"; tail -2 $O/abort_markers.log | cut -c1-300
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/abort/ext -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-pre --no-factors > $O/abort_ext.log 2>&1 || { echo "ext-event run failed"; tail -30 $O/abort_ext.log; exit 1; }
echo "ext-event run completed"; tail -2 $O/abort_ext.log | cut -c1-300

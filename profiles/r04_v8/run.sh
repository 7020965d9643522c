set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out/r04_v8; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  GVX_PREINT_COV8=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cov8_$v -- python3 $R/bench.py --config 4 --no-cpu --steps 10 --warmup 3 > $O/cov8_$v.log 2>&1
  f=$(find $O/cov8_$v -name "*kernel_stats.csv" | head -1)
  grep -i "preint" $f | cut -d, -f1-8
done

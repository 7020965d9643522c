# rocprofv3 kernel trace + stats of the configs[3] factor / preintegration legs
# Usage (through gpurun): bash tools/prof_fac.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof \
  -- python3 $R/bench.py --config 4 --no-cpu --steps 20 --warmup 10 > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;

# rocprofv3 kernel trace + stats of the configs[4] sequence replay (short sequence)
# Usage (through gpurun): bash tools/prof_seq.sh <tag> [frames]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1; F=${2:-300}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof \
  -- python3 $R/bench.py --config 5 --frames $F --no-cpu > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-4 $O/kernel_stats.csv | cut -c1-150

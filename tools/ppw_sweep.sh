# LK points-per-wave sweep: GPU parity tests + bench per setting.
# Usage: bash tools/ppw_sweep.sh <tag> <ppw>...
set -e
T=$1; shift
mkdir -p gpurun_out/$T
for p in "$@"; do
  GVX_KLT_PPW=$p timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/$T/t$p.log 2>&1
  GVX_KLT_PPW=$p timeout -k 10 200 python bench.py --no-cpu --steps 40 --warmup 30 > gpurun_out/$T/b$p.json 2> gpurun_out/$T/b$p.err
done

# Pyramid band-height variants (tools/variant.sh band40 / band48): parity, interleaved A/B, PMC traffic
set -e
mkdir -p gpurun_out/band
for b in 40 48; do
  GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_band$b.so timeout -k 10 300 python -u -m pytest tests/test_klt_gpu.py tests/test_sequence_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/band/t$b.log 2>&1 || { tail -20 gpurun_out/band/t$b.log; exit 1; }
  tail -1 gpurun_out/band/t$b.log
done
bash tools/ab.sh bandab 3 base band40 band48
for b in base 40 48; do
  L=""; [ $b != base ] && L=$PWD/ic-gvins_amd/gvx/variants/libgvx_band$b.so
  GVX_LIB=$L bash tools/pmc.sh bandpmc_$b FETCH_SIZE WRITE_SIZE
done

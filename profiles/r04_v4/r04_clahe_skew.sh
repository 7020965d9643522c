set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v6; mkdir -p $O
for r in 1 2; do
  for n in h257_t257 h264_t257 h272_t257 h257_t264 h264_t264 h272_t264; do
    L=$PWD/ic-gvins_amd/gvx/variants/libgvx_$n.so
    GVX_CLAHE_FUSED1=1 GVX_LIB=$L timeout -k 10 120 python tools/clahe_ab.py > $O/${n}_$r.json
    echo $n $(python3 -c "import json;print(round(json.load(open('$O/${n}_$r.json'))['ms_per_call'],4))")
  done
done

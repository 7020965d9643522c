set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v5; mkdir -p $O
for r in 1 2; do
  for n in base nohist nogather; do
    if [ $n = base ]; then L=""; else L=$PWD/ic-gvins_amd/gvx/variants/libgvx_$n.so; fi
    GVX_CLAHE_FUSED1=1 GVX_LIB=$L timeout -k 10 120 python tools/clahe_ab.py > $O/${n}_$r.json
    echo $n $(cat $O/${n}_$r.json)
  done
done

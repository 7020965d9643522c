set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v16; mkdir -p $O
for v in base wsf2 rsqp base wsf2 rsqp; do
  if [ $v = base ]; then lib=""; else lib=$PWD/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
  GVX_LIB="$lib" timeout -k 10 200 python3 tools/preint_loop.py > $O/loop_$v.json 2> $O/loop_$v.err || { tail -20 $O/loop_$v.err; exit 1; }
  echo $v $(cat $O/loop_$v.json)
done

set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v19; mkdir -p $O
GVX_LIB=$PWD/ic-gvins_amd/gvx/variants/libgvx_clk.so timeout -k 10 200 python3 tools/preint_clock.py > $O/clock.json 2> $O/clock.err || { tail -20 $O/clock.err; exit 1; }
cat $O/clock.json

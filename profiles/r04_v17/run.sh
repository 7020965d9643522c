set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r04_v17; mkdir -p $O
# timing probes only (wrong results by construction): no parity tests
bash tools/preint_prof.sh r04_v17/prof base fakemem norec

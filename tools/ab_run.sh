# r06: pyramid band height at HEAD (40, the default, against 56, 72 and 96 level-1 rows per wave)
set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
V=$PWD/ic-gvins_amd/gvx/variants
CFGS="b40||;b56|GVX_LIB=$V/libgvx_b56.so|;b72|GVX_LIB=$V/libgvx_b72.so|;b96|GVX_LIB=$V/libgvx_b96.so|;b72_nov|GVX_LIB=$V/libgvx_b72.so|--no-overlap --streams 1" bash tools/r06_ab.sh $TAG ${ROUNDS:-3}

#!/bin/bash
# Build libgvx with one source file replaced (or the current tree as is, when
# no replacement is given), for A/B timing on the GPU box:
#   tools/variant.sh <name> [<replacement file> [<target file in csrc>]]
# -> ic-gvins_amd/gvx/variants/libgvx_<name>.so ; select it with GVX_LIB=<path>.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; SRC=${2:-}; TGT=${3:-$(basename "${SRC:-x}")}
T=$(mktemp -d /tmp/gvx_variant_XXXX)
cp -r "$R/ic-gvins_amd/csrc/." "$T/"
rm -rf "$T/build"
if [ -n "$SRC" ]; then cp "$SRC" "$T/$TGT"; fi
mkdir -p "$R/ic-gvins_amd/gvx/variants"
make -s -C "$T" -j8 INC="$R/include" OUT="$R/ic-gvins_amd/gvx/variants/libgvx_$N.so" 2>&1 | grep -E "error" || true
rm -rf "$T"
ls -la "$R/ic-gvins_amd/gvx/variants/libgvx_$N.so"

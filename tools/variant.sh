#!/bin/bash
# Build libgvx with source files replaced (or the current tree as is, when no
# replacement is given), for A/B timing on the GPU box:
#   tools/variant.sh <name> [<replacement file> [<target file in csrc>]] ...
# (pairs may repeat; a lone replacement keeps its own file name)
# -> ic-gvins_amd/gvx/variants/libgvx_<name>.so ; select it with GVX_LIB=<path>.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
T=$(mktemp -d /tmp/gvx_variant_XXXX)
cp -r "$R/ic-gvins_amd/csrc/." "$T/"
rm -rf "$T/build"
while [ $# -gt 0 ]; do
  SRC=$1; TGT=${2:-$(basename "$1")}
  cp "$SRC" "$T/$TGT"
  shift; [ $# -gt 0 ] && shift
done
mkdir -p "$R/ic-gvins_amd/gvx/variants"
make -s -C "$T" -j8 EXTRA="$EXTRA" INC="$R/include" OUT="$R/ic-gvins_amd/gvx/variants/libgvx_$N.so" 2>&1 | grep -E "error" || true
rm -rf "$T"
ls -la "$R/ic-gvins_amd/gvx/variants/libgvx_$N.so"

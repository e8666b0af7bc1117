#!/bin/bash
# Build the library from a git revision (default HEAD) into
# halo2_svd041_amd/libsvdw_base.so, for same-box A/B runs against the working
# tree's build (tools/ab_lib.sh).
set -eu
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" halo2_svd041_amd/csrc include | tar -x -C "$TMP"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-function \
  -I"$TMP/include" -o "$ROOT/halo2_svd041_amd/libsvdw_base.so" \
  $(ls "$TMP"/halo2_svd041_amd/csrc/*.hip) "$TMP/halo2_svd041_amd/csrc/engine.cpp"
rm -rf "$TMP"
echo "built libsvdw_base.so from $REV"

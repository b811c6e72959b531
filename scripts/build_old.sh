#!/bin/bash
# Build the library of a git revision (default HEAD) into build/lib_old for scripts/ab_libs.sh.
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" gym-flock_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$ROOT/build/lib_old"
cd "$TMP/gym-flock_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result -Wno-unused-value -I"$TMP/include" -shared \
  -o "$ROOT/build/lib_old/libgymflock.so" flock_kernels.hip capi.hip coverage_kernels.hip coverage_expert.hip \
  cov_capi.hip graph_utils.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$TMP"
echo "built build/lib_old from $REV"

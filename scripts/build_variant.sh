#!/bin/bash
# Build the working tree's library with extra compiler flags into build/lib_<NAME>/ for
# A/B runs (scripts/ab_knn_libs.sh):  bash scripts/build_variant.sh w6 -DGF_STEP_WAVES_KNN=6
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/build/lib_$NAME"
cd "$ROOT/gym-flock_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result -Wno-unused-value -I"$ROOT/include" "$@" -shared \
  -o "$ROOT/build/lib_$NAME/libgymflock.so" flock_kernels.hip capi.hip coverage_kernels.hip coverage_expert.hip coverage_maps.hip \
  cov_capi.hip graph_utils.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built build/lib_$NAME ($*)"

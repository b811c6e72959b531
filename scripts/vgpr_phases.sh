#!/bin/bash
# Per-phase register study of the step kernel (CPU only, no GPU): flock_kernels.hip compiled
# once per phase with that phase removed at compile time (-DGF_CT_ABLATE=<mask>, the diag
# build's ablation switches as constants, csrc/flock_internal.h), each build's
# -Rpass-analysis=kernel-resource-usage summarised by scripts/resusage.py for the kernel
# instantiations named in $WANT. Usage: bash scripts/vgpr_phases.sh OUT_DIR [jobs]
set -e
cd "$(dirname "$0")/.."
O=${1:-build/vgpr_phases}
J=${2:-6}
mkdir -p "$O"
HIPCC=/opt/rocm/bin/hipcc
FLAGS="${EXTRA:-} -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Iinclude -c gym-flock_amd/csrc/flock_kernels.hip -Rpass-analysis=kernel-resource-usage"
# mask: phase removed (flock_kernels.hip's GF_ABLATE sites)
PHASES="0:none 1:knn_merge_and_outputs 2:feature_pass 32:neighbour_gather 256:row_outputs 0x200000:key_insertion 0x20000:predicted_rows 0x40000:inline_rim 8:pass1 16:tile_staging 0x200021:insertion+merge+gather"
run() {
  local m=${1%%:*} n=${1#*:}
  $HIPCC $FLAGS -DGF_CT_ABLATE=$m -o "$O/$n.o" 2> "$O/$n.log" || echo "build $n failed"
}
export -f run; export HIPCC FLAGS O
printf '%s\n' $PHASES | xargs -P "$J" -I{} bash -c 'run "$@"' _ {}
for p in $PHASES; do
  n=${p#*:}
  echo "== $n (GF_CT_ABLATE=${p%%:*})"
  python scripts/resusage.py "$O/$n.log" flock_step_kernel | grep -E "${WANT:-ILb1ELb0ELb0ELb0ELi0ELi7ELb0ELi0E|ILb1ELb0ELb0ELb0ELi0ELi0ELb0ELi0E}" || true
done

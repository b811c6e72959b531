#!/bin/bash
# VGPRs / spills / occupancy of the Flocking-v0 step instantiations (KN = 7, and the exact
# small-env KX = 7) for a build variant (extra -D flags as arguments), device code only.
cd "$(dirname "$0")/../gym-flock_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off --cuda-device-only -I../../include "$@" \
  -c flock_kernels.hip -o /tmp/vgpr_knn.o -Rpass-analysis=kernel-resource-usage 2> /tmp/vgpr_knn.log
python ../../scripts/resusage.py /tmp/vgpr_knn.log step | grep -E "Li0ELi7ELb0ELi0E|Li0ELi0ELb0ELi0E" | grep "ILb1ELb0E"

#!/bin/bash
# VGPRs / occupancy of the step kernel instantiations for a build variant (extra -D flags
# as arguments), device code only: bash scripts/vgpr.sh [-DFOO=1 ...]
cd "$(dirname "$0")/../gym-flock_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off --cuda-device-only -I../../include "$@" \
  -c flock_kernels.hip -o /tmp/vgpr_probe.o -Rpass-analysis=kernel-resource-usage 2> /tmp/vgpr_probe.log
python ../../scripts/resusage.py /tmp/vgpr_probe.log step | grep -E "Li7E|Lb0ELi0ELi0E" | grep "ILb1ELb0E"

#!/bin/bash
# Instruction counts (PMC) of the Flocking-v0 step on HEAD (lib_base), the balanced feature
# pass (lib_list) and lean pair terms (lib_lean): does the list cut VALU issue?
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/s29
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
for n in base list lean; do
  GYMFLOCK_LIB=$PWD/build/lib_$n/libgymflock.so KNN=1 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/k_$n -o pmc -- python3 scripts/pmc_step.py > $O/k_$n.log 2>&1
done
python3 scripts/pmc_mix.py $O

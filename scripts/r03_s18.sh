#!/bin/bash
# Instruction mix (SQ counters) of the current build's step kernels: plain, controller,
# Flocking-v0, N=8192 (one launch per step, 5 steps), one rocprofv3 --pmc pass each.
set -e
export TMPDIR=/tmp
O=$PWD/gpurun_out/s18
rm -rf $O; mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$n -o pmc -- python3 scripts/pmc_step.py > $O/$n.log 2>&1
}
run plain X=1 && run ctrl MODE=ctrl && run knn KNN=1 && run n8192 N=8192 B=32
python scripts/pmc_mix.py $O

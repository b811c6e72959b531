#!/bin/bash
# Round 5, session 20: per-wave instruction mix (PMC) of the product build's step kernels:
# plain, step + controller, Flocking-v0 (scripts/pmc_mix.py summarises).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r05_s20; mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
cd /tmp
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$n -o pmc -- python3 $R/scripts/pmc_step.py > $O/$n.log 2>&1
}
run plain MODE=plain && run ctrl MODE=ctrl && run knn KNN=1
r=$?; echo "pmc rc=$r"
cd $R && python scripts/pmc_mix.py $O
exit $r

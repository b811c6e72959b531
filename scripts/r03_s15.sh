#!/bin/bash
# VALU/SALU/LDS instruction counts of the step kernels with parts switched off (diagnostic
# build, fe_diag switches), one rocprofv3 --pmc pass per configuration.
set -e
export TMPDIR=/tmp
O=$PWD/gpurun_out/${S15_OUT:-s15}
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$n -o pmc -- python3 scripts/pmc_step.py > $O/$n.log 2>&1
}
run p_all DIAG=0 && run p_nofeat DIAG=2 && run p_nopass1 DIAG=8 && run p_nostage DIAG=16 && run p_conststore DIAG=1024 && run p_norowout DIAG=256 &&
run k_all KNN=1 DIAG=0 && run k_nomerge KNN=1 DIAG=1 && run k_noinsert KNN=1 DIAG=0x200000 && run k_nopred KNN=1 DIAG=0x20000 &&
run k_nogather KNN=1 DIAG=32 && run k_nofeat KNN=1 DIAG=2 && run k_norim KNN=1 DIAG=0x40000
echo "rc=$?"

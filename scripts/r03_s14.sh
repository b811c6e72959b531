#!/bin/bash
# Instruction mix of the plain and Flocking-v0 step kernels (one launch per step, 5 steps):
# SQ instruction/cycle counters + GRBM_GUI_ACTIVE, one rocprofv3 --pmc pass each.
set -e
export TMPDIR=/tmp
O=$PWD/gpurun_out/s14
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/plain -o pmc -- python3 scripts/pmc_step.py > $O/plain.log 2>&1
KNN=1 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/knn -o pmc -- python3 scripts/pmc_step.py > $O/knn.log 2>&1
C2="SQ_INSTS_VALU_FLOPS_FP64 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"
timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $O/plain2 -o pmc -- python3 scripts/pmc_step.py > $O/plain2.log 2>&1 || echo "pass2 plain rc=$?"
KNN=1 timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $O/knn2 -o pmc -- python3 scripts/pmc_step.py > $O/knn2.log 2>&1 || echo "pass2 knn rc=$?"
ls -R $O | head -30

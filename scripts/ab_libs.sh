#!/bin/bash
# Cross-build A/B: alternate processes of scripts/ab_kernels.py on the baseline library
# (build/lib_old) and the working tree's, same box, ROUNDS each. Extra arguments are
# passed to the working tree's runs as ab_kernels configs (default: "new:").
set -e
mkdir -p gpurun_out
NEW=("${@:-new:}")
for i in 1 2 3; do
  GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so ROUNDS=4 timeout -k 10 200 python scripts/ab_kernels.py "old:" > gpurun_out/ab_old_$i.log 2>&1
  ROUNDS=4 timeout -k 10 200 python scripts/ab_kernels.py "${NEW[@]}" > gpurun_out/ab_new_$i.log 2>&1
  grep -h "step" gpurun_out/ab_old_$i.log gpurun_out/ab_new_$i.log | grep -v identical
done

#!/bin/bash
# Plain step at 7 workgroups per CU (7-wave register budget, no LDS floor, rows read one
# at a time) against HEAD (6 per CU): headline-only bench A/B, 3 rounds, both 20 and 200 steps.
set -e
mkdir -p gpurun_out
X="--no-controller-line --no-packed-line --no-knn-line --no-other-configs"
ROUNDS=3 NEWLIB=$PWD/build/lib_w7/libgymflock.so bash scripts/ab_bench.sh $X > gpurun_out/s22_ab20.txt 2>&1
cat gpurun_out/s22_ab20.txt | grep -v "^setup\|^config\|^drop"

#!/bin/bash
# Step-kernel geometry sweep (rows per block x tile) with scripts/ablate.py QUICK rounds.
set -e
mkdir -p gpurun_out
for R in ${ROWS:-16 32 64}; do
  for T in ${TILES:-512 1024}; do
    GYMFLOCK_ROWS=$R GYMFLOCK_TILE=$T QUICK=1 ROUNDS=${ROUNDS:-5} timeout -k 10 120 python scripts/ablate.py > gpurun_out/sweep_R${R}_T${T}.log 2>&1
    echo "R=$R T=$T $(grep -E '^full' gpurun_out/sweep_R${R}_T${T}.log)"
  done
done

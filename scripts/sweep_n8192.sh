#!/bin/bash
# Geometry sweep (rows per block x tile) of the step kernel at config 5 (N=8192 x 32 envs).
mkdir -p gpurun_out
for R in ${ROWS:-4 8 16}; do
  for T in ${TILES:-256 512 1024}; do
    GYMFLOCK_ROWS=$R GYMFLOCK_TILE=$T timeout -k 10 120 python bench.py --n-agents 8192 --n-envs 32 --steps 10 --warmup 2 \
      --no-cpu-baseline --no-controller-line --no-packed-line > gpurun_out/sw8192_R${R}_T${T}.log 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/sw8192_R${R}_T${T}.log').read().strip().splitlines()[-1]); print('R=$R T=$T', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))"
  done
done

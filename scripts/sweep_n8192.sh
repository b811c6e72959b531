#!/bin/bash
# Geometry sweep of the step kernel at config 5 (N=8192 x 32 envs).
# CONFIGS: space-separated ROWS:TILE[:LDS_FLOOR] triples (LDS_FLOOR in bytes, 0 = no floor).
mkdir -p gpurun_out
for c in ${CONFIGS:-16:512 16:256 8:512 8:256 8:256:0 4:256:0 16:128 16:128:0 32:256}; do
  IFS=: read -r R T F <<< "$c"
  tag="R${R}_T${T}_F${F:-d}"
  env GYMFLOCK_ROWS=$R GYMFLOCK_TILE=$T ${F:+GYMFLOCK_LDS_FLOOR=$F} \
    timeout -k 10 120 python bench.py --n-agents 8192 --n-envs 32 --steps ${STEPS:-10} --warmup 2 \
    --no-cpu-baseline --no-controller-line --no-packed-line --no-knn-line > gpurun_out/sw8192_${tag}.log 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/sw8192_${tag}.log').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))"
done

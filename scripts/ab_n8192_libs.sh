#!/bin/bash
# Config 5 (N=8192 x 32 envs, plain step) on several libraries, interleaved, ROUNDS rounds:
#   bash scripts/ab_n8192_libs.sh tree gb16     (build/lib_<name>; "tree" = in-tree lib)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for n in "$@"; do
    lib=$PWD/build/lib_$n/libgymflock.so; [ "$n" = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
    GYMFLOCK_LIB=$lib timeout -k 10 150 python bench.py --n-agents 8192 --n-envs 32 --steps ${STEPS:-20} --warmup 3 \
      --no-cpu-baseline --no-controller-line --no-packed-line --no-knn-line > gpurun_out/ab8192_$n.log 2>/dev/null || { echo "$n failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab8192_$n.log').read().strip().splitlines()[-1]); print('round $r $n', round(d['ms_per_step'],4), 'ms', round(d['roofline']['frac'],3))"
  done
done

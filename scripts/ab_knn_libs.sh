#!/bin/bash
# Flocking-v0 line (scripts/knn_line.py: clock warm-up, reset, 5 warm-up steps, timed
# steps) on several libraries, interleaved, ROUNDS rounds, 20- and 200-step windows:
#   bash scripts/ab_knn_libs.sh base w6        (build/lib_<name>/libgymflock.so; "tree" = in-tree lib)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq ${ROUNDS:-3}); do
  for n in "$@"; do
    lib=$PWD/build/lib_$n/libgymflock.so; [ "$n" = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
    for s in 20 200; do
      out=$(GYMFLOCK_LIB=$lib KSTEPS=$s WARM=5 timeout -k 10 120 python scripts/knn_line.py 2>&1) || { echo "$n failed: $out"; exit 1; }
      echo "round $r $n steps=$s $(echo "$out" | tail -1)"
    done
  done
done

#!/bin/bash
# Flocking-v0 line under the diagnostic build's ablation switches (fe_diag), interleaved,
# 20- and 200-step windows:  bash scripts/knn_diag_line.sh 0 0x400 0x401 ...
# ("plain" = the FlockingRelative step without kNN)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export GYMFLOCK_LIB=$PWD/build/lib_diag/libgymflock.so
for r in $(seq ${ROUNDS:-2}); do
  for d in "$@"; do
    for s in 20 200; do
      if [ "$d" = plain ]; then out=$(KNN=0 KSTEPS=$s WARM=5 timeout -k 10 120 python scripts/knn_line.py 2>&1)
      else out=$(DIAG=$d KSTEPS=$s WARM=5 timeout -k 10 120 python scripts/knn_line.py 2>&1); fi || { echo "$d failed: $out"; exit 1; }
      echo "round $r diag=$d steps=$s $(echo "$out" | tail -1)"
    done
  done
done

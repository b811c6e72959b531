#!/bin/bash
# FlockingRelative step (scripts/knn_line.py with KNN=0) on several libraries, interleaved:
#   bash scripts/ab_plain_libs.sh tree f28       (build/lib_<name>; "tree" = in-tree lib)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq ${ROUNDS:-3}); do
  for n in "$@"; do
    lib=$PWD/build/lib_$n/libgymflock.so; [ "$n" = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
    for s in 20 200; do
      out=$(GYMFLOCK_LIB=$lib KNN=0 KSTEPS=$s WARM=5 timeout -k 10 120 python scripts/knn_line.py 2>&1) || { echo "$n failed: $out"; exit 1; }
      echo "round $r $n steps=$s $(echo "$out" | tail -1)"
    done
  done
done

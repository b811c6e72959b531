#!/bin/bash
# Greedy expert step (scripts/time_greedy.py) on several libraries, interleaved:
#   bash scripts/ab_greedy_libs.sh tree g4      (build/lib_<name>; "tree" = in-tree lib)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq ${ROUNDS:-3}); do
  for n in "$@"; do
    lib=$PWD/build/lib_$n/libgymflock.so; [ "$n" = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
    GYMFLOCK_LIB=$lib ROUNDS=3 timeout -k 10 150 python scripts/time_greedy.py "$n" 2>&1 | tail -1 || exit 1
  done
done

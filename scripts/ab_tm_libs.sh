#!/bin/bash
# Time-matrix build (scripts/time_tm.py) on several libraries, interleaved:
#   bash scripts/ab_tm_libs.sh base tree      (build/lib_<name>; "tree" = in-tree lib)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq ${ROUNDS:-3}); do
  for n in "$@"; do
    lib=$PWD/build/lib_$n/libgymflock.so; [ "$n" = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
    GYMFLOCK_LIB=$lib timeout -k 10 120 python scripts/time_tm.py "$n" 2>&1 | tail -1 || exit 1
  done
done

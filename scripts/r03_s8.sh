#!/bin/bash
# Round-3 session 8: the store skeleton of the tiled step at N=8192 (diagnostic build):
# what the network stores alone cost, to bound what any compute restructuring can win.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do
  for d in 0 0x1A 0x41A 0x71A; do
    GYMFLOCK_LIB=$PWD/build/lib_diag/libgymflock.so DIAG=$d N=8192 B=32 K=20 timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1
  done
  for d in 0 0x1A 0x41A 0x71A; do
    GYMFLOCK_LIB=$PWD/build/lib_diag/libgymflock.so DIAG=$d N=1024 B=256 K=100 timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1
  done
  GYMFLOCK_LIB=$PWD/gym-flock_amd/lib/libgymflock.so N=8192 B=32 K=20 timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1 | sed "s/^/grid /"
done

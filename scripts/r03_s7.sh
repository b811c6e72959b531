#!/bin/bash
# Round-3 session 7: cell-list step, one vs two launches per step, vs the tiled kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s7; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_grid_step_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_grid.log 2>&1 || { tail -40 $O/pytest_grid.log; exit 1; }
tail -1 $O/pytest_grid.log
for r in 1 2; do
for lib in old tree; do for st in 1 2; do
  GYMFLOCK_LIB=$PWD/build/lib_$lib/libgymflock.so N=8192 B=32 STREAMS=$st timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1 | sed "s/^/$lib /"
done; done
for lib in old grid1k; do for st in 1 2; do
  GYMFLOCK_LIB=$PWD/build/lib_$lib/libgymflock.so N=1024 B=256 K=100 STREAMS=$st timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1 | sed "s/^/$lib /"
done; done
done

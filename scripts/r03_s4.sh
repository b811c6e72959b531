#!/bin/bash
# Round-3 session 4: wide-env cell-list step: parity, then config 5 against the tiled build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s4; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_grid_step_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_grid.log 2>&1 || { tail -40 $O/pytest_grid.log; exit 1; }
tail -12 $O/pytest_grid.log
ROUNDS=3 timeout -k 10 600 bash scripts/ab_n8192_libs.sh old tree > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc

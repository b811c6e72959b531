#!/bin/bash
# Greedy expert geometry after the SWAR search: lanes per robot and loads in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s37; mkdir -p $O
set -o pipefail
GYMFLOCK_LIB=$PWD/build/lib_l4/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_coverage_greedy_gpu.py > $O/pytest_l4.txt 2>&1 || { tail -30 $O/pytest_l4.txt; exit 1; }
tail -1 $O/pytest_l4.txt
ROUNDS=2 bash scripts/ab_greedy_libs.sh tree l4 if2 l4if8 l16 2>&1 | tee $O/ab_greedy.txt

#!/bin/bash
# Greedy expert: bounded block search over the cost row (in-tree lib) vs the whole-row scan
# (lib_gscan): Coverage GPU tests on the in-tree lib, then expert-step and time-matrix A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s34; mkdir -p $O
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py > $O/pytest_cov.txt 2>&1 || { tail -30 $O/pytest_cov.txt; exit 1; }
tail -1 $O/pytest_cov.txt
ROUNDS=3 bash scripts/ab_greedy_libs.sh tree gscan 2>&1 | tee $O/ab_greedy.txt
for n in tree gscan; do
  lib=$PWD/build/lib_$n/libgymflock.so; [ "$n" = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$lib timeout -k 10 200 python scripts/time_tm.py $n 2>&1 | tail -1 | tee -a $O/ab_tm.txt
done

#!/bin/bash
# Fused kNN step with the plain step's paired row reads in pass 1 (GF_P1_PAIR_KNN):
# flock GPU tests on it, then Flocking-v0 A/B against HEAD (lib_base), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s31; mkdir -p $O
set -o pipefail
GYMFLOCK_LIB=$PWD/build/lib_pair/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_flock_gpu.py > $O/pytest_pair.txt 2>&1 || { tail -30 $O/pytest_pair.txt; exit 1; }
tail -1 $O/pytest_pair.txt
ROUNDS=3 bash scripts/ab_knn_libs.sh base pair 2>&1 | tee $O/ab_knn.txt

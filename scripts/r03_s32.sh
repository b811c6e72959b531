#!/bin/bash
# Fused kNN step: paired row reads (lib_pair) and, on top, the predicted rows' candidate
# bounds and order from LDS tables with the mostly-predicted loop paired too (lib_ptab):
# flock GPU tests on lib_ptab, then Flocking-v0 A/B against HEAD (lib_base), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s32; mkdir -p $O
set -o pipefail
GYMFLOCK_LIB=$PWD/build/lib_ptab/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py > $O/pytest_ptab.txt 2>&1 || { tail -30 $O/pytest_ptab.txt; exit 1; }
tail -1 $O/pytest_ptab.txt
ROUNDS=3 bash scripts/ab_knn_libs.sh base pair ptab 2>&1 | tee $O/ab_knn.txt

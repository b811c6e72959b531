#!/bin/bash
# Fused kNN merge with the exactness tests after the rounds (in-tree, GF_KNN_MERGE_LEAN=1)
# vs per round (lib_mold): flock GPU tests on the in-tree lib, then Flocking-v0 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s38; mkdir -p $O
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py > $O/pytest_flock.txt 2>&1 || { tail -30 $O/pytest_flock.txt; exit 1; }
tail -1 $O/pytest_flock.txt
ROUNDS=3 bash scripts/ab_knn_libs.sh tree mold 2>&1 | tee $O/ab_knn.txt

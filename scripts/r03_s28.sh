#!/bin/bash
# Balanced feature pass (GF_FEAT_LIST: a row's pairs listed in LDS, dealt round robin over
# its slices) and lean pair terms (GF_PAIR_LEAN): flock/kNN GPU tests on the changed build,
# then Flocking-v0 and plain-step A/B, interleaved, against HEAD (lib_base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s28; mkdir -p $O
set -o pipefail
GYMFLOCK_LIB=$PWD/build/lib_listlean/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py > $O/pytest_listlean.txt 2>&1 || { tail -30 $O/pytest_listlean.txt; exit 1; }
tail -1 $O/pytest_listlean.txt
ROUNDS=2 bash scripts/ab_knn_libs.sh base list lean listlean 2>&1 | tee $O/ab_knn.txt
ROUNDS=2 bash scripts/ab_plain_libs.sh base lean 2>&1 | tee $O/ab_plain.txt

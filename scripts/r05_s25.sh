#!/bin/bash
# Deferred kNN ranking A/B (GF_KNN_DEFER): kNN GPU tests on the variants, then the
# Flocking-v0 line interleaved over base / noinl / d1 / d2 / d2i.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s25; mkdir -p $O
for v in d2 d2i; do
  GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_flock_gpu.py -m gpu -k "knn or flocking_v0 or Flocking" > $O/tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
ROUNDS=2 timeout -k 10 700 bash scripts/ab_knn_libs.sh base noinl d1 d2 d2i 2>&1 | tee $O/ab.txt

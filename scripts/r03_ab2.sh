#!/bin/bash
# Round-3 A/B: N=8192 adjacency bits in a global scratch (L2) instead of LDS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ab2; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
for v in gb16 gb32; do
  GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "config5" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
ROUNDS=3 timeout -k 10 900 bash scripts/ab_n8192_libs.sh tree gb16 gb32 gb16w6 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc

#!/bin/bash
# Round-3 A/B: fused-kNN list insertion (med3) and rcp+Newton reciprocal; parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ab1; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ROUNDS=3 timeout -k 10 900 bash scripts/ab_knn_libs.sh base med3 tree nr2 > $O/ab_knn.txt 2>&1 || { cat $O/ab_knn.txt; exit 1; }
cat $O/ab_knn.txt
ROUNDS=2 timeout -k 10 600 bash scripts/ab_plain_libs.sh base tree nr2 > $O/ab_plain.txt 2>&1 || { cat $O/ab_plain.txt; exit 1; }
cat $O/ab_plain.txt
for o in 0 1; do OTHER=$([ $o = 1 ] && echo 1) KSTEPS=200 WARM=5 timeout -k 10 120 python scripts/knn_line.py > $O/other$o.txt 2>&1; echo "other=$o $(tail -1 $O/other$o.txt)"; done

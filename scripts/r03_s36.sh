#!/bin/bash
# Greedy expert, uint8 rows: four targets per 32-bit operation (SWAR, in-tree lib) vs one
# (lib_gold = HEAD): Coverage GPU tests on the in-tree lib, then the expert-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s36; mkdir -p $O
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py > $O/pytest_cov.txt 2>&1 || { tail -30 $O/pytest_cov.txt; exit 1; }
tail -1 $O/pytest_cov.txt
ROUNDS=3 bash scripts/ab_greedy_libs.sh ${LIBS:-tree gold} 2>&1 | tee $O/ab_greedy.txt

#!/bin/bash
# Branch-free one-Newton reciprocal for the feature pair terms: GPU suite, bench A/B vs HEAD.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s17_pytest.txt 2>&1 || { tail -30 gpurun_out/s17_pytest.txt; exit 1; }
tail -2 gpurun_out/s17_pytest.txt
ROUNDS=2 bash scripts/ab_bench.sh > gpurun_out/s17_ab.txt 2>&1
cat gpurun_out/s17_ab.txt

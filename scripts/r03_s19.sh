#!/bin/bash
# Coverage: hipLaunchKernel + bound Python call (host-bound split step): Coverage tests,
# time_cov A/B against HEAD's library (old Python path too: the tree's Python is used).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py > gpurun_out/s19_pytest.txt 2>&1
tail -1 gpurun_out/s19_pytest.txt
bash scripts/ab_cov_multi.sh > gpurun_out/s19_ab.txt 2>&1
cat gpurun_out/s19_ab.txt

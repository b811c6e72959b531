#!/bin/bash
# Coverage node records: GPU Coverage tests, interleaved A/B against HEAD's library, timeline.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py > gpurun_out/s10_pytest.txt 2>&1
tail -2 gpurun_out/s10_pytest.txt
bash scripts/ab_cov_multi.sh lds0 nt128 > gpurun_out/s10_ab.txt 2>&1
cat gpurun_out/s10_ab.txt
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/s10_timeline.txt 2>&1
cat gpurun_out/s10_timeline.txt

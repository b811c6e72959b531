#!/bin/bash
# Coverage: fewer dirty lines per step (constant tail stores skipped). GPU Coverage tests,
# A/B (split and one launch per step) against HEAD and the no-skip build, timeline.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py > gpurun_out/s13_pytest.txt 2>&1
tail -1 gpurun_out/s13_pytest.txt
bash scripts/ab_cov_multi.sh noskip > gpurun_out/s13_ab.txt 2>&1
for i in 1 2; do
  STREAMS=1 GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so timeout -k 10 200 python scripts/time_cov.py old-one
  STREAMS=1 timeout -k 10 200 python scripts/time_cov.py new-one
done >> gpurun_out/s13_ab.txt 2>&1
cat gpurun_out/s13_ab.txt
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/s13_timeline.txt 2>&1

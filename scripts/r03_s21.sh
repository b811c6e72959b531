#!/bin/bash
# Config 5 network store column-block-major: wide-env GPU tests, then N=8192 x 32 step
# time A/B (scripts/time_grid.py, two launches per step) against HEAD's library, plus the
# 8 GiB store probe of this box.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_wide_step_gpu.py tests/test_flock_gpu.py > gpurun_out/s21_pytest.txt 2>&1 || { tail -30 gpurun_out/s21_pytest.txt; exit 1; }
tail -1 gpurun_out/s21_pytest.txt
for i in 1 2 3; do
  GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so K=40 timeout -k 10 200 python scripts/time_grid.py 2>&1 | sed 's/^/old /'
  K=40 timeout -k 10 200 python scripts/time_grid.py 2>&1 | sed 's/^/new /'
done
hipcc -O3 --offload-arch=gfx950 scripts/storeprobe.hip -o /tmp/sp && timeout -k 10 200 /tmp/sp

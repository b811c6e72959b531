#!/bin/bash
# Contiguous buffers: config-5 store order A/B (row after row = HEAD vs column-block-major),
# wide-step tests on the block-major build, store probes in contiguous and default memory.
set -e
mkdir -p gpurun_out
GYMFLOCK_LIB=$PWD/build/lib_bm/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_wide_step_gpu.py > gpurun_out/s26_pytest.txt 2>&1 || { tail -30 gpurun_out/s26_pytest.txt; exit 1; }
tail -1 gpurun_out/s26_pytest.txt
for i in 1 2 3; do
  GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so K=40 timeout -k 10 200 python scripts/time_grid.py 2>&1 | sed 's/^/row-major /'
  GYMFLOCK_LIB=$PWD/build/lib_bm/libgymflock.so K=40 timeout -k 10 200 python scripts/time_grid.py 2>&1 | sed 's/^/block-major /'
done
hipcc -O3 --offload-arch=gfx950 scripts/storeprobe.hip -o /tmp/sp
timeout -k 10 100 /tmp/sp c
timeout -k 10 100 /tmp/sp m

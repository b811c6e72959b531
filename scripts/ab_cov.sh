#!/bin/bash
# Cross-build A/B of the Coverage step: alternate processes of scripts/time_cov.py on
# the baseline library (build/lib_old) and the working tree's, same box.
set -e
mkdir -p gpurun_out
for i in 1 2 3; do
  GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so timeout -k 10 200 python scripts/time_cov.py old
  timeout -k 10 200 python scripts/time_cov.py new
done

#!/bin/bash
# Contiguous output buffers (>= 256 MiB): bench A/B (headline and config 5) against HEAD.
set -e
mkdir -p gpurun_out
X="--no-controller-line --no-packed-line --no-knn-line"
ROUNDS=3 bash scripts/ab_bench.sh $X > gpurun_out/s25_ab.txt 2>&1
grep -v "^setup\|^config\|^drop" gpurun_out/s25_ab.txt

#!/bin/bash
# Coverage claim rounds tagged (no clears) with in-order LDS: A/B and both timelines.
set -e
mkdir -p gpurun_out
bash scripts/ab_cov_multi.sh covtag > gpurun_out/s20_ab.txt 2>&1
cat gpurun_out/s20_ab.txt
for v in stamps1 stamps_tag; do
  GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/s20_timeline_$v.json 2>&1
done

#!/bin/bash
# Cross-build A/B of the bench lines: bench.py (driver window: 20 steps after 5 warm-up
# steps, no CPU baseline) alternating HEAD's library (build/lib_old) and the working
# tree's (or NEWLIB's), ROUNDS times; one JSON line per run into
# gpurun_out/ab_bench_{old,new}.jsonl.
set -e
mkdir -p gpurun_out
: > gpurun_out/ab_bench_old.jsonl
: > gpurun_out/ab_bench_new.jsonl
for i in $(seq ${ROUNDS:-2}); do
  GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" >> gpurun_out/ab_bench_old.jsonl
  GYMFLOCK_LIB=${NEWLIB:-$PWD/gym-flock_amd/lib/libgymflock.so} timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" >> gpurun_out/ab_bench_new.jsonl
done
python scripts/ab_bench_report.py gpurun_out/ab_bench_old.jsonl gpurun_out/ab_bench_new.jsonl

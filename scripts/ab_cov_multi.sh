#!/bin/bash
# Coverage step A/B over HEAD (build/lib_old), the working tree and build variants given as
# arguments (build/lib_<name>), interleaved processes on one box, 3 rounds.
set -e
for i in 1 2 3; do
  GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so timeout -k 10 200 python scripts/time_cov.py old
  for v in "$@"; do
    GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 200 python scripts/time_cov.py $v
  done
  timeout -k 10 200 python scripts/time_cov.py new
done

#!/bin/bash
# Cross-build A/B of the greedy expert step (scripts/time_greedy.py): baseline library
# build/lib_old vs the working tree's, alternating processes on one box.
set -e
for i in 1 2 3; do
  GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so timeout -k 10 200 python scripts/time_greedy.py old
  timeout -k 10 200 python scripts/time_greedy.py new
done

#!/bin/bash
# Multi-wave time-matrix passes for launches of few chunks: Coverage GPU tests on the tree
# (the drop-in and small-batch matrices now take it), then the drop-in first-step probe and
# the config-4 matrices, tree vs the one-wave form (GF_TM_FEW_CHUNKS=0), two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s27; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py -m gpu > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in tree tm1w; do
    lib=$PWD/build/lib_$v/libgymflock.so; [ $v = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
    GYMFLOCK_LIB=$lib timeout -k 10 120 python scripts/cov_first_step_probe.py > $O/probe_${v}_$r.txt 2>&1 || exit 1
    echo "$v round $r first steps: $(grep 'step 0' $O/probe_${v}_$r.txt | awk '{print $5}' | tr '\n' ' ')"
  done
done
GYMFLOCK_LIB=$PWD/gym-flock_amd/lib/libgymflock.so R=200 timeout -k 10 120 python scripts/cov_first_step_probe.py > $O/probe_r200.txt 2>&1 || exit 1
echo "tree R=200 first steps: $(grep 'step 0' $O/probe_r200.txt | awk '{print $5}' | tr '\n' ' ')"

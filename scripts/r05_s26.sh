#!/bin/bash
# Time-matrix schedule kernel (staged in LDS) and batch width A/B: Coverage GPU tests on
# the tree, then the drop-in first-step probe and the config-4 time matrix per library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s26; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py -m gpu > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
GYMFLOCK_LIB=$PWD/build/lib_tb16/libgymflock.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_coverage_greedy_gpu.py -m gpu > $O/tests_tb16.log 2>&1
rc=$?; echo "tests tb16 rc=$rc $(tail -1 $O/tests_tb16.log)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in tb8 tb16; do
    GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 120 python scripts/cov_first_step_probe.py > $O/probe_${v}_$r.txt 2>&1 || exit 1
    echo "$v round $r first steps: $(grep 'step 0' $O/probe_${v}_$r.txt | awk '{print $5}' | tr '\n' ' ')"
    GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 300 python bench.py --workload coverage --steps 50 --warmup 10 --no-cpu-baseline > $O/cov_${v}_$r.json 2> $O/cov_${v}_$r.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$v round $r tm_all_envs_ms', round(d['greedy_expert']['time_matrix_ms_all_envs'],2))" $O/cov_${v}_$r.json
  done
done

#!/bin/bash
# Round-3 session 9: Coverage claim rounds tagged vs cleared (A/B, same box), the packed
# line's PMC, the Coverage timeline of the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r03s9; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
GYMFLOCK_LIB=$R/build/lib_covtag/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_coverage_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_covtag.log 2>&1 || { tail -30 $O/pytest_covtag.log; exit 1; }
tail -1 $O/pytest_covtag.log
for i in 1 2 3 4; do
  timeout -k 10 200 python scripts/time_cov.py tree 2>&1 | tail -1
  GYMFLOCK_LIB=$R/build/lib_covtag/libgymflock.so timeout -k 10 200 python scripts/time_cov.py tagged 2>&1 | tail -1
done
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  MODE=packed timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_packed_$c -o pmc -- python3 $R/scripts/pmc_step.py > $O/pmc_packed_$c.log 2>&1 || exit 1
done
echo pmc ok

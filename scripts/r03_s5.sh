#!/bin/bash
# Round-3 session 5: cell-list step after the parallel prep scan: parity, config-5 A/B,
# rocprofv3 kernel stats of the config-5 line, and config 2 through the cell list (A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s5; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_grid_step_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_grid.log 2>&1 || { tail -40 $O/pytest_grid.log; exit 1; }
tail -1 $O/pytest_grid.log
ROUNDS=3 timeout -k 10 600 bash scripts/ab_n8192_libs.sh old tree > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8192 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n-agents 8192 --n-envs 32 --steps 20 --warmup 3 --no-cpu-baseline --no-controller-line --no-packed-line --no-knn-line > $GRAFT_REPO_ROOT/$O/prof8192.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof8192.log; exit 1; }
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03s5/prof8192/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print("%-70s %6s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
ROUNDS=2 timeout -k 10 600 bash scripts/ab_plain_libs.sh tree grid1k > $O/ab_plain.txt 2>&1 || { cat $O/ab_plain.txt; exit 1; }
cat $O/ab_plain.txt
timeout -k 10 600 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_cov.log 2>&1 || { tail -30 $O/pytest_cov.log; exit 1; }
tail -1 $O/pytest_cov.log
timeout -k 10 500 bash scripts/ab_cov.sh > $O/ab_cov.txt 2>&1; rc=$?; grep -v "^$" $O/ab_cov.txt | tail -8; exit $rc

#!/bin/bash
# get_stats aggregates on the metrics path: the new GPU tests (summary vs oracle, RCCL
# all-gather at one rank), then the multi-rank bench path at one rank (--force-dist) with
# its gathered reward and stats checks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s30; mkdir -p $O
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_flock_gpu.py -k "stats" > $O/pytest_stats.txt 2>&1 || { tail -30 $O/pytest_stats.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_stats.txt | tail -5
timeout -k 10 300 python bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/bench_forcedist.json 2> $O/bench_forcedist.err || { tail -20 $O/bench_forcedist.err; exit 1; }
cat $O/bench_forcedist.json

#!/bin/bash
# A round-5 measurement set in one GPU session: the default bench line in the driver's
# window, the Coverage workload (with the greedy expert), rocprofv3 kernel trace + stats of
# a 100-step bench, and its per-grid kernel stats and step periods (scripts/trace_by_grid.py).
#   bash scripts/r05_profile.sh v1        -> gpurun_out/r05_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-v1}
R=$PWD
O=$R/gpurun_out/r05_$TAG
mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
echo "bench20 ok"
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
echo "bench_cov ok"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/rocprof_trace.log 2>&1 || { tail $O/rocprof_trace.log; exit 1; }
cd $R
python scripts/trace_by_grid.py $O/trace/trace_kernel_trace.csv $O/trace_by_grid --steps 100 > $O/trace_by_grid.txt && cat $O/trace_by_grid.txt

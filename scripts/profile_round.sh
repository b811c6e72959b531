#!/bin/bash
# A round's measurement set, one GPU session: the default bench line (driver window and
# 200 steps), rocprofv3 kernel stats of the bench, PMC HBM traffic of the step kernel,
# and a kernel trace of the Flocking-v0 line. Outputs under gpurun_out/prof_<TAG>/.
#   bash scripts/profile_round.sh v3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-v1}
O=gpurun_out/prof_$TAG
mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && tail -c 400 $O/bench20.json &&
timeout -k 10 400 python bench.py > $O/bench200.json 2> $O/bench200.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/rocprof_trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python scripts/pmc_step.py > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python scripts/pmc_step.py > $O/pmc_write.log 2>&1 &&
KSTEPS=200 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/knn -o knn -- python scripts/knn_line.py > $O/knn_line.log 2>&1 &&
python scripts/knn_line_report.py $O/knn/knn_kernel_trace.csv 200 > $O/knn_line_report.txt
echo "rc=$?"

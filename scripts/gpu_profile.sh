#!/bin/bash
# Bench + rocprofv3 kernel trace + PMC traffic passes for the bench workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && cat gpurun_out/bench.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-packed-line --no-knn-line > gpurun_out/rocprof_trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python scripts/pmc_step.py > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o pmc -- python scripts/pmc_step.py > gpurun_out/pmc_write.log 2>&1 &&
N=8192 B=32 timeout -k 10 300 python bench.py --n-agents 8192 --n-envs 32 --steps 20 --warmup 3 --no-cpu-baseline --no-knn-line > gpurun_out/bench_n8192.log 2>&1 && cat gpurun_out/bench_n8192.log &&
timeout -k 10 300 python bench.py --workload coverage --steps 50 --warmup 5 > gpurun_out/bench_coverage.log 2> gpurun_out/bench_coverage.err && cat gpurun_out/bench_coverage.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cov -o cov -- python bench.py --workload coverage --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/rocprof_cov.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_knn -o knn -- python scripts/time_knn.py > gpurun_out/rocprof_knn.log 2>&1 &&
python scripts/knn_trace.py gpurun_out/prof_knn/knn_kernel_trace.csv
echo "rc=$?"

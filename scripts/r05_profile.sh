#!/bin/bash
# A round-5 measurement set in one GPU session: the GPU suite, smoke, the default bench line
# (driver window and 200 steps), the Coverage workload (with the greedy expert), the
# multi-rank path at one rank (--force-dist: the RCCL reward and stats gathers), a rocprofv3
# kernel trace + stats of a 100-step bench with its per-grid kernel stats and step periods
# (scripts/trace_by_grid.py), and PMC HBM traffic (FETCH_SIZE and WRITE_SIZE passes) of every
# bench sub-line's kernel (summarised here by scripts/pmc_all.sh).
#   bash scripts/r05_profile.sh v2        -> gpurun_out/r05_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-v1}
R=$PWD
O=$R/gpurun_out/r05_$TAG
mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
echo "bench20 ok"
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench200.json 2> $O/bench200.err || { tail $O/bench200.err; exit 1; }
echo "bench200 ok"
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
echo "bench_cov ok"
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs > $O/bench_forcedist.json 2> $O/bench_forcedist.err || { tail $O/bench_forcedist.err; exit 1; }
echo "bench_forcedist ok"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/rocprof_trace.log 2>&1 || { tail $O/rocprof_trace.log; exit 1; }
cd $R
python scripts/trace_by_grid.py $O/trace/trace_kernel_trace.csv $O/trace_by_grid --steps 100 > $O/trace_by_grid.txt && cat $O/trace_by_grid.txt
cd /tmp
pmc() {  # pmc <name> <script> [env...]
  local name=$1 script=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    env "$@" timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${name}_$c -o pmc -- python3 $R/scripts/$script > $O/pmc_${name}_$c.log 2>&1 || return 1
  done
}
pmc plain pmc_step.py &&
pmc ctrl pmc_step.py MODE=ctrl &&
pmc packed pmc_step.py MODE=packed &&
pmc knn pmc_step.py KNN=1 &&
pmc n8192 pmc_step.py N=8192 B=32 &&
pmc cov pmc_cov.py
echo "pmc rc=$?"
# run-to-run spread of the headline on this box: three more driver-window lines
cd $R
for r in 1 2 3; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs > $O/bench20_rep$r.json 2>/dev/null; done
python - $O <<'PY'
import json, sys
for r in (1, 2, 3):
    d = json.loads(open("%s/bench20_rep%d.json" % (sys.argv[1], r)).read().strip().splitlines()[-1])
    print("rep", r, round(d["ms_per_step"] * 1e3, 2), "us", round(d["roofline"]["frac"], 3),
          "knn", round(d["flocking_v0_knn7"]["ms_per_step"] * 1e3, 2), round(d["flocking_v0_knn7"]["ratio_to_plain_step"], 3))
PY
# the GPU suite once more, after everything above (flakiness check)
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu_again.log 2>&1; echo "second suite rc=$?"; tail -1 $O/pytest_gpu_again.log

# Round 5, session 12: why the multi-rank path (--force-dist: one rank, reward all-gather
# every 8 steps) slows the plain step; kernel trace with queue ids.
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
O=$R/gpurun_out/r05_s12; mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --force-dist --steps 40 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
cd $R
timeout -k 10 300 python bench.py --force-dist --steps 40 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/fd.json 2> $O/fd.err; echo "fd rc=$?"
timeout -k 10 300 python bench.py --force-dist --metrics-every 64 --steps 40 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/fd64.json 2> $O/fd64.err; echo "fd64 rc=$?"
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/nofd.json 2> $O/nofd.err; echo "nofd rc=$?"
python - <<'PY'
import json
for f in ("fd", "fd64", "nofd"):
    d = json.loads(open("gpurun_out/r05_s12/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d["config"]["parallelism"])
PY
ls $O/trace

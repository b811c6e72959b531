# Round 5, session 6: the greedy expert's fallback draws on the device (COV_GREEDY_RNG):
# Coverage tests, then the Coverage bench workload with the expert lines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s6; mkdir -p $O
timeout -k 10 60 ./scripts/flagprobe.bin > $O/flagprobe.txt 2>&1; echo "flagprobe rc=$?"; cat $O/flagprobe.txt
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_cov.log 2>&1; r0=$?; echo "coverage tests rc=$r0"; tail -15 $O/pytest_cov.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
echo "bench_cov ok"
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s6/bench_cov.json").read().strip().splitlines()[-1])
def walk(o, p=""):
    for k, v in o.items():
        if isinstance(v, dict): walk(v, p + k + ".")
        elif "expert" in p + k or k in ("ms_per_step", "value"): print(p + k, "=", v)
walk(d)
PY

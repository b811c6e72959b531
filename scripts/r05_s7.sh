# Round 5, session 7: the drop-in steps wait for the kernel's completion flag; device
# fallback draws. Full GPU suite, the bench line (driver window) and the Coverage workload.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s7; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; r0=$?; echo "gpu tests rc=$r0"; tail -5 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
echo "bench20 ok"
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
echo "bench_cov ok"
python - <<'PY'
import json
for f in ("bench20", "bench_cov"):
    d = json.loads(open("gpurun_out/r05_s7/%s.json" % f).read().strip().splitlines()[-1])
    def walk(o, p=""):
        for k, v in o.items():
            if isinstance(v, dict): walk(v, p + k + ".")
            elif "expert" in p + k or "dropin" in p or k in ("ms_per_step", "frac"): print(p + k, "=", v)
    walk(d)
PY

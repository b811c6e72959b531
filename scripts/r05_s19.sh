# Round 5, session 19: reset()'s draws on the device (cov_reset_seeded): Coverage tests,
# the Coverage workload with the reset timings.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s19; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -15 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 300 python bench.py --workload coverage --steps 1000 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s19/bench_cov.json").read().strip().splitlines()[-1])
print(round(d["ms_per_step"] * 1e3, 2), {k: v for k, v in d["greedy_expert"].items() if "ms" in k})
PY

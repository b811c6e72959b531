# Round 5, session 16: Coverage steps with the automatic launch split (greedy steps in two
# halves, others one launch): tests, the Coverage workload, the greedy probe.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s16; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py tests/test_stream_ordering_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -3 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
for r in 1 2; do
timeout -k 10 300 python bench.py --workload coverage --steps 1000 --warmup 20 --no-cpu-baseline > $O/bench_cov_$r.json 2> $O/bench_cov_$r.err || { tail $O/bench_cov_$r.err; exit 1; }
done
timeout -k 10 300 python scripts/cov_greedy_probe.py > $O/probe.json 2> $O/probe.err; echo "probe rc=$?"
python - <<'PY'
import json
for r in (1, 2):
    d = json.loads(open("gpurun_out/r05_s16/bench_cov_%d.json" % r).read().strip().splitlines()[-1])
    print(r, round(d["ms_per_step"] * 1e3, 2), "us/step, frac", round(d["roofline"]["frac"], 3), "expert in episodes",
          round(d["greedy_expert"]["expert_step_ms_in_episodes"] * 1e3, 2), "us")
print(open("gpurun_out/r05_s16/probe.json").read())
PY

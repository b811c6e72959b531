# Round 5, session 23: one-env Flocking-v0 handles ranked exactly in the step (tile = env,
# up to 1024 agents): Flocking GPU tests, then the drop-in probe lines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s23; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -8 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s23/bench20.json").read().strip().splitlines()[-1])
for n in ("n100", "n1024"):
    print(n, {k: (round(v["step_ms"] * 1e3, 1), round(v["controller_plus_step_ms"] * 1e3, 1)) for k, v in d["dropin"][n].items() if isinstance(v, dict)})
print("plain", d["ms_per_step"], "knn", d["flocking_v0_knn7"]["ms_per_step"])
PY

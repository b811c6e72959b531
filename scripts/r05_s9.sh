# Round 5, session 9: the drop-in Flocking-v0 step of a larger env waits for its rim kNN's
# completion flag. Flocking GPU tests, then the bench line (driver window).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s9; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -5 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s9/bench20.json").read().strip().splitlines()[-1])
for n in ("n100", "n1024"):
    print(n, {k: {kk: round(vv * 1e3, 2) for kk, vv in v.items() if kk.endswith("_ms")} for k, v in d["dropin"][n].items() if isinstance(v, dict)})
print("plain", d["ms_per_step"], "knn", d["flocking_v0_knn7"]["ms_per_step"])
PY

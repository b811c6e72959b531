# Round 5, session 3: one bench line in the driver's window with every sub-object (drop-in
# probes for Flocking and Coverage included).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_cov.log 2>&1; r0=$?; echo "coverage tests rc=$r0"; tail -3 $O/pytest_cov.log
[ $r0 -gt 1 ] && exit $r0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --cpu-seconds 6 > $O/bench20.json 2> $O/bench20.err; rc=$?; echo "bench rc=$rc"; tail -3 $O/bench20.err
python - $O/bench20.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", d["ms_per_step"], d["roofline"]["frac"], "knn", d["flocking_v0_knn7"]["ms_per_step"], d["flocking_v0_knn7"]["ratio_to_plain_step"])
for n in ("n100", "n1024"):
    print(n, {k: {kk: round(vv * 1e3, 1) for kk, vv in v.items()} for k, v in d["dropin"][n].items()})
print(d.get("runtime"))
for r in ("r6", "r200"):
    print(r, {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()} for k, v in d["dropin_coverage"][r].items()})
PY
exit $rc

# Round 5, session 1: the GPU suite on the new tree (exact small-env kNN, fused
# Flocking-v0 expert action, staging stream of the metrics path, runtime binding tests),
# smoke, and one bench line in the driver's window with the drop-in probe.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -15 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --cpu-seconds 6 > $O/bench20.json 2> $O/bench20.err; rc=$?; echo "bench rc=$rc"
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

# Round 5, session 2: the GPU suite on the tree, the kNN tests on the lean A/B library,
# the Flocking-v0 A/B (tree / lean / lean6 / w6u1), then one bench line with the drop-in
# probes.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -12 $O/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
GYMFLOCK_LIB=$PWD/build/lib_lean6/libgymflock.so timeout -k 10 300 python -u -m pytest tests/test_flock_gpu.py -m gpu -q -k "knn or flocking_v0 or golden" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_lean6.log 2>&1; r2=$?; echo "lean6 knn tests rc=$r2"; tail -3 $O/pytest_lean6.log
[ $r2 -gt 1 ] && exit $r2
ROUNDS=2 timeout -k 10 400 bash scripts/ab_knn_libs.sh tree lean lean6 w6u1 > $O/ab_knn_lean.txt 2>&1; echo "ab rc=$?"; cat $O/ab_knn_lean.txt
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --cpu-seconds 6 > $O/bench20.json 2> $O/bench20.err; rc3=$?; echo "bench rc=$rc3"
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

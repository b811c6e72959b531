# Product build with the superset pass 1 + fast store loop for the fused kNN step:
# the GPU suite, smoke, a bench line, then phase timelines (GF_STAMPS build).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s20_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/s20_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s20_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/s20_smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/s20_bench.json 2> $O/s20_bench.err; rc=$?; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
python - $O/s20_bench.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", round(d["ms_per_step"] * 1e3, 1), "us frac", round(d["roofline"]["frac"], 3))
for k in ("step_with_controller", "packed_network", "flocking_v0_knn7", "coverage_config4", "n8192_config5"):
    v = d.get(k)
    if v:
        print(k, round(v["ms_per_step"] * 1e3, 2), "us frac", round(v["roofline"]["frac"], 3), "ratio", round(v.get("ratio_to_plain_step", 0), 3))
PY
L=$PWD/build/lib_st1/libgymflock.so
GYMFLOCK_LIB=$L timeout -k 10 200 python scripts/phase_timeline.py > $O/s20_tl_plain.txt 2>&1 && GYMFLOCK_LIB=$L KNN=1 timeout -k 10 200 python scripts/phase_timeline.py > $O/s20_tl_knn.txt 2>&1; echo tl rc=$?
head -18 $O/s20_tl_plain.txt; head -18 $O/s20_tl_knn.txt

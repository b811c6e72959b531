#!/bin/bash
# Round-4 GPU-box session. Modes (any combination, in order): test smoke bench bench200 prof
# Every GPU step has its own time limit; a crash/abort/timeout (exit >= 124, 134, 139)
# ends the session, an ordinary test failure (exit 1) does not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r04}; mkdir -p $O
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n ${TAILN:-15} "$O/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "ABORT after $name"; exit $rc; fi
  return 0
}
summ() {
python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", round(d["ms_per_step"] * 1e3, 1), "us frac", round(d["roofline"]["frac"], 3))
for k in ("step_with_controller", "packed_network", "flocking_v0_knn7", "coverage_config4", "n8192_config5"):
    v = d.get(k)
    if v:
        print(k, round(v["ms_per_step"] * 1e3, 2), "us frac", round(v["roofline"]["frac"], 3),
              "ratio", round(v.get("ratio_to_plain_step", 0), 3))
if d.get("dropin"):
    print("dropin", json.dumps(d["dropin"])[:900])
if d.get("coverage_config4", {}).get("greedy_expert"):
    print("greedy", json.dumps(d["coverage_config4"]["greedy_expert"])[:400])
PY
}
for MODE in "$@"; do
  case $MODE in
    test) step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider ;;
    testk) step pytest_gpu_k 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "$K" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench20 600 python bench.py --steps 20 --warmup 5 && (grep "^{" $O/bench20.log | tail -1 > $O/bench20.json; summ $O/bench20.json) ;;
    bench200) step bench200 600 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-other-configs && summ $O/bench200.log ;;
    prof) step rocprof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o trace -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    *) echo "unknown mode $MODE"; exit 2 ;;
  esac
done
echo "=== done"

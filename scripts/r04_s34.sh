# bench.py's dropin sub-object with the Flocking-v0 entries (driver window).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s34_bench.json 2> $O/s34_bench.err; rc=$?; echo "bench rc=$rc"
python - $O/s34_bench.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for n in ("n100", "n1024"):
    print(n, {k: {kk: round(vv * 1e3, 1) for kk, vv in v.items()} for k, v in d["dropin"][n].items()})
PY
exit $rc

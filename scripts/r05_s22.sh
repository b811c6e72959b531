# Round 5, session 22: the Coverage workload with whole expert episodes.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s22; mkdir -p $O
timeout -k 10 300 python bench.py --workload coverage --steps 1000 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s22/bench_cov.json").read().strip().splitlines()[-1])
print(round(d["ms_per_step"] * 1e3, 2), {k: v for k, v in d["greedy_expert"].items() if "ms" in k or "per_s" in k})
PY

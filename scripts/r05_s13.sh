# Round 5, session 13: the multi-rank path at one rank after re-warming the clocks that
# RCCL's initialisation let drop (bench.py REWARM_STEPS), against the plain line.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s13; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line"
for r in 1 2; do
timeout -k 10 300 python bench.py --force-dist $A > $O/fd_$r.json 2> $O/fd_$r.err || { tail $O/fd_$r.err; exit 1; }
timeout -k 10 300 python bench.py $A > $O/nofd_$r.json 2> $O/nofd_$r.err || { tail $O/nofd_$r.err; exit 1; }
done
python - <<'PY'
import json
for f in ("fd_1", "nofd_1", "fd_2", "nofd_2"):
    d = json.loads(open("gpurun_out/r05_s13/%s.json" % f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"] * 1e3, 2), "us/step", d["config"]["parallelism"], d.get("clock_warmup"), d.get("gathered_rewards_ok"))
PY

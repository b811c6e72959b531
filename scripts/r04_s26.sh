# One-tile envs take their rows from the tile staging; a single one-tile env's host actions travel
# in the kernel arguments (fe_step_host). GPU suite,
# the drop-in probe and a bench line (its dropin sub-object).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s26_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -2 $O/s26_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/dropin_probe.py > $O/s26_dropin_probe.txt 2>&1; echo "probe rc=$?"; tail -3 $O/s26_dropin_probe.txt
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s26_bench.json 2> $O/s26_bench.err; echo "bench rc=$?"
python - $O/s26_bench.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", round(d["ms_per_step"] * 1e3, 1), "knn", round(d["flocking_v0_knn7"]["ms_per_step"] * 1e3, 1))
dd = d["dropin"]; print("dropin n100 direct", dd["n100"]["direct"], "pooled", dd["n100"]["pooled"])
PY
for r in 0 1; do for s in 1 2; do STREAMS=$s ROUNDS=3 timeout -k 10 120 python scripts/time_cov.py s$s > $O/s26_cov_s${s}_$r.txt 2>&1; echo "cov streams=$s round $r: $(tail -2 $O/s26_cov_s${s}_$r.txt | tr '\n' ' ')"; done; done
GYMFLOCK_LIB=$PWD/build/lib_cand/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s26_cand_tests.log 2>&1; echo "cand kNN tests rc=$?"; tail -1 $O/s26_cand_tests.log
ROUNDS=3 OUT=gpurun_out/r04/ab_s26 timeout -k 10 900 python scripts/ab_multi.py head=build/lib_head/libgymflock.so new=gym-flock_amd/lib/libgymflock.so cand=build/lib_cand/libgymflock.so -- --no-other-configs --no-packed-line
STEPS=200 WARMUP=20 ROUNDS=2 OUT=gpurun_out/r04/ab_s26_200 timeout -k 10 900 python scripts/ab_multi.py new=gym-flock_amd/lib/libgymflock.so cand=build/lib_cand/libgymflock.so -- --no-other-configs --no-packed-line
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline > $O/s26_forcedist.json 2> $O/s26_forcedist.err; echo "forcedist rc=$?"
python - $O/s26_forcedist.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print({k: d.get(k) for k in ("ms_per_step", "n_gpus", "gathered_rewards_ok", "gathered_stats_ok", "rccl")})
PY

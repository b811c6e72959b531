# Round 5, session 24: A/B of the one-env exact in-step kNN threshold (1024: product build,
# 128: build/lib_exact128), drop-in Flocking-v0 per call over N, two rounds.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s24; mkdir -p $O
for r in 1 2; do
timeout -k 10 200 python scripts/dropin_exact_probe.py >> $O/ab.txt 2>&1 || exit 1
timeout -k 10 200 env GYMFLOCK_LIB=$PWD/build/lib_exact128/libgymflock.so python scripts/dropin_exact_probe.py >> $O/ab.txt 2>&1 || exit 1
done
cat $O/ab.txt

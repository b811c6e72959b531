# Flocking-v0 A/B 6: the predicted rows' candidate radius^2 factor (2.25 x the 7th-nearest
# r2 two states back, product) against 1.69 and 1.44, over 20 and 200 steps.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_cf144/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s28_tests.log 2>&1; rc=$?; echo "cf144 kNN tests rc=$rc"; tail -1 $O/s28_tests.log
[ $rc -ge 124 ] && exit $rc
STEPS=200 WARMUP=20 ROUNDS=2 OUT=gpurun_out/r04/ab_s28_200 timeout -k 10 900 python scripts/ab_multi.py cur=gym-flock_amd/lib/libgymflock.so cf169=build/lib_cf169/libgymflock.so cf144=build/lib_cf144/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
ROUNDS=3 OUT=gpurun_out/r04/ab_s28 timeout -k 10 900 python scripts/ab_multi.py cur=gym-flock_amd/lib/libgymflock.so cf169=build/lib_cf169/libgymflock.so cf144=build/lib_cf144/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line

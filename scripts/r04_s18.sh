# Flocking-v0 A/B 3: the fused kNN step at 6 waves per SIMD (80 VGPRs; the superset pass 1
# leaves its spills outside the loops) vs 5 (supsf2); w6n = 6 waves without the superset.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_w6s/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s18_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/s18_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s18 timeout -k 10 900 python scripts/ab_multi.py supsf2=build/lib_supsf2/libgymflock.so w6s=build/lib_w6s/libgymflock.so w6n=build/lib_w6n/libgymflock.so -- --no-other-configs --no-packed-line

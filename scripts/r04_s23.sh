# Flocking-v0 A/B 4: inline-rim scan with 1 column in flight per lane (u1; its register
# peak set the kernel's) at 5 and 6 waves per SIMD, vs the current build.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_u1w6/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s23_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/s23_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s23 timeout -k 10 900 python scripts/ab_multi.py cur=build/lib_cur/libgymflock.so u1w5=build/lib_u1w5/libgymflock.so u1w6=build/lib_u1w6/libgymflock.so -- --no-other-configs --no-packed-line

# Flocking-v0 A/B: superset pass 1 (sup), fast network store loop (sf), both (supsf) vs base.
# kNN-related GPU tests run on the sup+sf build first (parity), then the interleaved bench A/B.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_supsf/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s15_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/s15_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s15 timeout -k 10 900 python scripts/ab_multi.py base=build/lib_base/libgymflock.so sup=build/lib_sup/libgymflock.so sf=build/lib_sf/libgymflock.so supsf=build/lib_supsf/libgymflock.so -- --no-other-configs --no-packed-line

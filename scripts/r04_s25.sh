# Flocking-v0 A/B 5: hybrid pass 1 (superset on every tile but the last; the last tile's
# bits exact from the band sweep, its feature pass after the network stores) vs superset on
# every tile (cur).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_hyb/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s25_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/s25_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s25 timeout -k 10 900 python scripts/ab_multi.py cur=build/lib_cur/libgymflock.so hyb=build/lib_hyb/libgymflock.so -- --no-other-configs --no-packed-line

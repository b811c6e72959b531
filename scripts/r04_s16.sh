# Flocking-v0 A/B 2: kNN key by fma + saturating convert, exact words by LDS atomic clears
# (supsf2, sf2) vs supsf and base; sfp = supsf2 with the fast store loop for the plain step too.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_sfp/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py tests/test_stream_ordering_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s16_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/s16_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s16 timeout -k 10 900 python scripts/ab_multi.py base=build/lib_base/libgymflock.so supsf=build/lib_supsf/libgymflock.so supsf2=build/lib_supsf2/libgymflock.so sf2=build/lib_sf2/libgymflock.so sfp=build/lib_sfp/libgymflock.so -- --no-other-configs --no-packed-line

# A/B of the round-4 latency changes' effect on the batched lines: head (before them),
# new (one-tile rows in the staging lambda + kernel-argument actions), new2 (one-tile rows
# copied from the staged tile after a barrier, outside the staging lambda), nouin (new2
# without the kernel-argument-action template parameter).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_new2/libgymflock.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s27_tests.log 2>&1; rc=$?; echo "new2 gpu suite rc=$rc"; tail -1 $O/s27_tests.log
[ $rc -ne 0 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s27 timeout -k 10 1000 python scripts/ab_multi.py head=build/lib_head/libgymflock.so new=gym-flock_amd/lib/libgymflock.so new2=build/lib_new2/libgymflock.so nouin=build/lib_nouin/libgymflock.so -- --no-other-configs --no-packed-line

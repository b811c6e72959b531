# Debug: does the HEAD library (build/lib_base) abort in the full GPU suite too?
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_base/libgymflock.so GF_ABORT_BT=1 timeout -k 10 600 python -u -m pytest -s -p no:faulthandler tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/s21_g.log 2>&1; echo "d rc=$?"; grep -v "^Extension" $O/s21_g.log | grep -v PASSED | tail -30

# The inline-action boundary tests, then the final round-4 profile set (v3).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_flock_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "inline_actions or dropin" > $O/s29_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error|passed|failed" $O/s29_tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
bash scripts/r04_profile.sh v3

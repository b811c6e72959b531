# Round 5, session 10: the mid-run collective abort path (comm_event_wait timing out).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_metrics_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -30 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 timeout -k 10 300 ./build/asan/capi_asan > $O/asan.log 2>&1; ra=$?; echo "asan rc=$ra"; tail -5 $O/asan.log
[ $ra -ne 0 ] && exit $ra
timeout -k 10 120 python scripts/cov_launch_probe.py > $O/cov_launch_probe.json 2>&1; r1=$?; cat $O/cov_launch_probe.json
exit $r1

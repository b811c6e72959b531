# Round 5, session 10: the mid-run collective abort path (comm_event_wait timing out).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_metrics_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -30 $O/pytest.log
exit $r0

# Round 5, session 14: Coverage split steps with the second half from a launcher thread
# (cov_set_streams 3) against one thread (2) and one launch (1); then the Coverage tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s14; mkdir -p $O
timeout -k 10 180 python scripts/cov_launch_probe.py > $O/cov_launch_probe.json 2>&1; r1=$?; cat $O/cov_launch_probe.json
[ $r1 -ne 0 ] && exit $r1
timeout -k 10 300 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -3 $O/pytest.log
exit $r0

# Round 5, session 5: Coverage tests with the direct greedy path for short unvisited lists,
# then the greedy probe (steady state vs episodes).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_cov.log 2>&1; r0=$?; echo "coverage tests rc=$r0"; tail -15 $O/pytest_cov.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 300 python scripts/cov_greedy_probe.py > $O/probe2.json 2> $O/probe2.err; rc=$?; echo "probe rc=$rc"; cat $O/probe2.json
exit $rc

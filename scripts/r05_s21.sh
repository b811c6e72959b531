# Round 5, session 21: the Coverage expert / reset tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s21; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -8 $O/pytest.log
exit $r0

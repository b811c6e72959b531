# Round 5, session 18: the device fallback draws at the config-4 shape (64 envs, sampled).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s18; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py -m gpu -v -k "config4_batch" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -15 $O/pytest.log
exit $r0

# Round 5, session 17: page-locked (completion flag) vs pageable (stream wait) drop-in outputs.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s17; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_flock_gpu.py -m gpu -q -k "flag_and_stream or dropin" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -15 $O/pytest.log
exit $r0

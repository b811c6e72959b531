# Flocking-v0 drop-in step through fe_step_host_knn: GPU tests (flock file + the capi
# export check), then the latency probe (FlockingRelative direct, Flocking-v0 pooled/direct).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_flock_variants_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s30_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/s30_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/dropin_knn_probe.py

cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_metrics_gpu.py tests/test_flock_gpu.py -k "metrics or comm or gather or dropin or step_host or host_pool or stats" -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s9_tests.log 2>&1; echo "tests rc=$?"; grep -E "PASS|FAIL|ERROR|passed|failed|lone-rank" $O/s9_tests.log | tail -30
timeout -k 10 300 python -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench
class A: pass
print(json.dumps(bench.bench_dropin(A())))" > $O/dropin2.log 2>&1; tail -1 $O/dropin2.log | cut -c1-900

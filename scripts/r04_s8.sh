cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py tests/test_flock_gpu.py -k "coverage or greedy or wire or dropin or step_host" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/cov_tests.log 2>&1; echo "tests rc=$?"; tail -5 $O/cov_tests.log
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.log 2>&1 && grep "^{" $O/bench_cov.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1e3, json.dumps(d.get('greedy_expert')))"
timeout -k 10 300 python -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench
class A: pass
print(json.dumps(bench.bench_dropin(A())))" > $O/dropin.log 2>&1; tail -3 $O/dropin.log
ROUNDS=2 OUT=gpurun_out/r04/ab_mode1 timeout -k 10 600 python scripts/ab_multi.py new=gym-flock_amd/lib/libgymflock.so mode1=build/lib_mode1/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
timeout -k 5 40 ./build/comm_probe 1 && timeout -k 5 40 ./build/comm_probe 0
echo "probe rc=$?"

cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/cov_tests.log 2>&1; echo "cov tests rc=$?"; tail -5 $O/cov_tests.log
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.log 2>&1 && grep "^{" $O/bench_cov.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1e3, json.dumps(d.get('greedy_expert')))"
timeout -k 5 40 ./build/comm_probe 1 && timeout -k 5 40 ./build/comm_probe 0
echo "probe rc=$?"

cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s14_cov.log 2>&1; echo "cov tests rc=$?"; tail -2 $O/s14_cov.log
for r in 0 1 2; do for L in old:build/lib_old new:gym-flock_amd/lib; do n=${L%%:*}; d=${L#*:}
GYMFLOCK_LIB=$PWD/$d/libgymflock.so timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/s14_${n}_$r.log 2>&1 || { echo "bench failed $n"; exit 1; }
grep "^{" $O/s14_${n}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); g=d.get('greedy_expert',{}); print('$r $n step %.2f us  expert %.2f  two_launch %.2f  episodes %.2f  tm %.1f ms' % (d['ms_per_step']*1e3, g['expert_step_ms']*1e3, g['expert_step_ms_two_launches']*1e3, g['expert_step_ms_in_episodes']*1e3, g['time_matrix_ms_all_envs']))"
done; done
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so GREEDY=1 timeout -k 10 200 python scripts/cov_timeline.py > $O/cov_timeline_greedy2.json 2>&1; echo "tl rc=$?"; python -c "
import json; d=json.load(open('$O/cov_timeline_greedy2.json')); print(d['launch_span_us'], {k:(v['median'],v['p90'],v['max']) for k,v in d['phases_us'].items()})"

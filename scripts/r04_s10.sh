cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_metrics_gpu.py tests/test_flock_gpu.py -k "metrics or comm or gather or dropin or step_host or host_pool or stats" -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s10_tests.log 2>&1; echo "tests rc=$?"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/s10_tests.log | tail -40
timeout -k 10 300 python -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench
class A: pass
print(json.dumps(bench.bench_dropin(A())))" > $O/dropin3.log 2>&1; tail -1 $O/dropin3.log | cut -c1-900
GYMFLOCK_LIB=$PWD/build/lib_v2/libgymflock.so timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py tests/test_flock_variants_gpu.py tests/test_stream_ordering_gpu.py -k "knn or v0 or variant or flocking" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s10_knn_v2.log 2>&1; echo "knn v2 tests rc=$?"; tail -5 $O/s10_knn_v2.log
ROUNDS=3 OUT=gpurun_out/r04/ab_v2 timeout -k 10 700 python scripts/ab_multi.py base=gym-flock_amd/lib/libgymflock.so v2=build/lib_v2/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
echo "== ctrl instruction mix by part"
export TMPDIR=/tmp
P=$PWD/gpurun_out/r04/pmc_ctrl; mkdir -p $P
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P/$n -o pmc -- python3 scripts/pmc_step.py > $P/$n.log 2>&1
}
run p_all DIAG=0 && run c_all MODE=ctrl DIAG=0 && run c_nofeat MODE=ctrl DIAG=2 && run c_nopass1 MODE=ctrl DIAG=8 &&
run c_recip MODE=ctrl DIAG=2048 && run c_nograd MODE=ctrl DIAG=4096 && run c_norowout MODE=ctrl DIAG=256 && run c_noreward MODE=ctrl DIAG=512 &&
python scripts/pmc_mix.py $P > $P/mix.txt; cat $P/mix.txt
echo "== coverage greedy timeline"
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so GREEDY=1 timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/r04/cov_timeline_greedy.json 2>&1; echo "tl rc=$?"; head -c 1500 gpurun_out/r04/cov_timeline_greedy.json
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/r04/cov_timeline_random.json 2>&1; echo "tl rc=$?"

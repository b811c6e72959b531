cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s13_flock.log 2>&1; echo "flock tests rc=$?"; tail -2 $O/s13_flock.log
ROUNDS=3 OUT=gpurun_out/r04/ab_s13 timeout -k 10 900 python scripts/ab_multi.py c32=build/lib_c32/libgymflock.so new=gym-flock_amd/lib/libgymflock.so sf0=build/lib_sf0/libgymflock.so -- --no-other-configs --no-packed-line
P=$PWD/gpurun_out/r04/pmc_knn2; mkdir -p $P
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P/$n -o pmc -- python3 scripts/pmc_step.py > $P/$n.log 2>&1
}
run k_all KNN=1 DIAG=0 && run k_nomerge KNN=1 DIAG=1 && python scripts/pmc_mix.py $P > $P/mix.txt; cat $P/mix.txt

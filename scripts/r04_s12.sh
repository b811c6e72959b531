cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_w6/libgymflock.so timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py -k "knn or v0" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s12_knn_w6.log 2>&1; echo "knn w6 tests rc=$?"; tail -2 $O/s12_knn_w6.log
GYMFLOCK_LIB=$PWD/build/lib_c32/libgymflock.so timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py -k "controller or ctrl or expert or closed" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s12_ctrl_c32.log 2>&1; echo "ctrl c32 tests rc=$?"; tail -2 $O/s12_ctrl_c32.log
ROUNDS=3 OUT=gpurun_out/r04/ab_w6 timeout -k 10 900 python scripts/ab_multi.py base=gym-flock_amd/lib/libgymflock.so w6=build/lib_w6/libgymflock.so c32=build/lib_c32/libgymflock.so -- --no-other-configs --no-packed-line
echo "== knn instruction mix by part"
P=$PWD/gpurun_out/r04/pmc_knn; mkdir -p $P
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P/$n -o pmc -- python3 scripts/pmc_step.py > $P/$n.log 2>&1
}
run p_all DIAG=0 && run k_all KNN=1 DIAG=0 && run k_nomerge KNN=1 DIAG=1 && run k_noinsert KNN=1 DIAG=0x200000 && run k_nopred KNN=1 DIAG=0x20000 &&
run k_nogather KNN=1 DIAG=32 && run k_nofeat KNN=1 DIAG=2 && run k_nopass1 KNN=1 DIAG=8 && run k_norim KNN=1 DIAG=0x40000 &&
python scripts/pmc_mix.py $P > $P/mix.txt; cat $P/mix.txt

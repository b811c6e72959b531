# PMC instruction mix of the Flocking-v0 step with the superset pass 1 + fast store loop
# (diagnostic build of supsf2): whole kernel and with parts switched off.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
P=$PWD/gpurun_out/r04/pmc_knn3; mkdir -p $P
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag2/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P/$n -o pmc -- python3 scripts/pmc_step.py > $P/$n.log 2>&1
}
run k_all KNN=1 DIAG=0 && run k_nomerge KNN=1 DIAG=1 && run k_nogather KNN=1 DIAG=32 && run k_noinsert KNN=1 DIAG=0x200000 && run k_nofeat KNN=1 DIAG=2 && run k_nopred KNN=1 DIAG=0x20000 && run p_all DIAG=0 && python scripts/pmc_mix.py $P > $P/mix.txt; cat $P/mix.txt

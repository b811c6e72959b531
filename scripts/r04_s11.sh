cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r04/v2trace; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_v2/libgymflock.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O -o v2 -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other-configs --no-packed-line --no-controller-line > $O/bench.log 2>&1; echo "rc=$?"
find $O -name "*kernel_stats.csv" | head -3
for f in $(find $O -name "*kernel_stats.csv"); do cut -d, -f1-8 $f | head -12; done

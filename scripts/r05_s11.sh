# Round 5, session 11: host launch cost of two streams from one thread vs two threads.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s11; mkdir -p $O
timeout -k 10 120 ./scripts/flagprobe.bin > $O/flagprobe.txt 2>&1; r=$?; cat $O/flagprobe.txt; exit $r

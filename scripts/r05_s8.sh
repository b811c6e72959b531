# Round 5, session 8: phase timelines of the plain and the Flocking-v0 step (config 2, one
# launch per step) from the stamps build (make -C gym-flock_amd/csrc stamps STAMPS=2).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s8; mkdir -p $O
export GYMFLOCK_LIB=$PWD/build/lib_stamps2/libgymflock.so
timeout -k 10 120 python scripts/phase_timeline.py > $O/tl_plain.txt 2>&1 || { tail $O/tl_plain.txt; exit 1; }
timeout -k 10 120 env KNN=1 python scripts/phase_timeline.py > $O/tl_knn.txt 2>&1 || { tail $O/tl_knn.txt; exit 1; }
head -22 $O/tl_plain.txt; echo ----; head -22 $O/tl_knn.txt

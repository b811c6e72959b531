# Phase timelines (GF_STAMPS=1) of the plain and the Flocking-v0 step (supsf2 code).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
L=$PWD/build/lib_st1/libgymflock.so
GYMFLOCK_LIB=$L timeout -k 10 200 python scripts/phase_timeline.py > $O/s19_plain.txt 2>&1 && GYMFLOCK_LIB=$L KNN=1 timeout -k 10 200 python scripts/phase_timeline.py > $O/s19_knn.txt 2>&1; echo rc=$?
head -22 $O/s19_plain.txt; head -22 $O/s19_knn.txt

# Phase timeline of the kNN step built for 6 waves per SIMD (inline rim U=1), to see where
# the 6-wave build loses (A/B: 225 vs 197 us) against the 5-wave timeline (s20_tl_knn.txt).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_st6/libgymflock.so KNN=1 timeout -k 10 200 python scripts/phase_timeline.py > $O/s24_tl_knn_w6.txt 2>&1; echo tl rc=$?
head -18 $O/s24_tl_knn_w6.txt

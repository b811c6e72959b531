# Small envs (N <= 128): every unranked row of the fused kNN step ranked by its wave's inline
# scan (no rim work). kNN tests on that build, then the drop-in probe: product vs ilim.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_ilim/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking or dropin" > $O/s32_tests.log 2>&1; rc=$?; echo "ilim tests rc=$rc"; tail -1 $O/s32_tests.log
[ $rc -ne 0 ] && exit $rc
for L in gym-flock_amd/lib build/lib_ilim; do echo $L; GYMFLOCK_LIB=$PWD/$L/libgymflock.so timeout -k 10 200 python scripts/dropin_knn_probe.py; done

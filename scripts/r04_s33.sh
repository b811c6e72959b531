# Fused kNN step: up to 4 unranked rows per wave ranked inline (ir4) vs 2 (ir2, product),
# 20 and 200 steps; kNN tests on ir4.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_ir4/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s33_tests.log 2>&1; rc=$?; echo "ir4 tests rc=$rc"; tail -1 $O/s33_tests.log
ROUNDS=3 OUT=gpurun_out/r04/ab_s33 timeout -k 10 900 python scripts/ab_multi.py ir2=build/lib_ir2/libgymflock.so ir4=build/lib_ir4/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
STEPS=200 WARMUP=20 ROUNDS=2 OUT=gpurun_out/r04/ab_s33_200 timeout -k 10 900 python scripts/ab_multi.py ir2=build/lib_ir2/libgymflock.so ir4=build/lib_ir4/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line

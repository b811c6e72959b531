# Final check of the round-4 tree: GPU suite, smoke, a bench line (driver window) and the
# Flocking-v0 drop-in probe on the in-tree library.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04_final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -1 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.txt
[ $rc -ne 0 ] && exit $rc

timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err; rc=$?; echo "bench rc=$rc"
timeout -k 10 200 python scripts/dropin_knn_probe.py > $O/dropin_knn_probe.txt 2>&1; cat $O/dropin_knn_probe.txt

exit $rc

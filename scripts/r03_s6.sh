#!/bin/bash
# Round-3 session 6: hashed cell-list step with the many-workgroup prep (bin, scan,
# scatter, order): parity at wide N and through the N=1024 variant; A/B and profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s6; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_grid_step_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_grid.log 2>&1 || { tail -40 $O/pytest_grid.log; exit 1; }
tail -1 $O/pytest_grid.log
GYMFLOCK_LIB=$PWD/build/lib_grid1k/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "not knn and not variant" > $O/pytest_grid1k.log 2>&1 || { tail -40 $O/pytest_grid1k.log; exit 1; }
tail -1 $O/pytest_grid1k.log
ROUNDS=3 timeout -k 10 600 bash scripts/ab_n8192_libs.sh old tree > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
ROUNDS=3 timeout -k 10 600 bash scripts/ab_plain_libs.sh tree grid1k > $O/ab_plain.txt 2>&1 || { cat $O/ab_plain.txt; exit 1; }
cat $O/ab_plain.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8192 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n-agents 8192 --n-envs 32 --steps 20 --warmup 3 --no-cpu-baseline --no-controller-line --no-packed-line --no-knn-line > $GRAFT_REPO_ROOT/$O/prof8192.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof8192.log; exit 1; }
GYMFLOCK_LIB=$GRAFT_REPO_ROOT/build/lib_grid1k/libgymflock.so KNN=0 KSTEPS=100 WARM=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof1k -o run -- python3 $GRAFT_REPO_ROOT/scripts/knn_line.py > $GRAFT_REPO_ROOT/$O/prof1k.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof1k.log; exit 1; }
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob
for tag in ("prof8192", "prof1k"):
    f = glob.glob("gpurun_out/r03s6/%s/**/*kernel_stats.csv" % tag, recursive=True)[0]
    print(tag)
    for r in list(csv.DictReader(open(f)))[:8]:
        print("  %-66s %6s %10.1f us" % (r["Name"][:66], r["Calls"], float(r["AverageNs"]) / 1e3))
PY

#!/bin/bash
# Ablations of the Flocking-v0 kernels (diagnostic build), one rocprofv3 trace each:
#   bash scripts/knn_ablate.sh [DIAG values...]   (default: 0 0x1000000 0x2000000 0x800000 1 32; kNN kernel switches are fe_diag bits << 12)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
export GYMFLOCK_LIB=$PWD/build/lib_diag/libgymflock.so
for d in ${@:-0 0x1000000 0x2000000 0x800000 1 32}; do
  echo "=== DIAG=$d"
  DIAG=$d timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kab_$d -o run -- python scripts/knn_phases.py > gpurun_out/kab_$d.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/kab_$d.log; exit 1; }
  python scripts/knn_phases_report.py gpurun_out/kab_$d/run_kernel_trace.csv
done

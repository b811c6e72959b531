#!/bin/bash
# kNN kernel A/B under rocprofv3 kernel trace: baseline library (build/lib_old) vs the
# working tree, then the working tree's ablation switches (DIAGS). Device time per launch
# (scripts/knn_trace.py), init and dispersed states.
set -e
mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/knn_$tag -o run -- \
    python $R/scripts/time_knn.py > $R/gpurun_out/knn_$tag.log 2>&1
  echo "== $tag"; python $R/scripts/knn_trace.py $(find $R/gpurun_out/knn_$tag -name "*kernel_trace.csv" | head -1)
}
run old GYMFLOCK_LIB=$R/build/lib_old/libgymflock.so
run new X=1
for d in ${DIAGS:-0x4000 0x8000}; do run diag$d DIAG=$d; done

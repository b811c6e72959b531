#!/bin/bash
# Coverage bench under rocprofv3 kernel trace; prints the top kernels. Run on the GPU box.
set -e
mkdir -p gpurun_out
tag=${1:-cov}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run -- python bench.py --workload coverage --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1
python - "$tag" <<'PY'
import sqlite3, sys, glob
db = sqlite3.connect(glob.glob("gpurun_out/prof_%s/**/*.db" % sys.argv[1], recursive=True)[0])
for r in db.execute("select name, total_calls, average from top_kernels limit 8"):
    print("%-90s %5d %10.1f us" % (r[0][:90], r[1], r[2]))
PY
tail -1 gpurun_out/prof_$tag.log

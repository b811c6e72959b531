# Kernel trace of the drop-in Flocking-v0 step at N=100 (where its 68 us go).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04/s31; mkdir -p $O
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o knn -- python3 $R/scripts/dbg/knn_dropin_loop.py > $O/log.txt 2>&1; echo rc=$?
cut -c1-200 $O/knn_kernel_stats.csv
python3 - $O/knn_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-12:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    print("%-60s start %8.1f us  dur %6.1f us" % (r["Kernel_Name"][:60], (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY

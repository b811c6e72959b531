"""Per-state kernel durations from a rocprofv3 kernel trace of scripts/knn_phases.py."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "flock_" in r["Kernel_Name"]]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
REPS = 5
# per state: (plain steps to reach it), then REPS x (fused step, rim kNN), REPS x full kNN, 1 stats
i = 0
for t in (0, 25, 50, 100, 200):
    while i < len(rows) and "stats" not in rows[i]["Kernel_Name"]:
        i += 1
    i += 1  # the stats kernel of h.stats()
    fused = [dur(rows[i + 2 * k]) for k in range(REPS)]
    rim = [dur(rows[i + 2 * k + 1]) for k in range(REPS)]
    i += 2 * REPS
    full = [dur(rows[i + k]) for k in range(REPS)]
    i += REPS
    med = lambda v: sorted(v)[len(v) // 2]
    print("t=%3d  fused step %.1f us  rim kNN %.1f us  full kNN %.1f us" % (t, med(fused), med(rim), med(full)))

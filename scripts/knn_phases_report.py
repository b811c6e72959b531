"""Per-state kernel durations from a rocprofv3 kernel trace of scripts/knn_phases.py."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "flock_" in r["Kernel_Name"]]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
med = lambda v: sorted(v)[len(v) // 2] if v else float("nan")
# groups start after each stats kernel (h.stats() of a new state)
groups, cur = [], None
for r in rows:
    if "stats" in r["Kernel_Name"]:
        cur = []
        groups.append(cur)
    elif cur is not None:
        cur.append(r)
for t, g in zip((0, 25, 50, 100, 200), groups):
    plain = [dur(r) for r in g if "step" in r["Kernel_Name"] and r["Kernel_Name"].rstrip(")").split(",")[-2:] != [] and ", 7>" not in r["Kernel_Name"]]
    fused = [dur(r) for r in g if ", 7>" in r["Kernel_Name"]]
    knn = [dur(r) for r in g if "knn" in r["Kernel_Name"]]
    rim, full = knn[:len(fused)], knn[len(fused):]
    print("t=%3d  plain step %.1f us  fused step %.1f us  rim kNN %.1f us  full kNN %.1f us"
          % (t, med(plain[:5]), med(fused), med(rim), med(full)))

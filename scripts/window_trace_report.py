"""Per-step timeline of 20-step windows from a rocprofv3 kernel trace of
scripts/window_probe.py: for each window (launches separated by an idle
gap > 30 us), the time from the first launch's start to each step's end (the later end
of its two half-batch launches), and the window's step period."""
import csv
import sys

rows = sorted((r for r in csv.DictReader(open(sys.argv[1])) if "flock_step" in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
wins, cur, last_end = [], [], None
for s, e in ev:
    if last_end is not None and s - last_end > 30000 and cur:
        wins.append(cur)
        cur = []
    cur.append((s, e))
    last_end = max(last_end or 0, e)
wins.append(cur)
for w in wins[-6:]:
    if len(w) != 40:
        continue
    t0 = w[0][0]
    ends = [max(w[2 * k][1], w[2 * k + 1][1]) - t0 for k in range(20)]
    gaps = [ends[0]] + [ends[k] - ends[k - 1] for k in range(1, 20)]
    print("window %.1f us: first step ends %.1f, steps 2-20 avg %.1f, last 5 avg %.1f; starts of halves %s"
          % ((ends[-1]) / 1e3, ends[0] / 1e3, (ends[-1] - ends[0]) / 19e3, (ends[-1] - ends[-6]) / 5e3,
             [round((w[k][0] - t0) / 1e3, 1) for k in range(4)]))

"""Fused-step and rim-kNN launch durations over the timed steps of scripts/knn_line.py
(rocprofv3 kernel trace): the last KSTEPS steps, in blocks of 20."""
import csv
import os
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
fused = [dur(r) for r in rows if ", 7>" in r["Kernel_Name"]][-2 * steps:]
rim = [dur(r) for r in rows if "knn_kernel" in r["Kernel_Name"]][-steps:]
for b in range(0, steps, 20):
    f = fused[2 * b:2 * b + 40]
    k = rim[b:b + 20]
    print("steps %3d-%3d  fused half-launch avg %.1f us  rim kNN avg %.1f us" % (b, b + 19, sum(f) / len(f), sum(k) / len(k)))

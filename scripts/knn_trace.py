"""Durations of the kNN and step kernels from a rocprofv3 --kernel-trace CSV of
scripts/time_knn.py, in dispatch order: the first half of the kNN dispatches ran on the
synthetic init state, the second half on the dispersed state.
Usage: python scripts/knn_trace.py <kernel_trace.csv>"""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
knn = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "knn_kernel" in r["Kernel_Name"]]
h = len(knn) // 2
for label, v in (("init", knn[:h]), ("dispersed", knn[h:])):
    v = np.array(v) / 1e3
    print("flock_knn_kernel %-10s n=%3d median %7.1f us  min %7.1f us" % (label, len(v), np.median(v), v.min()))

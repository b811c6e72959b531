"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of scripts/pmc_step.py into
profiles/pmc_traffic.json (per-launch HBM bytes of the step kernel).

gfx950 corrections (/opt/skills/guides/MI355X_MICROARCH.md §HBM): both counters are in
KiB; FETCH_SIZE reports half the bytes of a wide coalesced read, so it is doubled.
usage: python scripts/pmc_summary.py <fetch_csv> <write_csv> <N> <B> [out.json]"""
import csv
import json
import os
import sys


def per_kernel(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals


def main():
    fetch_csv, write_csv, n, b = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    # the plain step: <DYN=true, UF64=false, CTRL=false[, VAR=false]>
    key = [k for k in f if "flock_step_kernel<true, false, false" in k][0]
    fetch_kib = sum(f[key]) / len(f[key])
    write_kib = sum(w[key]) / len(w[key])
    total = (2 * fetch_kib + write_kib) * 1024
    alg = b * (4 * n * n + 96 * n + 8)
    d = json.load(open(out)) if os.path.exists(out) else {}
    d["%dx%d" % (n, b)] = {
        "kernel": key, "launches": len(f[key]),
        "FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib,
        "bytes_per_launch": total, "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": total / alg,
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE reads half)"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d["%dx%d" % (n, b)], indent=1))


if __name__ == "__main__":
    main()

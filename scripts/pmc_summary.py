"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json
(per-launch HBM bytes of one kernel, next to its algorithmic bytes per launch).

gfx950 corrections (/opt/skills/guides/MI355X_MICROARCH.md §HBM): both counters are in
KiB; FETCH_SIZE reports half the bytes of a wide coalesced read, so it is doubled.
usage: python scripts/pmc_summary.py <fetch_csv> <write_csv> <key> <kernel substring>
                                     <algorithmic bytes per launch> [skip launches] [out.json]
e.g.   ... 1024x256 "flock_step_kernel<true, false, false" 1098909696"""
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
    fetch_csv, write_csv, key, sub, alg = sys.argv[1:6]
    alg = float(alg)
    skip = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    out = sys.argv[7] if len(sys.argv) > 7 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    kern = [k for k in f if sub in k][0]
    fv, wv = f[kern][skip:], w[kern][skip:]
    fetch_kib = sum(fv) / len(fv)
    write_kib = sum(wv) / len(wv)
    total = (2 * fetch_kib + write_kib) * 1024
    d = json.load(open(out)) if os.path.exists(out) else {}
    d[key] = {
        "kernel": kern, "launches": len(fv), "skipped_first_launches": skip,
        "FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib,
        "bytes_per_launch": total, "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": total / alg,
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE reads half)"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d[key], indent=1))


if __name__ == "__main__":
    main()

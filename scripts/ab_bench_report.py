"""Side-by-side ms_per_step of bench.py lines (scripts/ab_bench.sh): the headline and every
sub-object that has ms_per_step, per run, for two JSONL files."""
import json
import sys


def lines(path):
    out = []
    for ln in open(path):
        ln = ln.strip()
        if ln.startswith("{"):
            d = json.loads(ln)
            row = {"headline": d["ms_per_step"]}
            for k, v in d.items():
                if isinstance(v, dict) and "ms_per_step" in v:
                    row[k] = v["ms_per_step"]
            out.append(row)
    return out


a, b = lines(sys.argv[1]), lines(sys.argv[2])
keys = list(a[0]) if a else []
for k in keys:
    print("%-22s old %s   new %s" % (k, " ".join("%8.4f" % r.get(k, float("nan")) for r in a),
                                      " ".join("%8.4f" % r.get(k, float("nan")) for r in b)))

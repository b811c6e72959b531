"""Interleaved A/B of bench.py lines over several library builds on one box: ROUNDS
rounds, each running bench.py once per library (GYMFLOCK_LIB) in rotation, then the
median ms per step of every line per library.
  python scripts/ab_multi.py name=path/to/libgymflock.so ... [-- extra bench.py args]
Environment: ROUNDS (default 3), STEPS (20), WARMUP (5), OUT (gpurun_out/ab_multi)."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
argv = sys.argv[1:]
extra = []
if "--" in argv:
    i = argv.index("--")
    argv, extra = argv[:i], argv[i + 1:]
libs = [a.split("=", 1) for a in argv]
rounds = int(os.environ.get("ROUNDS", 3))
out = os.environ.get("OUT", os.path.join(ROOT, "gpurun_out", "ab_multi"))
os.makedirs(out, exist_ok=True)
res = {name: [] for name, _ in libs}
for r in range(rounds):
    for name, path in libs:
        env = dict(os.environ, GYMFLOCK_LIB=os.path.abspath(path))
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", os.environ.get("STEPS", "20"),
               "--warmup", os.environ.get("WARMUP", "5"), "--no-cpu-baseline"] + extra
        p = subprocess.run(cmd, env=env, capture_output=True, timeout=600)
        open(os.path.join(out, "%s_%d.err" % (name, r)), "wb").write(p.stderr)
        lines = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not lines:
            print("FAILED", name, r, p.returncode, p.stderr.decode()[-800:], flush=True)
            sys.exit(1)
        d = json.loads(lines[-1])
        open(os.path.join(out, "%s_%d.json" % (name, r)), "w").write(lines[-1] + "\n")
        row = {"plain": d["ms_per_step"]}
        for k, v in d.items():
            if isinstance(v, dict) and "ms_per_step" in v:
                row[k] = v["ms_per_step"]
        res[name].append(row)
        print("round %d %-10s %s" % (r, name, " ".join("%s=%.2f" % (k, 1e3 * v) for k, v in row.items())), flush=True)
print("median us per step")
keys = list(res[libs[0][0]][0])
for k in keys:
    print("%-22s %s" % (k, "  ".join("%s %8.2f" % (n, 1e3 * statistics.median(r[k] for r in res[n] if k in r))
                                     for n, _ in libs)))

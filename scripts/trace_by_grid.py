"""Kernel statistics of a rocprofv3 kernel trace split by kernel AND grid size, and the
step period of every bench workload, so the bench line's roofline fractions can be
rebuilt from tracked files (rocprofv3's own --stats lumps every grid of a kernel name
together: e.g. the drop-in N=100 launches with config 2's half batches).

  python scripts/trace_by_grid.py trace_kernel_trace.csv OUT_PREFIX [--steps K] [--skip 0]

writes OUT_PREFIX_kernels.csv (kernel, template args, grid, launches, avg / median / min /
max duration in ns) and OUT_PREFIX_periods.json: for each flock_step_kernel instantiation
and grid of the bench's workloads, its runs of back-to-back launches (an idle gap of more
than 30 us, e.g. the bench's sync and barrier around a timed region, splits runs; the
first `skip` launches of a run dropped; with --steps K only runs of 2K launches, the
bench's timed regions of K steps, are kept), the step period (two concurrent
half-batch launches per step: span of the run / (launches / 2), and the median distance
between the starts of launches k and k + 2), the algorithmic bytes per step and the
fraction of the 8 TB/s HBM peak. The bytes follow DESIGN.md §4 / bench.py: 4N^2 + 96N + 8
per env-step, + 16N with the controller's output, + N * (7*4 + 28*4 + 4 + 4) with the
7-nearest observation."""
import csv
import json
import re
import statistics
import sys

HBM_PEAK_GBS = 8000.0
# workgroups of one half-batch launch -> (agents, envs in the half, envs of the whole step)
HALVES = {128 * 32: (1024, 128, 256), 16 * 512: (8192, 16, 32)}


def short(name):
    m = re.search(r"(\w+)<([^()]*)>", name)
    return (m.group(1), m.group(2)) if m else (name.split("(")[0], "")


def main():
    path, out = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else None
    rows = list(csv.DictReader(open(path)))
    groups = {}
    for r in rows:
        k, targs = short(r["Kernel_Name"])
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0)
        groups.setdefault((k, targs, grid, wg), []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    with open(out + "_kernels.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "template_args", "grid_x", "workgroup_x", "workgroups", "launches", "avg_ns",
                    "median_ns", "min_ns", "max_ns"])
        for (k, targs, grid, wg), ev in sorted(groups.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
            d = [e - s for s, e in ev]
            w.writerow([k, targs, grid, wg, grid // max(wg, 1), len(d), round(statistics.mean(d)),
                        round(statistics.median(d)), min(d), max(d)])
    periods = []
    for (k, targs, grid, wg), ev in groups.items():
        if k != "flock_step_kernel" or wg == 0 or (grid // wg) not in HALVES:
            continue
        N, half_envs, envs = HALVES[grid // wg]
        a = [t.strip() for t in targs.split(",")]
        ctrl = len(a) > 2 and a[2] == "true"
        knn = len(a) > 5 and a[5] not in ("0", "")
        per_env = 4 * N * N + 96 * N + 8 + (16 * N if ctrl else 0) + (N * (7 * 4 + 28 * 4 + 4 + 4) if knn else 0)
        # the packed-output line runs the plain instantiation: told apart by its period,
        # which the dense bytes would put above the HBM peak
        packed_env = 8 * N * ((N + 63) // 64) + 4 * N + 96 * N + 8
        label = "step_with_controller" if ctrl else "flocking_v0_knn7" if knn else "plain"
        ev.sort()
        runs, cur = [], [ev[0]]
        for s, e in ev[1:]:
            if s - max(x[1] for x in cur[-4:]) > 30_000:
                runs.append(cur)
                cur = []
            cur.append((s, e))
        runs.append(cur)
        for run in runs:
            if steps is not None and abs(len(run) - 2 * steps) > 2:
                continue
            run = run[skip:]
            if len(run) < 20:
                continue
            span = max(e for _, e in run) - run[0][0]
            per = span / (len(run) / 2.0)
            med = statistics.median(run[i + 2][0] - run[i][0] for i in range(len(run) - 2))
            lab, step_bytes = label, per_env * envs
            if label == "plain" and step_bytes / (med * 1e-9) / 1e9 > HBM_PEAK_GBS:
                lab, step_bytes = "packed_network", packed_env * envs
            if N == 8192:
                lab = "n8192_config5"
            periods.append({"line": lab, "start_ns": run[0][0], "kernel": k, "template_args": targs, "N": N,
                            "envs_per_step": envs,
                            "launches": len(run), "span_us": span / 1e3,
                            "step_period_us_span": per / 1e3, "step_period_us_median": med / 1e3,
                            "algorithmic_bytes_per_step": step_bytes,
                            "frac_span": step_bytes / (per * 1e-9) / 1e9 / HBM_PEAK_GBS,
                            "frac_median": step_bytes / (med * 1e-9) / 1e9 / HBM_PEAK_GBS})
    periods.sort(key=lambda p: p["start_ns"])
    json.dump({"source": path, "skip_per_run": skip, "hbm_peak_gbs": HBM_PEAK_GBS, "runs": periods},
              open(out + "_periods.json", "w"), indent=1)
    for p in periods:
        print("%-22s %-62s N=%d launches %4d  period %.1f us (median %.1f)  frac %.3f / %.3f" % (
            p["line"], p["kernel"] + "<" + p["template_args"] + ">", p["N"], p["launches"], p["step_period_us_span"],
            p["step_period_us_median"], p["frac_span"], p["frac_median"]))


if __name__ == "__main__":
    main()

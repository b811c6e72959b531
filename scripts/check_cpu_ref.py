"""Check oracle/cpu_ref.py (bench.py's CPU baseline) against the reference itself.

Runs in the build container only (it imports /root/reference read-only through the
shims of tests/golden/make_golden.py). For N = 256 and 1024 (config 2's agent count),
from the same synthetic state and float32 actions:
  * outputs: state, state_values, network, reward and controller of the reference's
    FlockingRelativeEnv and of CpuFlock must be bitwise equal (same array operations);
  * time: step() and step()+controller() of both, interleaved, best of several rounds,
    one thread; CpuFlock must be within +-15 % of the reference.
Coverage (config 4: R=200 robots, the map of global seed 8, max_nodes 1000): the
reference's CoverageEnv and oracle/cpu_ref_coverage.CpuCoverage from the same starts,
unvisited set and random actions: every step's observation, reward and done bitwise
equal, and the step time within +-15 %.
Writes the result to profiles/r03/cpu_ref_check.json.

  OMP_NUM_THREADS=1 python scripts/check_cpu_ref.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import make_golden as mg  # noqa: E402
from oracle.cpu_ref import CpuFlock  # noqa: E402
from oracle.flocking import synthetic_state  # noqa: E402


def ref_env(x, n):
    mg._install_shims()
    import importlib
    fr = importlib.import_module("gym_flock.envs.flocking.flocking_relative")
    env = fr.FlockingRelativeEnv()
    env.params_from_cfg(mg._Cfg(comm_radius=0.9, n_agents=n, v_max=5.0, dt=0.01))
    env.x = np.array(x, dtype=np.float64)
    return env


def coverage_case(rounds=3, steps=30):
    import importlib
    from oracle.cpu_ref_coverage import CpuCoverage
    mg._install_shims()
    cov = importlib.import_module("gym_flock.envs.spatial.coverage")
    R, M = 200, 1000
    np.random.seed(8)
    ref = cov.CoverageEnv(n_robots=R, nearby_starts=False, max_nodes=M)
    ref.seed(9)
    np.random.seed(8)
    ref.reset()
    T = ref.n_targets
    ours = CpuCoverage(ref.x[R:, :2], R, M)
    start = ref.closest_targets - R
    ours.reset(start, np.nonzero(ref.visited[:, 0] == 0)[0])
    rs = np.random.RandomState(7)
    acts = [rs.randint(0, 4, size=(R, 1)) for _ in range(steps)]
    same = True
    for a in acts[:10]:
        o1, r1, d1, _ = ref.step(a)
        o2, r2, d2, _ = ours.step(a)
        same &= bool(r1 == r2 and d1 == d2 and np.array_equal(ref.x, ours.x) and
                     all(np.array_equal(o1[k], o2[k]) for k in ref.keys))
    t = {"ref_step": [], "ours_step": []}
    for _ in range(rounds):
        for name, env in (("ref", ref), ("ours", ours)):
            t0 = time.perf_counter()
            for a in acts:
                env.step(a)
            t[name + "_step"].append((time.perf_counter() - t0) / steps)
    best = {k: 1e3 * min(v) for k, v in t.items()}
    ratio = best["ours_step"] / best["ref_step"]
    return {"workload": "Coverage-v0 R=%d T=%d max_nodes %d" % (R, T, M), "bitwise_equal": bool(same), "ms": best,
            "ratio_step": ratio, "within_15pct": bool(abs(ratio - 1) <= 0.15)}


def main():
    out = {"cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "numpy": np.__version__, "cases": []}
    ok = True
    for n, rounds, steps in ((256, 5, 20), (1024, 3, 6)):
        x0 = synthetic_state(n, 0)
        u = np.random.RandomState(1234).uniform(-1, 1, size=(n, 2)).astype(np.float32)
        ref, ours = ref_env(x0, n), CpuFlock(x0)
        (sv_r, net_r), rw_r, _, _ = ref.step(u)
        (sv_o, net_o), rw_o, _, _ = ours.step(u)
        same = (np.array_equal(ref.x, ours.x) and np.array_equal(sv_r, sv_o) and np.array_equal(net_r, net_o)
                and rw_r == rw_o and np.array_equal(ref.controller(), ours.controller())
                and np.array_equal(ref.controller(False), ours.controller(False)))
        t = {"ref_step": [], "ours_step": [], "ref_ctrl": [], "ours_ctrl": []}
        for _ in range(rounds):
            for name, env in (("ref", ref), ("ours", ours)):
                t0 = time.perf_counter()
                for _ in range(steps):
                    env.step(u)
                t1 = time.perf_counter()
                for _ in range(steps):
                    env.step(u)
                    env.controller()
                t2 = time.perf_counter()
                t[name + "_step"].append((t1 - t0) / steps)
                t[name + "_ctrl"].append((t2 - t1) / steps)
        best = {k: 1e3 * min(v) for k, v in t.items()}
        ratio = best["ours_step"] / best["ref_step"]
        ratio_c = best["ours_ctrl"] / best["ref_ctrl"]
        case = {"n_agents": n, "bitwise_equal": bool(same), "ms": best, "ratio_step": ratio, "ratio_step_ctrl": ratio_c,
                "within_15pct": bool(abs(ratio - 1) <= 0.15 and abs(ratio_c - 1) <= 0.15)}
        ok &= case["bitwise_equal"] and case["within_15pct"]
        out["cases"].append(case)
        print(json.dumps(case))
    case = coverage_case()
    ok &= case["bitwise_equal"] and case["within_15pct"]
    out["cases"].append(case)
    print(json.dumps(case))
    out["ok"] = bool(ok)
    os.makedirs(os.path.join(ROOT, "profiles", "r03"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r03", "cpu_ref_check.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("ok" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())

"""Check oracle/cpu_ref.py (bench.py's CPU baseline) against the reference itself.

Runs in the build container only (it imports /root/reference read-only through the
shims of tests/golden/make_golden.py). For N = 256 and 1024 (config 2's agent count),
from the same synthetic state and float32 actions:
  * outputs: state, state_values, network, reward and controller of the reference's
    FlockingRelativeEnv and of CpuFlock must be bitwise equal (same array operations);
  * time: step() and step()+controller() of both, interleaved, best of several rounds,
    one thread; CpuFlock must be within +-15 % of the reference.
Writes the result to profiles/r02/cpu_ref_check.json.

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
    out["ok"] = bool(ok)
    os.makedirs(os.path.join(ROOT, "profiles", "r02"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r02", "cpu_ref_check.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("ok" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())

"""Coverage config 4 (512 envs x R=200, max_nodes 1000, map seed 8) greedy expert step
(COV_ACTIONS_GREEDY: greedy actions and the step in one launch per half batch) in the
steady state (thousands of steps from one reset: every target visited, every robot on
its fallback) and inside episodes (reset every 75 steps, EPISODE_LENGTH): device time
per step over windows of 5 steps through an episode, and the wall time per step.

  python scripts/cov_greedy_probe.py            (JSON on stdout)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]

from oracle.maps_host import generate_targets  # noqa: E402
from gym_flock.vec import VecCoverage  # noqa: E402


def main():
    R, B, M = 200, 512, 1000
    np.random.seed(8)
    targets = generate_targets()
    v = VecCoverage(B, R, max_nodes=M, episode_length=10 ** 9)
    v.set_targets(targets)
    v.reset(seed=0)
    t0 = time.perf_counter()
    v.h.controller_greedy(fetch=False)
    v.sync()
    out = {"time_matrix_ms": 1e3 * (time.perf_counter() - t0), "n_targets": len(targets)}
    streams = int(os.environ.get("STREAMS", "0"))
    v.h.set_streams(streams)
    out["streams"] = streams

    def window(k, fn):
        v.sync()
        v.h.timing_start(1)
        t = time.perf_counter()
        for _ in range(k):
            fn()
        v.sync()
        wall = time.perf_counter() - t
        ms, n = v.h.timing_stop()
        return 1e3 * wall / k, ms

    greedy = lambda: v.step(greedy=True)  # noqa: E731
    for _ in range(3000):  # the steady state: every target visited
        greedy()
    out["steady_wall_ms"], out["steady_device_ms"] = window(500, greedy)
    per_win = np.zeros((15, 2))
    eps = 6
    for e in range(eps):
        v.reset(seed=100 + e)
        for w in range(15):
            wall, dev = window(5, greedy)
            per_win[w] += (wall / eps, dev / eps)
    out["episode_windows_wall_ms"] = per_win[:, 0].round(5).tolist()
    out["episode_windows_device_ms"] = per_win[:, 1].round(5).tolist()
    ep_wall = 0.0
    for e in range(eps):
        v.reset(seed=200 + e)
        v.sync()
        t = time.perf_counter()
        for _ in range(75):
            greedy()
        v.sync()
        ep_wall += time.perf_counter() - t
    out["episode_wall_ms_per_step"] = 1e3 * ep_wall / (75 * eps)
    rs = np.random.RandomState(7)
    v.set_actions(rs.randint(0, 4, size=(B, R)))
    ep_wall = 0.0
    for e in range(eps):
        v.reset(seed=300 + e)
        v.sync()
        t = time.perf_counter()
        for _ in range(75):
            v.step(resident=True)
        v.sync()
        ep_wall += time.perf_counter() - t
    out["episode_random_wall_ms_per_step"] = 1e3 * ep_wall / (75 * eps)
    v.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Kernel makeup of a drop-in Coverage-v0 greedy episode's first step (the new map's time
matrix): one CoverageEnv (R from the environment, default 6), greedy expert episodes in the
default direct mode; run under rocprofv3 --kernel-trace and split by step."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock.envs.spatial import CoverageEnv  # noqa: E402

R = int(os.environ.get("R", 6))
np.random.seed(8)
env = CoverageEnv(n_robots=R, nearby_starts=R <= 6, max_nodes=1000)
env.seed(3)
for ep in range(int(os.environ.get("EPISODES", 4))):
    env.reset()
    done, k = False, 0
    while not done:
        t0 = time.perf_counter()
        _, _, done, _ = env.step(env.controller(greedy=True))
        if k < 2:
            print("episode %d step %d: %.1f us" % (ep, k, 1e6 * (time.perf_counter() - t0)), flush=True)
        k += 1
env.close()

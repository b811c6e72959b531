"""Greedy-expert step timing for A/B work (run on the GPU box): config 4's batch (512
envs x 200 robots, one generated map); after the time matrices are built, ROUNDS rounds
of K (device greedy controller + resident step); prints the wall time per expert step.
GYMFLOCK_LIB selects the library (default: the working tree's)."""
import os
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."), os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-flock_amd")]
from oracle.maps_host import generate_targets  # noqa: E402
from gym_flock.vec import VecCoverage  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "run"
R, B, M, K = 200, 512, 1000, 200
np.random.seed(8)
targets = generate_targets()
v = VecCoverage(B, R, max_nodes=M, episode_length=10 ** 9)
v.set_targets(targets)
walls = []
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    v.reset(seed=rnd)
    v.h.controller_greedy(fetch=False)
    v.sync()
    t0 = time.perf_counter()
    for _ in range(K):
        v.h.controller_greedy(fetch=False)
        v.step(resident=True)
    v.sync()
    walls.append(1e6 * (time.perf_counter() - t0) / K)
print("%-8s expert step median %6.2f us (min %6.2f)" % (tag, np.median(walls), np.min(walls)))
v.close()

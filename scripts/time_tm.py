"""Time-matrix build time (construct_time_matrix for all envs) at config 4: 512 envs x
200 robots on one generated map; ROUNDS rebuilds (set_targets invalidates every env's
matrix), each followed by one greedy step. GYMFLOCK_LIB selects the library."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-flock_amd"))
from oracle.maps_host import generate_targets  # noqa: E402
from gym_flock.vec import VecCoverage  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "run"
R, B, M = 200, 512, 1000
np.random.seed(8)
targets = generate_targets()
v = VecCoverage(B, R, max_nodes=M, episode_length=10 ** 9)
v.set_targets(targets)
v.reset(seed=0)
ms = []
for rnd in range(int(os.environ.get("ROUNDS", "4"))):
    v.set_targets(targets)
    v.sync()
    t0 = time.perf_counter()
    v.h.controller_greedy(fetch=False)
    v.sync()
    ms.append(1e3 * (time.perf_counter() - t0))
print("%-8s time matrix + greedy step, all %d envs: median %.2f ms (min %.2f)" % (tag, B, np.median(ms), np.min(ms)))
v.close()

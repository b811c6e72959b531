"""Time-matrix build time (construct_time_matrix + greedy lists for all envs) at config 4:
512 envs x 200 robots, each env its own device map (cov_generate_maps, streams seeded
8 + b); ROUNDS rebuilds (a new map for every env each round, untimed), each followed by
one greedy step's actions. GYMFLOCK_LIB selects the library. Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock.vec import VecCoverage  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "run"
R, B, M = 200, 512, 1000
v = VecCoverage(B, R, max_nodes=M, episode_length=75)
v.reset(seed=0, new_maps=True, map_seed=8)
v.h.controller_greedy(fetch=False)
ms = []
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    v.reset(seed=rnd, new_maps=True)
    v.sync()
    t0 = time.perf_counter()
    v.h.controller_greedy(fetch=False)
    v.sync()
    ms.append(1e3 * (time.perf_counter() - t0))
print(json.dumps({"tag": tag, "envs": B, "tm_and_lists_ms_median": float(np.median(ms)), "min": float(np.min(ms)),
                  "all": ms}))
v.close()

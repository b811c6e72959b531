"""The batched reset with device draws (cov_seed_reset_kernel + cov_reset), for A/B work (run
on the GPU box): config 4's batch (512 envs x 200 robots, the bench's map), ROUNDS rounds of
10 timed reset(seed) calls each; prints the median and min ms per reset over the rounds.
GYMFLOCK_LIB selects the library (default: the working tree's)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from oracle.maps_host import generate_targets  # noqa: E402
from gym_flock.vec import VecCoverage  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "run"
R, B, M = 200, 512, 1000
np.random.seed(8)
v = VecCoverage(B, R, max_nodes=M, episode_length=75)
v.set_targets(generate_targets())
for s in range(5):
    v.reset(seed=s)
v.sync()
per = []
for r in range(int(os.environ.get("ROUNDS", "10"))):
    t0 = time.perf_counter()
    for e in range(10):
        v.reset(seed=100 + 10 * r + e)
    v.sync()
    per.append(1e3 * (time.perf_counter() - t0) / 10)
print(json.dumps({"tag": tag, "ms_per_reset_median": float(np.median(per)), "min": float(np.min(per)),
                  "all": [round(x, 4) for x in per]}))
v.close()

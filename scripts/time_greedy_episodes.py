"""Fused greedy expert steps in episodes, for A/B work (run on the GPU box): config 4's
batch (512 envs x 200 robots, the bench's map), after the time matrices are built,
EPISODES episodes of reset(seed) + 75 v.step(greedy=True) (the device fallback draws),
the resets untimed; prints the median and min us per expert step over the episodes.
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
if os.environ.get("STREAMS"):  # launches per step (cov_set_streams: 1 or 2; default: 2 for greedy steps)
    v.h.set_streams(int(os.environ["STREAMS"]))
v.reset(seed=0)
v.step(greedy=True)  # builds the time matrices and greedy lists
v.sync()
per = []
for e in range(int(os.environ.get("EPISODES", "8"))):
    v.reset(seed=100 + e)
    v.sync()
    t0 = time.perf_counter()
    for _ in range(75):
        v.step(greedy=True)
    v.sync()
    per.append(1e6 * (time.perf_counter() - t0) / 75)
print(json.dumps({"tag": tag, "us_per_expert_step_median": float(np.median(per)), "min": float(np.min(per)),
                  "all": [round(x, 2) for x in per]}))
v.close()

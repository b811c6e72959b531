"""Expert episodes as one launch each (cov_step_expert), for A/B work (run on the GPU box):
config 4's batch (512 envs x 200 robots, the bench's map), after the time matrices are built,
EPISODES episodes of reset(seed) + expert_steps(75, fetch=False), timed together with their
resets as bench.py's expert_episode_ms_all_envs_one_launch; prints the median and min ms per
episode over ROUNDS rounds. GYMFLOCK_LIB selects the library (default: the working tree's)."""
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
v.reset(seed=0)
v.step(greedy=True)  # builds the time matrices and greedy lists
v.expert_steps(75, fetch=False)
v.sync()
per = []
eps = int(os.environ.get("EPISODES", "4"))
for r in range(int(os.environ.get("ROUNDS", "10"))):
    t0 = time.perf_counter()
    for e in range(eps):
        v.reset(seed=600 + e)
        v.expert_steps(75, fetch=False)
    v.sync()
    per.append(1e3 * (time.perf_counter() - t0) / eps)
print(json.dumps({"tag": tag, "ms_per_episode_median": float(np.median(per)), "min": float(np.min(per)),
                  "all": [round(x, 3) for x in per]}))
v.close()

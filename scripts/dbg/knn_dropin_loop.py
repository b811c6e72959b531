"""200 drop-in Flocking-v0 steps at N=100 (fetch_mode "direct"), for a rocprofv3 kernel trace."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock.envs.flocking.flocking import FlockingEnv  # noqa: E402
from gym_flock.init_states import synthetic_state  # noqa: E402

n = int(os.environ.get("N", 100))
env = FlockingEnv()
env.n_agents = n
env._make_spaces()
env.x = synthetic_state(n, 0)
env.compute_helpers()
u = np.random.RandomState(5).uniform(-1, 1, size=(n, 2)).astype(np.float32)
for _ in range(200):
    env.step(u)
env.close()
print("done")

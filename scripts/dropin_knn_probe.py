"""Drop-in Flocking-v0 step latency (run on the GPU box): FlockingEnv.step(u) per call at
N=100 and 1024, B=1 (observation = the 7-nearest-neighbour rows), beside
FlockingRelativeEnv.step(u).
  python scripts/dropin_knn_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock.envs.flocking.flocking import FlockingEnv  # noqa: E402
from gym_flock.envs.flocking.flocking_relative import FlockingRelativeEnv  # noqa: E402
from gym_flock.init_states import synthetic_state  # noqa: E402


def per_call(fn, k=300):
    for _ in range(20):
        fn()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    return 1e6 * (time.perf_counter() - t0) / k


for n in (100, 1024):
    out = []
    for cls, mode in ((FlockingRelativeEnv, "direct"), (FlockingEnv, "pooled"), (FlockingEnv, "direct")):
        env = cls()
        env.fetch_mode = mode
        env.n_agents = n
        env._make_spaces()
        env.x = synthetic_state(n, 0)
        env.compute_helpers()
        u = np.random.RandomState(5).uniform(-1, 1, size=(n, 2)).astype(np.float32)
        out.append("%s[%s] %.1f us" % (cls.__name__, mode, per_call(lambda: env.step(u))))
        env.close()
    print("N=%d  " % n + "  ".join(out), flush=True)

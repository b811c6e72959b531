"""Drop-in Flocking-v0 step (FlockingEnv.step(u), one env, direct mode) per call over a
range of N, for an A/B of the one-env exact in-step ranking (run with GYMFLOCK_LIB set to
each build).   python scripts/dropin_exact_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock.envs.flocking.flocking import FlockingEnv  # noqa: E402
from gym_flock.init_states import synthetic_state  # noqa: E402


def per_call(fn, k=300):
    for _ in range(30):
        fn()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    return 1e6 * (time.perf_counter() - t0) / k


out = []
for n in (128, 192, 256, 384, 512, 768, 1024):
    env = FlockingEnv()
    env.n_agents = n
    env._make_spaces()
    env.x = synthetic_state(n, 0)
    env.compute_helpers()
    u = np.random.RandomState(5).uniform(-1, 1, size=(n, 2)).astype(np.float32)
    out.append("N=%d %.1f" % (n, per_call(lambda: env.step(u))))
    env.close()
print(os.environ.get("GYMFLOCK_LIB", "product"), "  ".join(out), flush=True)

"""Where the drop-in single-env step's time goes (run on the GPU box): per call at N=100 and
1024, B=1, the pieces of FlockingRelativeEnv.step: the host-action step alone (upload +
launch, no wait), a stream sync after it, the batched output fetch into pool arrays, and
the whole env.step; plus a resident-action step + sync (no upload) for the launch floor.
  python scripts/dropin_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock import _native as nat  # noqa: E402
from gym_flock.envs.flocking.flocking_relative import FlockingRelativeEnv  # noqa: E402
from gym_flock.init_states import synthetic_state  # noqa: E402


def per_call(fn, k=400):
    for _ in range(20):
        fn()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    return 1e6 * (time.perf_counter() - t0) / k


for n in (100, 1024):
    env = FlockingRelativeEnv()
    env.n_agents = n
    env._make_spaces()
    env.fetch_mode = "pooled"
    env.x = synthetic_state(n, 0)
    env.compute_helpers()
    h = env._handle()
    u = np.random.RandomState(5).uniform(-1, 1, size=(n, 2)).astype(np.float32)
    u32 = u[None]
    pool = nat.host_pool()
    res = {}
    res["step(u)+sync"] = per_call(lambda: (h.step(u32), h.sync()))
    h.set_actions(u32)  # (a host-action step replaces the resident actions)
    res["resident step+sync"] = per_call(lambda: (h.step(None, nat.FE_U_RESIDENT), h.sync()))
    res["sync only"] = per_call(lambda: h.sync())
    res["outputs(pool)"] = per_call(lambda: h.outputs(0, pool=pool))
    res["step(u)+outputs(pool)"] = per_call(lambda: (h.step(u32), h.outputs(0, pool=pool)))
    res["env.step(u)"] = per_call(lambda: env.step(u))
    print("N=%d " % n + "  ".join("%s %.1f us" % (k, v) for k, v in res.items()))
    env.close()

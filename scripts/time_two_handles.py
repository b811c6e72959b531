"""Launch overlap across HIP streams at config 2 (256 envs x N=1024): wall time per
256-env step for the batch on one handle (1 or 2 launches per step, fe_set_streams)
and split over several handles, each with its own stream(s), launched alternately."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock import _native as nat  # noqa: E402
from gym_flock.init_states import synthetic_batch  # noqa: E402

N, B, K = int(os.environ.get("N", 1024)), int(os.environ.get("B", 256)), 100
x0 = synthetic_batch(B, N)
u = np.random.RandomState(0).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)


def make(parts, streams):
    cuts = np.linspace(0, B, parts + 1).round().astype(int)
    hs = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        h = nat.FlockHandle(N, int(b - a))
        h.set_streams(streams)
        h.set_actions(u[a:b])
        hs.append((h, a, b))
    return hs


setups = {"1 handle, 1 stream": make(1, 1), "1 handle, 2 streams": make(1, 2),
          "2 handles, 1 stream each": make(2, 1), "3 handles, 1 stream each": make(3, 1),
          "2 handles, 2 streams each": make(2, 2)}
res = {k: [] for k in setups}
for rnd in range(4):
    for name, hs in setups.items():
        for h, a, b in hs:
            h.set_state(x0[a:b])
        for _ in range(10):
            for h, _, _ in hs:
                h.step(None, nat.FE_U_RESIDENT)
        for h, _, _ in hs:
            h.sync()
        t0 = time.perf_counter()
        for _ in range(K):
            for h, _, _ in hs:
                h.step(None, nat.FE_U_RESIDENT)
        for h, _, _ in hs:
            h.sync()
        res[name].append((time.perf_counter() - t0) / K * 1e6)
for name, v in res.items():
    print("%-28s %.1f us per %d-env step (median of 4; min %.1f)" % (name, np.median(v), B, min(v)))

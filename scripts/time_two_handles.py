"""Does splitting the config-2 batch over two handles (two HIP streams, 128 envs each,
launched alternately) overlap one launch's store tail with the other's compute head?
Prints wall time per step of the whole 256-env batch for 1 handle vs 2 (and 4)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock import _native as nat  # noqa: E402
from gym_flock.init_states import synthetic_batch  # noqa: E402

N, B, K = 1024, 256, 200
x0 = synthetic_batch(B, N)
u = np.random.RandomState(0).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)


def make(parts):
    hs = []
    per = B // parts
    for p in range(parts):
        h = nat.FlockHandle(N, per)
        h.set_state(x0[p * per:(p + 1) * per])
        h.set_actions(u[p * per:(p + 1) * per])
        hs.append(h)
    return hs


setups = {p: make(p) for p in (1, 2, 4)}
res = {p: [] for p in setups}
for rnd in range(5):
    for p, hs in setups.items():
        for i, h in enumerate(hs):
            h.set_state(x0[i * (B // p):(i + 1) * (B // p)])
        for _ in range(10):
            for h in hs:
                h.step(None, nat.FE_U_RESIDENT)
        for h in hs:
            h.sync()
        t0 = time.perf_counter()
        for _ in range(K):
            for h in hs:
                h.step(None, nat.FE_U_RESIDENT)
        for h in hs:
            h.sync()
        res[p].append((time.perf_counter() - t0) / K * 1e6)
for p, v in res.items():
    print("%d handle(s) x %3d envs: %.1f us per 256-env step (median of 5; min %.1f)" % (p, B // p, np.median(v), min(v)))

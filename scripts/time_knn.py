"""Flocking-v0 step (step + 7-NN observation) at config 2: wall time per step on a
fixed workload (state reset before every step) for the synthetic init and for the
same swarm after 300 random steps (dispersed: more agents below 7 neighbours)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock import _native as nat  # noqa: E402
from gym_flock.init_states import synthetic_batch  # noqa: E402

N, B, K = int(os.environ.get("N", 1024)), int(os.environ.get("B", 256)), 30
h = nat.FlockHandle(N, B, n_neighbors=7)
if os.environ.get("DIAG"):  # ablation switches (fe_diag), e.g. DIAG=0x4000
    h.diag_switches(int(os.environ["DIAG"], 0))
x0 = synthetic_batch(B, N)
h.set_actions(np.random.RandomState(0).uniform(-1, 1, size=(B, N, 2)).astype(np.float32))
h.set_state(x0)
for _ in range(300):
    h.step(None, nat.FE_U_RESIDENT)
x300 = h.get_state()
for label, x in (("init", x0), ("after 300 steps", x300)):
    h.set_state(x)
    _, _, deg = h.stats()
    for flags, name in ((nat.FE_U_RESIDENT, "step"), (nat.FE_U_RESIDENT | nat.FE_WITH_KNN, "step+knn")):
        ts = []
        for _ in range(K):
            h.set_state(x)
            h.sync()
            t0 = time.perf_counter()
            h.step(None, flags)
            h.sync()
            ts.append(time.perf_counter() - t0)
        print("%-16s %-9s median %.1f us   (agents with < 7 neighbours: %.1f%%)"
              % (label, name, 1e6 * np.median(ts), 100 * np.mean(deg < 7)))

"""Flocking-v0 kernel costs in isolation along the bench workload's trajectory (config 2,
synthetic init, the same resident random actions every step): for the states after
0, 25, 50, 100 and 200 steps, REPS x [set_state, plain step, sync], REPS x [set_state,
fused step + rim kNN, sync] and REPS x
[set_state, full kNN (fe_get_knn without a step)]. Run under rocprofv3 --kernel-trace;
scripts/knn_phases_report.py splits the trace by state."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock import _native as nat  # noqa: E402
from gym_flock.init_states import synthetic_batch  # noqa: E402

N, B, REPS = int(os.environ.get("N", 1024)), int(os.environ.get("B", 256)), 5
h = nat.FlockHandle(N, B, n_neighbors=7)
if os.environ.get("DIAG"):  # ablation switches (diagnostic build: GYMFLOCK_LIB=build/lib_diag/...)
    h.diag_switches(int(os.environ["DIAG"], 0))
h.set_actions(np.random.RandomState(1234).uniform(-1, 1, size=(B, N, 2)).astype(np.float32))
h.set_state(synthetic_batch(B, N, seed0=0))
t = 0
for target in (0, 25, 50, 100, 200):
    while t < target:
        h.step(None, nat.FE_U_RESIDENT)
        t += 1
    x = h.get_state()
    _, _, deg = h.stats()
    print("state t=%d: %.1f%% of agents below 7 neighbours" % (t, 100 * np.mean(deg < 7)), flush=True)
    for _ in range(REPS):
        h.set_state(x)
        h.step(None, nat.FE_U_RESIDENT)
        h.sync()
    for _ in range(REPS):
        h.set_state(x)
        h.step(None, nat.FE_U_RESIDENT | nat.FE_WITH_KNN)
        h.sync()
    for _ in range(REPS):
        h.set_state(x)
        h.knn(0)
    h.set_state(x)
h.close()

"""Cell-list step A/B helper (run on the GPU box): wall us per step of the plain step at
N agents x B envs with one or two launches per step (fe_set_streams), synthetic init,
resident random actions, clock warm-up, K steps. GYMFLOCK_LIB selects the library.
  N=8192 B=32 STREAMS=1 python scripts/time_grid.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-flock_amd"))
from gym_flock.vec import VecFlockingRelative  # noqa: E402

N, B = int(os.environ.get("N", 8192)), int(os.environ.get("B", 32))
K = int(os.environ.get("K", 20))
env = VecFlockingRelative(B, N)
env.h.set_streams(int(os.environ.get("STREAMS", 2)))
if os.environ.get("DIAG"):  # ablation switches (diagnostic build: GYMFLOCK_LIB=build/lib_diag/...)
    env.h.diag_switches(int(os.environ["DIAG"], 0))
x0 = env.reset(seed=0)
env.set_actions(np.random.RandomState(1234).uniform(-1, 1, size=(B, N, 2)).astype(np.float32))
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    for _ in range(4):
        env.step(resident=True)
    env.sync()
env.reset(x=x0)
for _ in range(3):
    env.step(resident=True)
env.sync()
t0 = time.perf_counter()
for _ in range(K):
    env.step(resident=True)
env.sync()
el = time.perf_counter() - t0
print("N=%d B=%d streams=%s diag=%s: %.1f us/step" % (N, B, os.environ.get("STREAMS", 2), os.environ.get("DIAG", "0"),
                                                     1e6 * el / K))
env.close()

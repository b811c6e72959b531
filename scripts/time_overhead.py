"""Per-step wall time of the bench workload with and without per-launch HIP event
timing (fe_kernel_timing), to size the timing overhead inside bench.py's timed region."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock.vec import VecFlockingRelative  # noqa: E402

v = VecFlockingRelative(256, 1024)
v.reset(seed=0)
v.set_actions(np.random.RandomState(1234).uniform(-1, 1, size=(256, 1024, 2)).astype(np.float32))
K = 200
for rnd in range(3):
    for timed in (False, True):
        v.reset(seed=0)
        for _ in range(20):
            v.step(resident=True)
        v.sync()
        if timed:
            v.h.timing_start()
        t0 = time.perf_counter()
        for _ in range(K):
            v.step(resident=True)
        v.sync()
        el = time.perf_counter() - t0
        kms = v.h.timing_stop()[0] if timed else float("nan")
        print("round %d timed=%d: %.1f us/step wall, kernel %.1f us" % (rnd, timed, 1e6 * el / K, 1e3 * kms))

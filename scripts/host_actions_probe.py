"""Host-action steps in short and long windows (run on the GPU box): the bench's config-2
workload (256 envs x 1024 agents), env.step(u) with the same pageable float32 (B,N,2)
array every call, against the resident-action step. Each window is bracketed by a device
sync like bench.py's timed(); prints ms per step per window, the ratio to the resident
step, and the host time of each of the first 6 calls of the window (where a fixed cost
of the window would show)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock.vec import VecFlockingRelative  # noqa: E402

B, N = 256, 1024
env = VecFlockingRelative(B, N)
x0 = env.reset(seed=0)
u = np.random.RandomState(1234).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
env.set_actions(u)


def window(k, fn):
    env.sync()
    calls = []
    t0 = time.perf_counter()
    for _ in range(k):
        c0 = time.perf_counter()
        fn()
        calls.append(1e6 * (time.perf_counter() - c0))
    env.sync()
    return 1e3 * (time.perf_counter() - t0) / k, calls


for _ in range(300):
    env.step(resident=True)
res = {}
for k in (20, 200):
    res[k] = min(window(k, lambda: env.step(resident=True))[0] for _ in range(3))
    print("resident  K=%3d  %.4f ms/step" % (k, res[k]))
for warm in (1, 5, 50):
    for k in (20, 200):
        env.reset(x=x0)
        for _ in range(warm):
            env.step(u)
        ms, calls = window(k, lambda: env.step(u))
        print("host u    warm %2d  K=%3d  %.4f ms/step  ratio %.3f  first calls (us) %s  median call %.1f us" %
              (warm, k, ms, ms / res[k], " ".join("%.0f" % c for c in calls[:6]), float(np.median(calls))))
# the bench's sequence: packed-output steps, a reset, 5 host-action warm-up steps, then
# the window with and without the HIP-event timing window bench.py's timed() opens
for timing in (False, True, False, True):
    for _ in range(50):
        env.step(resident=True, network="packed")
    env.reset(x=x0)
    for _ in range(5):
        env.step(u)
    if timing:
        env.h.timing_start(every=8)
    ms, calls = window(20, lambda: env.step(u))
    if timing:
        env.h.timing_stop()
    print("bench seq timing %d  K= 20  %.4f ms/step  ratio %.3f  first calls (us) %s  median call %.1f us" %
          (timing, ms, ms / res[20], " ".join("%.0f" % c for c in calls[:6]), float(np.median(calls))))
# after closed-loop controller steps (the bench's controller line runs before the host line)
for rep in range(2):
    env.reset(x=x0)
    env.controller()
    for _ in range(300):
        env.step(expert=True, controller=True)
    env.reset(x=x0)
    for _ in range(5):
        env.step(u)
    ms, calls = window(20, lambda: env.step(u))
    print("after ctrl       K= 20  %.4f ms/step  ratio %.3f  first calls (us) %s  median call %.1f us" %
          (ms, ms / res[20], " ".join("%.0f" % c for c in calls[:6]), float(np.median(calls))))
env.close()

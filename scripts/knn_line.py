"""Flocking-v0 line alone (config 2 + 7-NN observation), for rocprofv3 kernel traces.

  rocprofv3 --kernel-trace --stats -d gpurun_out/knnprof -o run -- python scripts/knn_line.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-flock_amd"))
sys.path.insert(0, ROOT)

from gym_flock.vec import VecFlockingRelative  # noqa: E402


def main():
    N, B = 1024, 256
    steps = int(os.environ.get("KSTEPS", "50"))
    knn = os.environ.get("KNN", "1") == "1"
    other = None
    if os.environ.get("OTHER"):  # a second config-2 handle alive beside it (as in bench.py)
        other = VecFlockingRelative(B, N)
        other.reset(seed=0)
    env = VecFlockingRelative(B, N, n_neighbors=7)
    if os.environ.get("DIAG"):  # ablation switches (diagnostic build: GYMFLOCK_LIB=build/lib_diag/...)
        env.h.diag_switches(int(os.environ["DIAG"], 0))
    x0 = env.reset(seed=0)
    u = np.random.RandomState(1234).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    if os.environ.get("LAYOUT") == "lattice":  # worst case: exact ties in every row, every step
        w = int(np.ceil(np.sqrt(N)))
        x0 = np.zeros((B, N, 4))
        x0[:, :, 0] = 0.25 * (np.arange(N) % w)
        x0[:, :, 1] = 0.25 * (np.arange(N) // w)
        u[:] = 0.0
        env.reset(x=x0)
    env.set_actions(u)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < float(os.environ.get("CLOCK_S", "0.3")):
        for _ in range(8):
            env.step(resident=True, knn=knn)
        env.sync()
    env.reset(x=x0)
    for _ in range(int(os.environ.get("WARM", "0"))):  # warm-up steps after the reset (bench: 5)
        env.step(resident=True, knn=knn)
    env.sync()
    if os.environ.get("TIMING"):  # the bench's device timing window
        env.h.timing_start(every=8)
    t0 = time.perf_counter()
    for _ in range(steps):
        env.step(resident=True, knn=knn)
    env.sync()
    if os.environ.get("TIMING"):
        env.h.timing_stop()
    print("knn=%d %.1f us/step" % (knn, 1e6 * (time.perf_counter() - t0) / steps))
    env.close()


if __name__ == "__main__":
    main()

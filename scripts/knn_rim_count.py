"""Rows the fused Flocking-v0 step leaves to the rim kNN, per step of the bench workload
(diagnostic build, ablation 0x400: the rim kernel does no work, so those rows keep
idx = -1). Prints, every few steps, the fraction of rows and of 256-row blocks and of
32-row step blocks holding such rows.
  GYMFLOCK_LIB=build/lib_diag/libgymflock.so python scripts/knn_rim_count.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-flock_amd"))

from gym_flock.vec import VecFlockingRelative  # noqa: E402


def main():
    N, B = 1024, 256
    steps = int(os.environ.get("KSTEPS", "200"))
    env = VecFlockingRelative(B, N, n_neighbors=7)
    env.h.diag_switches(0x400)
    env.reset(seed=0)
    env.set_actions(np.random.RandomState(1234).uniform(-1, 1, size=(B, N, 2)).astype(np.float32))
    for t in range(steps):
        env.step(resident=True, knn=True)
        if t < 30 or t % 10 == 0:
            idx, _ = env.knn()
            slow = idx[:, :, 0] < 0
            b256 = slow.reshape(B, N // 256, 256).any(axis=2)
            b32 = slow.reshape(B, N // 32, 32).any(axis=2)
            per32 = slow.reshape(B, N // 32, 32).sum(axis=2)
            print("step %3d rows %.4f blocks256 %.3f blocks32 %.3f max/32-block %d" %
                  (t, slow.mean(), b256.mean(), b32.mean(), per32.max()), flush=True)
    env.close()


if __name__ == "__main__":
    main()

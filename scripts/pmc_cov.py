"""A few Coverage steps of the bench's config-4 workload (512 envs x R=200, the bench's map,
resident random actions), one launch per step, for rocprofv3 --pmc passes (no timing)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from oracle.maps_host import generate_targets  # noqa: E402
from gym_flock.vec import VecCoverage  # noqa: E402

R, B, M = 200, 512, 1000
np.random.seed(8)
targets = generate_targets()
v = VecCoverage(B, R, max_nodes=M, episode_length=10 ** 9)
v.set_targets(targets)
v.h.set_streams(1)
v.reset(seed=0)
v.set_actions(np.random.RandomState(7).randint(0, 4, size=(B, R)))
for _ in range(int(os.environ.get("STEPS", 20))):
    v.step(resident=True)
v.sync()
print("done")

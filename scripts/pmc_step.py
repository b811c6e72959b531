"""A few steps of the bench workload, for rocprofv3 --pmc passes (no timing)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock import _native as nat  # noqa: E402
from gym_flock.init_states import synthetic_batch  # noqa: E402

N = int(os.environ.get("N", 1024))
B = int(os.environ.get("B", 256))
STEPS = int(os.environ.get("STEPS", 5))
KNN = os.environ.get("KNN") == "1"  # the Flocking-v0 step (fused 7-NN) instead of the plain one
h = nat.FlockHandle(N, B, n_neighbors=7 if KNN else 0)
# one launch per step (fe_set_streams(1)) so each counter row is a whole step's bytes;
# the split launches of the default write the same bytes in two halves
h.set_streams(1)
h.set_state(synthetic_batch(B, N))
h.set_actions(np.random.RandomState(0).uniform(-1, 1, size=(B, N, 2)).astype(np.float32))
if os.environ.get("DIAG"):  # ablation switches: diagnostic build only (GYMFLOCK_LIB=build/lib_diag/...)
    h.diag_switches(int(os.environ["DIAG"], 0))
# MODE: "plain" (default), "ctrl" (closed loop: step + fused controller), "packed"
MODE = os.environ.get("MODE", "plain")
flags = nat.FE_U_RESIDENT | (nat.FE_WITH_KNN if KNN else 0)
if MODE == "ctrl":
    h.controller()
    flags = nat.FE_U_EXPERT | nat.FE_WITH_CONTROLLER
elif MODE == "packed":
    flags |= nat.FE_PACKED_NETWORK | nat.FE_NO_NETWORK  # as bench.py network="packed"
for _ in range(STEPS):
    h.step(None, flags)
if os.environ.get("FILL"):
    h.diag_fill(os.environ["FILL"] == "nt", STEPS)
h.sync()
print("done")

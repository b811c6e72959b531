"""Debug probe: a one-rank RCCL communicator on a FlockHandle created, used and torn down
(optionally with torch imported first, so libgymflock binds torch's HIP runtime and RCCL).
  TORCH=1 MODE=stats|init|rewards python scripts/dbg/comm_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
if os.environ.get("GF_BT") == "1":
    import ctypes
    ctypes.CDLL(os.path.join(ROOT, "scripts", "dbg", "libabort_bt.so"))
if os.environ.get("TORCH") == "1":
    import torch  # noqa: F401
import numpy as np  # noqa: E402
from gym_flock import _native as nat  # noqa: E402
from gym_flock.init_states import synthetic_batch  # noqa: E402

mode = os.environ.get("MODE", "stats")
B, N = 6, 128
for it in range(int(os.environ.get("REPS", 3))):
    h = nat.FlockHandle(N, B)
    h.set_state(synthetic_batch(B, N))
    u = np.random.RandomState(5).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    h.comm_init(1, 0, nat.FlockHandle.comm_unique_id(), timeout=60.0)
    for _ in range(3):
        h.step(u, 0)
    if mode == "stats":
        h.allgather_stats()
        h.gathered_stats()
    elif mode == "rewards":
        h.allgather_rewards()
        h.gathered_rewards()
    h.close()
    print("rep", it, "ok", flush=True)
print("done", mode, flush=True)

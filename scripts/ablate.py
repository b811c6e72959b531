"""In-process A/B of step-kernel variants (MI355X_MICROARCH rule 24: interleaved rounds,
one process). Prints median/min device time per variant and the implied GB/s."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock import _native as nat  # noqa: E402
from gym_flock.init_states import synthetic_batch  # noqa: E402

N = int(os.environ.get("N", 1024))
B = int(os.environ.get("B", 256))
STEPS, ROUNDS = 30, int(os.environ.get("ROUNDS", 5))
h = nat.FlockHandle(N, B)
h.set_state(synthetic_batch(B, N))
h.set_actions(np.random.RandomState(0).uniform(-1, 1, size=(B, N, 2)).astype(np.float32))
alg = B * (4 * N * N + 96 * N + 8)

variants = {} if os.environ.get("QUICK") else {
    "full": (0, 0),
    "nt_stores": (4, 0),
    "no_pass1_no_feat": (10, 0),
    "no_tile_no_pass1_no_feat": (26, 0),
    "nonet_no_pass1_no_feat": (10, nat.FE_NO_NETWORK),
    "nonet_no_tile_no_p1_no_feat": (26, nat.FE_NO_NETWORK),
    "no_feature_pass": (2, 0),
    "no_network": (0, nat.FE_NO_NETWORK),
    "compute_only_no_feat": (2, nat.FE_NO_NETWORK),
    "ctrl_fused": (0, nat.FE_WITH_CONTROLLER),
    "plain_order": (32, 0),
    "ctrl_no_feature_pass": (2, nat.FE_WITH_CONTROLLER),
    "ctrl_no_network": (0, nat.FE_WITH_CONTROLLER | nat.FE_NO_NETWORK),
}
if os.environ.get("QUICK"):
    variants = {"full": (0, 0), "nt_stores": (4, 0), "ctrl_fused": (0, nat.FE_WITH_CONTROLLER)}
res = {k: [] for k in list(variants) + ["fill", "fill_nt"]}
x0 = synthetic_batch(B, N)
for r in range(ROUNDS):
    for name, (diag, flags) in variants.items():
        h.diag_switches(diag)
        h.set_state(x0)  # same workload every time (the swarm spreads as it steps)
        h.step(None, nat.FE_U_RESIDENT | flags)
        h.timing_start()
        for _ in range(STEPS):
            h.step(None, nat.FE_U_RESIDENT | flags)
        ms, n = h.timing_stop()
        res[name].append(ms)
    h.diag_switches(0)
    res["fill"].append(h.diag_fill(False, STEPS))
    res["fill_nt"].append(h.diag_fill(True, STEPS))
net_bytes = B * N * N * 4
print("R=%s T=%s pad=%s" % (os.environ.get("GYMFLOCK_ROWS"), os.environ.get("GYMFLOCK_TILE"),
                           os.environ.get("GYMFLOCK_LDS_PAD")))
print("N=%d B=%d  algorithmic bytes/launch %.3f GB, network %.3f GB" % (N, B, alg / 1e9, net_bytes / 1e9))
for k, v in res.items():
    v = np.array(v)
    by = net_bytes if k.startswith("fill") else alg
    print("%-22s median %8.1f us  min %8.1f us  -> %7.0f GB/s" % (k, 1e3 * np.median(v), 1e3 * v.min(),
                                                            by / (np.median(v) * 1e-3) / 1e9))

"""In-process interleaved A/B of step-kernel configurations (each a separate handle
created under its own GYMFLOCK_* environment), plus an output-equality check between
them. Usage: python scripts/ab_kernels.py 'A:GYMFLOCK_FRONT=0' 'B:GYMFLOCK_FRONT=1' ..."""
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
x0 = synthetic_batch(B, N)
u = np.random.RandomState(0).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
alg = B * (4 * N * N + 96 * N + 8)

configs, extra = {}, {}
for spec in sys.argv[1:] or ["tiled:GYMFLOCK_FRONT=0", "front:GYMFLOCK_FRONT=1"]:
    name, _, kv = spec.partition(":")
    env = dict(p.split("=") for p in kv.split(",") if p)
    diag = int(env.pop("diag", 0))
    extra[name] = int(env.pop("flags", "0"), 0)  # extra fe_step flags, e.g. 0x20 = FE_NO_NETWORK
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    h = nat.FlockHandle(N, B)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
    h.set_state(x0)
    h.set_actions(u)
    if diag:
        h.diag_switches(diag)
    configs[name] = h

flags_list = {"step": nat.FE_U_RESIDENT, "step+ctrl": nat.FE_U_RESIDENT | nat.FE_WITH_CONTROLLER}
res = {(c, f): [] for c in configs for f in flags_list}
for r in range(ROUNDS):
    for c, h in configs.items():
        for f, flags in flags_list.items():
            h.set_state(x0)
            h.step(None, flags | extra[c])
            h.timing_start()
            for _ in range(STEPS):
                h.step(None, flags | extra[c])
            ms, n = h.timing_stop()
            res[(c, f)].append(ms)
for (c, f), v in res.items():
    v = np.array(v)
    print("%-10s %-10s median %8.1f us  min %8.1f us  -> %7.0f GB/s" % (c, f, 1e3 * np.median(v), 1e3 * v.min(),
                                                                      alg / (np.median(v) * 1e-3) / 1e9))
# outputs of every config after one step from the same state must agree exactly
ref = None
for c, h in configs.items():
    h.set_state(x0)
    h.step(u, nat.FE_WITH_CONTROLLER)
    out = (h.get_state(), h.state_values(), h.network(0), h.network(B - 1), h.rewards(), h.controls())
    if ref is None:
        ref = out
        continue
    same = [np.array_equal(a, b) for a, b in zip(out, ref)]
    print("outputs of %s identical to the first config:" % c, same)

"""Coverage step phase timeline (config 4: 512 envs x R=200, the bench's map and resident
random actions) from the stamps build (make -C gym-flock_amd/csrc stamps; GYMFLOCK_LIB=
build/lib_stamps1/libgymflock.so). One launch per step (cov_set_streams(1)) so every
workgroup of a step has its own stamp slots; after W warm-up steps, each of K steps is
followed by a read of the stamps of that launch. Per workgroup (s_memrealtime, 100 MHz):
  t0 start, t1 first round trip done (robot nodes/actions/offers, env words; the node
  prefetch issued), t2 claim rounds done, t3 tail writes issued, t4 all writes done.
Prints medians / p90 / max of each phase over all workgroups and steps, the launch span
(min t0 .. max t4), and the phases of the workgroup that ends last.

  GYMFLOCK_LIB=build/lib_stamps1/libgymflock.so python scripts/cov_timeline.py
GREEDY=1: the fused greedy expert step (COV_ACTIONS_GREEDY: greedy actions picked inside
the step launch, between stamps 1 and 2), in episodes (reset every 75 steps, the
reference's EPISODE_LENGTH) so robots still have unvisited targets to head for.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock import _native as nat  # noqa: E402
from oracle.maps_host import generate_targets  # noqa: E402
from gym_flock.vec import VecCoverage  # noqa: E402

R, B, M = 200, 512, 1000
W, K = int(os.environ.get("WARM", "50")), int(os.environ.get("K", "30"))
np.random.seed(8)
targets = generate_targets()
v = VecCoverage(B, R, max_nodes=M, episode_length=10 ** 9)
v.set_targets(targets)
v.h.set_streams(1)
v.reset(seed=0)
v.set_actions(np.random.RandomState(7).randint(0, 4, size=(B, R)))
GREEDY = os.environ.get("GREEDY") == "1"
if GREEDY:
    v.h.controller_greedy(fetch=False)  # builds every env's time matrix and greedy lists
    v.sync()
nstep = [0]


def one_step():
    if GREEDY:
        if nstep[0] % 75 == 0:
            v.reset(seed=1000 + nstep[0])
        nstep[0] += 1
        v.step(greedy=True)
    else:
        v.step(resident=True)
lib = nat.load()
fn = lib.cov_diag_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros((4096, 8), np.uint64)
for _ in range(W):
    one_step()
v.sync()
ph = {k: [] for k in ("first_round_trip", "claims", "tail_issue", "write_drain", "block_total")}
spans, last = [], []
for _ in range(K):
    one_step()
    v.sync()
    assert fn(buf.ctypes.data, buf.size) == 0
    t = buf[:B, :5].astype(np.int64)
    t = t - t[:, 0].min()
    d = np.diff(t, axis=1) * 10.0  # ns (100 MHz)
    for k, col in zip(("first_round_trip", "claims", "tail_issue", "write_drain"), d.T):
        ph[k].extend(col.tolist())
    ph["block_total"].extend(((t[:, 4] - t[:, 0]) * 10.0).tolist())
    spans.append(float((t[:, 4].max() - t[:, 0].min()) * 10.0))
    e = int(np.argmax(t[:, 4]))
    last.append({"start_ns": float(t[e, 0] * 10.0), "phases_ns": [float(x) for x in d[e]]})
out = {"workload": "Coverage-v0 R=200, T=%d, max_nodes 1000, 512 envs, one launch per step%s" % (
           len(targets), ", fused greedy expert in episodes of 75" if GREEDY else ", resident random actions"),
       "steps": K, "launch_span_us": {"median": float(np.median(spans)) / 1e3, "max": max(spans) / 1e3},
       "phases_us": {k: {"median": float(np.median(x)) / 1e3, "p90": float(np.percentile(x, 90)) / 1e3,
                         "max": float(np.max(x)) / 1e3} for k, x in ph.items()},
       "last_block_of_median_step": last[int(np.argsort(spans)[len(spans) // 2])]}
print(json.dumps(out, indent=1))
v.close()

"""Is the Coverage config-4 step (512 envs x R=200, resident random actions) bound by the
host's launch cost or by the device? For 1 and 2 launches per step (cov_set_streams):
the host time spent enqueueing K steps (the calls return before the device is done; K
small enough that the HIP queue never fills) and the wall time until the device is done.

  python scripts/cov_launch_probe.py            (JSON on stdout)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from oracle.maps_host import generate_targets  # noqa: E402
from gym_flock.vec import VecCoverage  # noqa: E402


def main():
    R, B, M = 200, 512, 1000
    np.random.seed(8)
    v = VecCoverage(B, R, max_nodes=M, episode_length=10 ** 9)
    v.set_targets(generate_targets())
    v.reset(seed=0)
    v.set_actions(np.random.RandomState(7).randint(0, 4, size=(B, R)))
    step = v.h._step_resident
    out = {}
    for streams in (2, 1) * int(os.environ.get("REPS", "2")):
        v.h.set_streams(streams)
        for _ in range(2000):  # clocks up
            step()
        v.sync()
        res = []
        for K in (100, 300):
            v.sync()
            t0 = time.perf_counter()
            for _ in range(K):
                step()
            t1 = time.perf_counter()
            v.sync()
            t2 = time.perf_counter()
            res.append({"steps": K, "enqueue_us_per_step": 1e6 * (t1 - t0) / K,
                        "wall_us_per_step": 1e6 * (t2 - t0) / K})
        out.setdefault("streams_%d" % streams, []).append(res)
    v.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

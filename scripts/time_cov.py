"""Coverage step timing for A/B work (run on the GPU box): the bench's config 4 workload
(512 envs x 200 robots, one generated map, resident random actions), ROUNDS rounds of
K steps; prints wall us/step and the sampled cov_step_kernel time per round.
GYMFLOCK_LIB selects the library (default: the working tree's)."""
import os
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."), os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-flock_amd")]
from oracle.maps_host import generate_targets  # noqa: E402
from gym_flock.vec import VecCoverage  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "run"
R, B, M, K = 200, 512, 1000, 400
np.random.seed(8)
targets = generate_targets()
v = VecCoverage(B, R, max_nodes=M, episode_length=10 ** 9)
v.set_targets(targets)
if os.environ.get("STREAMS"):  # launches per step (cov_set_streams: 1 or 2)
    v.h.set_streams(int(os.environ["STREAMS"]))
rs = np.random.RandomState(7)
walls, kern, enq = [], [], []
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    v.reset(seed=rnd)
    v.set_actions(rs.randint(0, 4, size=(B, R)))
    for _ in range(20):
        v.step(resident=True)
    v.sync()
    v.h.timing_start(every=8)
    t0 = time.perf_counter()
    for _ in range(K):
        v.step(resident=True)
    enq.append(1e6 * (time.perf_counter() - t0) / K)  # host time to enqueue a step
    v.sync()
    walls.append(1e6 * (time.perf_counter() - t0) / K)
    kern.append(1e3 * v.h.timing_stop()[0])
print("%-8s wall median %6.2f us/step (min %6.2f)  kernel median %6.2f us  enqueue %6.2f us/step" %
      (tag, np.median(walls), np.min(walls), np.median(kern), np.median(enq)))
v.close()

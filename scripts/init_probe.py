"""Where does a step from the dense synthetic init spend its time? (diagnostic)

After a 300-step GPU warm-up, each row resets config 2 (256 x 1024) to the synthetic
init and times 20 steps with a set of ablation switches (fe_diag; timing only, the
outputs are wrong with most of them), then 20 more steps after 200 steps of
dispersal. Interleaved over 3 rounds.

  python scripts/init_probe.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-flock_amd"))

from gym_flock.init_states import synthetic_batch  # noqa: E402
from gym_flock.vec import VecFlockingRelative  # noqa: E402

CASES = {"full": 0, "no_features": 2, "no_pass1": 8, "no_pass1_no_feat": 10, "no_tile_loads": 16,
         "no_row_outputs": 256, "no_reward": 512, "const_rows": 1024, "const_rows_no_pass1_feat": 1024 | 10}


def main():
    N, B = int(os.environ.get("PN", 1024)), int(os.environ.get("PB", 256))
    env = VecFlockingRelative(B, N)
    x0 = synthetic_batch(B, N, 0)
    u = np.random.RandomState(1234).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    env.set_state(x0)
    env.set_actions(u)
    for _ in range(300):
        env.step(resident=True)
    env.sync()

    def window(k):
        env.sync()
        t0 = time.perf_counter()
        for _ in range(k):
            env.step(resident=True)
        env.sync()
        return 1e6 * (time.perf_counter() - t0) / k

    res = {k: {"init": [], "dispersed": []} for k in CASES}
    for _ in range(3):
        for name, bits in CASES.items():
            env.h.diag_switches(0)
            env.set_state(x0)
            env.h.diag_switches(bits)
            res[name]["init"].append(window(20))
            env.h.diag_switches(0)
            window(200)
            env.h.diag_switches(bits)
            res[name]["dispersed"].append(window(20))
    env.h.diag_switches(0)
    for name, r in res.items():
        print("%-26s init %7.1f us   dispersed %7.1f us" % (name, min(r["init"]), min(r["dispersed"])))
    print(json.dumps(res))
    env.close()


if __name__ == "__main__":
    main()

"""Short-window probe: why does a 20-step bench window run slower than a 200-step one?

From a cold process, times consecutive windows of config 2 (256 x 1024) steps, each
bracketed by a device sync (host wall time and the handle's device window), under
one and two streams per step, and with idle gaps between windows. A clock/power ramp
shows as windows that speed up over the first tens of ms of GPU activity; a per-window
fixed cost shows as a constant excess of short windows over long ones.

  python scripts/window_probe.py > gpurun_out/window_probe.json
"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-flock_amd"))

from gym_flock.vec import VecFlockingRelative  # noqa: E402


def smi():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--json"], capture_output=True,
                             text=True, timeout=20).stdout
        d = json.loads(out)
        card = d[sorted(d)[0]]
        return {k: v for k, v in card.items() if any(s in k for s in ("sclk", "mclk", "fclk", "Power"))}
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)}


def main():
    N, B = 1024, 256
    env = VecFlockingRelative(B, N)
    env.reset(seed=0)
    u = np.random.RandomState(1234).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    env.set_actions(u)
    rec = {"smi_idle": smi()}
    t_start = time.perf_counter()

    def window(k, streams=2):
        env.h.set_streams(streams)
        env.sync()
        env.h.timing_start(every=8)
        t0 = time.perf_counter()
        for _ in range(k):
            env.step(resident=True)
        env.sync()
        el = time.perf_counter() - t0
        ms, _ = env.h.timing_stop()
        return {"t": round(t0 - t_start, 4), "k": k, "streams": streams, "host_us": 1e6 * el / k,
                "dev_us": 1e3 * ms}

    rows = []
    # exactly what the driver does: 5 warmup steps, then windows of 20
    for _ in range(5):
        env.step(resident=True)
    env.sync()
    for i in range(40):
        rows.append(window(20))
        if i == 5:
            rec["smi_after_6_windows"] = smi()
    for i in range(10):
        rows.append(window(20, streams=1))
    for i in range(3):
        rows.append(window(200))
    for i in range(3):
        rows.append(window(200, streams=1))
    # idle gaps: does the device fall back between windows?
    for gap in (0.001, 0.01, 0.05, 0.2, 1.0):
        time.sleep(gap)
        r = window(20)
        r["gap_s"] = gap
        rows.append(r)
    # a fresh state: is the slowdown state dependent (reset = init swarm)?
    env.reset(seed=0)
    for i in range(5):
        rows.append(dict(window(20), after_reset=True))
    rec["smi_end"] = smi()
    rec["rows"] = rows
    for r in rows:
        print("%8.4f k=%3d s=%d host %7.1f dev %7.1f %s" % (r["t"], r["k"], r["streams"], r["host_us"], r["dev_us"],
                                                          "gap=%s" % r.get("gap_s", "")), file=sys.stderr)
    print(json.dumps(rec))
    env.close()


if __name__ == "__main__":
    main()

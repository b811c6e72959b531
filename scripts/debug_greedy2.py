import sys
import numpy as np
sys.path.insert(0, "gym-flock_amd"); sys.path.insert(0, ".")
from gym_flock.envs.spatial.maps import generate_targets
from gym_flock import _native as nat
np.random.seed(8)
targets = generate_targets()
T = len(targets)
for R, M in ((200, 1000), (16, 1000), (200, 800)):
    for B in (8, 16, 32, 64, 65, 128, 512):
        h = nat.CoverageHandle(R, B, M)
        h.set_targets(targets)
        bad = [b for b in range(B) if (h.time_matrix(b, T)[0] == 0).all()]
        print("R", R, "M", M, "B", B, "bad", len(bad), bad[:3], flush=True)
        h.close()

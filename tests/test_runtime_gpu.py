"""Which HIP runtime and RCCL libgymflock runs on (include/gymflock.h fe_runtime_info).

The GPU test process itself is torch-free, so the library binds the ROCm runtime and
RCCL it was built against. A trainer that imports torch first makes it bind torch's
bundled copies (same sonames; RTLD_DEEPBIND cannot undo a library already loaded): a
child process does exactly that, then steps an env, writes a Coverage observation into
a torch device tensor, and runs a communicator initialisation that times out (the abort
path that once corrupted the heap under torch's runtime), reporting the libraries mapped
into it. Needs an MI355X."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")


def _mapped(name):
    with open("/proc/self/maps") as f:
        return sorted({ln.split()[-1] for ln in f if name in ln and "/" in ln})


def test_gpu_suite_process_is_torch_free():
    """No test module imported torch into this process (collection included): the
    library is bound to /opt/rocm's HIP runtime and RCCL, as the bench is."""
    assert "torch" not in sys.modules
    nat.load()
    info = nat.runtime_info()
    assert info["hip_lib"].startswith("/opt/rocm"), info
    assert info["rccl_lib"].startswith("/opt/rocm"), info
    assert info["hip_runtime"] > 0 and info["rccl"] > 0, info
    hip = _mapped("libamdhip64")
    assert hip and all(p.startswith("/opt/rocm") for p in hip), hip
    print("bound:", json.dumps(info))


_TORCH_FIRST = r"""
import json, sys, time
import numpy as np
import torch
assert torch.cuda.is_available()
sys.path[:0] = [{root!r}, {pkg!r}]
from gym_flock import _native as nat
from gym_flock.init_states import synthetic_batch
from gym_flock.vec import VecCoverage
from oracle.maps_host import generate_targets
from oracle import flocking as orc
from oracle import coverage as oc
out = {{"runtime": nat.runtime_info()}}
with open("/proc/self/maps") as f:
    maps = f.read().splitlines()
out["hip_mapped"] = sorted({{ln.split()[-1] for ln in maps if "libamdhip64" in ln and "/" in ln}})
out["rccl_mapped"] = sorted({{ln.split()[-1] for ln in maps if "librccl" in ln and "/" in ln}})
B, N = 2, 48
h = nat.FlockHandle(N, B, n_neighbors=7)
x0 = synthetic_batch(B, N, seed0=4)
h.set_state(x0)
u = np.random.RandomState(2).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
h.step(u, nat.FE_WITH_KNN | nat.FE_WITH_CONTROLLER)
x1, idx = h.get_state(), h.knn()[0]
out["step_ok"] = all(np.array_equal(x1[b], orc.step(x0[b], u[b])["x"]) and
                     np.array_equal(idx[b], orc.knn_observation(x1[b])[0]) for b in range(B))
# a Coverage observation written into a torch device tensor (zero-copy consumer)
np.random.seed(400)
v = VecCoverage(1, 10, max_nodes=700)
v.set_targets(generate_targets(), env=0)
v.reset(seed=3)
v.step(np.random.RandomState(9).randint(0, 4, size=(1, 10)))
flat = v.flat_obs()
dst = torch.empty((1, 15 * 700 + 1), dtype=torch.float32, device="cuda")
v.flat_obs(f32=True, device_ptr=dst.data_ptr())
v.sync()
out["flat_ok"] = bool(np.array_equal(dst.cpu().numpy(), flat.astype(np.float32))) and \
    bool(np.array_equal(flat[0], oc.flatten_obs(v.obs(0))))
v.close()
# a lone rank of a 2-rank communicator: the bounded init fails, the handle keeps stepping
t0 = time.monotonic()
try:
    h.comm_init(2, 0, nat.FlockHandle.comm_unique_id(), timeout=5.0)
    out["comm"] = "INIT_OK"
except nat.GymFlockError as e:
    out["comm"] = e.code
out["comm_seconds"] = time.monotonic() - t0
h.step(u, 0)
x2 = h.get_state()
out["step_after_ok"] = all(np.array_equal(x2[b], orc.step(x1[b], u[b])["x"]) for b in range(B))
h.close()
print("RESULT " + json.dumps(out))
"""


def test_torch_first_child_binds_torch_runtime_and_survives_comm_abort():
    code = _TORCH_FIRST.format(root=ROOT, pkg=os.path.join(ROOT, "gym-flock_amd"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=240)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    line = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("RESULT ")][-1]
    out = json.loads(line[len("RESULT "):])
    print(json.dumps(out, indent=1))
    assert out["step_ok"] and out["flat_ok"] and out["step_after_ok"], out
    assert out["comm"] == nat.GF_ECOMM and out["comm_seconds"] < 15.0, out
    # the library runs on whichever HIP runtime the process mapped first: report it, and
    # check that fe_runtime_info names a library that is actually mapped
    assert out["hip_mapped"], out
    assert os.path.realpath(out["runtime"]["hip_lib"]) in {os.path.realpath(p) for p in out["hip_mapped"]}, out

"""Coverage observation wire formats on the device: the
FlattenDictWrapper rows (test.py:33, keys coverage.py:90) and the batched unpack_obs
graph tuple (coverage.py:689-741). Integer and float32 values are copied, so every
comparison is exact. The flat rows are pinned to the reference's recorded observations.
The unpack restatement is pinned only by the oracle, because TensorFlow is absent.
Needs an MI355X."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import coverage as oc

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")
from gym_flock.vec import VecCoverage  # noqa: E402


def test_flat_obs_matches_reference_episode():
    f = np.load(os.path.join(GOLDEN, "coverage_r6_random.npz"))
    R, T, M = int(f["n_robots"]), int(f["n_targets"]), int(f["max_nodes"])
    h = nat.CoverageHandle(R, 1, M)
    h.set_targets(f["targets"], env=0)
    start = oc.closest_targets(f["x0"][:R], f["targets"], R) - R
    visited = np.ones((1, M - R), np.uint8)
    visited[0, :T] = f["visited0"][R:].astype(np.uint8)
    h.reset(start[None], visited)
    ref0 = oc.flatten_obs({k: f[k + "0"] for k in oc.KEYS})
    np.testing.assert_array_equal(h.flat_obs()[0], ref0)
    for t in range(5):
        h.step(f["actions"][t][None])
        ref = oc.flatten_obs({k: f[k][t] for k in oc.KEYS})
        flat = h.flat_obs()
        assert flat.dtype == np.float64 and flat.shape == (1, 15 * M + 1)
        np.testing.assert_array_equal(flat[0], ref)
        np.testing.assert_array_equal(h.flat_obs(f32=True)[0], ref.astype(np.float32))
    h.close()


def _batch(B=3, R=10, M=700, steps=4):
    from oracle.maps_host import generate_targets
    maps = []
    for b in range(B):
        np.random.seed(400 + b)
        maps.append(generate_targets())
    v = VecCoverage(B, R, max_nodes=M)
    for b in range(B):
        v.set_targets(maps[b], env=b)
    v.reset(seed=3)
    rs = np.random.RandomState(9)
    for _ in range(steps):
        v.step(rs.randint(0, 4, size=(B, R)))
    return v


def test_batched_flat_obs():
    """Every env's flat row (the device-pointer output into a torch tensor is checked in a
    torch-first child process, tests/test_runtime_gpu.py: this process stays torch-free)."""
    v = _batch()
    B = v.n_envs
    flat = v.flat_obs()
    for b in range(B):
        np.testing.assert_array_equal(flat[b], oc.flatten_obs(v.obs(b)))
    v.close()


@pytest.mark.parametrize("mask_all", [False, True])
def test_graphs_tuple_vs_oracle_unpack(mask_all):
    v = _batch()
    B, M = v.n_envs, v.h.max_nodes
    flat32 = v.flat_obs(f32=True)
    if mask_all:  # every graph masked: unpack each graph alone, then offset and concatenate
        parts = [oc.unpack_obs(flat32[b:b + 1]) for b in range(B)]
        ref = dict(n_node=np.concatenate([p["n_node"] for p in parts]),
                   nodes=np.concatenate([p["nodes"] for p in parts]),
                   n_edge=np.concatenate([p["n_edge"] for p in parts]),
                   edges=np.concatenate([p["edges"] for p in parts]),
                   senders=np.concatenate([p["senders"] + b * M for b, p in enumerate(parts)]),
                   receivers=np.concatenate([p["receivers"] + b * M for b, p in enumerate(parts)]),
                   globs=np.concatenate([p["globs"] for p in parts]))
    else:
        ref = oc.unpack_obs(flat32)
        assert ref["n_edge"][1] == 4 * M  # the reference keeps graph 1's padding
    g = v.graphs_tuple(mask_all=mask_all)
    for k in ("n_node", "nodes", "n_edge", "edges", "senders", "receivers", "globs"):
        np.testing.assert_array_equal(g[k], ref[k], err_msg=k)
    from gym_flock.envs.spatial import CoverageEnv

    class Space:
        shape = (15 * M + 1,)
    host = CoverageEnv.unpack_obs(flat32, Space())
    if not mask_all:
        assert host[0] == B
        for a, k in zip(host[1:], ("n_node", "nodes", "n_edge", "edges", "senders", "receivers", "globs")):
            np.testing.assert_array_equal(a, ref[k], err_msg=k)
    v.close()

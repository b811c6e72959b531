"""Pin the Coverage oracle (oracle/coverage.py) against the reference's recorded
episodes (tests/golden/coverage_*.npz from tests/golden/make_golden_coverage.py)."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import coverage as oc

EPISODES = sorted(glob.glob(os.path.join(GOLDEN, "coverage_r*.npz")))


def check_obs(obs, f, t=None):
    sfx = "" if t is None else None
    get = (lambda k: f[k + "0"]) if t is None else (lambda k: f[k][t])
    np.testing.assert_array_equal(obs["nodes"], get("nodes"))
    np.testing.assert_array_equal(obs["edges"], get("edges"))
    np.testing.assert_array_equal(obs["senders"], get("senders"))
    np.testing.assert_array_equal(obs["receivers"], get("receivers"))
    np.testing.assert_array_equal(obs["step"], get("step"))
    return sfx


@pytest.mark.parametrize("path", EPISODES, ids=os.path.basename)
def test_episode_matches_reference(path):
    f = np.load(path)
    R, T = int(f["n_robots"]), int(f["n_targets"])
    env = oc.CoverageOracle(f["targets"], R, int(f["max_nodes"]))
    np.testing.assert_array_equal(env.motion[0], f["motion_senders"])
    np.testing.assert_array_equal(env.motion[1], f["motion_receivers"])
    start = oc.closest_targets(f["x0"][:R], f["targets"], R) - R
    unvisited = np.nonzero(f["visited0"][R:] == 0)[0] + R
    # reset() marks the start nodes visited; the fixture holds visited after that, so
    # the unvisited set before reset's observation is visited0 == 0 minus nothing
    obs = env.reset(start, unvisited)
    check_obs(obs, f)
    for t in range(len(f["actions"])):
        obs, r, d = env.step(f["actions"][t])
        np.testing.assert_array_equal(env.xr, f["xr"][t])
        np.testing.assert_array_equal(env.closest(), f["closest"][t])
        assert r == f["reward"][t] and d == f["done"][t]
        check_obs(obs, f, t)
        np.testing.assert_array_equal(env.visited.astype(np.int8), f["visited"][t])


def test_lattice_matches_reference():
    f = np.load(os.path.join(GOLDEN, "coverage_maps.npz"))
    np.testing.assert_array_equal(oc.generate_lattice(-120, 120, -120, 120), f["lattice"])


GREEDY = sorted(glob.glob(os.path.join(GOLDEN, "coverage_r*_greedy.npz")))
ENV_SEED = {"coverage_r6_greedy.npz": 6, "coverage_r20_greedy.npz": 13}


@pytest.mark.parametrize("path", GREEDY, ids=os.path.basename)
def test_greedy_expert_matches_reference(path):
    f = np.load(path)
    R, T = int(f["n_robots"]), int(f["n_targets"])
    env = oc.CoverageOracle(f["targets"], R, int(f["max_nodes"]))
    cost, prev = oc.time_matrix(T, env.motion[0] - R, env.motion[1] - R)
    np.testing.assert_array_equal(cost, f["graph_cost"])
    np.testing.assert_array_equal(prev, f["graph_previous"])
    start = oc.closest_targets(f["x0"][:R], f["targets"], R) - R
    env.reset(start, np.nonzero(f["visited0"][R:] == 0)[0] + R)
    rs = np.random.RandomState(ENV_SEED[os.path.basename(path)])
    rs.choice(np.arange(T), size=(R,), replace=False)
    rs.choice(np.arange(T) + R, size=(int(T * 0.5),), replace=False)
    n_random = 0
    for t in range(len(f["actions"])):
        cur = env.closest()
        recv = oc.action_receivers(cur, env.nbr, env.cnt, R)
        a, rand = oc.greedy_actions(cost, prev, cur, env.visited[R:], recv, R)
        for i in np.nonzero(rand)[0]:
            a[i] = rs.choice(4)  # the reference's fallback draw, robot order (:864)
            n_random += 1
        np.testing.assert_array_equal(a, f["actions"][t])
        env.step(a)
    if "r20" in path:
        assert n_random > 0  # the long episode exercises the random fallback


def test_flatten_and_unpack_round_trip():
    """FlattenDictWrapper rows (test.py:33) of a recorded reference observation and the
    unpack_obs restatement (coverage.py:689-741) recover it. The reference offsets the
    senders before its padding test, so only graph 0 drops padding."""
    f = np.load(os.path.join(GOLDEN, "coverage_r6_random.npz"))
    M = int(f["max_nodes"])
    obs = {k: f[k + "0"] for k in oc.KEYS}
    flat = oc.flatten_obs(obs)
    assert flat.dtype == np.float64 and flat.shape == (15 * M + 1,)
    u = oc.unpack_obs(np.stack([flat, flat]))
    np.testing.assert_array_equal(u["nodes"][:M], obs["nodes"])
    valid = obs["senders"] != -1
    assert u["n_edge"][0] == valid.sum() and u["n_edge"][1] == 4 * M
    np.testing.assert_array_equal(u["senders"][:valid.sum()], obs["senders"][valid])
    np.testing.assert_array_equal(u["senders"][valid.sum():], obs["senders"] + M)
    assert u["globs"][0, 0] == obs["step"][0, 0]


@pytest.mark.parametrize("path", EPISODES, ids=os.path.basename)
def test_cpu_ref_coverage_matches_reference(path):
    """oracle/cpu_ref_coverage.py (bench.py's config-4 CPU baseline, the reference's own
    loop-and-np.where op sequence) reproduces the recorded episodes bit for bit."""
    from oracle.cpu_ref_coverage import CpuCoverage
    f = np.load(path)
    R = int(f["n_robots"])
    env = CpuCoverage(f["targets"], R, int(f["max_nodes"]))
    np.testing.assert_array_equal(env.motion_edges[0], f["motion_senders"])
    np.testing.assert_array_equal(env.motion_edges[1], f["motion_receivers"])
    start = oc.closest_targets(f["x0"][:R], f["targets"], R) - R
    obs = env.reset(start, np.nonzero(f["visited0"] == 0)[0])
    check_obs(obs, f)
    np.testing.assert_array_equal(env.x, f["x0"])
    for t in range(len(f["actions"])):
        obs, r, d, _ = env.step(np.array(f["actions"][t]).reshape(-1, 1))
        np.testing.assert_array_equal(env.x[:R], f["xr"][t])
        assert r == f["reward"][t] and d == f["done"][t]
        check_obs(obs, f, t)
        np.testing.assert_array_equal(env.visited[:, 0].astype(np.int8), f["visited"][t])

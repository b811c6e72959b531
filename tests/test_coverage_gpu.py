"""Parity of the HIP Coverage-v0 path with the reference's recorded episodes and the
CPU oracle, through the C-ABI. Integer outputs (nodes, senders/receivers, step,
rewards, done, robot nodes, visited) and the float32 edge features are compared
bit-exactly. Needs an MI355X."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import coverage as oc

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")
from gym_flock.vec import VecCoverage  # noqa: E402

EPISODES = sorted(glob.glob(os.path.join(GOLDEN, "coverage_r*.npz")))


def assert_obs(o, f, t=None):
    get = (lambda k: f[k + "0"]) if t is None else (lambda k: f[k][t])
    np.testing.assert_array_equal(o["nodes"], get("nodes"))
    np.testing.assert_array_equal(o["edges"], get("edges"))
    np.testing.assert_array_equal(o["senders"], get("senders"))
    np.testing.assert_array_equal(o["receivers"], get("receivers"))
    np.testing.assert_array_equal(o["step"], get("step"))


@pytest.mark.parametrize("path", EPISODES, ids=os.path.basename)
def test_episode_matches_reference_golden(path):
    f = np.load(path)
    R, T, M = int(f["n_robots"]), int(f["n_targets"]), int(f["max_nodes"])
    h = nat.CoverageHandle(R, 1, M)
    h.set_targets(f["targets"], env=0)
    assert h.n_motion()[0] == len(f["motion_senders"])
    start = oc.closest_targets(f["x0"][:R], f["targets"], R) - R
    visited = np.ones((1, M - R), np.uint8)
    visited[0, :T] = f["visited0"][R:].astype(np.uint8)
    h.reset(start[None], visited)
    assert_obs(h.obs(0), f)
    for t in range(len(f["actions"])):
        h.step(f["actions"][t][None])
        assert_obs(h.obs(0), f, t)
        r, d = h.rewards()
        assert r[0] == f["reward"][t] and d[0] == f["done"][t]
        xr, nodes = h.robots(0)
        np.testing.assert_array_equal(xr, f["xr"][t])
        np.testing.assert_array_equal(nodes, f["closest"][t])
        np.testing.assert_array_equal(h.visited(0)[:T], f["visited"][t][R:])
    h.close()


def test_batched_envs_with_distinct_graphs_vs_oracle():
    """4 envs, each its own map and random actions, 20 steps against the oracle."""
    from oracle.maps_host import generate_targets
    B, R, M = 4, 12, 600
    maps = []
    for b in range(B):
        np.random.seed(100 + b)
        maps.append(generate_targets())
    v = VecCoverage(B, R, max_nodes=M)
    for b in range(B):
        v.set_targets(maps[b], env=b)
    start, visited = v.reset(seed=5)
    orcs = []
    for b in range(B):
        o = oc.CoverageOracle(maps[b], R, M)
        T = len(maps[b])
        obs0 = o.reset(start[b], np.nonzero(visited[b, :T] == 0)[0] + R)
        assert_obs(v.obs(b), {k + "0": val for k, val in obs0.items()})
        orcs.append(o)
    rs = np.random.RandomState(0)
    for t in range(20):
        acts = rs.randint(0, 4, size=(B, R))
        v.step(acts)
        r, d = v.rewards()
        for b in range(B):
            obs, rr, dd = orcs[b].step(acts[b])
            assert_obs(v.obs(b), {k + "0": val for k, val in obs.items()})
            assert r[b] == rr and d[b] == dd
    v.close()


def test_collisions_and_blocking_order():
    """Crowded start (robots on adjacent nodes of a small grid) so that moves collide:
    stays claim first, then index order decides, blocked robots stay (:187-200)."""
    xs, ys = np.meshgrid(np.arange(6) * 5.5, np.arange(6) * 5.5)
    targets = np.stack([ys.ravel(), xs.ravel()], axis=1)
    R, M = 10, 200
    h = nat.CoverageHandle(R, 1, M)
    h.set_targets(targets, env=0)
    o = oc.CoverageOracle(targets, R, M)
    start = np.arange(R)
    visited = np.zeros((1, M - R), np.uint8)
    h.reset(start[None], visited)
    o.reset(start, np.arange(len(targets)) + R)
    rs = np.random.RandomState(3)
    for t in range(40):
        a = rs.randint(0, 4, size=R)
        h.step(a[None])
        obs, rr, dd = o.step(a)
        assert_obs(h.obs(0), {k + "0": val for k, val in obs.items()})
        np.testing.assert_array_equal(h.robots(0)[1], o.closest())
        assert h.rewards()[0][0] == rr
    h.close()


def test_step_after_close_is_refused():
    """A closed handle's resident and greedy steps (bound to the C handle object) pass NULL
    and are refused with GF_EINVAL, never the freed handle (advisor r03)."""
    f = np.load(EPISODES[0])
    R, M = int(f["n_robots"]), int(f["max_nodes"])
    h = nat.CoverageHandle(R, 1, M)
    h.set_targets(f["targets"], env=0)
    h.close()
    for kw in ({"resident": True}, {"greedy": True}):
        with pytest.raises(nat.GymFlockError):
            h.step(**kw)


def test_external_robot_positions_recompute_closest():
    f = np.load(EPISODES[0])
    R, T, M = int(f["n_robots"]), int(f["n_targets"]), int(f["max_nodes"])
    h = nat.CoverageHandle(R, 1, M)
    h.set_targets(f["targets"], env=0)
    o = oc.CoverageOracle(f["targets"], R, M)
    start = np.arange(R) * (T // R)
    h.reset(start[None], np.ones((1, M - R), np.uint8))
    o.reset(start, [])
    rs = np.random.RandomState(2)
    # two placements, each followed by steps: the full pass after a placement (blocked
    # robots keep their off-node positions and edges) and the node-record steps after it
    for place in range(2):
        xr = f["targets"][start] + np.random.RandomState(1 + place).uniform(-2.0, 2.0, size=(R, 2))
        h.set_robot_positions(0, xr)
        o.xr = xr.copy()
        for t in range(8):
            a = rs.randint(0, 4, size=R)
            h.step(a[None])
            obs, rr, dd = o.step(a)
            assert_obs(h.obs(0), {k + "0": val for k, val in obs.items()})
            np.testing.assert_array_equal(h.robots(0)[0], o.xr)
            assert h.rewards()[0][0] == rr
    h.close()


@pytest.mark.parametrize("mode", ["direct", "getters"])
def test_env_api_reproduces_reference_reset_and_episode(mode):
    """CoverageEnv with the fixture's seeds regenerates the reference's map, starts and
    unvisited set (global and env RNGs in the reference's call order), then replays the
    recorded random episode. "direct" (the default) is one cov_step_host call per step:
    every observation, reward and done flag as recorded, last_loc the robots' nodes
    before the move (:183), and the arrays a step returned stay as they were after
    later steps (fresh arrays per call)."""
    from gym_flock.envs.spatial import CoverageEnv
    f = np.load(os.path.join(GOLDEN, "coverage_r6_random.npz"))
    np.random.seed(3)
    env = CoverageEnv(n_robots=6, nearby_starts=False, max_nodes=500)
    env.fetch_mode = mode
    env.seed(4)
    np.random.seed(3)
    obs = env.reset()
    assert_obs(obs, f)
    kept = []
    prev = env.closest_targets
    for t in range(len(f["actions"])):
        obs, r, d, _ = env.step(f["actions"][t].reshape(-1, 1))
        np.testing.assert_array_equal(env.last_loc, prev)
        prev = f["closest"][t]
        assert_obs(obs, f, t)
        assert r == f["reward"][t] and d == f["done"][t]
        kept.append((t, obs))
    for t, o in kept[::7]:
        assert_obs(o, f, t)
    with pytest.raises(IndexError):
        env.step(np.full((6, 1), 4))
    env.close()


def test_env_get_action_edges_and_unpack_state():
    """get_action_edges (coverage.py:206-232) from the device observation, and the
    NumPy unpack_obs_state (:744-798) on a flattened observation."""
    from gym_flock.envs.spatial import CoverageEnv
    f = np.load(os.path.join(GOLDEN, "coverage_r6_random.npz"))
    np.random.seed(3)
    env = CoverageEnv(n_robots=6, nearby_starts=False, max_nodes=500)
    env.seed(4)
    np.random.seed(3)
    env.reset()
    env.step(f["actions"][0].reshape(-1, 1))
    (snd, rcv), dists, diff = env.get_action_edges()
    R = 6
    o = oc.CoverageOracle(f["targets"], R, 500)
    cur = f["closest"][0]
    np.testing.assert_array_equal(snd, np.repeat(np.arange(R), 4))
    np.testing.assert_array_equal(rcv, oc.action_receivers(cur, o.nbr, o.cnt, R).reshape(-1))
    x = np.vstack([f["xr"][0], f["targets"]])
    np.testing.assert_array_equal(diff, x[snd] - x[rcv])
    np.testing.assert_array_equal(dists, np.linalg.norm(x[snd] - x[rcv], axis=1))
    flat = oc.flatten_obs(env._h.obs(0))[None].astype(np.float32)

    class Space:
        shape = flat.shape[1:]
    state = np.arange(500 * 4, dtype=np.float32).reshape(500, 4)
    out = CoverageEnv.unpack_obs_state(flat, Space(), state, 2)
    assert out[2].shape == (500, 5) and out[3].shape == (500, 5)
    np.testing.assert_array_equal(out[2][:, 3:], state[:, :2])
    np.testing.assert_array_equal(out[3][:, 3:], state[:, 2:])
    env.close()


@pytest.mark.parametrize("R", [64, 255, 256, 300])
def test_crowded_grid_claims_vs_oracle(R):
    """Dense robots on a 25x25 grid (long claim chains), at the one-wave claim path's
    limits (R = 64, 255, 256 robots: up to 4 per lane) and past them (R = 300 takes the
    multi-wave path); 25 random steps against the oracle."""
    xs, ys = np.meshgrid(np.arange(25) * 5.5, np.arange(25) * 5.5)
    targets = np.stack([ys.ravel(), xs.ravel()], axis=1)
    M = 1300
    h = nat.CoverageHandle(R, 1, M)
    h.set_targets(targets, env=0)
    o = oc.CoverageOracle(targets, R, M)
    rs = np.random.RandomState(R)
    start = rs.choice(len(targets), R, replace=False)
    h.reset(start[None], np.zeros((1, M - R), np.uint8))
    o.reset(start, np.arange(len(targets)) + R)
    for t in range(25):
        a = rs.randint(0, 4, size=R)
        h.step(a[None])
        obs, rr, dd = o.step(a)
        assert_obs(h.obs(0), {k + "0": val for k, val in obs.items()})
        np.testing.assert_array_equal(h.robots(0)[1], o.closest())
        assert h.rewards()[0][0] == rr
    h.close()


def test_split_steps_match_single_stream():
    """Back-to-back resident steps go out as two half-batch launches on two streams;
    the observations, rewards and robots equal the one-launch-per-step run."""
    from oracle.maps_host import generate_targets
    B, R, M = 5, 12, 600
    np.random.seed(7)
    targets = generate_targets()
    runs = []
    for streams in (2, 1):
        h = nat.CoverageHandle(R, B, M)
        h.set_streams(streams)
        h.set_targets(targets)
        T = len(targets)
        rs = np.random.RandomState(11)
        start = np.stack([rs.choice(T, R, replace=False) for _ in range(B)]).astype(np.int32)
        h.reset(start, np.zeros((B, M - R), np.uint8))
        got = []
        for k in range(3):
            h.set_actions(rs.randint(0, 4, size=(B, R)))
            for _ in range(4):
                h.step(resident=True)
            got += [h.rewards()[0]] + [h.obs(b)[key] for b in range(B) for key in ("nodes", "edges", "senders")]
            got += [h.robots(b)[1] for b in range(B)]
        runs.append(got)
        h.close()
    for a, b in zip(*runs):
        np.testing.assert_array_equal(a, b)


def test_full_config4_batch_properties_and_sampled_parity():
    """BASELINE.json configs[3] at full size: 512 envs x 200 robots, max_nodes 1000, one
    generated ~550-target map (global seed 8, as bench.py), random actions for 8 steps.
    Whole batch: every env's robots sit on target nodes (two can share one: a robot
    blocked after an earlier robot claimed its node stays, coverage.py:187-200, as the
    oracle shows on the sampled envs), rewards are the newly visited counts (summed
    rewards = visited growth), and the observation tails name only robots and targets. Sampled envs (first, middle, last): full observations, rewards, robots and
    visited sets bit-exact against the oracle every step."""
    from oracle.maps_host import generate_targets
    B, R, M = 512, 200, 1000
    np.random.seed(8)
    targets = generate_targets()
    T = len(targets)
    v = VecCoverage(B, R, max_nodes=M, episode_length=10 ** 9)
    v.set_targets(targets)
    start, visited0 = v.reset(seed=0)
    # the reset's own observation already marks the start nodes visited (no reward)
    vis0 = np.stack([v.h.visited(b)[:T].astype(np.int64) for b in range(B)])
    sample = (0, 257, 511)
    orcs = {}
    for b in sample:
        o = oc.CoverageOracle(targets, R, M)
        o.reset(start[b], np.nonzero(visited0[b, :T] == 0)[0] + R)
        orcs[b] = o
    rs = np.random.RandomState(9)
    total = np.zeros(B)
    for t in range(8):
        acts = rs.randint(0, 4, size=(B, R)).astype(np.int32)
        v.step(acts)
        r, d = v.rewards()
        assert not d.any() and (r >= 0).all()
        total += r
        for b in sample:
            obs, rr, dd = orcs[b].step(acts[b])
            assert_obs(v.obs(b), {k + "0": val for k, val in obs.items()})
            assert r[b] == rr and d[b] == dd
            np.testing.assert_array_equal(v.h.robots(b)[1], orcs[b].closest())
    for b in range(B):
        nodes = v.h.robots(b)[1]
        assert nodes.min() >= R and nodes.max() < R + T
        vis = v.h.visited(b)[:T].astype(np.int64)
        assert (vis >= vis0[b]).all() and vis.sum() - vis0[b].sum() == total[b]
    for b in (1, 300):
        o = v.obs(b)
        s, rcv = o["senders"], o["receivers"]
        live = s >= 0
        assert (s[live] < R + T).all() and (rcv[live] < R + T).all()
    v.close()


def test_default_env_nearby_starts():
    """CoverageEnv() with the module defaults (NEARBY_STARTS, 500 padded nodes) builds its
    start region from the motion graph before any reset (get_n_nearest, coverage.py:655-673,
    reading the graph's static observation) and resets inside it: the region equals the
    oracle's breadth-first growth from the drawn node over the reference's motion edges
    (utils.py:8-24), and the robots start on distinct targets of it. One direct step and
    its observation against the CPU reference op sequence."""
    from gym_flock.envs.spatial import CoverageEnv
    from oracle.cpu_ref_coverage import CpuCoverage
    seen = []
    orig = CoverageEnv.get_n_nearest

    def spy(self, i, n):
        seen.append(int(i))
        return orig(self, i, n)

    CoverageEnv.get_n_nearest = spy
    try:
        np.random.seed(3)  # a map of 431 targets (coverage_r6_random's)
        env = CoverageEnv()
        env.seed(11)
        np.random.seed(3)
        obs = env.reset()
    finally:
        CoverageEnv.get_n_nearest = orig
    R, T = env.n_robots, env.n_targets
    cpu = CpuCoverage(env.targets, R, env.max_nodes)
    s, q = cpu.motion_edges[0] - R, cpu.motion_edges[1] - R
    want = {seen[-1]}
    while len(want) < 5 * R:
        want |= set(q[np.isin(s, list(want))].tolist())
    np.testing.assert_array_equal(np.nonzero(env.start_region)[0], sorted(want))
    starts = env.closest_targets - R
    assert len(set(starts.tolist())) == R and all(env.start_region[t] for t in starts)
    vis = env.visited[R:, 0]
    cpu.reset(starts, np.nonzero(vis[:T] == 0)[0] + R)
    a = np.random.RandomState(2).randint(0, 4, size=(R, 1))
    obs, r, d, _ = env.step(a)
    ref, rr, dd, _ = cpu.step(a)
    for k in ("nodes", "edges", "senders", "receivers"):
        np.testing.assert_array_equal(obs[k].reshape(ref[k].shape), ref[k], err_msg=k)
    assert r == rr and d == dd
    env.close()


def _jittered_grid(nx, ny, seed, spacing=5.5, jitter=0.3):
    rs = np.random.RandomState(seed)
    xs, ys = np.meshgrid(np.arange(nx) * spacing, np.arange(ny) * spacing)
    p = np.stack([xs.ravel(), ys.ravel()], axis=1)
    return p + rs.uniform(-jitter, jitter, size=p.shape)


def test_motion_graph_edge_cases_vs_oracle():
    """The motion-graph kernel (cell grid over the targets' box, the radius test from
    squared distances except at the edge) against the oracle's radius graph: a jittered
    grid with pairs at exactly the radius and one ulp either side, coincident targets
    (distance 0: no edge), and a map spread so wide that the grid gives way to the scan
    of every target; a target with more than 4 neighbours is refused."""
    r = 5.5 * 1.2
    g = _jittered_grid(8, 7, 1)
    edge = np.array([[200.0, 0.0], [200.0 + r, 0.0], [300.0, 0.0], [np.nextafter(300.0 + r, np.inf), 0.0],
                     [400.0, 0.0], [np.nextafter(400.0 + r, 0.0), 0.0], [500.0, 500.0], [500.0, 500.0],
                     [500.0, 500.0 + r]])
    wide = np.concatenate([_jittered_grid(6, 1, 2), [[1.0e5, 3.0], [1.0e5 + r, 3.0], [-2.0e5, -7.0]]])
    maps = [np.concatenate([g, edge]), wide, g[::-1].copy()]
    B, R, M = len(maps), 3, 200
    v = VecCoverage(B, R, max_nodes=M)
    for b in range(B):
        v.set_targets(maps[b], env=b)
    start, visited = v.reset(seed=5)
    for b in range(B):
        o = oc.CoverageOracle(maps[b], R, M)
        T = len(maps[b])
        assert v.h.n_motion()[b] == o.n_motion
        obs0 = o.reset(start[b], np.nonzero(visited[b, :T] == 0)[0] + R)
        assert_obs(v.obs(b), {k + "0": val for k, val in obs0.items()})
    s, q, _ = oc.radius_graph(maps[0], r)
    pairs = set(zip(s.tolist(), q.tolist()))
    T0 = len(g)
    assert (T0, T0 + 1) in pairs and (T0 + 2, T0 + 3) not in pairs and (T0 + 4, T0 + 5) in pairs
    assert (T0 + 6, T0 + 7) not in pairs  # coincident
    v.close()
    crowded = np.array([[0.0, 0.0], [1.0, 0.0], [0.0, 1.0], [-1.0, 0.0], [0.0, -1.0], [1.0, 1.0]])
    h = nat.CoverageHandle(2, 1, 50)
    with pytest.raises(nat.GymFlockError):
        h.set_targets(crowded, env=0)
    h.close()

"""Parity of the HIP greedy expert (construct_time_matrix :621-653, controller(greedy=True)
:800-872) with the reference's recorded greedy episodes and the CPU oracle, through the
C-ABI. Time matrices, predecessors and actions are integers: compared bit-exactly.
Needs an MI355X."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import coverage as oc

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")
from gym_flock.vec import VecCoverage  # noqa: E402

GREEDY = sorted(glob.glob(os.path.join(GOLDEN, "coverage_r*_greedy.npz")))
ENV_SEED = {"coverage_r6_greedy.npz": 6, "coverage_r20_greedy.npz": 13}
MAP_SEED = {"coverage_r6_greedy.npz": 5, "coverage_r20_greedy.npz": 12}


def _handle_for(f, horizon=10):
    R, T, M = int(f["n_robots"]), int(f["n_targets"]), int(f["max_nodes"])
    h = nat.CoverageHandle(R, 1, M, horizon=horizon)
    h.set_targets(f["targets"], env=0)
    return h, R, T, M


@pytest.mark.parametrize("path", GREEDY, ids=os.path.basename)
def test_time_matrix_matches_reference(path):
    f = np.load(path)
    h, R, T, M = _handle_for(f)
    cost, prev = h.time_matrix(0, T)
    np.testing.assert_array_equal(cost, f["graph_cost"])
    np.testing.assert_array_equal(prev, f["graph_previous"])
    h.close()


@pytest.mark.parametrize("path", GREEDY, ids=os.path.basename)
def test_greedy_episode_matches_reference(path):
    """The whole recorded greedy episode through the handle, random fallbacks drawn on
    the host from the replayed env RNG."""
    f = np.load(path)
    h, R, T, M = _handle_for(f)
    start = oc.closest_targets(f["x0"][:R], f["targets"], R) - R
    visited = np.ones((1, M - R), np.uint8)
    visited[0, :T] = f["visited0"][R:].astype(np.uint8)
    h.reset(start[None], visited)
    rs = np.random.RandomState(ENV_SEED[os.path.basename(path)])
    rs.choice(np.arange(T), size=(R,), replace=False)
    rs.choice(np.arange(T) + R, size=(int(T * 0.5),), replace=False)
    for t in range(len(f["actions"])):
        a, rnd = h.controller_greedy()
        a = a[0].copy()
        for i in np.nonzero(rnd[0])[0]:
            a[i] = rs.choice(4)
        np.testing.assert_array_equal(a, f["actions"][t])
        h.step(a[None])
        np.testing.assert_array_equal(h.robots(0)[1], f["closest"][t])
    h.close()


@pytest.mark.parametrize("mode", ["direct", "getters"])
@pytest.mark.parametrize("path", GREEDY, ids=os.path.basename)
def test_env_api_greedy_controller(path, mode):
    """CoverageEnv.controller(greedy=True) with the fixture's seeds reproduces the
    reference's expert episode, including its np_random fallback draws. "direct" (the
    default): after the first controller() call every step is one cov_step_host launch
    that also computes the expert's actions for the resulting state, which the next
    controller() call takes (the fallback draws on the host, in robot order) without a
    device call. Observations, rewards, done flags and the robots' nodes as recorded."""
    from gym_flock.envs.spatial import CoverageEnv
    f = np.load(path)
    name = os.path.basename(path)
    np.random.seed(MAP_SEED[name])
    env = CoverageEnv(n_robots=int(f["n_robots"]), nearby_starts=False, max_nodes=int(f["max_nodes"]))
    env.fetch_mode = mode
    env.seed(ENV_SEED[name])
    np.random.seed(MAP_SEED[name])
    env.reset()
    for t in range(len(f["actions"])):
        if mode == "direct" and t > 0:
            assert env._greedy_cache is not None  # made by the previous step's launch
        a = env.controller(random=False, greedy=True)
        assert a.shape == (int(f["n_robots"]), 1) and a.dtype == np.int32
        np.testing.assert_array_equal(a[:, 0], f["actions"][t])
        obs, r, d, _ = env.step(a)
        assert r == f["reward"][t] and d == f["done"][t]
        for k in ("nodes", "edges", "senders", "receivers", "step"):
            np.testing.assert_array_equal(obs[k].reshape(f[k][t].shape), f[k][t], err_msg=k)
        np.testing.assert_array_equal(env.closest_targets, f["closest"][t])
    np.testing.assert_array_equal(env.graph_cost, f["graph_cost"])
    np.testing.assert_array_equal(env.graph_previous, f["graph_previous"])
    with pytest.raises(AssertionError):
        env.controller(random=False, greedy=False)  # OR-Tools routing: not available
    env.close()


def _two_clusters():
    """A disconnected map: two lattice patches 60 m apart (inf entries never clear, so
    the reference's loop stops on "no change")."""
    xs, ys = np.meshgrid(np.arange(7) * 5.5, np.arange(5) * 5.5)
    a = np.stack([xs.ravel(), ys.ravel()], axis=1)
    return np.concatenate([a, a + np.array([60.0, 0.0])])


def _line(n=300):
    """A 300-target path: hop counts up to 299 exceed the uint8 entries, so the device
    reruns the env with uint16 entries."""
    return np.stack([np.arange(n) * 5.5, np.zeros(n)], axis=1)


@pytest.mark.parametrize("horizon", [-1, 0, 1, 3, 10])
@pytest.mark.parametrize("which", ["map", "clusters", "line"])
def test_time_matrix_horizons_vs_oracle(horizon, which):
    """Sweep counts set by each arm of the stop rule: the horizon break, no inf left,
    and no change (disconnected graph), for several horizons including unbounded; the
    line exercises the wide (uint16) fallback."""
    if which == "map":
        from oracle.maps_host import generate_targets
        np.random.seed(21)
        targets = generate_targets()
    elif which == "clusters":
        targets = _two_clusters()
    else:
        targets = _line()
    R, M = 8, len(targets) + 8 + 2
    h = nat.CoverageHandle(R, 1, M, horizon=horizon)
    h.set_targets(targets, env=0)
    o = oc.CoverageOracle(targets, R, M)
    cost, prev = h.time_matrix(0, len(targets))
    ec, ep = oc.time_matrix(len(targets), o.motion[0] - R, o.motion[1] - R, horizon=horizon)
    np.testing.assert_array_equal(cost, ec)
    np.testing.assert_array_equal(prev, ep)
    h.close()


def _lattice(n):
    xs, ys = np.meshgrid(np.arange(n) * 5.5, np.arange(n) * 5.5)
    return np.stack([xs.ravel(), ys.ravel()], axis=1)


@pytest.mark.parametrize("case", ["one_env_676", "one_env_900", "batch_28", "batch_30"])
def test_time_matrix_wave_forms_vs_oracle(case):
    """Both forms of the time-matrix passes against the oracle: four waves per 64-source
    chunk when a launch has at most 256 chunks and their LDS fits (one env of 676 targets;
    28 envs of a 552-target map: 252 chunks), one wave per chunk otherwise (900 targets: the
    predecessors no longer fit in LDS beside the entries; 30 envs: 270 chunks)."""
    if case.startswith("one_env"):
        targets = _lattice(26 if case.endswith("676") else 30)
        B = 1
    else:
        from oracle.maps_host import generate_targets
        np.random.seed(21)
        targets = generate_targets()
        B = int(case.split("_")[1])
    T = len(targets)
    R, M = 8, T + 8 + 2
    h = nat.CoverageHandle(R, B, M, horizon=-1)
    for b in range(B):
        h.set_targets(targets, env=b)
    o = oc.CoverageOracle(targets, R, M)
    ec, ep = oc.time_matrix(T, o.motion[0] - R, o.motion[1] - R, horizon=-1)
    for b in sorted({0, B - 1}):
        cost, prev = h.time_matrix(b, T)
        np.testing.assert_array_equal(cost, ec)
        np.testing.assert_array_equal(prev, ep)
    h.close()


def _greedy_phase(v, maps, R, M, seed, steps):
    B = len(maps)
    start, visited = v.reset(seed=seed)
    orcs, mats = [], []
    for b in range(B):
        o = oc.CoverageOracle(maps[b], R, M)
        T = len(maps[b])
        o.reset(start[b], np.nonzero(visited[b, :T] == 0)[0] + R)
        orcs.append(o)
        mats.append(oc.time_matrix(T, o.motion[0] - R, o.motion[1] - R))
    rngs = [np.random.RandomState(1000 + b) for b in range(B)]
    n_rand = 0
    for t in range(steps):
        a, rnd = v.h.controller_greedy()
        for b in range(B):
            cur = orcs[b].closest()
            recv = oc.action_receivers(cur, orcs[b].nbr, orcs[b].cnt, R)
            ea, er = oc.greedy_actions(mats[b][0], mats[b][1], cur, orcs[b].visited[R:], recv, R)
            np.testing.assert_array_equal(rnd[b], er)
            np.testing.assert_array_equal(a[b][~er], ea[~er])
            for i in np.nonzero(er)[0]:
                a[b, i] = rngs[b].choice(4)
                n_rand += 1
        v.step(a)
        r, d = v.rewards()
        for b in range(B):
            _, rr, dd = orcs[b].step(a[b])
            assert r[b] == rr and d[b] == dd
    for b in range(B):
        cost, prev = v.h.time_matrix(b, len(maps[b]))
        np.testing.assert_array_equal(cost, mats[b][0])
        np.testing.assert_array_equal(prev, mats[b][1])
    return n_rand


def test_batched_greedy_vs_oracle():
    """6 envs, each its own map (different target counts, so per-env chunk counts
    differ), greedy for 20 steps against the oracle with per-env fallback RNGs; then a
    new graph for env 2 (only its matrix is stale) and another phase."""
    from oracle.maps_host import generate_targets
    B, R, M = 6, 16, 800
    maps = []
    for b in range(B):
        np.random.seed(300 + b)
        maps.append(generate_targets())
    v = VecCoverage(B, R, max_nodes=M)
    for b in range(B):
        v.set_targets(maps[b], env=b)
    _greedy_phase(v, maps, R, M, seed=11, steps=20)
    np.random.seed(999)
    maps[2] = generate_targets()
    v.set_targets(maps[2], env=2)
    _greedy_phase(v, maps, R, M, seed=12, steps=20)
    v.close()


def test_greedy_resident_actions_and_external_positions():
    """controller_greedy(fetch=False) leaves the actions on the device for
    step(resident=True); robots placed off-node use freshly computed closest nodes."""
    f = np.load(GREEDY[0])
    h, R, T, M = _handle_for(f)
    o = oc.CoverageOracle(f["targets"], R, M)
    cost, prev = oc.time_matrix(T, o.motion[0] - R, o.motion[1] - R)
    start = np.arange(R) * (T // R)
    h.reset(start[None], np.zeros((1, M - R), np.uint8))
    o.reset(start, np.arange(T) + R)
    xr = f["targets"][start] + np.random.RandomState(4).uniform(-2.0, 2.0, size=(R, 2))
    h.set_robot_positions(0, xr)
    o.xr = xr.copy()
    cur = o.closest()
    ea, er = oc.greedy_actions(cost, prev, cur, o.visited[R:], oc.action_receivers(cur, o.nbr, o.cnt, R), R)
    assert not er.any()
    a, rnd = h.controller_greedy()
    np.testing.assert_array_equal(a[0], ea)
    for t in range(5):
        h.controller_greedy(fetch=False)
        h.step(resident=True)
        cur = o.closest()
        ea, er = oc.greedy_actions(cost, prev, cur, o.visited[R:], oc.action_receivers(cur, o.nbr, o.cnt, R), R)
        ea[er] = 0  # the device leaves action 0 where the host would draw
        o.step(ea)
        np.testing.assert_array_equal(h.robots(0)[1], o.closest())
    h.close()


def test_mixed_width_batch_greedy_vs_oracle():
    """One batch with a 33x33 grid (1089 targets, more than one 512-target sweep of the
    row scan) and the 300-target line (hop counts past 254: the uint16 rerun), greedy
    against the oracle."""
    xs, ys = np.meshgrid(np.arange(33) * 5.5, np.arange(33) * 5.5)
    grid = np.stack([xs.ravel(), ys.ravel()], axis=1)
    maps = [grid, _line()]
    R, M = 8, 1100
    v = VecCoverage(2, R, max_nodes=M)
    for b in range(2):
        v.set_targets(maps[b], env=b)
    _greedy_phase(v, maps, R, M, seed=5, steps=15)
    v.close()


def test_fused_greedy_step_equals_separate():
    """cov_step(COV_ACTIONS_GREEDY): the greedy actions computed inside the step's launch
    from the per-node greedy lists, against controller_greedy (its own kernel) followed
    by a resident step, fallback robots taking action 0 in both. A batch of different
    maps over a whole episode (robots placed off-node in one env at step 10): the actions
    taken, needs_random, robots, rewards and observations are equal at every step."""
    from oracle.maps_host import generate_targets
    B, R, M = 4, 20, 800
    maps = []
    for b in range(B):
        np.random.seed(700 + b)
        maps.append(generate_targets())
    va, vb = VecCoverage(B, R, max_nodes=M), VecCoverage(B, R, max_nodes=M)
    for v in (va, vb):
        for b in range(B):
            v.set_targets(maps[b], env=b)
        v.reset(seed=21)
    n_rand = 0
    for t in range(75):
        if t == 10:
            xr = va.h.robots(1)[0] + np.random.RandomState(8).uniform(-2.0, 2.0, size=(R, 2))
            va.h.set_robot_positions(1, xr)
            vb.h.set_robot_positions(1, xr)
        ea, er = va.h.controller_greedy()
        va.step(resident=True)
        vb.step(greedy=True, fallback="zero")
        ga, gr = vb.h.actions()
        np.testing.assert_array_equal(ga, ea)
        np.testing.assert_array_equal(gr, er)
        n_rand += int(er.sum())
        ra, da = va.rewards()
        rb, db = vb.rewards()
        np.testing.assert_array_equal(ra, rb)
        np.testing.assert_array_equal(da, db)
        for b in range(B):
            np.testing.assert_array_equal(va.h.robots(b)[1], vb.h.robots(b)[1])
        if t % 15 == 0:
            oa, ob = va.obs(t % B), vb.obs(t % B)
            for k in oa:
                np.testing.assert_array_equal(oa[k], ob[k])
    print("fallback robots over the episode:", n_rand)
    va.close()
    vb.close()


def test_fused_greedy_step_vs_oracle():
    """The fused greedy step against the oracle's greedy actions (fallbacks as action 0)
    on the recorded r20 map, 30 steps: robots' nodes equal every step."""
    f = np.load(GREEDY[-1])
    h, R, T, M = _handle_for(f)
    o = oc.CoverageOracle(f["targets"], R, M)
    cost, prev = oc.time_matrix(T, o.motion[0] - R, o.motion[1] - R)
    start = np.arange(R) * (T // R)
    h.reset(start[None], np.zeros((1, M - R), np.uint8))
    o.reset(start, np.arange(T) + R)
    for t in range(30):
        cur = o.closest()
        ea, er = oc.greedy_actions(cost, prev, cur, o.visited[R:], oc.action_receivers(cur, o.nbr, o.cnt, R), R)
        ea[er] = 0
        h.step(greedy=True)
        np.testing.assert_array_equal(h.actions()[0][0], ea)
        o.step(ea)
        np.testing.assert_array_equal(h.robots(0)[1], o.closest())
    h.close()


def test_fused_greedy_deep_list_scans_vs_oracle():
    """Late-episode shape: every target visited but a few, so each robot's greedy list is
    scanned far past its first load of entries (the list loader fetches 32 entries per
    round trip). The fused greedy step against the oracle for 25 steps on the r20 map, with
    the remaining targets at depths 7..213 of the robots' lists; the robots reach all six
    within the 25 steps, after which every robot falls back."""
    f = np.load(GREEDY[-1])
    h, R, T, M = _handle_for(f)
    o = oc.CoverageOracle(f["targets"], R, M)
    cost, prev = oc.time_matrix(T, o.motion[0] - R, o.motion[1] - R)
    rs = np.random.RandomState(3)
    start = rs.choice(T, R, replace=False)
    left = rs.choice(np.setdiff1d(np.arange(T), start), size=6, replace=False)
    vis = np.ones((1, M - R), np.uint8)
    vis[0, left] = 0
    h.reset(start[None], vis)
    o.reset(start, left + R)
    depths = []
    for t in range(25):
        cur = o.closest()
        if t == 0:  # how deep the first unvisited target sits in each robot's list
            for c in cur - R:
                order = np.lexsort((np.arange(T), cost[c]))
                depths.append(int(np.nonzero(np.isin(order, left))[0][0]))
        ea, er = oc.greedy_actions(cost, prev, cur, o.visited[R:], oc.action_receivers(cur, o.nbr, o.cnt, R), R)
        ea[er] = 0
        h.step(greedy=True)
        ga, gr = h.actions()
        np.testing.assert_array_equal(gr[0], er)
        np.testing.assert_array_equal(ga[0], ea)
        o.step(ea)
        np.testing.assert_array_equal(h.robots(0)[1], o.closest())
    assert max(depths) > 64, depths  # scans past two round trips of the loader
    h.close()


def test_cov_step_host_batched_matches_step_and_getters():
    """cov_step_host on a batch of 3 envs with distinct maps, page-locked destinations
    (written by the step's own workgroups) on even steps and pageable numpy arrays (copies
    after the launch) on odd steps, with COV_NEXT_GREEDY: every env's observation, step,
    reward, done, robot nodes and next greedy actions equal those of cov_step + the
    getters + cov_controller_greedy on a second handle stepped with the same actions."""
    from oracle.maps_host import generate_targets
    B, R, M = 3, 10, 700
    maps = []
    for b in range(B):
        np.random.seed(300 + b)
        maps.append(generate_targets())
    hs = [nat.CoverageHandle(R, B, M) for _ in range(2)]
    rs = np.random.RandomState(31)
    start = np.stack([rs.choice(len(maps[b]), R, replace=False) for b in range(B)]).astype(np.int32)
    visited = np.ones((B, M - R), np.uint8)
    for b in range(B):
        visited[b, :len(maps[b])] = rs.randint(0, 2, len(maps[b]))
    for h in hs:
        for b in range(B):
            h.set_targets(maps[b], env=b)
        h.reset(start, visited)
    pool = nat.host_pool()
    for t in range(12):
        a = rs.randint(0, 4, size=(B, R)).astype(np.int32)
        new = pool.array if t % 2 == 0 else (lambda shape, dt: np.empty(shape, dt))
        o = dict(nodes=new((B, M, 3), np.float32), edges=new((B, 4 * M), np.float32),
                 senders=new((B, 4 * M), np.int32), receivers=new((B, 4 * M), np.int32),
                 step=new((B,), np.int64), reward=new((B,), np.float64), done=new((B,), np.uint8),
                 closest=new((B, R), np.int32), nxt=new((B, R), np.int32), nrd=new((B, R), np.uint8))
        hs[0].step_host(a, *(o[k].ctypes.data for k in ("nodes", "edges", "senders", "receivers", "step", "reward",
                                                         "done", "closest", "nxt", "nrd")))
        hs[1].step(a)
        r1, d1 = hs[1].rewards()
        np.testing.assert_array_equal(o["reward"], r1)
        np.testing.assert_array_equal(o["done"].astype(bool), d1)
        ga, gr = hs[1].controller_greedy()
        np.testing.assert_array_equal(o["nxt"], ga)
        np.testing.assert_array_equal(o["nrd"].astype(bool), gr)
        for b in range(B):
            ob = hs[1].obs(b)
            np.testing.assert_array_equal(o["nodes"][b], ob["nodes"])
            np.testing.assert_array_equal(o["edges"][b], ob["edges"][:, 0])
            np.testing.assert_array_equal(o["senders"][b], ob["senders"])
            np.testing.assert_array_equal(o["receivers"][b], ob["receivers"])
            assert o["step"][b] == ob["step"][0, 0]
            np.testing.assert_array_equal(o["closest"][b], hs[1].robots(b)[1])
    for h in hs:
        h.close()


def test_greedy_list_and_direct_paths_vs_oracle():
    """60 unvisited targets on the r20 map, 40 greedy steps: the greedy actions come from
    the list scan while more than 32 targets are unvisited and from the direct minimum over
    the short candidate list after that (until none is left). Through the three device
    forms at once: the fused greedy step (COV_ACTIONS_GREEDY), cov_step_host's next-state
    actions (COV_NEXT_GREEDY) and the standalone controller (cov_controller_greedy), each
    against the oracle's greedy expert, robots' nodes checked every step."""
    f = np.load(GREEDY[-1])
    hs = [_handle_for(f)[0] for _ in range(2)]
    R, T, M = int(f["n_robots"]), int(f["n_targets"]), int(f["max_nodes"])
    o = oc.CoverageOracle(f["targets"], R, M)
    cost, prev = oc.time_matrix(T, o.motion[0] - R, o.motion[1] - R)
    rs = np.random.RandomState(8)
    start = rs.choice(T, R, replace=False)
    left = rs.choice(np.setdiff1d(np.arange(T), start), size=60, replace=False)
    vis = np.ones((1, M - R), np.uint8)
    vis[0, left] = 0
    for h in hs:
        h.reset(start[None], vis)
    o.reset(start, left + R)
    pool = nat.host_pool()
    outs = {k: pool.array(shape, dt) for k, shape, dt in (("nxt", (1, R), np.int32), ("nrd", (1, R), np.uint8))}
    n_left = []
    for t in range(40):
        cur = o.closest()
        ea, er = oc.greedy_actions(cost, prev, cur, o.visited[R:], oc.action_receivers(cur, o.nbr, o.cnt, R), R)
        ea[er] = 0
        n_left.append(int((o.visited[R:] == 0).sum()))
        ga, gr = hs[1].controller_greedy()  # standalone kernel on the second handle's state
        np.testing.assert_array_equal(ga[0], ea)
        np.testing.assert_array_equal(gr[0], er)
        if t > 0:  # the previous cov_step_host computed this state's actions already
            np.testing.assert_array_equal(outs["nxt"][0], ea)
            np.testing.assert_array_equal(outs["nrd"][0].astype(bool), er)
        hs[0].step(greedy=True)
        a0, r0 = hs[0].actions()
        np.testing.assert_array_equal(a0[0], ea)
        np.testing.assert_array_equal(r0[0], er)
        hs[1].step_host(ea[None].astype(np.int32), None, None, None, None, None, None, None, None,
                        outs["nxt"].ctypes.data, outs["nrd"].ctypes.data)
        o.step(ea)
        for h in hs:
            np.testing.assert_array_equal(h.robots(0)[1], o.closest())
    assert max(n_left) > 32 and min(n_left) <= 32, n_left  # both paths taken
    for h in hs:
        h.close()


def _reset_stream(seed, T, R):
    """A reference env's np_random after reset's two draws (coverage.py:405-424)."""
    rs = np.random.RandomState(seed)
    rs.choice(np.arange(T), size=(R,), replace=False)
    rs.choice(np.arange(T) + R, size=(int(T * 0.5),), replace=False)
    return rs


@pytest.mark.parametrize("path", GREEDY, ids=os.path.basename)
def test_device_rng_greedy_episode_matches_reference(path):
    """COV_GREEDY_RNG: the recorded greedy episode as fused greedy steps, the fallback
    robots' np_random.choice(4) (coverage.py:861-864) drawn on the device from the env's
    stream (the fixture's seed after reset's draws): actions, rewards and robots' nodes
    bit-exact at every step, and the device stream afterwards equals the host RandomState
    after as many draws."""
    f = np.load(path)
    h, R, T, M = _handle_for(f)
    start = oc.closest_targets(f["x0"][:R], f["targets"], R) - R
    visited = np.ones((1, M - R), np.uint8)
    visited[0, :T] = f["visited0"][R:].astype(np.uint8)
    h.reset(start[None], visited)
    rs = _reset_stream(ENV_SEED[os.path.basename(path)], T, R)
    h.set_rng([rs])
    n_draws = 0
    for t in range(len(f["actions"])):
        h.step(greedy=True, rng=True)
        a, rnd = h.actions()
        np.testing.assert_array_equal(a[0], f["actions"][t])
        n_draws += int(rnd.sum())
        r, d = h.rewards()
        assert r[0] == f["reward"][t] and d[0] == f["done"][t]
        np.testing.assert_array_equal(h.robots(0)[1], f["closest"][t])
    if "r20" in path:
        assert n_draws > 0  # (the r6 episode never falls back)
    rs.randint(0, 4, size=n_draws)
    keys, pos = h.get_rng()
    st = rs.get_state()
    assert pos[0] == st[2]
    np.testing.assert_array_equal(keys[0], st[1])
    h.close()


@pytest.mark.parametrize("R", [16, 200])
def test_device_rng_batched_vs_oracle(R):
    """VecCoverage.step(greedy=True) with the reference's fallback draws (the default):
    4 envs with their own maps and streams (seed + b after reset's draws), two half-batch
    launches per step, against the oracle's greedy expert with per-env RandomStates drawing
    in robot order. At R=200 most robots fall back once the targets near them are visited,
    so each stream passes several key regenerations. Actions, fallback flags, rewards and
    nodes bit-exact every step; the device streams equal the host's at the end."""
    from oracle.maps_host import generate_targets
    B, M, steps = 4, 1000, 40
    maps = []
    for b in range(B):
        np.random.seed(500 + b)
        maps.append(generate_targets())
    v = VecCoverage(B, R, max_nodes=M)
    for b in range(B):
        v.set_targets(maps[b], env=b)
    start, visited = v.reset(seed=40)
    orcs, mats, rngs = [], [], []
    for b in range(B):
        T = len(maps[b])
        o = oc.CoverageOracle(maps[b], R, M)
        o.reset(start[b], np.nonzero(visited[b, :T] == 0)[0] + R)
        orcs.append(o)
        mats.append(oc.time_matrix(T, o.motion[0] - R, o.motion[1] - R))
        rngs.append(_reset_stream(40 + b, T, R))
    n_draws = 0
    for t in range(steps):
        v.step(greedy=True)
        ga, gr = v.h.actions()
        r, d = v.rewards()
        for b in range(B):
            o = orcs[b]
            cur = o.closest()
            ea, er = oc.greedy_actions(mats[b][0], mats[b][1], cur, o.visited[R:],
                                       oc.action_receivers(cur, o.nbr, o.cnt, R), R)
            k = np.nonzero(er)[0]
            ea[k] = rngs[b].choice(4, size=len(k))
            n_draws += len(k)
            np.testing.assert_array_equal(gr[b], er)
            np.testing.assert_array_equal(ga[b], ea)
            _, rr, dd = o.step(ea)
            assert r[b] == rr and d[b] == dd
            np.testing.assert_array_equal(v.h.robots(b)[1], o.closest())
    if R == 200:
        assert n_draws > 4 * 2 * 624, n_draws  # regenerations in every stream
    for b in range(B):
        st, want = v.np_random(b).get_state(), rngs[b].get_state()
        assert st[2] == want[2]
        np.testing.assert_array_equal(st[1], want[1])
    v.close()


def test_device_rng_argument_checks():
    """COV_GREEDY_RNG before cov_set_rng is GF_ESTATE; positions outside [0, 624] and more
    than 624 robots are refused."""
    f = np.load(GREEDY[0])
    h, R, T, M = _handle_for(f)
    start = np.arange(R, dtype=np.int32)[None]
    h.reset(start, np.zeros((1, M - R), np.uint8))
    with pytest.raises(nat.GymFlockError, match="cov_set_rng"):
        h.step(greedy=True, rng=True)
    st = list(np.random.RandomState(1).get_state())
    st[2] = 625
    with pytest.raises(nat.GymFlockError, match="position"):
        h.set_rng([tuple(st)])
    h.close()
    h = nat.CoverageHandle(700, 1, 2400)  # room for 8 * 700 action edges beside the motion graph
    with pytest.raises(nat.GymFlockError, match="624"):
        h.set_rng([np.random.RandomState(1)])
    # streams from the device reset do not lift the limit either
    xs, ys = np.meshgrid(np.arange(28) * 5.5, np.arange(28) * 5.5)  # 784 targets >= 700 robots
    h.set_targets(np.stack([xs.ravel(), ys.ravel()], axis=1), env=0)
    h.reset_seeded(3)
    with pytest.raises(nat.GymFlockError, match="624"):
        h.step(greedy=True, rng=True)
    h.close()


def test_device_rng_config4_batch_sampled_vs_oracle():
    """The bench's config-4 shape (R=200, the map of seed 8, max_nodes 1000) at 64 envs: a
    whole episode (75 steps, EPISODE_LENGTH) of VecCoverage.step(greedy=True) with the
    fallback draws on the device, every env stepping in the same two half-batch launches;
    envs 0, 31 and 63 checked against the oracle's expert with their own RandomStates at
    every step (actions, nodes, rewards and done flags), and their streams at the end."""
    from oracle.maps_host import generate_targets
    R, B, M = 200, 64, 1000
    np.random.seed(8)
    targets = generate_targets()
    T = len(targets)
    v = VecCoverage(B, R, max_nodes=M)
    v.set_targets(targets)
    start, visited = v.reset(seed=0)
    o0 = oc.CoverageOracle(targets, R, M)
    cost, prev = oc.time_matrix(T, o0.motion[0] - R, o0.motion[1] - R)
    picks = (0, 31, 63)
    orcs, rngs = {}, {}
    for b in picks:
        o = oc.CoverageOracle(targets, R, M)
        o.reset(start[b], np.nonzero(visited[b, :T] == 0)[0] + R)
        orcs[b] = o
        rngs[b] = _reset_stream(b, T, R)
    draws = 0
    for t in range(75):
        v.step(greedy=True)
        ga, gr = v.h.actions()
        r, d = v.rewards()
        for b in picks:
            o = orcs[b]
            cur = o.closest()
            ea, er = oc.greedy_actions(cost, prev, cur, o.visited[R:], oc.action_receivers(cur, o.nbr, o.cnt, R), R)
            k = np.nonzero(er)[0]
            ea[k] = rngs[b].choice(4, size=len(k))
            draws += len(k)
            np.testing.assert_array_equal(gr[b], er, err_msg="env %d step %d" % (b, t))
            np.testing.assert_array_equal(ga[b], ea, err_msg="env %d step %d" % (b, t))
            _, rr, dd = o.step(ea)
            assert r[b] == rr and d[b] == dd, (b, t)
            np.testing.assert_array_equal(v.h.robots(b)[1], o.closest())
    assert draws > 624  # the sampled streams pass a key regeneration
    for b in picks:
        st, want = v.np_random(b).get_state(), rngs[b].get_state()
        assert st[2] == want[2]
        np.testing.assert_array_equal(st[1], want[1])
    v.close()


@pytest.mark.parametrize("R", [6, 200])
def test_device_reset_draws_equal_host_draws(R):
    """VecCoverage.reset on the device (cov_reset_seeded: RandomState(seed + b)'s two
    choices without replacement, one wave per env) against the host draws (RandomState
    loops, cov_reset + cov_set_rng): starts, visited flags, the observations reset()
    returns and the envs' streams equal, for envs with different maps (target counts), and
    the first greedy steps after it take the same actions."""
    from oracle.maps_host import generate_targets
    B, M = 5, 1000
    maps = []
    for b in range(B):
        np.random.seed(600 + b)
        maps.append(generate_targets())
    vs = [VecCoverage(B, R, max_nodes=M, env_offset=3) for _ in range(2)]
    for v in vs:
        for b in range(B):
            v.set_targets(maps[b], env=b)
    sd, vd = vs[0].reset(seed=77)
    sh, vh = vs[1].reset(seed=77, draws="host")
    np.testing.assert_array_equal(sd, sh)
    np.testing.assert_array_equal(vd, vh)
    kd, pd = vs[0].h.get_rng()
    kh, ph = vs[1].h.get_rng()
    np.testing.assert_array_equal(kd, kh)
    np.testing.assert_array_equal(pd, ph)
    for b in range(B):
        od, oh = vs[0].obs(b), vs[1].obs(b)
        for k in od:
            np.testing.assert_array_equal(od[k], oh[k])
    for t in range(10):
        for v in vs:
            v.step(greedy=True)
        np.testing.assert_array_equal(vs[0].h.actions()[0], vs[1].h.actions()[0])
    # and the host RandomState of env 2 (seed 77 + 3 + 2) matches the device stream after reset
    rs = np.random.RandomState(77 + 3 + 2)
    T = len(maps[2])
    np.testing.assert_array_equal(sd[2], rs.choice(np.arange(T), size=(R,), replace=False))
    for v in vs:
        v.close()


@pytest.mark.parametrize("frac", [0.0, 0.3, 1.0])
def test_device_reset_fraction_edges(frac):
    """cov_reset_seeded at the ends of frac_active_targets (nothing unvisited, everything
    unvisited) and between: the draws and visited flags equal the host loops'."""
    from oracle.maps_host import generate_targets
    np.random.seed(31)
    targets = generate_targets()
    vs = [VecCoverage(3, 8, max_nodes=800, frac_active_targets=frac) for _ in range(2)]
    for v in vs:
        v.set_targets(targets)
    sd, vd = vs[0].reset(seed=5)
    sh, vh = vs[1].reset(seed=5, draws="host")
    np.testing.assert_array_equal(sd, sh)
    np.testing.assert_array_equal(vd, vh)
    np.testing.assert_array_equal(vs[0].h.get_rng()[0], vs[1].h.get_rng()[0])
    for v in vs:
        v.close()


@pytest.mark.parametrize("R", [20, 200])
def test_expert_steps_one_launch_equals_single_steps(R):
    """VecCoverage.expert_steps(n) (cov_step_expert: n fused greedy expert steps with the
    device fallback draws in ONE launch) against n calls of step(greedy=True) on a twin
    batch: 4 envs with their own device maps and streams, 75 steps (an episode) then 40 more
    (at R=200 most robots draw once their targets are visited: several key regenerations
    inside one launch). Every step's rewards and done flags, the final observations,
    robots' nodes, visited flags, last actions and the streams bit-exact."""
    B, M = 4, 1000
    v1, v2 = VecCoverage(B, R, max_nodes=M), VecCoverage(B, R, max_nodes=M)
    for v in (v1, v2):
        v.reset(seed=21, new_maps=True, map_seed=5)
    for n in (75, 40):
        rw = np.empty((n, B))
        dn = np.empty((n, B), bool)
        for t in range(n):
            v1.step(greedy=True)
            rw[t], dn[t] = v1.rewards()
        r2, d2 = v2.expert_steps(n)
        np.testing.assert_array_equal(r2, rw)
        np.testing.assert_array_equal(d2, dn)
        for b in range(B):
            o1, o2 = v1.obs(b), v2.obs(b)
            for k in ("nodes", "edges", "senders", "receivers", "step"):
                np.testing.assert_array_equal(o2[k], o1[k], err_msg="%s env %d" % (k, b))
            np.testing.assert_array_equal(v2.h.robots(b)[1], v1.h.robots(b)[1])
            np.testing.assert_array_equal(v2.h.visited(b), v1.h.visited(b))
            s1, s2 = v1.np_random(b).get_state(), v2.np_random(b).get_state()
            assert s1[2] == s2[2]
            np.testing.assert_array_equal(s1[1], s2[1])
        for x1, x2 in zip(v1.h.actions(), v2.h.actions()):
            np.testing.assert_array_equal(x2, x1)
    assert rw.sum() >= 0
    with pytest.raises(nat.GymFlockError):
        v2.h.step_expert(0)
    v1.close()
    v2.close()

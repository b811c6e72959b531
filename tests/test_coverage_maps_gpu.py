"""Per-episode Coverage maps on the device (cov_generate_maps; SURVEY.md §8f row 2,
coverage.py:516-527 with make_map.py:30-67, :207-231) against the reference's recorded
maps (tests/golden/coverage_maps.npz: 100 seeds, and the second map of 10 of those
streams), the host generator with scipy's Delaunay (oracle/maps_host.py) and the
restatement of the device algorithm (oracle/coverage_maps.py). Targets are compared
bit-exactly, and so are the cities the device draws from each env's stream and the
motion graphs built from the maps. Needs an MI355X."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import coverage_maps as cmo
from oracle.maps_host import generate_targets as host_targets

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")
from gym_flock.vec import VecCoverage  # noqa: E402


def _fixture():
    f = np.load(os.path.join(GOLDEN, "coverage_maps.npz"))
    lat = f["lattice"]

    def split(lens, idx):
        out, o = [], 0
        for n in lens:
            out.append(lat[idx[o:o + n]])
            o += n
        return out

    return f, split(f["many_len"], f["many_idx"]), split(f["next_len"], f["next_idx"])


def _targets(h, n):
    return [h.targets(b, int(n[b])) for b in range(len(n))]


def test_device_maps_match_reference_maps():
    """Env b's stream seeded as np.random.seed(b): its cities are RandomState(b)'s 24
    uniform draws and its targets the reference's map for seed b, for 100 seeds; the
    next call (streams continued) gives the reference's second map of each stream."""
    f, many, nxt = _fixture()
    B = len(many)
    h = nat.CoverageHandle(6, B, 1000)
    n, st, cities = h.generate_maps(map_seed=0)
    assert not (st & ~nat.COV_MAP_NEAR_DEGENERATE).any(), st
    for b in range(B):
        np.testing.assert_array_equal(cities[b], cmo.cities(np.random.RandomState(b)))
        assert n[b] == len(many[b]), (b, n[b], len(many[b]))
    for b, t in enumerate(_targets(h, n)):
        np.testing.assert_array_equal(t, many[b], err_msg="seed %d" % b)
    for s in range(3):
        np.testing.assert_array_equal(h.targets(s, n[s]), f["targets_seed%d" % s])
    n2, st2, _ = h.generate_maps()  # continue every stream
    for b in range(len(nxt)):
        np.testing.assert_array_equal(h.targets(b, n2[b]), nxt[b], err_msg="second map of seed %d" % b)
    h.close()


def test_device_maps_given_cities_vs_host_and_restatement():
    """Cities given by the caller (the drop-in env's np.random draws): 40 streams beyond the
    fixture's seeds against the scipy host generator and the restated device algorithm,
    one env at a time and as a batch."""
    seeds = list(range(1000, 1040))
    cities = np.stack([cmo.cities(np.random.RandomState(s)) for s in seeds])
    h = nat.CoverageHandle(6, len(seeds), 1000)
    n, st, _ = h.generate_maps(cities=cities)
    h1 = nat.CoverageHandle(6, 1, 1000)
    for b, s in enumerate(seeds):
        np.random.seed(s)
        ref = host_targets(120, 120, 5.5, 5.5 * 1.2)
        got = h.targets(b, n[b])
        np.testing.assert_array_equal(got, ref, err_msg="seed %d" % s)
        rt, amb = cmo.generate_targets(cities[b])
        np.testing.assert_array_equal(got, rt)
        assert bool(st[b] & nat.COV_MAP_NEAR_DEGENERATE) == amb
        if b < 8:
            n1, _, _ = h1.generate_maps(cities=cities[b:b + 1], env=0)
            np.testing.assert_array_equal(h1.targets(0, n1[0]), ref)
    h.close()
    h1.close()


def test_device_map_motion_graph_equals_uploaded_map():
    """The motion graph and static observation built after a device map equal those of the
    same targets uploaded with cov_set_targets (both through cov_graph_kernel)."""
    B, R, M = 6, 20, 800
    h = nat.CoverageHandle(R, B, M)
    n, _, _ = h.generate_maps(map_seed=7)
    g = nat.CoverageHandle(R, B, M)
    for b in range(B):
        g.set_targets(h.targets(b, n[b]), env=b)
    np.testing.assert_array_equal(h.n_motion(), g.n_motion())
    for b in range(B):
        oh, og = h.obs(b), g.obs(b)
        for k in ("nodes", "edges", "senders", "receivers"):
            np.testing.assert_array_equal(oh[k], og[k])
    h.close()
    g.close()


def test_map_too_large_for_max_nodes_fails():
    """Seed 4's map has 648 targets: with max_nodes 606 and 6 robots (600 slots; seeds
    0-5 have 536, 410, 437, 431, 648, 394) the call fails with GF_EINVAL naming env 4,
    like the reference, whose padded observation cannot hold it (with its default
    max_nodes 500, 10 of the 100 recorded maps are too large); the other envs keep their
    maps."""
    f, many, _ = _fixture()
    assert len(many[4]) == 648 and max(len(many[b]) for b in (0, 1, 2, 3, 5)) <= 600
    h = nat.CoverageHandle(6, 6, 606)
    with pytest.raises(nat.GymFlockError) as e:
        h.generate_maps(map_seed=0)
    assert e.value.code == nat.GF_EINVAL and "env 4" in str(e.value) and "648" in str(e.value)
    np.testing.assert_array_equal(h.targets(3, len(many[3])), many[3])
    h.close()


def test_vec_reset_new_maps_then_expert_episode_vs_oracle():
    """VecCoverage.reset(seed, new_maps=True, map_seed): every env its own device map,
    the device reset draws and the fused greedy expert with the fallback draws on the
    device; every env replayed on the CPU oracle from the reference's maps and the same
    seeds matches step for step (rewards, observations); a second reset with new_maps
    draws the next map of each stream."""
    from oracle import coverage as oc
    B, R, M = 4, 20, 800
    f, many, nxt = _fixture()
    v = VecCoverage(B, R, max_nodes=M)
    start, visited = v.reset(seed=11, new_maps=True, map_seed=0)
    orcs, mats, rngs = [], [], []
    for b in range(B):
        T = len(many[b])
        assert v.n_targets[b] == T
        np.testing.assert_array_equal(v.h.targets(b, T), many[b])
        rs = np.random.RandomState(11 + b)  # the reference env's np_random, reset's draws
        st = rs.choice(np.arange(T), size=(R,), replace=False)
        drop = rs.choice(np.arange(T) + R, size=(int(T * 0.5),), replace=False)
        np.testing.assert_array_equal(start[b], st)
        o = oc.CoverageOracle(many[b], R, M)
        o.reset(st, drop)
        orcs.append(o)
        mats.append(oc.time_matrix(T, o.motion[0] - R, o.motion[1] - R))
        rngs.append(rs)
    for t in range(12):
        v.step(greedy=True)
        r, d = v.rewards()
        for b in range(B):
            o = orcs[b]
            cur = o.closest()
            recv = oc.action_receivers(cur, o.nbr, o.cnt, R)
            a, rnd = oc.greedy_actions(mats[b][0], mats[b][1], cur, o.visited[R:], recv, R)
            for i in np.nonzero(rnd)[0]:
                a[i] = rngs[b].choice(4)
            ref, rr, dd = o.step(a)
            assert r[b] == rr and d[b] == dd, (t, b)
            got = v.obs(b)
            for key in ("nodes", "senders", "receivers"):
                np.testing.assert_array_equal(got[key].reshape(ref[key].shape), ref[key], err_msg="t=%d b=%d" % (t, b))
    v.reset(seed=12, new_maps=True)
    for b in range(B):
        np.testing.assert_array_equal(v.targets(b), nxt[b])
    v.close()


def test_dropin_default_env_map_capacity():
    """The reference's default Coverage-v0 (max_nodes 500, 6 robots) with np.random.seed(4)
    builds a 648-target map in its constructor without complaint and resets onto the next
    map (393 targets); with seed 0 both maps (536, 554) are too large and reset() raises
    ValueError (the reference's broadcast error, coverage.py:325). The same here."""
    from gym_flock.envs.spatial.coverage import CoverageEnv
    f, many, nxt = _fixture()
    np.random.seed(4)
    env = CoverageEnv()
    env.reset()
    np.testing.assert_array_equal(env.targets, nxt[4])
    env.close()
    np.random.seed(0)
    env = CoverageEnv()
    with pytest.raises(ValueError):
        env.reset()
    env.close()


def test_dropin_reset_draws_reference_maps():
    """CoverageEnv.reset() after np.random.seed(s): the map the reference's reset draws
    (its cities from the global np.random, the rest on the device), for three seeds, and
    the global stream left where the reference leaves it."""
    from gym_flock.envs.spatial.coverage import CoverageEnv
    f, many, _ = _fixture()
    env = CoverageEnv(n_robots=6, nearby_starts=False, max_nodes=1000, init_graph=False)
    for s in (0, 5, 9):
        np.random.seed(s)
        env.reset()
        np.testing.assert_array_equal(env.targets, many[s])
        after = np.random.random_sample()
        rs = np.random.RandomState(s)
        rs.random_sample(24)
        assert after == rs.random_sample()
    env.close()


@pytest.mark.parametrize("world_radius", [260.0, 3000.0], ids=["grid", "scan"])
def test_device_map_far_cities_grid_and_scan(world_radius):
    """A small arena (30 x 30 half-widths) with 4 of the 12 given cities ~250 away: the
    near-road test through the waypoint grid (world_radius 260: a 113-cell grid, most of
    it far from the arena) and through the scan of every waypoint (world_radius 3000: the
    grid would need more than 256 cells a side) give the restated algorithm's map."""
    rs = np.random.RandomState(3)
    c = np.concatenate([rs.uniform(-28, 28, size=(8, 2)), [[-250, -240], [255, -235], [-245, 258], [252, 248]]])
    mc = nat.map_config_default(xmax=30, ymax=30)
    mc.world_radius = world_radius
    ref, amb = cmo.generate_targets(c, 30, 30)
    assert 2 <= len(ref) < 500 and not amb
    h = nat.CoverageHandle(2, 1, 500)
    n, st, _ = h.generate_maps(cities=c[None], env=0, map_config=mc)
    assert n[0] == len(ref) and st[0] == 0
    np.testing.assert_array_equal(h.targets(0, n[0]), ref)
    h.close()

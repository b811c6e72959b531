"""Parity of the HIP FlockingRelative / Flocking-v0 path against the reference's golden
vectors and the CPU oracle, through the C-ABI (ctypes). Needs an MI355X.

Tolerances (north star: 1e-5 rtol in float32, integer indices bit-exact):
  state x (float64)          bit-exact (same op order, no FMA contraction)
  adjacency / network        bit-exact (network = float32(1/deg) on set bits)
  state_values (float32)     |d| <= 1e-5*|ref| + 1e-9 (float64 sums, order differs)
  controller (float64)       |d| <= 1e-9*|ref| + 1e-12
  reward (float64)           rtol 1e-12
  kNN indices                bit-exact; kNN obs float32 of float64 differences
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import flocking as orc

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")
from gym_flock.init_states import synthetic_batch  # noqa: E402
from gym_flock.vec import VecFlockingRelative  # noqa: E402

STEP_FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "flock_n*_s*_step.npz")))


def adj_from_bits(bits, n):
    return np.unpackbits(bits, axis=1, count=n).astype(bool)


def close_sv(ours, ref):
    np.testing.assert_allclose(ours, ref, rtol=1e-5, atol=1e-9)


def check_against_oracle(h, x0, u, b=None, ctrl=True):
    """Compare env b of handle h (after one step from x0 with u) to the oracle."""
    ref = orc.step(x0, u, with_controller=ctrl)
    env = 0 if b is None else b
    np.testing.assert_array_equal(h.get_state(env), ref["x"])
    net = h.network(env)
    np.testing.assert_array_equal(net > 0, ref["adj"])
    np.testing.assert_array_equal(net, ref["network"].astype(np.float32))
    close_sv(h.state_values(env), ref["state_values"])
    np.testing.assert_allclose(h.rewards()[env], ref["reward"], rtol=1e-12)
    if ctrl:
        np.testing.assert_allclose(h.controls(env), ref["ctrl"], rtol=1e-9, atol=1e-12)
    return ref


@pytest.mark.parametrize("path", STEP_FIXTURES, ids=os.path.basename)
def test_step_matches_reference_golden(path):
    f = np.load(path)
    n = f["x0"].shape[0]
    h = nat.FlockHandle(n, 1, n_neighbors=7)
    h.set_state(f["x0"][None])
    h.step(f["u"][None], nat.FE_WITH_CONTROLLER | nat.FE_WITH_KNN)
    np.testing.assert_array_equal(h.get_state(0), f["x1"])
    net = h.network(0)
    adj = adj_from_bits(f["adj_bits"], n)
    np.testing.assert_array_equal(net > 0, adj)
    deg = np.maximum(f["deg"], 1).astype(np.float64)
    np.testing.assert_array_equal(net, (adj / deg[:, None]).astype(np.float32))
    close_sv(h.state_values(0), f["state_values"])
    np.testing.assert_allclose(h.rewards()[0], f["reward"], rtol=1e-12)
    np.testing.assert_allclose(h.controls(0), f["ctrl"], rtol=1e-9, atol=1e-12)
    idx, obs = h.knn(0)
    np.testing.assert_array_equal(idx, f["knn_idx"])
    x1 = f["x1"]
    want_obs = np.concatenate([x1 - x1[f["knn_idx"][:, m]] for m in range(7)], axis=1)
    if "knn_obs" in f:
        np.testing.assert_array_equal(want_obs, f["knn_obs"])
    np.testing.assert_array_equal(obs, want_obs.astype(np.float32))
    vd, md, _ = h.stats(0)
    np.testing.assert_allclose(vd, f["vel_diffs"], rtol=1e-12)
    np.testing.assert_array_equal(md, f["min_dists"])
    dec = h.controller(centralized=False)[0]
    np.testing.assert_allclose(dec, f["ctrl_decentralized"], rtol=1e-9, atol=1e-12)
    # float64 actions take the float64 arithmetic path of the reference
    h.set_state(f["x0"][None])
    h.step(f["u64"][None])
    np.testing.assert_array_equal(h.get_state(0), f["x1_u64"])
    np.testing.assert_array_equal((h.network(0) > 0).sum(axis=1), f["deg_u64"])
    close_sv(h.state_values(0), f["sv_u64"])
    np.testing.assert_allclose(h.rewards()[0], f["reward_u64"], rtol=1e-12)
    h.close()


def test_n10_episode_trajectory_bit_exact():
    """Config 1: the reference's 40-step N=10 episode (20 expert, 20 float32 random
    actions) replayed through the engine: state bit-exact at every step."""
    f = np.load(os.path.join(GOLDEN, "flock_n10_episode.npz"))
    h = nat.FlockHandle(10, 1)
    h.set_state(f["x0"][None])
    h.compute_helpers()
    close_sv(h.state_values(0), f["sv0"])
    np.testing.assert_array_equal(h.network(0), f["net0"].astype(np.float32))
    for t in range(40):
        u = f["u"][t].astype(np.float32) if f["u_is_f32"][t] else f["u"][t]
        if not f["u_is_f32"][t]:
            np.testing.assert_allclose(h.controller()[0], u, rtol=1e-9, atol=1e-12)
        h.step(u[None], nat.FE_WITH_CONTROLLER)
        np.testing.assert_array_equal(h.get_state(0), f["x"][t])
        close_sv(h.state_values(0), f["sv"][t])
        np.testing.assert_array_equal(h.network(0), f["net"][t].astype(np.float32))
        np.testing.assert_allclose(h.rewards()[0], f["reward"][t], rtol=1e-12)
        np.testing.assert_allclose(h.controls(0), f["ctrl"][t], rtol=1e-9, atol=1e-12)
    h.close()


@pytest.mark.parametrize("mode", ["direct", "pooled"])
def test_dropin_expert_loop_episode(mode):
    """The reference's 40-step N=10 episode (20 expert steps u = env.controller(), then 20
    float32 random actions) through the drop-in env API. In "direct" mode every step is
    one fe_step_host launch that also computes the next expert action, which the next
    controller() returns without a launch. State bit-exact every step; observations,
    reward and controller as the fixture (tolerances of the module docstring)."""
    from gym_flock.envs.flocking.flocking_relative import FlockingRelativeEnv
    f = np.load(os.path.join(GOLDEN, "flock_n10_episode.npz"))
    env = FlockingRelativeEnv()
    env.n_agents = 10
    env._make_spaces()
    env.fetch_mode = mode
    env.x = f["x0"]
    env.compute_helpers()
    close_sv(env.state_values, f["sv0"])
    np.testing.assert_array_equal(env.state_network, f["net0"].astype(np.float32))
    for t in range(40):
        if not f["u_is_f32"][t]:
            got = env.controller()
            np.testing.assert_allclose(got, f["u"][t], rtol=1e-9, atol=1e-12)
            if t > 0 and mode == "direct":
                assert env._ctrl_cache is not None  # the fused result, no extra launch
            np.testing.assert_array_equal(env.controller(), got)  # same state, same answer
            u = f["u"][t]
        else:
            u = f["u"][t].astype(np.float32)
        (sv, net), r, done, info = env.step(u)
        assert not done and info == {}
        np.testing.assert_array_equal(env.x, f["x"][t])
        close_sv(sv, f["sv"][t])
        np.testing.assert_array_equal(net, f["net"][t].astype(np.float32))
        np.testing.assert_allclose(r, f["reward"][t], rtol=1e-12)
        if mode == "direct" and t >= 1:
            np.testing.assert_allclose(env._ctrl_cache, f["ctrl"][t], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(env.controller(), f["ctrl"][t], rtol=1e-9, atol=1e-12)
    # the arrays a step returned stay valid after later steps (fresh arrays per call)
    (sv_a, net_a), _, _, _ = env.step(np.zeros((10, 2), np.float32))
    keep = (sv_a.copy(), net_a.copy())
    env.step(np.ones((10, 2), np.float32))
    np.testing.assert_array_equal(sv_a, keep[0])
    np.testing.assert_array_equal(net_a, keep[1])
    env.close()


@pytest.mark.parametrize("n,f64", [(384, False), (385, False), (192, True), (193, True), (600, False)])
def test_dropin_inline_actions_boundaries(n, f64):
    """fe_step_host passes one env's actions in the kernel arguments up to 3 KiB (N <= 384
    float32, 192 float64) and an env of one tile; past either bound the kernel reads
    them in place from page-locked memory. Both sides of each bound agree with the batched
    path: state and network bit for bit; state_values, reward and the expert action within
    the module's tolerances (the direct step fuses the controller, whose instantiation
    takes the IEEE division for its pair terms)."""
    from gym_flock.envs.flocking.flocking_relative import FlockingRelativeEnv
    from gym_flock.init_states import synthetic_state
    envs = []
    for mode in ("direct", "pooled"):
        env = FlockingRelativeEnv()
        env.n_agents = n
        env._make_spaces()
        env.fetch_mode = mode
        env.x = synthetic_state(n, 3)
        env.compute_helpers()
        env.controller()  # later steps fuse the expert action (direct mode)
        envs.append(env)
    rs = np.random.RandomState(11)
    for t in range(4):
        u = rs.uniform(-1, 1, size=(n, 2))
        u = u if f64 else u.astype(np.float32)
        out = [env.step(u) for env in envs]
        (sv0, net0), r0 = out[0][0], out[0][1]
        (sv1, net1), r1 = out[1][0], out[1][1]
        np.testing.assert_array_equal(envs[0].x, envs[1].x)
        np.testing.assert_array_equal(net0, net1)
        close_sv(sv0, sv1)
        np.testing.assert_allclose(r0, r1, rtol=1e-12)
        np.testing.assert_allclose(envs[0].controller(), envs[1].controller(), rtol=1e-9, atol=1e-12)
    for env in envs:
        env.close()


def test_step_host_pageable_and_pinned_destinations():
    """fe_step_host with pageable destinations (device buffers, copied after the launch)
    and with page-locked ones (written by the kernel through their mapped addresses)
    equals the device-buffer step. After a page-locked step the device observation
    getters refuse (their buffers were not written) while rewards and state stay
    readable; a device step makes them readable again."""
    B, N = 2, 40
    x0 = synthetic_batch(B, N, seed0=9)
    u = np.random.RandomState(4).uniform(-1, 1, size=(B, N, 2))
    ha, hb = nat.FlockHandle(N, B), nat.FlockHandle(N, B)
    ha.set_state(x0)
    hb.set_state(x0)
    ha.step(u, nat.FE_WITH_CONTROLLER)
    sv = np.empty((B, N, 6), np.float32)
    net = np.empty((B, N, N), np.float32)
    rw = np.empty(B)
    ct = np.empty((B, N, 2))
    hb.step_host(u.ctypes.data, True, sv.ctypes.data, net.ctypes.data, rw.ctypes.data, ct.ctypes.data)
    np.testing.assert_array_equal(hb.get_state(), ha.get_state())
    np.testing.assert_array_equal(sv, ha.state_values())
    np.testing.assert_array_equal(net, ha.network())
    np.testing.assert_array_equal(rw, ha.rewards())
    np.testing.assert_array_equal(ct, ha.controls())
    np.testing.assert_array_equal(hb.network(), net)  # pageable: the device copy is current
    # page-locked actions and destinations: read and written in place by the kernel
    pu = nat.PinnedArray((B, N, 2), np.float64)
    pu.a[...] = u
    ps = [nat.PinnedArray(shape, dt) for shape, dt in (((B, N, 6), np.float32), ((B, N, N), np.float32),
                                                        ((B,), np.float64), ((B, N, 2), np.float64))]
    ha.step(u, nat.FE_WITH_CONTROLLER)
    hb.step_host(pu.addr, True, *[p.addr for p in ps])
    np.testing.assert_array_equal(hb.get_state(), ha.get_state())
    for p, want in zip(ps, (ha.state_values(), ha.network(), ha.rewards(), ha.controls())):
        np.testing.assert_array_equal(p.a, want)
    np.testing.assert_array_equal(hb.rewards(), ha.rewards())
    with pytest.raises(nat.GymFlockError) as e:
        hb.network()
    assert e.value.code == nat.GF_ESTATE
    hb.step(u, 0)  # a device step makes them readable again
    ha.step(u, 0)
    np.testing.assert_array_equal(hb.network(), ha.network())
    for p in ps + [pu]:
        p.close()
    ha.close()
    hb.close()


@pytest.mark.parametrize("n", [7, 10, 63, 100, 130, 1000, 1030, 2049])
def test_sizes_vs_oracle(n):
    """Ragged N (scalar network path when N % 4 != 0, partial ballot words, several LDS
    tiles above 1024) on a batch of 3 envs."""
    B = 3
    x0 = synthetic_batch(B, n, seed0=100 + n)
    u = np.random.RandomState(n).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B, n_neighbors=7 if n >= 7 else 0)
    h.set_state(x0)
    h.step(u, nat.FE_WITH_CONTROLLER | (nat.FE_WITH_KNN if n >= 7 else 0))
    for b in range(B):
        ref = check_against_oracle(h, x0[b], u[b], b)
        if n >= 7:
            idx, obs = h.knn(b)
            ridx, robs = orc.knn_observation(ref["x"])
            np.testing.assert_array_equal(idx, ridx)
            np.testing.assert_array_equal(obs, robs.astype(np.float32))
    h.close()


def test_n1_and_isolated_agents():
    """Edge cases: one agent (no pairs), and a sparse swarm with isolated agents
    (deg 0 -> network row of zeros, state_values 0)."""
    h = nat.FlockHandle(1, 2)
    x0 = np.array([[[0.1, 0.2, 1.0, -1.0]], [[0.0, 0.0, 0.0, 0.0]]])
    u = np.zeros((2, 1, 2), np.float32)
    h.set_state(x0)
    h.step(u, nat.FE_WITH_CONTROLLER)
    for b in range(2):
        check_against_oracle(h, x0[b], u[b], b)
    h.close()
    rs = np.random.RandomState(5)
    x = np.zeros((1, 50, 4))
    x[0, :, :2] = rs.uniform(-20, 20, size=(50, 2))
    x[0, :, 2:] = rs.uniform(-1, 1, size=(50, 2))
    h = nat.FlockHandle(50, 1)
    h.set_state(x)
    u = rs.uniform(-1, 1, size=(1, 50, 2)).astype(np.float32)
    h.step(u, nat.FE_WITH_CONTROLLER)
    ref = check_against_oracle(h, x[0], u[0])
    assert (ref["deg"] == 0).any()
    h.close()


def test_noncentralized_and_sum_pooling():
    n, B = 200, 2
    x0 = synthetic_batch(B, n, seed0=42)
    u = np.random.RandomState(1).uniform(-1, 1, size=(B, n, 2))  # float64 actions
    h = nat.FlockHandle(n, B, mean_pooling=False, centralized=False)
    h.set_state(x0)
    h.step(u, nat.FE_WITH_CONTROLLER)
    for b in range(B):
        ref = orc.step(x0[b], u[b], mean_pooling=False, with_controller=True, centralized=False)
        np.testing.assert_array_equal(h.get_state(b), ref["x"])
        np.testing.assert_array_equal(h.network(b), ref["network"].astype(np.float32))
        close_sv(h.state_values(b), ref["state_values"])
        np.testing.assert_allclose(h.controls(b), ref["ctrl"], rtol=1e-9, atol=1e-12)
    h.close()


def test_closed_loop_expert_matches_oracle_rollout():
    """FE_U_EXPERT feeds the fused controller output back as the next action (the
    reference's env.step(env.controller()) loop): 30 steps against the oracle, the
    oracle consuming the engine's own actions so both follow one trajectory."""
    n, B = 64, 2
    x = synthetic_batch(B, n, seed0=9)
    h = nat.FlockHandle(n, B)
    h.set_state(x)
    h.compute_helpers(nat.FE_WITH_CONTROLLER)
    for t in range(30):
        u = h.controls()
        for b in range(B):
            np.testing.assert_allclose(u[b], orc.controller(x[b]), rtol=1e-9, atol=1e-12)
        h.step(None, nat.FE_U_EXPERT | nat.FE_WITH_CONTROLLER)
        x = np.stack([orc.integrate(x[b], u[b]) for b in range(B)])
        np.testing.assert_array_equal(h.get_state(), x)
    h.close()


def test_full_config2_properties_and_sampled_parity():
    """Config 2 (N=1024 x 256 envs): size-independent properties on the whole batch
    (row sums of the mean-pooled network, symmetric adjacency, determinism) and
    oracle parity on sampled envs."""
    B, N = 256, 1024
    x0 = synthetic_batch(B, N, seed0=0)
    u = np.random.RandomState(0).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    v = VecFlockingRelative(B, N)
    v.set_state(x0)
    v.step(u, controller=True)
    net = v.network()
    sv = v.state_values()
    rew = v.rewards()
    adj = net > 0
    deg = adj.sum(axis=2)
    rows = net.sum(axis=2, dtype=np.float64)
    np.testing.assert_allclose(rows[deg > 0], 1.0, rtol=1e-5)
    assert np.all(rows[deg == 0] == 0)
    assert np.array_equal(adj, adj.transpose(0, 2, 1))
    assert not adj[:, np.arange(N), np.arange(N)].any()
    v.set_state(x0)
    v.step(u, controller=True)
    assert np.array_equal(v.network(), net) and np.array_equal(v.state_values(), sv)
    assert np.array_equal(v.rewards(), rew)
    for b in (0, 97, 255):
        check_against_oracle(v.h, x0[b], u[b], b)
    v.close()


def test_env_api_reset_matches_reference_fixture():
    """FlockingRelativeEnv.reset() reproduces the reference's rejection-sampled state
    from the same global seed, with the acceptance test run on the device."""
    import gym_flock

    f = np.load(os.path.join(GOLDEN, "flock_n64_reset.npz"))

    class Cfg:
        def getfloat(self, k):
            return {"comm_radius": 0.9, "v_max": 5.0, "dt": 0.01}[k]

        def getint(self, k):
            return 64

    env = gym_flock.make("FlockingRelative-v0")
    env.params_from_cfg(Cfg())
    np.random.seed(int(f["seed"]))
    sv, net = env.reset()
    np.testing.assert_array_equal(env.x, f["x0"])
    close_sv(sv, f["state_values"])
    np.testing.assert_array_equal(net > 0, adj_from_bits(f["adj_bits"], 64))
    (sv1, net1), r, done, info = env.step(np.zeros((64, 2), np.float32))
    assert done is False and info == {} and isinstance(r, float)
    with pytest.raises(AssertionError):
        env.step(np.zeros((63, 2)))
    u = env.controller()
    assert u.shape == (64, 2) and u.dtype == np.float64
    st = env.get_stats()
    assert set(st) == {"vel_diffs", "min_dists"}
    env.close()


def test_flocking_v0_env_api():
    import gym_flock

    class Cfg:  # params_from_cfg scales r_max by sqrt(N) (:75), so reset() accepts quickly
        def getfloat(self, k):
            return {"comm_radius": 0.9, "v_max": 5.0, "dt": 0.01}[k]

        def getint(self, k):
            return 100

    env = gym_flock.make("Flocking-v0")
    env.params_from_cfg(Cfg())
    np.random.seed(3)
    obs, net = env.reset()
    assert obs.shape == (100, 28) and net.shape == (100, 100)
    x = env.x
    u = np.random.RandomState(2).uniform(-1, 1, size=(100, 2)).astype(np.float32)
    (obs, net), r, done, _ = env.step(u)
    ref = orc.step(x, u)
    ridx, robs = orc.knn_observation(ref["x"])
    np.testing.assert_array_equal(env.nearest, ridx)
    np.testing.assert_array_equal(obs, robs.astype(np.float32))
    env.close()


@pytest.mark.parametrize("n,f64", [(100, False), (300, True)])
def test_flocking_v0_dropin_direct_matches_oracle(n, f64):
    """Flocking-v0's drop-in step in the default fetch mode: one fe_step_host_knn call
    returns the neighbour rows, indices, network and reward of the new state. Against the
    oracle (indices bit-exact, observation rows as float32 of the float64 differences,
    network bit-exact) over several steps, and equal to the pooled mode's getters."""
    from gym_flock.envs.flocking.flocking import FlockingEnv
    from gym_flock.init_states import synthetic_state
    envs = []
    for mode in ("direct", "pooled"):
        env = FlockingEnv()
        env.n_agents = n
        env._make_spaces()
        env.fetch_mode = mode
        env.x = synthetic_state(n, 4)
        env.compute_helpers()
        envs.append(env)
    rs = np.random.RandomState(12)
    for t in range(5):
        x = envs[0].x
        u = rs.uniform(-1, 1, size=(n, 2))
        u = u if f64 else u.astype(np.float32)
        (obs, net), r, done, _ = envs[0].step(u)
        (obs_p, net_p), r_p, _, _ = envs[1].step(u)
        ref = orc.step(x, u)
        ridx, robs = orc.knn_observation(ref["x"])
        np.testing.assert_array_equal(envs[0].x, ref["x"])
        np.testing.assert_array_equal(envs[0].nearest, ridx)
        np.testing.assert_array_equal(obs, robs.astype(np.float32))
        np.testing.assert_array_equal(net, ref["network"].astype(np.float32))
        np.testing.assert_allclose(r, ref["reward"], rtol=1e-12)
        np.testing.assert_array_equal(obs, obs_p)
        np.testing.assert_array_equal(envs[0].nearest, envs[1].nearest)
        np.testing.assert_array_equal(net, net_p)
        assert r == r_p
        np.testing.assert_array_equal(envs[0].get_observation(), obs)  # the fetched rows, no relaunch
    idx, kobs = envs[0]._handle().knn(0)  # fe_get_knn after fe_step_host_knn: the same rows
    np.testing.assert_array_equal(idx, envs[0].nearest)
    np.testing.assert_array_equal(kobs, obs)
    for env in envs:
        env.close()


@pytest.mark.parametrize("n", [10, 100, 300])
def test_flocking_v0_dropin_expert_loop(n):
    """Flocking-v0's expert loop through the env API, `u = env.controller(); env.step(u)`
    for 20 steps (N = 10 and 100: the exact in-step ranking with the actions in the kernel
    arguments; 300: the fused-key ranking with the controller, actions read from
    page-locked memory). After the first controller() call every step computes the next
    expert action in its own launch (fe_step_host_knn_ctrl) and controller() returns it.
    Against the oracle stepped with the same actions: state bit-exact, kNN indices
    bit-exact and observations exact, controller rtol 1e-9, network exact."""
    from gym_flock.envs.flocking.flocking import FlockingEnv
    from gym_flock.init_states import synthetic_state
    env = FlockingEnv()
    env.n_agents = n
    env._make_spaces()
    env.x = synthetic_state(n, 31)
    env.compute_helpers()
    for t in range(20):
        x = env.x
        if t > 0:
            assert env._ctrl_cache is not None  # computed by the previous step's launch
        u = env.controller()
        np.testing.assert_allclose(u, orc.controller(x), rtol=1e-9, atol=1e-12)
        (obs, net), r, done, _ = env.step(u)
        ref = orc.step(x, u, with_controller=True)
        ridx, robs = orc.knn_observation(ref["x"])
        np.testing.assert_array_equal(env.x, ref["x"])
        np.testing.assert_array_equal(env.nearest, ridx)
        np.testing.assert_array_equal(obs, robs.astype(np.float32))
        np.testing.assert_array_equal(net, ref["network"].astype(np.float32))
        np.testing.assert_allclose(r, ref["reward"], rtol=1e-12)
        assert env._ctrl_cache is not None  # fused into the step's launch
        np.testing.assert_allclose(env._ctrl_cache, ref["ctrl"], rtol=1e-9, atol=1e-12)
    env.close()


@pytest.mark.parametrize("mode", ["direct", "pooled"])
def test_flocking_v0_episode_fixture(mode):
    """The reference's recorded N=10 episode (20 expert then 20 float32 random actions)
    through Flocking-v0's env API: the same states and networks, the 7-nearest rows of
    each recorded state, and controller() as recorded."""
    from gym_flock.envs.flocking.flocking import FlockingEnv
    f = np.load(os.path.join(GOLDEN, "flock_n10_episode.npz"))
    env = FlockingEnv()
    env.n_agents = 10
    env._make_spaces()
    env.fetch_mode = mode
    env.x = f["x0"]
    env.compute_helpers()
    for t in range(40):
        if not f["u_is_f32"][t]:
            np.testing.assert_allclose(env.controller(), f["u"][t], rtol=1e-9, atol=1e-12)
            u = f["u"][t]
        else:
            u = f["u"][t].astype(np.float32)
        (obs, net), r, _, _ = env.step(u)
        np.testing.assert_array_equal(env.x, f["x"][t])
        ridx, robs = orc.knn_observation(f["x"][t])
        np.testing.assert_array_equal(env.nearest if mode == "direct" else env._handle().knn(0)[0], ridx)
        np.testing.assert_array_equal(obs, robs.astype(np.float32))
        np.testing.assert_array_equal(net, f["net"][t].astype(np.float32))
        np.testing.assert_allclose(r, f["reward"][t], rtol=1e-12)
        np.testing.assert_allclose(env.controller(), f["ctrl"][t], rtol=1e-9, atol=1e-12)
    env.close()


def _small_knn_cases(n, rs):
    """The nine kNN shapes of _knn_cases rebuilt at a small N (exact in-step ranking at
    N <= 128, the fused-key ranking above): sparse, tied lattices, coincident agents,
    large offsets, dense lattices and swarms, a detached sparse group."""
    w = int(np.ceil(np.sqrt(n)))
    g = np.stack(np.meshgrid(np.arange(w), np.arange(w)), -1).reshape(-1, 2)[:n] * 2.0
    side = np.sqrt(n / 100.0)
    cases = {}
    x = np.zeros((n, 4))
    x[:, :2] = rs.uniform(-12, 12, size=(n, 2)) * side  # dispersed: almost every row below k neighbours
    cases["dispersed"] = x
    x = np.zeros((n, 4))
    x[:, :2] = g[rs.permutation(n)]  # lattice: exact r2 ties everywhere, no neighbours
    cases["lattice"] = x
    x = cases["lattice"].copy()
    x[:, :2] += rs.uniform(-1, 1, size=(n, 2)) * 1e-12
    cases["lattice_jitter"] = x
    x = np.zeros((n, 4))
    x[:, :2] = rs.uniform(-8, 8, size=(n, 2)) * side
    x[10:20, :2] = x[0, :2]  # coincident agents (r2 = 0 ties)
    cases["coincident_ragged"] = x
    x = cases["dispersed"].copy()
    x[:, :2] += 3.0e6
    cases["offset"] = x
    x = np.zeros((n, 4))
    x[:, :2] = g[rs.permutation(n)] * 0.125  # ~20 neighbours each, exact ties
    cases["dense_lattice"] = x
    x = cases["dense_lattice"].copy()
    x[:, :2] += rs.uniform(-1, 1, size=(n, 2)) * 1e-3
    x[:, 2:] = rs.uniform(-1, 1, size=(n, 2))
    cases["dense_jitter"] = x
    x = np.zeros((n, 4))
    x[:, :2] = rs.uniform(-1.8, 1.8, size=(n, 2)) * side
    x[:, 2:] = rs.uniform(-1, 1, size=(n, 2))
    x[50:54, :2] = x[7, :2]
    x[60, :2] = x[61, :2] + np.array([3e-9, 0.0])  # closer than one key step
    cases["dense_random"] = x
    x = cases["dense_random"].copy()
    x[:12, :2] += 30.0 + rs.uniform(-5, 5, size=(12, 2))  # a detached, sparse group
    cases["dense_with_rim"] = x
    return cases


KNN_CASES = ["dispersed", "lattice", "lattice_jitter", "coincident_ragged", "offset", "dense_lattice",
             "dense_jitter", "dense_random", "dense_with_rim"]


@pytest.mark.parametrize("n", [100, 128, 129])
def test_knn_small_env_cases_vs_oracle(n):
    """Flocking-v0 at the reference's default size and around the exact-ranking limit
    (N <= 128: every row ranked exactly in the step from the env's LDS tile; 129: the
    fused-key ranking with inline scans and the rim kernel): the nine kNN shapes, both
    agent orders, k = 7, through the batched step (FE_WITH_KNN, zero actions) and through
    FlockingEnv.step in direct mode (one fe_step_host_knn call). Indices bit-exact,
    observations exact, against the oracle's stable argsort."""
    from gym_flock.envs.flocking.flocking import FlockingEnv
    cases = _small_knn_cases(n, np.random.RandomState(2100 + n))
    env = FlockingEnv()
    env.n_agents = n
    env._make_spaces()
    for case in KNN_CASES:
        x0 = cases[case]
        xb = np.stack([x0, x0[::-1].copy()])
        h = nat.FlockHandle(n, 2, n_neighbors=7)
        h.set_state(xb)
        u0 = np.zeros((2, n, 2), np.float32)
        h.step(u0, nat.FE_WITH_KNN)
        for b in range(2):
            x1 = h.get_state(b)
            np.testing.assert_array_equal(x1, orc.integrate(xb[b], u0[b]), err_msg=case)
            idx, obs = h.knn(b)
            ridx, robs = orc.knn_observation(x1, 7)
            np.testing.assert_array_equal(idx, ridx, err_msg=case)
            np.testing.assert_array_equal(obs, robs.astype(np.float32), err_msg=case)
            # the drop-in step from the same state
            env.x = xb[b]
            (eobs, enet), _, _, _ = env.step(np.zeros((n, 2), np.float32))
            np.testing.assert_array_equal(env.nearest, ridx, err_msg=case + " (env)")
            np.testing.assert_array_equal(eobs, robs.astype(np.float32), err_msg=case + " (env)")
        h.close()
    env.close()


@pytest.mark.parametrize("n", [192, 193])
def test_knn_one_env_window_edges_vs_oracle(n):
    """The one-env exact kNN window at its upper edge (kStepExactKnnMaxOneEnv = 192,
    csrc/flock_internal.h): a handle of one env with N = 192 takes the exact in-step
    ranking (the largest KX tile of one env), N = 193 the fused-key ranking with the rim
    kernel. The nine kNN shapes in both agent orders through FlockingEnv.step in direct
    mode (one fe_step_host_knn call), then `u = env.controller(); env.step(u)` with the
    next expert action fused into the step (fe_step_host_knn_ctrl), and through a
    one-env batched handle (FE_WITH_KNN). Indices bit-exact, observations exact, states
    bit-exact, controls rtol 1e-9, against the oracle (flocking.py:20-25)."""
    from gym_flock.envs.flocking.flocking import FlockingEnv
    cases = _small_knn_cases(n, np.random.RandomState(3300 + n))
    env = FlockingEnv()
    env.n_agents = n
    env._make_spaces()
    h = nat.FlockHandle(n, 1, n_neighbors=7)
    for case in KNN_CASES:
        for x0 in (cases[case], cases[case][::-1].copy()):
            u0 = np.zeros((n, 2), np.float32)
            x1 = orc.integrate(x0, u0)
            ridx, robs = orc.knn_observation(x1, 7)
            h.set_state(x0[None])
            h.step(u0[None], nat.FE_WITH_KNN)
            idx, obs = h.knn(0)
            np.testing.assert_array_equal(idx, ridx, err_msg=case + " (handle)")
            np.testing.assert_array_equal(obs, robs.astype(np.float32), err_msg=case + " (handle)")
            env.x = x0
            (eobs, _), _, _, _ = env.step(u0)
            np.testing.assert_array_equal(env.x, x1, err_msg=case)
            np.testing.assert_array_equal(env.nearest, ridx, err_msg=case + " (env)")
            np.testing.assert_array_equal(eobs, robs.astype(np.float32), err_msg=case + " (env)")
            u = env.controller()
            np.testing.assert_allclose(u, orc.controller(x1), rtol=1e-9, atol=1e-12, err_msg=case)
            (eobs, _), _, _, _ = env.step(u)
            ref = orc.step(x1, u, with_controller=True)
            ridx2, robs2 = orc.knn_observation(ref["x"], 7)
            np.testing.assert_array_equal(env.x, ref["x"], err_msg=case + " (fused)")
            np.testing.assert_array_equal(env.nearest, ridx2, err_msg=case + " (fused)")
            np.testing.assert_array_equal(eobs, robs2.astype(np.float32), err_msg=case + " (fused)")
            assert env._ctrl_cache is not None  # made by the step's own launch
            np.testing.assert_allclose(env.controller(), ref["ctrl"], rtol=1e-9, atol=1e-12, err_msg=case)
    h.close()
    env.close()


@pytest.mark.parametrize("n", [100, 128, 129])
def test_knn_small_env_continuous(n):
    """30 continuous Flocking-v0 steps of 4 envs at N around the exact-ranking limit
    (split steps, resident actions, a spread swarm: most rows below k neighbours), the
    state chain bit-exact and indices / observations against the oracle every 3rd step."""
    B = 4
    x0 = synthetic_batch(B, n, seed0=6100 + n)
    x0[:, :, :2] *= 2.0
    u = np.random.RandomState(n).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B, n_neighbors=7)
    h.set_state(x0)
    h.set_actions(u)
    x = x0.copy()
    for t in range(1, 31):
        h.step(None, nat.FE_U_RESIDENT | nat.FE_WITH_KNN)
        x = np.stack([orc.integrate(x[b], u[b]) for b in range(B)])
        if t % 3 == 0:
            np.testing.assert_array_equal(h.get_state(), x)
            idx, obs = h.knn()
            for b in range(B):
                ridx, robs = orc.knn_observation(x[b])
                np.testing.assert_array_equal(idx[b], ridx)
                np.testing.assert_array_equal(obs[b], robs.astype(np.float32))
    h.close()


def test_params_change_mid_episode_keeps_state():
    """Changing centralized, comm_radius, dt, action_scalar or mean_pooling between steps
    keeps the episode's state (the reference reads them at call time, :200-201): each
    step and controller() against the oracle with the parameters of that call, the
    state chain bit-exact. Flocking-v0 too (its kNN under the new radius)."""
    from gym_flock.envs.flocking.flocking import FlockingEnv
    from gym_flock.envs.flocking.flocking_relative import FlockingRelativeEnv
    from gym_flock.init_states import synthetic_state
    n = 100
    rs = np.random.RandomState(77)
    plan = [dict(), dict(centralized=False), dict(comm_radius=1.2), dict(dt=0.02),
            dict(mean_pooling=False), dict(action_scalar=5.0), dict(centralized=True, comm_radius=0.9)]
    for cls in (FlockingRelativeEnv, FlockingEnv):
        env = cls()
        env.n_agents = n
        env._make_spaces()
        env.x = synthetic_state(n, 5)
        env.compute_helpers()
        env.controller()  # the expert action is fused from here on
        for change in plan:
            for k, v in change.items():
                setattr(env, k, v)
            p = dict(comm_radius=env.comm_radius, dt=env.dt, action_scalar=env.action_scalar,
                     mean_pooling=env.mean_pooling)
            x = env.x
            np.testing.assert_allclose(env.controller(), orc.controller(x, p["comm_radius"], p["action_scalar"],
                                                                       env.centralized), rtol=1e-9, atol=1e-12)
            u = rs.uniform(-1, 1, size=(n, 2)).astype(np.float32)
            (o, net), r, _, _ = env.step(u)
            ref = orc.step(x, u, with_controller=True, centralized=env.centralized, **p)
            np.testing.assert_array_equal(env.x, ref["x"])
            np.testing.assert_array_equal(net, ref["network"].astype(np.float32))
            np.testing.assert_allclose(r, ref["reward"], rtol=1e-12)
            np.testing.assert_allclose(env.controller(), ref["ctrl"], rtol=1e-9, atol=1e-12)
            np.testing.assert_allclose(env.controller(centralized=not env.centralized),
                                       orc.step(x, u, with_controller=True, centralized=not env.centralized,
                                                **p)["ctrl"], rtol=1e-9, atol=1e-12)
            if cls is FlockingEnv:
                ridx, robs = orc.knn_observation(ref["x"])
                np.testing.assert_array_equal(env.nearest, ridx)
                np.testing.assert_array_equal(o, robs.astype(np.float32))
        env.close()


def test_float16_actions_take_float32_arithmetic():
    """float16 actions are computed as float32 actions of the same values (the kernels have
    float32 and float64 arithmetic; the reference's float16 rounding is parity unpinned)."""
    from gym_flock.envs.flocking.flocking_relative import FlockingRelativeEnv
    from gym_flock.init_states import synthetic_state
    n = 64
    x0 = synthetic_state(n, 9)
    u16 = np.random.RandomState(9).uniform(-1, 1, size=(n, 2)).astype(np.float16)
    outs = []
    for u in (u16, u16.astype(np.float32)):
        env = FlockingRelativeEnv()
        env.n_agents = n
        env._make_spaces()
        env.x = x0
        (sv, net), r, _, _ = env.step(u)
        outs.append((env.x, sv.copy(), net.copy(), r))
        env.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(outs[0][0], orc.step(x0, u16.astype(np.float32))["x"])


def test_config5_size_sampled_rows():
    """N=8192 (BASELINE.json configs[4]'s agent count; 16-row blocks, 16 LDS tiles per
    row sweep): the whole state and reward, and 40 sampled rows of the network,
    state_values and controller (first/last rows, tile and block edges, random rows)
    against the oracle restricted to those rows."""
    n, B = 8192, 2
    x0 = synthetic_batch(B, n, seed0=8192)
    u = np.random.RandomState(81).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    rs = np.random.RandomState(82)
    rows = np.unique(np.concatenate([[0, 1, 15, 16, 511, 512, 4095, 4096, 8190, 8191],
                                     rs.choice(n, 30, replace=False)]))
    h = nat.FlockHandle(n, B)
    h.set_state(x0)
    h.step(u, nat.FE_WITH_CONTROLLER)
    x1, sv, rew, ctrl = h.get_state(), h.state_values(), h.rewards(), h.controls()
    for b in range(B):
        ref = orc.step_rows(x0[b], u[b], rows, with_controller=True)
        np.testing.assert_array_equal(x1[b], ref["x"])
        np.testing.assert_allclose(rew[b], ref["reward"], rtol=1e-12)
        for k, r in enumerate(rows):
            net = h.network_rows(b, int(r), 1)[0]
            np.testing.assert_array_equal(net, ref["network"][k].astype(np.float32))
        close_sv(sv[b][rows], ref["state_values"])
        np.testing.assert_allclose(ctrl[b][rows], ref["ctrl"], rtol=1e-9, atol=1e-12)
    h.close()


@pytest.mark.parametrize("B", [3, 5, 8])
def test_split_steps_match_single_stream(B):
    """Two half-batch launches per step on two streams (the default) give the same bits
    as one launch per step, over resident, host and closed-loop steps mixed with
    getters, kNN and packed outputs (the join / ordering rules of fe_set_streams), and
    back-to-back fused kNN steps (de-phased first split step, rim kNN per half)."""
    n = 300
    x0 = synthetic_batch(B, n, seed0=3000)
    rs = np.random.RandomState(3001)
    us = [rs.uniform(-1, 1, size=(B, n, 2)).astype(np.float32) for _ in range(6)]
    outs = []
    for streams in (2, 1):
        h = nat.FlockHandle(n, B, n_neighbors=7)
        h.set_streams(streams)
        h.set_state(x0)
        h.set_actions(us[0])
        got = []
        for _ in range(4):  # back-to-back resident steps (split when streams == 2)
            h.step(None, nat.FE_U_RESIDENT)
        got += [h.get_state(), h.network(), h.rewards()]
        h.step(us[1], nat.FE_WITH_CONTROLLER | nat.FE_WITH_KNN)  # host actions, kNN
        got += [h.knn()[0], h.state_values(), h.controls()]
        for _ in range(3):  # closed loop on the device
            h.step(None, nat.FE_U_EXPERT | nat.FE_WITH_CONTROLLER)
        got += [h.controls()]
        h.step(us[2], nat.FE_PACKED_NETWORK)
        got += [h.get_state(), h.network_packed()[0], h.rewards()]
        h.set_actions(us[3])
        for _ in range(5):  # back-to-back Flocking-v0 steps
            h.step(None, nat.FE_U_RESIDENT | nat.FE_WITH_KNN)
        idx, obs = h.knn()
        got += [h.get_state(), idx, obs, h.rewards()]
        outs.append(got)
        h.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def test_network_store_loops():
    """Both forms of the network store loop write the oracle's rows: at N % 1024 == 0 the
    plain step uses the generic nibble select and the step + controller the fast
    bit-extract form (capi.hip store_fast)."""
    n, B = 1024, 2
    x0 = synthetic_batch(B, n, seed0=77)
    u = np.random.RandomState(78).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    for ctrl in (False, True):
        h = nat.FlockHandle(n, B)
        h.set_state(x0)
        h.step(u, nat.FE_WITH_CONTROLLER if ctrl else 0)
        for b in range(B):
            check_against_oracle(h, x0[b], u[b], b, ctrl=ctrl)
        h.close()


@pytest.mark.parametrize("n", [100, 1030])
def test_packed_network_vs_oracle(n):
    """FE_PACKED_NETWORK: adjacency bits and degrees (the packed output mode) match the
    oracle bit for bit, alone or next to the dense rows."""
    from gym_flock.vec import VecFlockingRelative
    B = 3
    x0 = synthetic_batch(B, n, seed0=500 + n)
    u = np.random.RandomState(n).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    v = VecFlockingRelative(B, n)
    for mode in ("both", "packed"):
        v.reset(x=x0)
        v.step(u, network=mode)
        bits, deg = v.network_packed()
        assert bits.shape == (B, n, (n + 63) // 64) and bits.dtype == np.uint64
        for b in range(B):
            ref = orc.step(x0[b], u[b])
            adj = np.unpackbits(bits[b].view(np.uint8), axis=1, bitorder="little")[:, :n].astype(bool)
            np.testing.assert_array_equal(adj, ref["adj"])
            np.testing.assert_array_equal(deg[b], ref["deg"])
            np.testing.assert_array_equal(v.get_state()[b], ref["x"])
            close_sv(v.state_values(b), ref["state_values"])
            if mode == "both":
                np.testing.assert_array_equal(v.network(b), ref["network"].astype(np.float32))
    v.close()


def test_reset_synthetic_matches_numpy_draws():
    """fe_reset_synthetic reproduces synthetic_batch (NumPy RandomState(seed + b)):
    velocities bit-exact (same uniforms), positions to the last ulp of cos/sin."""
    B, n = 4, 300
    h = nat.FlockHandle(n, B)
    h.reset_synthetic(seed=17)
    ref = synthetic_batch(B, n, seed0=17)
    x = h.get_state()
    np.testing.assert_array_equal(x[..., 2:], ref[..., 2:])
    np.testing.assert_allclose(x[..., :2], ref[..., :2], rtol=4e-16, atol=1e-300)
    h.close()


def test_degenerate_states_match_oracle():
    """Edge states: coincident agents (r2 = 0: the reference's 0/0 features are NaN),
    agents exactly on the comm-radius boundary, coordinates above the float32
    prefilter's range (every pair decided in float64), and a non-finite agent."""
    n = 40
    rs = np.random.RandomState(9)
    base = rs.uniform(-2, 2, size=(n, 4))
    cases = []
    x = base.copy()
    x[1, :2] = x[0, :2]  # coincident pair
    cases.append(x)
    x = base.copy()
    x[:, 1] = 0.0
    x[:, 0] = np.arange(n) * 0.9  # neighbours exactly 0.9 apart: r2 = 0.81 is not < 0.81
    cases.append(x)
    x = base.copy()
    x[:, :2] += 3.0e5  # |coordinates| beyond the float32 band's validity
    cases.append(x)
    x = base.copy()
    x[5, 0] = np.inf
    cases.append(x)
    for x0 in cases:
        u = rs.uniform(-1, 1, size=(n, 2)).astype(np.float32)
        h = nat.FlockHandle(n, 1)
        h.set_state(x0[None])
        h.step(u[None], nat.FE_WITH_CONTROLLER)
        with np.errstate(all="ignore"):
            ref = orc.step(x0, u, with_controller=True)
        np.testing.assert_array_equal(h.get_state(0), ref["x"])
        np.testing.assert_array_equal(h.network(0) > 0, ref["adj"])
        sv = h.state_values(0)
        np.testing.assert_array_equal(np.isnan(sv), np.isnan(ref["state_values"].astype(np.float32)))
        ok = ~np.isnan(ref["state_values"])
        np.testing.assert_allclose(sv[ok], ref["state_values"][ok], rtol=1e-5, atol=1e-9)
        h.close()


def _knn_cases():
    rs = np.random.RandomState(21)
    cases = {}
    n = 1024
    x = np.zeros((n, 4))
    x[:, :2] = rs.uniform(-60, 60, size=(n, 2))  # dispersed: almost every agent below k neighbours
    cases["dispersed"] = x
    g = np.stack(np.meshgrid(np.arange(32), np.arange(32)), -1).reshape(-1, 2) * 2.0
    x = np.zeros((n, 4))
    x[:, :2] = g[rs.permutation(n)]  # lattice: exact r2 ties everywhere, no neighbours
    cases["lattice"] = x
    x = cases["lattice"].copy()
    x[:, :2] += rs.uniform(-1, 1, size=(n, 2)) * 1e-12  # ties broken below float32 resolution
    cases["lattice_jitter"] = x
    x = np.zeros((1000, 4))
    x[:, :2] = rs.uniform(-40, 40, size=(1000, 2))
    x[10:20, :2] = x[0, :2]  # coincident agents (r2 = 0 ties); N not a multiple of 2k
    cases["coincident_ragged"] = x
    x = cases["dispersed"].copy()
    x[:, :2] += 3.0e6  # large coordinates: the float32 margin is wide (candidate overflow path)
    cases["offset"] = x
    # dense states (k = 7: the step's fused selection ranks the rows it can)
    x = np.zeros((n, 4))
    x[:, :2] = g[rs.permutation(n)] * 0.125  # ~20 neighbours each, exact r2 ties: equal keys
    cases["dense_lattice"] = x
    x = cases["dense_lattice"].copy()
    x[:, :2] += rs.uniform(-1, 1, size=(n, 2)) * 1e-3  # ties broken: fused ranking, a few rim rows
    x[:, 2:] = rs.uniform(-1, 1, size=(n, 2))
    cases["dense_jitter"] = x
    x = np.zeros((n, 4))
    x[:, :2] = rs.uniform(-2.5, 2.5, size=(n, 2))
    x[:, 2:] = rs.uniform(-1, 1, size=(n, 2))
    x[100:104, :2] = x[7, :2]  # coincident agents inside a dense swarm (r2 = 0 ties)
    x[500, :2] = x[501, :2] + np.array([3e-9, 0.0])  # keys differ by less than the q step
    cases["dense_random"] = x
    x = cases["dense_random"].copy()
    x[:40, :2] += 30.0  # a detached, sparse group: rows below k neighbours in a dense env
    x[:40, :2] += rs.uniform(-5, 5, size=(40, 2))
    cases["dense_with_rim"] = x
    return cases


@pytest.mark.parametrize("k", [1, 7, 16])
@pytest.mark.parametrize("case", ["dispersed", "lattice", "lattice_jitter", "coincident_ragged", "offset",
                                  "dense_lattice", "dense_jitter", "dense_random", "dense_with_rim"])
def test_knn_full_scan_rows_vs_oracle(case, k):
    """Flocking-v0 observation, indices bit-exact vs the oracle's stable argsort (ties to
    the lower index) and observations exact. Sparse states: (nearly) every agent has
    fewer than k neighbours, so each row is a full scan (bounded two-pass scan: float32
    group-minimum bound, candidate list, exact float64 ranking). Dense states (k = 7):
    the step's fused selection ranks rows whose k + 1 nearest keys are distinct, and
    the rim kNN the rows with exact ties, near-equal keys or too few neighbours."""
    x0 = _knn_cases()[case]
    n = x0.shape[0]
    xb = np.stack([x0, x0[::-1].copy()])  # second env: reversed agent order (other tie winners)
    h = nat.FlockHandle(n, 2, n_neighbors=k)
    h.set_state(xb)
    u0 = np.zeros((2, n, 2), np.float32)
    h.step(u0, nat.FE_WITH_KNN)
    for b in range(2):
        x1 = h.get_state(b)
        np.testing.assert_array_equal(x1, orc.integrate(xb[b], u0[b]))
        idx, obs = h.knn(b)
        ridx, robs = orc.knn_observation(x1, k)
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_array_equal(obs, robs.astype(np.float32))
    h.close()


def test_knn_pipelined_back_to_back():
    """Flocking-v0 steps issued back to back: each step's kNN runs on its own stream
    beside the next step, with double-buffered adjacency bits. The state chain stays
    bit-exact, and the kNN outputs read after 1, 2, 3 ... pipelined steps (and after a
    packed-output step in between) equal the oracle's on that step's state."""
    n, B = 300, 6
    x0 = synthetic_batch(B, n, seed0=4242)
    rs = np.random.RandomState(4243)
    u = rs.uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B, n_neighbors=7)
    h.set_state(x0)
    h.set_actions(u)
    x = x0.copy()
    for burst in (1, 2, 3, 5):
        for s in range(burst):
            flags = nat.FE_U_RESIDENT | nat.FE_WITH_KNN
            if burst == 3 and s == 1:  # a packed-output step writes the other bits buffer
                flags |= nat.FE_PACKED_NETWORK
            h.step(None, flags)
            x = np.stack([orc.step(x[b], u[b], with_controller=False)["x"] for b in range(B)])
        np.testing.assert_array_equal(h.get_state(), x)
        idx, obs = h.knn()
        for b in range(B):
            ridx, robs = orc.knn_observation(x[b])
            np.testing.assert_array_equal(idx[b], ridx)
            np.testing.assert_array_equal(obs[b], robs.astype(np.float32))
    h.close()


@pytest.mark.parametrize("spread", [1.0, 2.5])
def test_knn_radius_history_continuous(spread):
    """Flocking-v0 over 30 continuous steps (split steps, resident actions): from the
    third step on, the fused step ranks the rows whose k-th nearest two states back lay
    beyond 0.8 comm_radius against candidates within 1.5x that distance, and leaves the
    rest of the sparse rows to the rim kNN. spread 2.5: a swarm 2.5x wider (most agents
    below 7 neighbours). Indices bit-exact and observations exact against the oracle
    every third step, and the state chain bit-exact."""
    n, B = 300, 4
    x0 = synthetic_batch(B, n, seed0=77)
    x0[:, :, :2] *= spread
    rs = np.random.RandomState(78)
    u = rs.uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B, n_neighbors=7)
    h.set_state(x0)
    h.set_actions(u)
    x = x0.copy()
    for t in range(1, 31):
        h.step(None, nat.FE_U_RESIDENT | nat.FE_WITH_KNN)
        x = np.stack([orc.integrate(x[b], u[b]) for b in range(B)])
        if t % 3 == 0:
            np.testing.assert_array_equal(h.get_state(), x)
            idx, obs = h.knn()
            for b in range(B):
                ridx, robs = orc.knn_observation(x[b])
                np.testing.assert_array_equal(idx[b], ridx)
                np.testing.assert_array_equal(obs[b], robs.astype(np.float32))
    h.close()


@pytest.mark.parametrize("n,per_wave", [(256, 1), (256, 2), (256, 3), (256, 8), (128, 3), (128, 8), (129, 3),
                                        (129, 8)])
def test_knn_unranked_rows_inline_and_rim(n, per_wave):
    """Rows the fused step cannot rank (here: outliers 3 comm radii from everyone, with
    no radius history yet) go to the wave's own exact scan when a wave (8 rows at N=256)
    holds at most two of them, and to the rim kNN kernel otherwise. per_wave outliers in
    every 8-row group: 1 and 2 take the inline scan, 3 and 8 the rim kernel (env 1 mixes
    the two: outliers only in its even groups). N=128: the exact in-step ranking takes
    every row; 129: the first size past it. Indices bit-exact and observations exact
    against the oracle for 4 continuous steps (the history then ranks them in the step)."""
    B = 3
    x0 = synthetic_batch(B, n, seed0=91)
    for b in range(B):
        for g in range(n // 8):
            if b == 1 and g % 2:
                continue
            for k in range(per_wave):
                i = 8 * g + k
                ang = 2.399963 * i  # spread on a circle far outside the swarm
                x0[b, i, 0] = (30.0 + 2.7 * i) * np.cos(ang)
                x0[b, i, 1] = (30.0 + 2.7 * i) * np.sin(ang)
    u = np.random.RandomState(92).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B, n_neighbors=7)
    h.set_state(x0)
    h.set_actions(u)
    x = x0.copy()
    for t in range(4):
        h.step(None, nat.FE_U_RESIDENT | nat.FE_WITH_KNN)
        x = np.stack([orc.integrate(x[b], u[b]) for b in range(B)])
        np.testing.assert_array_equal(h.get_state(), x)
        idx, obs = h.knn()
        for b in range(B):
            ridx, robs = orc.knn_observation(x[b])
            np.testing.assert_array_equal(idx[b], ridx)
            np.testing.assert_array_equal(obs[b], robs.astype(np.float32))
    h.close()


@pytest.mark.parametrize("n,layout", [(1024, "line"), (300, "line"), (4096, "grid")])
def test_knn_spatially_indexed_line(n, layout):
    """Agents indexed in spatial order: along a jittered line (spacing 0.1 < comm_radius)
    each row's 8 nearest sit in one feature-pass slice (consecutive columns), which holds
    more than 7 of the row's neighbours and drops the rest. The merge must see that the
    dropped keys may include the row's 8th nearest (needed for the exactness test of the
    7th) and leave the row to the exact scan. "grid": a jittered square lattice indexed
    row-major (spacing 0.3). Indices and observations against the oracle for 3 steps."""
    B = 2
    rs = np.random.RandomState(93)
    x0 = np.zeros((B, n, 4))
    for b in range(B):
        if layout == "line":
            x0[b, :, 0] = 0.1 * np.arange(n) + 1e-9 * rs.standard_normal(n)
            x0[b, :, 1] = 0.02 * np.sin(0.37 * np.arange(n)) * b
        else:
            w = int(np.sqrt(n))
            x0[b, :, 0] = 0.3 * (np.arange(n) % w) + 1e-3 * rs.standard_normal(n)
            x0[b, :, 1] = 0.3 * (np.arange(n) // w) + 1e-3 * rs.standard_normal(n)
        x0[b, :, 2:] = rs.uniform(-0.01, 0.01, size=(n, 2))
    u = rs.uniform(-0.01, 0.01, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B, n_neighbors=7)
    h.set_state(x0)
    h.set_actions(u)
    x = x0.copy()
    for t in range(3):
        h.step(None, nat.FE_U_RESIDENT | nat.FE_WITH_KNN)
        x = np.stack([orc.integrate(x[b], u[b]) for b in range(B)])
        idx, obs = h.knn()
        for b in range(B):
            ridx, robs = orc.knn_observation(x[b])
            np.testing.assert_array_equal(idx[b], ridx)
            np.testing.assert_array_equal(obs[b], robs.astype(np.float32))
    h.close()


def _ordered_layout(kind, n, rs):
    """Agent positions whose indices follow space (users often build swarms that way)."""
    if kind == "disk_by_x":
        p = rs.uniform(-1, 1, size=(4 * n, 2))
        p = p[np.hypot(p[:, 0], p[:, 1]) < 1][:n] * np.sqrt(n) ** 0.5
        return p[np.argsort(p[:, 0], kind="stable")]
    if kind == "clusters":
        c = rs.uniform(-6, 6, size=(8, 2))
        lab = np.sort(rs.randint(0, 8, size=n))
        return c[lab] + 0.25 * rs.standard_normal((n, 2))
    if kind == "zorder":
        p = rs.uniform(0, 4, size=(n, 2)) * np.sqrt(n) / 8
        q = (p / p.max() * 1023).astype(np.int64)
        key = np.zeros(n, np.int64)
        for bit in range(10):
            key |= ((q[:, 0] >> bit) & 1) << (2 * bit) | ((q[:, 1] >> bit) & 1) << (2 * bit + 1)
        return p[np.argsort(key, kind="stable")]
    raise ValueError(kind)


@pytest.mark.parametrize("n", [64, 513, 1024])
@pytest.mark.parametrize("kind", ["disk_by_x", "clusters", "zorder"])
def test_knn_fused_spatial_orders(kind, n):
    """Flocking-v0 on swarms whose agent indices follow space (sorted by x, grouped by
    cluster, Z-order), so a row's nearest crowd into few feature-pass slices: 4
    continuous steps (radius history included), states, adjacency, indices and
    observations against the oracle every step."""
    B = 2
    rs = np.random.RandomState(1000 + n)
    x0 = np.zeros((B, n, 4))
    for b in range(B):
        x0[b, :, :2] = _ordered_layout(kind, n, rs)
        x0[b, :, 2:] = rs.uniform(-1, 1, size=(n, 2))
    u = rs.uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B, n_neighbors=7)
    h.set_state(x0)
    h.set_actions(u)
    x = x0.copy()
    for t in range(4):
        h.step(None, nat.FE_U_RESIDENT | nat.FE_WITH_KNN)
        x = np.stack([orc.integrate(x[b], u[b]) for b in range(B)])
        np.testing.assert_array_equal(h.get_state(), x)
        idx, obs = h.knn()
        net = h.network()
        for b in range(B):
            ridx, robs = orc.knn_observation(x[b])
            np.testing.assert_array_equal(idx[b], ridx)
            np.testing.assert_array_equal(obs[b], robs.astype(np.float32))
            np.testing.assert_array_equal(net[b] > 0, orc.pair_geometry(x[b])[4] < 0.9 * 0.9)
    h.close()


def test_full_config5_batch_sampled_parity():
    """BASELINE.json configs[4] at full size: 32 envs x N=8192 (8.6 GB of network), one
    step with the fused controller. Whole batch: every env's state bit-exact and its
    reward (rtol 1e-12) against the oracle, and the mean-pooled rows of 6 rows per env
    summing to 1. Sampled envs (0, 13, 31): 24 rows each (tile and block edges, random
    rows) of the network bit-exact, state_values and controller against the oracle."""
    n, B = 8192, 32
    x0 = synthetic_batch(B, n, seed0=5)
    u = np.random.RandomState(55).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B)
    h.set_state(x0)
    h.step(u, nat.FE_WITH_CONTROLLER)
    x1, rew, sv, ctrl = h.get_state(), h.rewards(), h.state_values(), h.controls()
    rs = np.random.RandomState(56)
    for b in range(B):
        xo = orc.integrate(x0[b], u[b])
        np.testing.assert_array_equal(x1[b], xo)
        np.testing.assert_allclose(rew[b], orc.reward(xo), rtol=1e-12)
        for r in rs.choice(n, 6, replace=False):
            row = h.network_rows(b, int(r), 1)[0].astype(np.float64)
            assert row.sum() == 0 or abs(row.sum() - 1.0) < 1e-5
    for b in (0, 13, 31):
        rows = np.unique(np.concatenate([[0, 15, 16, 511, 512, 8191], rs.choice(n, 18, replace=False)]))
        ref = orc.step_rows(x0[b], u[b], rows, with_controller=True)
        for k, r in enumerate(rows):
            np.testing.assert_array_equal(h.network_rows(b, int(r), 1)[0], ref["network"][k].astype(np.float32))
        close_sv(sv[b][rows], ref["state_values"])
        np.testing.assert_allclose(ctrl[b][rows], ref["ctrl"], rtol=1e-9, atol=1e-12)
    h.close()


def test_knn_bench_workload_long_run():
    """The bench's Flocking-v0 line at full size (BASELINE.json configs[1]: 256 envs x
    N=1024, the bench's synthetic init and resident random actions, split steps) for 220
    continuous steps, over which the swarm spreads until every agent is sparse (rows
    ranked from the radius history, the inline scan and the rim kernel all take part).
    Whole batch: the state chain bit-exact against the oracle; every row's 7 indices
    distinct, not the row itself, and in non-decreasing distance. Sampled envs: indices
    bit-exact and observations exact against the oracle at t = 1, 2, 3, 25, 60, 120, 220."""
    n, B = 1024, 256
    env = VecFlockingRelative(B, n, n_neighbors=7)
    x = env.reset(seed=0).copy()
    u = np.random.RandomState(1234).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    env.set_actions(u)
    sampled = (0, 1, 77, 128, 200, 255)
    checks = {1, 2, 3, 25, 60, 120, 220}
    rows = np.arange(n)[:, None]
    for t in range(1, 221):
        env.step(resident=True, knn=True)
        x = np.stack([orc.integrate(x[b], u[b]) for b in range(B)])
        if t not in checks:
            continue
        np.testing.assert_array_equal(env.get_state(), x)
        idx_all, obs_all = env.knn()
        for b in range(B):
            idx, obs = idx_all[b], obs_all[b]
            assert idx.min() >= 0 and idx.max() < n
            assert not (idx == rows).any()
            s = np.sort(idx, axis=1)
            assert not (s[:, 1:] == s[:, :-1]).any()
            d = x[b][idx, :2] - x[b][:, None, :2]
            r2 = (d * d).sum(-1)
            assert (np.diff(r2, axis=1) >= 0).all()
            if b in sampled:
                ridx, robs = orc.knn_observation(x[b])
                np.testing.assert_array_equal(idx, ridx)
                np.testing.assert_array_equal(obs, robs.astype(np.float32))
    env.close()


def test_batched_outputs_match_getters():
    """fe_get_outputs (one call, one sync; into numpy or page-locked pool arrays) returns
    the same state_values, network and rewards as the three getters, per env and for the
    whole batch; the drop-in env's fetch modes give the same step() tuple."""
    import gym_flock
    B, n = 3, 130
    x0 = synthetic_batch(B, n, seed0=77)
    u = np.random.RandomState(78).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B)
    h.set_state(x0)
    h.step(u)
    pool = nat.HostPool(cap_bytes=1 << 20)
    for env in (None, 0, 2):
        for p in (None, pool):
            sv, net, rw = h.outputs(env, pool=p)
            np.testing.assert_array_equal(sv, h.state_values(env))
            np.testing.assert_array_equal(net, h.network(env))
            np.testing.assert_array_equal(rw, h.rewards())
    h.close()
    outs = []
    for mode in ("getters", "batched", "pooled"):
        e = gym_flock.make("FlockingRelative-v0")
        e.n_agents = n
        e._make_spaces()
        e.fetch_mode = mode
        e.x = x0[0]
        (sv, net), r, _, _ = e.step(u[0])
        outs.append((sv, net, r))
        e.close()
    for sv, net, r in outs[1:]:
        np.testing.assert_array_equal(sv, outs[0][0])
        np.testing.assert_array_equal(net, outs[0][1])
        assert r == outs[0][2]


def test_host_pool_recycles_and_caps():
    """The drop-in env's page-locked output pool: distinct buffers while arrays live, a
    buffer comes back only once the array and every view of it are released, and past
    the cap arrays are ordinary numpy memory."""
    import gc
    pool = nat.HostPool(cap_bytes=3 * 4096)
    a = pool.array((1024,), np.float32)
    b = pool.array((1024,), np.float32)
    assert a.ctypes.data != b.ctypes.data and pool.live == 2 * 4096
    pa = a.ctypes.data
    del a
    gc.collect()
    c = pool.array((1024,), np.float32)
    assert c.ctypes.data == pa
    d = pool.array((1024,), np.float32)
    e = pool.array((1024,), np.float32)  # over the cap: plain numpy
    assert pool.live == 3 * 4096 and e.flags["OWNDATA"]
    view = b[10:20]
    pb = b.ctypes.data
    del b
    gc.collect()
    assert pool.live == 3 * 4096  # the view keeps b's buffer
    del view
    gc.collect()
    assert pool.live == 2 * 4096
    f = pool.array((1024,), np.float32)
    assert f.ctypes.data == pb
    f[:] = 1.0
    del c, d, e, f
    gc.collect()
    assert pool.live == 0
    pool.trim()


def test_stats_summary_matches_oracle():
    """fe_stats_summary: per-env np.mean of get_stats' two arrays (flocking_relative.py:
    136-143), taken on the device for every env of the batch (the metrics path's payload)."""
    B, N = 5, 200
    h = nat.FlockHandle(N, B)
    x0 = synthetic_batch(B, N)
    h.set_state(x0)
    u = np.random.RandomState(3).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    h.step(u, 0)
    summ = h.stats_summary()
    assert summ.shape == (B, 2)
    for b in range(B):
        st = orc.stats(h.get_state(b))
        np.testing.assert_allclose(summ[b], [st["vel_diffs"].mean(), st["min_dists"].mean()], rtol=1e-13)
        vd, md, _ = h.stats(b)  # the same device arrays the summary reduces
        np.testing.assert_allclose(summ[b], [vd.mean(), md.mean()], rtol=1e-13)


def test_allgather_stats_one_rank_equals_local_summary():
    """The RCCL all-gather of the stats summaries (fe_allgather_stats) at one rank: the
    gathered (1, B, 2) block is the local summary, bit for bit, and stays valid while the
    next steps run; before any all-gather the getter refuses."""
    B, N = 6, 128
    h = nat.FlockHandle(N, B)
    h.set_state(synthetic_batch(B, N))
    u = np.random.RandomState(5).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    h.comm_init(1, 0, nat.FlockHandle.comm_unique_id(), timeout=60.0)
    with pytest.raises(nat.GymFlockError):
        h.gathered_stats()
    for _ in range(3):
        h.step(u, 0)
    h.allgather_stats()
    want = h.stats_summary()
    got = h.gathered_stats()
    assert got.shape == (1, B, 2)
    np.testing.assert_array_equal(got[0], want)
    h.step(u, 0)  # a new summary waits for the pending gather before overwriting its source
    h.allgather_stats()
    np.testing.assert_array_equal(h.gathered_stats()[0], h.stats_summary())


@pytest.mark.parametrize("n", [100, 300])
def test_step_host_flag_and_stream_waits_agree(n):
    """fe_step_host_knn_ctrl into page-locked destinations (written by the kernels in place;
    the host waits for the last kernel's completion flag: the step's at N=100, the rim
    kNN's at N=300) and into pageable numpy arrays (copies after the launches; the host
    waits for the stream), on two handles from the same state and actions: every output
    equal at each of 300 steps, and the first step's against the oracle."""
    B, K = 1, 7
    hs = [nat.FlockHandle(n, B, n_neighbors=K) for _ in range(2)]
    x0 = synthetic_batch(B, n, seed0=21)
    for h in hs:
        h.set_state(x0)
    pool = nat.host_pool()
    shapes = dict(sv=((B, n, 6), np.float32), net=((B, n, n), np.float32), rew=((B,), np.float64),
                  ctrl=((B, n, 2), np.float64), idx=((B, n, K), np.int32), obs=((B, n, 4 * K), np.float32))
    pinned = {k: pool.array(*v) for k, v in shapes.items()}
    plain = {k: np.empty(*v) for k, v in shapes.items()}
    rs = np.random.RandomState(3)
    for t in range(300):
        u = rs.uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
        for h, o in ((hs[0], pinned), (hs[1], plain)):
            h.step_host_knn(u.ctypes.data, False, o["sv"].ctypes.data, o["net"].ctypes.data, o["rew"].ctypes.data,
                            o["idx"].ctypes.data, o["obs"].ctypes.data, ctrl=o["ctrl"].ctypes.data)
        for k in shapes:
            np.testing.assert_array_equal(pinned[k], plain[k], err_msg="%s at step %d" % (k, t))
        if t == 0:
            want = orc.step(x0[0], u[0])
            np.testing.assert_array_equal(pinned["net"][0], np.asarray(want["network"], np.float32))
            np.testing.assert_array_equal(pinned["idx"][0], orc.knn_observation(want["x"], K)[0])
    for h in hs:
        h.close()

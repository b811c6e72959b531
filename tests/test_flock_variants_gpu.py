"""Parity of the flocking variants on the HIP step kernel
with the reference's recorded episodes (tests/golden/variant_*.npz) and the variant
oracle. States are compared bit-exactly; float32 observations within rtol 1e-5; the
controller within rtol 1e-9 (its centralised sums are reordered). Needs an MI355X."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import flocking as fo
from oracle import flocking_variants as fv

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")
from gym_flock.envs import flocking as envs  # noqa: E402
from gym_flock.vec import VARIANTS, VecFlockingRelative  # noqa: E402


class Cfg:
    def __init__(self, n):
        self.n = n

    def getfloat(self, k):
        return {"comm_radius": 0.9, "v_max": 5.0, "dt": 0.01}[k]

    def getint(self, k):
        return self.n


def adj_from_bits(bits, n):
    return np.unpackbits(bits, axis=1, count=n).astype(bool)


def close_sv(ours, ref):
    np.testing.assert_allclose(ours, ref, rtol=1e-5, atol=1e-9)


def replay(env, f, n, check_dt=False):
    for t in range(len(f["x"])):
        if f["u_is_f32"][t]:
            u = f["u"][t].astype(np.float32)
        else:
            np.testing.assert_allclose(env.controller(), f["u"][t], rtol=1e-9, atol=1e-12)
            u = f["u"][t]  # continue from the reference's exact action
        (sv, net), r, done, info = env.step(u)
        assert done is False and info == {}
        if check_dt:
            assert env.dt == f["dt"][t]
        np.testing.assert_array_equal(env.x, f["x"][t])
        close_sv(sv, f["sv"][t])
        adj = adj_from_bits(f["adj_bits"][t], n)
        np.testing.assert_array_equal(net > 0, adj)
        deg = np.maximum(f["deg"][t], 1).astype(np.float32)
        np.testing.assert_array_equal(net, np.where(adj, (1.0 / deg.astype(np.float64)).astype(np.float32)[:, None], 0))
        np.testing.assert_allclose(r, f["reward"][t], rtol=1e-12)
        np.testing.assert_allclose(env.controller(), f["ctrl"][t], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(env.controller(centralized=False), f["ctrl_dec"][t], rtol=1e-9, atol=1e-12)


def test_leader_episode_matches_reference():
    f = np.load(os.path.join(GOLDEN, "variant_leader.npz"))
    np.random.seed(int(f["seed"]))
    env = envs.FlockingLeaderEnv()
    env.params_from_cfg(Cfg(12))
    sv0, net0 = env.reset()
    np.testing.assert_array_equal(env.x, f["x0"])
    close_sv(sv0, f["sv0"])  # pre-override observation, as the reference returns
    np.testing.assert_array_equal(net0, f["net0"].astype(np.float32))
    replay(env, f, 12)
    env.close()


def test_obstacle_episode_matches_reference():
    f = np.load(os.path.join(GOLDEN, "variant_obstacle.npz"))
    env = envs.FlockingObstacleEnv()
    sv0, net0 = env.reset()
    np.testing.assert_array_equal(env.x, f["x0"])
    close_sv(sv0, f["sv0"])
    np.testing.assert_array_equal(net0 > 0, adj_from_bits(f["adj_bits0"], 100))
    np.testing.assert_allclose(env.controller(), f["ctrl0"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(env.controller(centralized=False), f["ctrl0_dec"], rtol=1e-9, atol=1e-12)
    replay(env, f, 100)
    env.close()


def test_obstacle_mask_size_quirk():
    """The reference sizes the obstacle mask at __init__ (100 agents); another n_agents
    from params_from_cfg breaks its step with a broadcasting error. Reset still works."""
    env = envs.FlockingObstacleEnv()
    env.params_from_cfg(Cfg(50))
    env.reset()
    with pytest.raises(ValueError):
        env.step(np.zeros((50, 2)))
    env.close()


def test_stochastic_episode_matches_reference():
    f = np.load(os.path.join(GOLDEN, "variant_stochastic.npz"))
    np.random.seed(int(f["seed"]))
    env = envs.FlockingStochasticEnv()
    env.params_from_cfg(Cfg(10))
    sv0, _ = env.reset()
    np.testing.assert_array_equal(env.x, f["x0"])
    close_sv(sv0, f["sv0"])
    replay(env, f, 10, check_dt=True)
    env.close()


def test_twoflocks_episode_matches_reference():
    f = np.load(os.path.join(GOLDEN, "variant_twoflocks.npz"))
    np.random.seed(int(f["seed"]))
    env = envs.FlockingTwoFlocksEnv()
    env.params_from_cfg(Cfg(20))
    sv0, _ = env.reset()
    np.testing.assert_array_equal(env.x, f["x0"])
    close_sv(sv0, f["sv0"])
    replay(env, f, 20)
    env.close()


def test_registered_ids():
    import gym_flock
    for env_id, cls in (("FlockingLeader-v0", envs.FlockingLeaderEnv),
                        ("FlockingObstacle-v0", envs.FlockingObstacleEnv),
                        ("FlockingStochastic-v0", envs.FlockingStochasticEnv),
                        ("FlockingTwoFlocks-v0", envs.FlockingTwoFlocksEnv)):
        assert isinstance(gym_flock.make(env_id), cls)


@pytest.mark.parametrize("n,nz", [(300, 4), (1030, 600), (97, 0)])
@pytest.mark.parametrize("u_f64", [False, True])
def test_batched_variant_vs_oracle(n, nz, u_f64):
    """A batch of 3 envs with every switch on: frozen prefix, zeroed velocity pairs
    (across LDS tiles when nz > the 512-agent tile), clip, scale, per-env dt, controller
    clip; against the oracle."""
    B = 3
    var = dict(u_scale=6.0, u_clip=0.5, x_scale=6.0, ctrl_clip=0.5, n_frozen=min(nz, 7), n_vel_zero=nz)
    v = VecFlockingRelative(B, n, variant=var)
    x0 = np.stack([fo.synthetic_state(n, 70 + b) for b in range(B)])
    v.reset(x=x0)
    rs = np.random.RandomState(n + nz)
    u = rs.uniform(-1, 1, size=(B, n, 2))
    if not u_f64:
        u = u.astype(np.float32)
    dt = rs.normal(0.12, 0.018, size=B)
    v.step(u, controller=True, dt=dt)
    for b in range(B):
        x1 = fv.integrate(x0[b], u[b], dt[b], 6.0, min(nz, 7), 0.5, 6.0)
        np.testing.assert_array_equal(v.get_state()[b], x1)
        sv, net, adj, deg = fv.helpers(x1, n_vel_zero=nz)
        np.testing.assert_array_equal(v.network(b) > 0, adj)
        close_sv(v.state_values(b), sv)
        np.testing.assert_allclose(v.rewards()[b], fo.reward(x1), rtol=1e-12)
        np.testing.assert_allclose(v.controls(b), fv.controller(x1, n_vel_zero=nz, clip=0.5), rtol=1e-9, atol=1e-12)
    dec = v.controller(centralized=False)
    for b in range(B):
        x1 = v.get_state()[b]
        np.testing.assert_allclose(dec[b], fv.controller(x1, centralized=False, n_vel_zero=nz, clip=0.5),
                                   rtol=1e-9, atol=1e-12)
    v.close()


def test_variant_presets_and_clear():
    """The VARIANTS presets step like the oracle; clearing the variant restores the
    FlockingRelative step exactly."""
    n, B = 64, 2
    x0 = np.stack([fo.synthetic_state(n, 90 + b) for b in range(B)])
    u = np.random.RandomState(1).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    for name in ("leader", "obstacle"):
        v = VecFlockingRelative(B, n, variant=name)
        v.reset(x=x0)
        v.step(u)
        p = VARIANTS[name]
        for b in range(B):
            x1 = fv.integrate(x0[b], u[b], 0.01, p["u_scale"], p["n_frozen"])
            np.testing.assert_array_equal(v.get_state()[b], x1)
            close_sv(v.state_values(b), fv.helpers(x1, n_vel_zero=p.get("n_vel_zero", 0))[0])
        v.h.clear_variant()
        v.reset(x=x0)
        v.step(u)
        for b in range(B):
            np.testing.assert_array_equal(v.get_state()[b], fo.integrate(x0[b], u[b]))
        v.close()

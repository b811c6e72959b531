"""Pin the variant oracle (oracle/flocking_variants.py) against the reference's
recorded episodes (tests/golden/variant_*.npz, made by make_golden_variants.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import flocking as fo
from oracle import flocking_variants as fv

# the constants each reference variant hard-codes
VARIANTS = {
    "leader": dict(u_scale=1.0, n_frozen=2),
    "obstacle": dict(u_scale=1.0, n_frozen=4, n_vel_zero=4),
    "stochastic": dict(u_scale=6.0, u_clip=0.5, x_scale=6.0, ctrl_clip=0.5),
    "twoflocks": dict(u_scale=10.0),
}


def adj_from_bits(bits, n):
    return np.unpackbits(bits, axis=1, count=n).astype(bool)


def replay(name, x, f, dt_fn):
    p = VARIANTS[name]
    nvz = p.get("n_vel_zero", 0)
    n = x.shape[0]
    for t in range(len(f["x"])):
        if f["u_is_f32"][t]:
            u = f["u"][t].astype(np.float32)
        else:
            u = f["u"][t]
        dt = dt_fn(t)
        x = fv.integrate(x, u, dt, p["u_scale"], p.get("n_frozen", 0), p.get("u_clip"), p.get("x_scale"))
        np.testing.assert_array_equal(x, f["x"][t])
        sv, net, adj, deg = fv.helpers(x, n_vel_zero=nvz)
        np.testing.assert_array_equal(adj, adj_from_bits(f["adj_bits"][t], n))
        np.testing.assert_array_equal(deg, f["deg"][t])
        np.testing.assert_allclose(sv, f["sv"][t], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(fo.reward(x), f["reward"][t], rtol=1e-13)
        c = fv.controller(x, n_vel_zero=nvz, clip=p.get("ctrl_clip"))
        np.testing.assert_allclose(c, f["ctrl"][t], rtol=1e-12, atol=1e-13)
        cd = fv.controller(x, centralized=False, n_vel_zero=nvz, clip=p.get("ctrl_clip"))
        np.testing.assert_allclose(cd, f["ctrl_dec"][t], rtol=1e-12, atol=1e-13)
    return x


def test_leader_episode():
    f = np.load(os.path.join(GOLDEN, "variant_leader.npz"))
    n = int(f["n_agents"])
    np.random.seed(int(f["seed"]))
    x, before = fv.leader_reset(n, r_max=np.sqrt(n))
    np.testing.assert_array_equal(x, f["x0"])
    sv0, net0, _, _ = fo.helpers(before)  # reset() returns the pre-override observation
    np.testing.assert_allclose(sv0, f["sv0"], rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(net0, f["net0"])
    replay("leader", x, f, lambda t: 0.01)
    assert (f["x"][:, :2, 2:4] == f["x0"][None, :2, 2:4]).all()  # leaders keep their velocity


def test_obstacle_episode():
    f = np.load(os.path.join(GOLDEN, "variant_obstacle.npz"))
    x = fv.obstacle_reset()
    np.testing.assert_array_equal(x, f["x0"])
    sv, _, adj, deg = fv.helpers(x, n_vel_zero=4)
    np.testing.assert_array_equal(adj, adj_from_bits(f["adj_bits0"], 100))
    np.testing.assert_allclose(sv, f["sv0"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(fv.controller(x, n_vel_zero=4), f["ctrl0"], rtol=1e-12, atol=1e-13)
    replay("obstacle", x, f, lambda t: 0.01)


def test_stochastic_episode():
    f = np.load(os.path.join(GOLDEN, "variant_stochastic.npz"))
    n = int(f["n_agents"])
    np.random.seed(int(f["seed"]))
    x = fo.reset_rejection(n, r_max=np.sqrt(n))
    np.testing.assert_array_equal(x, f["x0"])
    dts = []

    def dt_fn(t):
        dts.append(np.random.normal(0.12, 0.018))  # flocking_stoch.py:24, global RNG
        assert dts[-1] == f["dt"][t]
        return dts[-1]

    replay("stochastic", x, f, dt_fn)


def test_twoflocks_episode():
    f = np.load(os.path.join(GOLDEN, "variant_twoflocks.npz"))
    n = int(f["n_agents"])
    np.random.seed(int(f["seed"]))
    x = fv.twoflocks_reset(n)
    np.testing.assert_array_equal(x, f["x0"])
    sv, _, _, _ = fo.helpers(x)
    np.testing.assert_allclose(sv, f["sv0"], rtol=1e-12, atol=1e-12)
    replay("twoflocks", x, f, lambda t: 0.01)


@pytest.mark.parametrize("side", [2, 5])
def test_grid_shape(side):
    g = fv.grid(20, side)
    assert g.shape == (20, 2)

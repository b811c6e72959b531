"""CPU oracle for the flocking variants.

TEST INFRASTRUCTURE ONLY, like oracle/flocking.py. It restates what each variant
changes against FlockingRelative-v0. It is pinned by tests/golden/variant_*.npz,
which were made from the reference by tests/golden/make_golden_variants.py.

The four variants (paths relative to gym_flock/envs/flocking/):
  flocking_leader.py     FlockingLeaderEnv      step :21-35, reset :37-41, mask :13-15
  flocking_obstacle.py   FlockingObstacleEnv    step :34-52, reset :59-74, helpers :75-104
  flocking_stoch.py      FlockingStochasticEnv  step :14-36, controller :39-46
  flocking_twoflocks.py  FlockingTwoFlocksEnv   reset :8-28
"""
import numpy as np

from . import flocking as fo


def integrate(x, u, dt, u_scale=10.0, n_frozen=0, u_clip=None, x_scale=None):
    """The variants' double-integrator update, in the reference's operation order.

    u_scale: the action multiplier. It is 10 in FlockingRelative (:96). The leader and
      obstacle steps leave u unscaled, so 1. The stochastic step scales by 6 (:21).
    n_frozen: agents [0, n_frozen) get mask 0. Their action terms are multiplied by
      the float64 mask after the float32 arithmetic (leader :27-33, obstacle :41-49).
    u_clip: np.clip(u, -c, c) first (stochastic :20). It keeps u's dtype.
    x_scale: the state is multiplied by it before the update and divided after
      (stochastic :22, :36).
    """
    x = np.array(x, dtype=np.float64, copy=True)
    u = np.asarray(u)
    assert u.shape == (x.shape[0], 2), "u must be (n_agents, 2)"
    if u.dtype not in (np.float32, np.float64):
        u = u.astype(np.float64)
    t = u.dtype.type
    if u_clip is not None:
        u = np.clip(u, -u_clip, u_clip)
    us = u * t(u_scale)
    acc_pos = ((us * t(dt)) * t(dt)) * t(0.5)
    acc_vel = us * t(dt)
    if n_frozen:
        mask = np.ones(x.shape[0])
        mask[:n_frozen] = 0
        acc_pos = acc_pos * mask[:, None]
        acc_vel = acc_vel * mask[:, None]
    if x_scale is not None:
        x = x * x_scale
    x[:, 0] = (x[:, 0] + x[:, 2] * dt) + acc_pos[:, 0]
    x[:, 1] = (x[:, 1] + x[:, 3] * dt) + acc_pos[:, 1]
    x[:, 2] = x[:, 2] + acc_vel[:, 0]
    x[:, 3] = x[:, 3] + acc_vel[:, 1]
    if x_scale is not None:
        x = x / x_scale
    return x


def pair_geometry(x, n_vel_zero=0):
    """flocking_relative.py:113-115, plus flocking_obstacle.py:79-80: velocity
    differences are zero for every pair that involves one of the first n_vel_zero
    agents."""
    dx, dy, dvx, dvy, r2 = fo.pair_geometry(x)
    if n_vel_zero:
        dvx = dvx.copy()
        dvy = dvy.copy()
        for d in (dvx, dvy):
            d[:n_vel_zero, :] = 0
            d[:, :n_vel_zero] = 0
    return dx, dy, dvx, dvy, r2


def helpers(x, comm_radius=0.9, mean_pooling=True, n_vel_zero=0):
    return fo.helpers(x, comm_radius, mean_pooling, pair_geometry(x, n_vel_zero))


def controller(x, comm_radius=0.9, action_scalar=10.0, centralized=True, n_vel_zero=0, clip=None):
    """controller() on the variant's diff (obstacle) and with the stochastic env's
    extra clip (flocking_stoch.py:44-45). action_scalar stays 10 in every variant
    (only the step's scaling changes)."""
    u = fo.controller(x, comm_radius, action_scalar, centralized, pair_geometry(x, n_vel_zero))
    if clip is not None:
        u = np.clip(u, -clip, clip)
    return u


def grid(n, side=5):
    """utils.py:26-33 (and its copy in flocking_obstacle.py:4-11)."""
    side2 = int(n / side)
    xs = np.arange(0, side) - side / 2.0
    ys = np.arange(0, side2) - side2 / 2.0
    xs, ys = np.meshgrid(xs, ys)
    return 0.8 * np.hstack((xs.reshape((n, 1)), ys.reshape((n, 1))))


def obstacle_reset(n_agents=100, n_obstacles=4):
    """flocking_obstacle.py:59-74: deterministic grid, velocity (0, -7); the obstacles
    sit on a small grid 10 below, at rest."""
    x = np.zeros((n_agents, 4))
    x[:, 0:2] = grid(n_agents)
    x[:, 2:4] = [0, -7.0]
    x[:n_obstacles, 0:2] = grid(n_obstacles, side=2) * 0.5
    x[:n_obstacles, 1] -= 10.0
    x[:n_obstacles, 2:4] = 0
    return x


def twoflocks_reset(n_agents, v_bias=5.0, rng=np.random):
    """flocking_twoflocks.py:8-28: grid positions, velocities -grid plus one global
    uniform bias per axis."""
    x = np.zeros((n_agents, 4))
    bias = rng.uniform(low=-v_bias / 2.0, high=v_bias / 2.0, size=(2,))
    g = grid(n_agents, side=int(n_agents / 10))
    x[:, 0:2] = g
    x[:, 2:4] = -g
    x[:, 2] = x[:, 2] + bias[0]
    x[:, 3] = x[:, 3] + bias[1]
    return x


def leader_reset(n_agents, r_max, v_max=5.0, n_leaders=2, rng=np.random):
    """flocking_leader.py:37-41: the relative env's rejection-sampled reset, then both
    leaders get velocity (w, w) for one draw w ~ U(-v_max, v_max). The observation the
    reference returns is the one computed before that override."""
    x = fo.reset_rejection(n_agents, r_max, v_max, rng=rng)
    before = x.copy()
    x[:n_leaders, 2:4] = np.ones((n_leaders, 2)) * rng.uniform(low=-v_max, high=v_max, size=(1, 1))
    return x, before

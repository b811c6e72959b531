"""Golden vectors for the flocking variants, generated from
the reference. make_golden.py imports this module after installing its gym stub.

Variants and what they change against FlockingRelative-v0:
  leader      flocking_leader.py: actions unscaled, first 2 agents ignore actions,
              reset sets the leaders' velocity to one global uniform draw
  obstacle    flocking_obstacle.py: actions unscaled, first 4 agents ignore actions,
              velocity differences zeroed for pairs that touch them, grid reset
  stochastic  flocking_stoch.py: clip +-0.5, scale 6, dt ~ N(0.12, 0.018) per step
              (global RNG), controller clipped to +-0.5
  twoflocks   flocking_twoflocks.py: grid reset with opposing velocities

Each episode records the reset state and observation, then per step: the action, the
state, state_values, adjacency bits/degree (the network is adj/deg), reward, and the
controller on the new state (centralised and not).
"""
import importlib
import os

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))


class _Cfg:
    def __init__(self, **kv):
        self.kv = kv

    def getfloat(self, k):
        return float(self.kv[k])

    def getint(self, k):
        return int(self.kv[k])


def _record(env, steps, u_fn, out):
    rec = {k: [] for k in ("u", "x", "sv", "adj_bits", "deg", "reward", "ctrl", "ctrl_dec", "dt")}
    for t in range(steps):
        u = u_fn(t, env)
        (sv, net), r, _, _ = env.step(u)
        adj = env.adj_mat > 0
        rec["u"].append(np.asarray(u, np.float64))
        rec["x"].append(env.x.copy())
        rec["sv"].append(np.array(sv))
        rec["adj_bits"].append(np.packbits(adj, axis=1))
        rec["deg"].append(adj.sum(axis=1).astype(np.int32))
        rec["reward"].append(r)
        rec["ctrl"].append(env.controller())
        rec["ctrl_dec"].append(env.controller(centralized=False))
        rec["dt"].append(env.dt)
    out.update({k: np.array(v) for k, v in rec.items()})
    return out


def gen_variants():
    mods = {name: importlib.import_module("gym_flock.envs.flocking." + name)
            for name in ("flocking_leader", "flocking_obstacle", "flocking_stoch", "flocking_twoflocks")}
    cfg = dict(comm_radius=0.9, v_max=5.0, dt=0.01)

    # leader, N=12: 15 closed-loop steps (float64 actions), 10 float32 random steps
    np.random.seed(31)
    env = mods["flocking_leader"].FlockingLeaderEnv()
    env.params_from_cfg(_Cfg(n_agents=12, **cfg))
    sv0, net0 = env.reset()
    out = dict(seed=31, n_agents=12, x0=env.x.copy(), sv0=np.array(sv0), net0=np.array(net0))
    rs = np.random.RandomState(5)
    u_f32 = [rs.uniform(-1, 1, size=(12, 2)).astype(np.float32) for _ in range(10)]
    out["u_is_f32"] = np.array([0] * 15 + [1] * 10, np.int8)
    _record(env, 25, lambda t, e: e.controller() if t < 15 else u_f32[t - 15], out)
    np.savez_compressed(os.path.join(OUT, "variant_leader.npz"), **out)

    # obstacle, N=100 (its mask is sized at __init__, so only the default N works)
    env = mods["flocking_obstacle"].FlockingObstacleEnv()
    sv0, net0 = env.reset()
    adj0 = env.adj_mat > 0
    out = dict(n_agents=100, x0=env.x.copy(), sv0=np.array(sv0), deg0=adj0.sum(axis=1).astype(np.int32),
               adj_bits0=np.packbits(adj0, axis=1), ctrl0=env.controller(),
               ctrl0_dec=env.controller(centralized=False))
    rs = np.random.RandomState(6)
    u_f32 = [rs.uniform(-1, 1, size=(100, 2)).astype(np.float32) for _ in range(5)]
    out["u_is_f32"] = np.array([0] * 20 + [1] * 5, np.int8)
    _record(env, 25, lambda t, e: e.controller() if t < 20 else u_f32[t - 20], out)
    np.savez_compressed(os.path.join(OUT, "variant_obstacle.npz"), **out)

    # stochastic, N=10: reset (rejection, global RNG) then 20 closed-loop steps, each
    # drawing dt from the global RNG; then 5 float32 steps
    np.random.seed(41)
    env = mods["flocking_stoch"].FlockingStochasticEnv()
    env.params_from_cfg(_Cfg(n_agents=10, **cfg))
    sv0, net0 = env.reset()
    out = dict(seed=41, n_agents=10, x0=env.x.copy(), sv0=np.array(sv0))
    rs = np.random.RandomState(7)
    u_f32 = [rs.uniform(-1, 1, size=(10, 2)).astype(np.float32) for _ in range(5)]
    out["u_is_f32"] = np.array([0] * 20 + [1] * 5, np.int8)
    _record(env, 25, lambda t, e: e.controller() if t < 20 else u_f32[t - 20], out)
    np.savez_compressed(os.path.join(OUT, "variant_stochastic.npz"), **out)

    # two flocks, N=20: grid reset with a global-RNG bias, 20 closed-loop steps
    np.random.seed(51)
    env = mods["flocking_twoflocks"].FlockingTwoFlocksEnv()
    env.params_from_cfg(_Cfg(n_agents=20, **cfg))
    sv0, net0 = env.reset()
    out = dict(seed=51, n_agents=20, x0=env.x.copy(), sv0=np.array(sv0))
    out["u_is_f32"] = np.zeros(20, np.int8)
    _record(env, 20, lambda t, e: e.controller(), out)
    np.savez_compressed(os.path.join(OUT, "variant_twoflocks.npz"), **out)
    print("variants: leader, obstacle, stochastic, twoflocks written")

"""Initial swarm states (host-side RNG, per-episode; not the step hot path).

reset() of the reference (flocking_relative.py:156-192) draws positions uniformly in
a disk of radius sqrt(r_max) and velocities U(-v_max, v_max) plus a common bias
U(-v_bias, v_bias), and rejects the draw until every agent has >= 2 neighbours and
the minimum pairwise distance is >= 0.1. The draws come from the GLOBAL NumPy RNG in
the order (length, angle, bias, vx, vy); `draw_swarm` reproduces that order exactly
so a seeded np.random gives the reference's states bit for bit.

At N >~ 150 the rejection loop never terminates (SURVEY.md finding 5), so batched
runs use `synthetic_state`: one draw of the same distribution from
np.random.RandomState(seed).
"""
import numpy as np


def draw_swarm(n_agents, r_max, v_max, v_bias, rng=np.random):
    """One candidate of reset()'s distribution (flocking_relative.py:167-174)."""
    x = np.zeros((n_agents, 4))
    length = np.sqrt(rng.uniform(0, r_max, size=(n_agents,)))
    angle = np.pi * rng.uniform(0, 2, size=(n_agents,))
    x[:, 0] = length * np.cos(angle)
    x[:, 1] = length * np.sin(angle)
    bias = rng.uniform(low=-v_bias, high=v_bias, size=(2,))
    x[:, 2] = rng.uniform(low=-v_max, high=v_max, size=(n_agents,)) + bias[0]
    x[:, 3] = rng.uniform(low=-v_max, high=v_max, size=(n_agents,)) + bias[1]
    return x


def synthetic_state(n_agents, seed, v_max=5.0, r_max=None):
    """SURVEY.md §8d synthetic init for env seed `seed` (r_max defaults to sqrt(N),
    the value params_from_cfg sets, flocking_relative.py:75)."""
    rs = np.random.RandomState(seed)
    if r_max is None:
        r_max = np.sqrt(n_agents)
    return draw_swarm(n_agents, r_max, v_max, v_max, rs)


def synthetic_batch(n_envs, n_agents, seed0=0, v_max=5.0):
    """(B,N,4) float64: env b uses synthetic_state(N, seed0 + b)."""
    out = np.empty((n_envs, n_agents, 4))
    for b in range(n_envs):
        out[b] = synthetic_state(n_agents, seed0 + b, v_max)
    return out

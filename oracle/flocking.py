"""CPU oracle for the FlockingRelative / Flocking-v0 env-step hot path.

TEST INFRASTRUCTURE ONLY. This module is a NumPy restatement of the reference
algorithm, used as the parity checker by tests/, by __graft_entry__.smoke() and as
the `cpu_baseline` leg of bench.py. The product (gym-flock_amd/) never imports it;
the product path runs on the HIP kernels and fails loudly without them.

Pinned against the reference's own outputs: tests/golden/*.npz were produced by
importing /root/reference (tests/golden/make_golden.py) and tests/test_oracle_golden.py
checks this restatement against every one of them.

Every function cites the reference lines it restates (paths relative to the
reference root, gym_flock/envs/flocking/...).
"""
import numpy as np


def integrate(x, u, dt=0.01, action_scalar=10.0):
    """Double-integrator update, flocking_relative.py:91-105.

    The action terms are evaluated in u's own dtype, exactly as NumPy does in the
    reference: `u * action_scalar` with a float32 `u` stays float32 (NEP 50 weak
    Python scalars), and so do `u*dt*dt*0.5` and `u*dt`; they are then added to the
    float64 state. Positions use the OLD velocity (:99-101 run before :103-105).
    """
    x = np.array(x, dtype=np.float64, copy=True)
    u = np.asarray(u)
    assert u.shape == (x.shape[0], 2), "u must be (n_agents, 2)"  # :94
    if u.dtype not in (np.float32, np.float64):
        u = u.astype(np.float64)
    t = u.dtype.type
    us = u * t(action_scalar)                     # :96
    acc_pos = ((us * t(dt)) * t(dt)) * t(0.5)     # u*dt*dt*0.5, left to right
    acc_vel = us * t(dt)                          # u*dt
    x[:, 0] = (x[:, 0] + x[:, 2] * dt) + acc_pos[:, 0]   # :99
    x[:, 1] = (x[:, 1] + x[:, 3] * dt) + acc_pos[:, 1]   # :101
    x[:, 2] = x[:, 2] + acc_vel[:, 0]                    # :103
    x[:, 3] = x[:, 3] + acc_vel[:, 1]                    # :105
    return x


def pair_geometry(x):
    """diff and r2 with an infinite diagonal, flocking_relative.py:113-115.

    r2 = dx*dx + dy*dy as two products and one sum (no fused multiply-add)."""
    px, py, vx, vy = x[:, 0], x[:, 1], x[:, 2], x[:, 3]
    dx = px[:, None] - px[None, :]
    dy = py[:, None] - py[None, :]
    dvx = vx[:, None] - vx[None, :]
    dvy = vy[:, None] - vy[None, :]
    r2 = dx * dx + dy * dy
    np.fill_diagonal(r2, np.inf)
    return dx, dy, dvx, dvy, r2


def pair_geometry_rows(x, rows):
    """pair_geometry() for the rows `rows` only (each against every agent), the same
    operations in the same order, so large N can be checked on sampled rows without the
    (N,N) temporaries."""
    rows = np.asarray(rows)
    px, py, vx, vy = x[:, 0], x[:, 1], x[:, 2], x[:, 3]
    dx = px[rows, None] - px[None, :]
    dy = py[rows, None] - py[None, :]
    dvx = vx[rows, None] - vx[None, :]
    dvy = vy[rows, None] - vy[None, :]
    r2 = dx * dx + dy * dy
    r2[np.arange(len(rows)), rows] = np.inf
    return dx, dy, dvx, dvy, r2


def step_rows(x, u, rows, comm_radius=0.9, dt=0.01, action_scalar=10.0, with_controller=False):
    """step() restricted to the rows `rows` of the per-agent outputs (helpers() and
    controller() take the row geometry unchanged); x and the reward are the whole env's."""
    x1 = integrate(x, u, dt, action_scalar)
    geom = pair_geometry_rows(x1, rows)
    sv, net, adj, deg = helpers(x1, comm_radius, True, geom)
    out = dict(x=x1, state_values=sv, network=net, adj=adj, deg=deg, reward=reward(x1))
    if with_controller:
        out["ctrl"] = controller(x1, comm_radius, action_scalar, True, geom)
    return out


def helpers(x, comm_radius=0.9, mean_pooling=True, geom=None):
    """compute_helpers(), flocking_relative.py:111-134.

    Returns (state_values (N,6), state_network (N,N), adjacency (N,N) bool, degree).
    Features per neighbour j of i (strict r2 < comm_radius**2, :117):
      [vx_i-vx_j, dx/r2^2, dx/r2, vy_i-vy_j, dy/r2^2, dy/r2]   (:124-125)
    summed over neighbours (:128). The network is adj/deg with deg 0 -> 1 (:120-122)
    when mean pooling (:131-134), else the 0/1 adjacency.
    """
    dx, dy, dvx, dvy, r2 = geom if geom is not None else pair_geometry(x)
    adj = r2 < comm_radius * comm_radius
    deg = adj.sum(axis=1)
    deg_safe = np.where(deg == 0, 1, deg).astype(np.float64)
    network = adj / deg_safe[:, None] if mean_pooling else adj.astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        rr = r2 * r2
        terms = (dvx, dx / rr, dx / r2, dvy, dy / rr, dy / r2)
    state_values = np.stack([np.where(adj, t, 0.0).sum(axis=1) for t in terms], axis=1)
    return state_values, network, adj, deg


def reward(x):
    """instant_cost(), flocking_relative.py:145-147: -(var(vx) + var(vy)), ddof 0."""
    return -1.0 * np.sum(np.var(x[:, 2:4], axis=0))


def controller(x, comm_radius=0.9, action_scalar=10.0, centralized=True, geom=None):
    """Turner-2003 expert, flocking_relative.py:194-226.

    grad = -2*d/r2^2 + 2*d/r2, zeroed where r2 > comm_radius (NOT comm_radius**2, :225).
    Centralised (:28, :200-208) sums [dvx, dvy, gx, gy] over ALL j; otherwise only over
    adjacent j (:205-206). u = clip([-gx - dvx, -dvy - gy], -10, 10) / action_scalar.
    """
    dx, dy, dvx, dvy, r2 = geom if geom is not None else pair_geometry(x)
    with np.errstate(divide="ignore", invalid="ignore"):
        rr = r2 * r2
        gx = -2.0 * (dx / rr) + 2.0 * (dx / r2)
        gy = -2.0 * (dy / rr) + 2.0 * (dy / r2)
    far = r2 > comm_radius
    gx = np.where(far, 0.0, gx)
    gy = np.where(far, 0.0, gy)
    if not centralized:
        adj = r2 < comm_radius * comm_radius
        gx, gy = np.where(adj, gx, 0.0), np.where(adj, gy, 0.0)
        dvx, dvy = np.where(adj, dvx, 0.0), np.where(adj, dvy, 0.0)
    s_dvx, s_dvy = dvx.sum(axis=1), dvy.sum(axis=1)
    s_gx, s_gy = gx.sum(axis=1), gy.sum(axis=1)
    u = np.stack([-s_gx - s_dvx, -s_dvy - s_gy], axis=1)   # :209
    return np.clip(u, -10, 10) / action_scalar              # :210-211


def stats(x, geom=None):
    """get_stats(), flocking_relative.py:136-143."""
    r2 = (geom if geom is not None else pair_geometry(x))[4]
    v = x[:, 2:4]
    vel_diffs = np.sqrt(np.sum((v - v.mean(axis=0)) ** 2, axis=1))
    min_dists = np.sqrt(r2.min(axis=0))
    return {"vel_diffs": vel_diffs, "min_dists": min_dists}


def knn_observation(x, k=7, geom=None):
    """Flocking-v0 get_observation(), flocking.py:20-25.

    Neighbours are the k smallest r2 (self has r2=inf so it sorts last). The
    reference's argsort is an unstable quicksort; this oracle breaks ties by the
    lower index (stable sort), the rule the HIP kernel implements. Returns
    (indices (N,k) int32, obs (N,4k) with obs[:,4m:4m+4] = x - x[nn_m]).
    """
    r2 = (geom if geom is not None else pair_geometry(x))[4]
    idx = np.argsort(r2, axis=1, kind="stable")[:, :k].astype(np.int32)
    obs = np.concatenate([x - x[idx[:, m]] for m in range(k)], axis=1)
    return idx, obs


def step(x, u, comm_radius=0.9, dt=0.01, action_scalar=10.0, mean_pooling=True,
         with_controller=False, centralized=True):
    """One FlockingRelativeEnv.step (flocking_relative.py:91-109) from state x.

    Returns dict(x, state_values, network, adj, deg, reward[, ctrl])."""
    x1 = integrate(x, u, dt, action_scalar)
    geom = pair_geometry(x1)
    sv, net, adj, deg = helpers(x1, comm_radius, mean_pooling, geom)
    out = dict(x=x1, state_values=sv, network=net, adj=adj, deg=deg, reward=reward(x1))
    if with_controller:
        out["ctrl"] = controller(x1, comm_radius, action_scalar, centralized, geom)
    return out


def reset_rejection(n_agents, r_max, v_max=5.0, comm_radius=0.9, rng=np.random):
    """reset(), flocking_relative.py:156-192: rejection-sample until every agent has
    degree >= 2 and the minimum pairwise distance is >= 0.1, drawing from the GLOBAL
    NumPy RNG in the reference's call order (length, angle, bias, vx, vy)."""
    x = np.zeros((n_agents, 4))
    degree, min_dist = 0, 0.0
    while degree < 2 or min_dist < 0.1:
        length = np.sqrt(rng.uniform(0, r_max, size=(n_agents,)))
        angle = np.pi * rng.uniform(0, 2, size=(n_agents,))
        x[:, 0] = length * np.cos(angle)
        x[:, 1] = length * np.sin(angle)
        bias = rng.uniform(low=-v_max, high=v_max, size=(2,))
        x[:, 2] = rng.uniform(low=-v_max, high=v_max, size=(n_agents,)) + bias[0]
        x[:, 3] = rng.uniform(low=-v_max, high=v_max, size=(n_agents,)) + bias[1]
        d = x[:, None, 0:2] - x[None, :, 0:2]
        a = np.sum(d * d, axis=2)
        np.fill_diagonal(a, np.inf)
        min_dist = np.sqrt(a.min())
        degree = int(np.min(np.sum(a < comm_radius * comm_radius, axis=1)))
    return x


def synthetic_state(n_agents, seed, v_max=5.0):
    """SURVEY §8d synthetic init (reset()'s distribution without rejection), with
    np.random.RandomState(seed) drawn in reset()'s call order."""
    rs = np.random.RandomState(seed)
    r_max = np.sqrt(n_agents)
    x = np.zeros((n_agents, 4))
    length = np.sqrt(rs.uniform(0, r_max, size=(n_agents,)))
    angle = np.pi * rs.uniform(0, 2, size=(n_agents,))
    x[:, 0] = length * np.cos(angle)
    x[:, 1] = length * np.sin(angle)
    bias = rs.uniform(low=-v_max, high=v_max, size=(2,))
    x[:, 2] = rs.uniform(low=-v_max, high=v_max, size=(n_agents,)) + bias[0]
    x[:, 3] = rs.uniform(low=-v_max, high=v_max, size=(n_agents,)) + bias[1]
    return x

"""CPU oracle for the Coverage-v0 env step (graph coverage with robot collision checks).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; never by the product. Restates gym_flock/envs/spatial/coverage.py of
the reference (lines cited per function) for the module configuration the reference
ships with (PAD_ACTIONS, COLLISION_CHECKS, no comm edges, no node history, no hidden
nodes, distance edge features). Pinned against tests/golden/coverage_*.npz.

Indexing follows the reference: agents 0..R-1 are robots, R..R+T-1 are targets
("global" node indices); robots always sit on target nodes.
"""
import numpy as np

N_ACTIONS = 4        # coverage.py:60
MAX_EDGES = 4        # coverage.py:56 (edges per node in the padded observation)
EPISODE_LENGTH = 75  # coverage.py:64
RES = 5.5            # coverage.py:80 (DELTA)


def radius_graph(targets, radius):
    """_get_graph_edges(radius, targets, self_loops=True), utils.py:8-24: every ordered
    pair at distance <= radius, zero distances dropped (so no self loops), row-major
    order; returns (senders, receivers, dists) in target-local indices."""
    d = targets[:, None, :] - targets[None, :, :]
    r = np.sqrt(d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1])
    r[r > radius] = 0
    s, q = np.nonzero(r)
    return s, q, r[s, q]


def neighbour_table(n_targets, senders, receivers):
    """Per target, its motion-graph out-neighbours in ascending order (the order
    np.where returns them in get_action_edges, coverage.py:216), padded with -1."""
    nbr = -np.ones((n_targets, N_ACTIONS), np.int64)
    cnt = np.zeros(n_targets, np.int64)
    for s, q in zip(senders, receivers):
        nbr[s, cnt[s]] = q
        cnt[s] += 1
    return nbr, cnt


def closest_targets(xr, targets, n_robots):
    """coverage.py:427-432: argmin over targets of the Euclidean distance (first index
    on ties), as global node indices."""
    d = xr[:, None, :] - targets[None, :, :]
    r = np.sqrt(d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1])
    return np.argmin(r, axis=1) + n_robots


def action_receivers(cur, nbr, cnt, n_robots):
    """get_action_edges, coverage.py:206-232: the 4 action targets of each robot = the
    out-neighbours of its current node, padded with the current node."""
    out = np.empty((len(cur), N_ACTIONS), np.int64)
    for i, c in enumerate(cur):
        t = c - n_robots
        k = cnt[t]
        out[i, :k] = nbr[t, :k] + n_robots
        out[i, k:] = c
    return out


def resolve_moves(cur, recv, actions):
    """step(), coverage.py:184-200: robots whose action stays claim their node first;
    then, in index order, each other robot takes its chosen node unless an earlier claim
    holds it (then it stays, and its node joins the claims). Returns the new nodes."""
    R = len(cur)
    chosen = recv[np.arange(R), actions]
    claims = -np.ones(R, np.int64)
    stay = chosen == cur
    claims[stay] = chosen[stay]
    taken = set(claims[stay].tolist())
    for i in range(R):
        if claims[i] == -1:
            if chosen[i] not in taken:
                claims[i] = chosen[i]
            else:
                claims[i] = cur[i]
            taken.add(int(claims[i]))
    return claims


class CoverageOracle:
    """State and observation arrays of one CoverageEnv (coverage.py:82-364)."""

    def __init__(self, targets, n_robots, max_nodes, motion_radius=RES * 1.2):
        self.R, self.T = n_robots, len(targets)
        self.n_agents = self.R + self.T
        self.max_nodes = max_nodes
        self.max_edges = max_nodes * MAX_EDGES
        self.targets = np.asarray(targets, dtype=np.float64)
        s, q, dist = radius_graph(self.targets, motion_radius)
        self.motion = (s + self.R, q + self.R)
        self.n_motion = len(s)
        self.nbr, self.cnt = neighbour_table(self.T, s, q)
        # static parts of the padded observation (_initialize_graph, coverage.py:551-594)
        self.edges = np.zeros((self.max_edges, 1), np.float32)
        self.senders = -np.ones(self.max_edges, np.int32)
        self.receivers = -np.ones(self.max_edges, np.int32)
        self.senders[:self.n_motion] = self.motion[0]
        self.receivers[:self.n_motion] = self.motion[1]
        self.edges[:self.n_motion, 0] = dist
        self.nodes = np.zeros((self.max_nodes, 3), np.float32)
        self.robot_flag = np.r_[np.ones(self.R), np.zeros(self.T)]
        self.landmark_flag = np.r_[np.zeros(self.R), np.ones(self.T)]

    def reset(self, start_targets, unvisited_targets):
        """reset() after the random draws (coverage.py:405-424): robots start on
        start_targets (target-local), unvisited_targets (global) are unvisited."""
        self.xr = self.targets[np.asarray(start_targets)].copy()
        self.visited = np.ones(self.n_agents)
        self.visited[np.asarray(unvisited_targets, dtype=np.int64)] = 0
        self.step_counter = 0
        return self._obs_reward()[0]

    def closest(self):
        return closest_targets(self.xr, self.targets, self.R)

    def step(self, actions):
        """step(), coverage.py:174-204; returns (obs, reward, done)."""
        actions = np.asarray(actions).reshape(-1).astype(np.int64)
        cur = self.closest()
        recv = action_receivers(cur, self.nbr, self.cnt, self.R)
        new = resolve_moves(cur, recv, actions)
        moved = new != cur
        self.xr[moved] = self.targets[new[moved] - self.R]
        return self._obs_reward()

    def _obs_reward(self):
        """_get_obs_reward(), coverage.py:234-364."""
        R = self.R
        cur = self.closest()
        recv = action_receivers(cur, self.nbr, self.cnt, R)
        robots = np.repeat(np.arange(R), N_ACTIONS)
        nodes = recv.reshape(-1)
        d = self.xr[robots] - self.targets[nodes - R]
        dist = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
        old_sum = np.sum(self.visited[R:])
        self.visited[cur] = 1
        snd = np.concatenate([nodes, robots])   # action_edges[1]
        rcv = np.concatenate([robots, nodes])   # action_edges[0]
        self.senders[self.n_motion:] = -1
        self.receivers[self.n_motion:] = -1
        self.nodes.fill(0)
        self.senders[-len(snd):] = snd
        self.receivers[-len(rcv):] = rcv
        self.edges[-len(snd):, 0] = np.concatenate([dist, dist]) / RES
        self.nodes[:self.n_agents, 0] = self.robot_flag
        self.nodes[:self.n_agents, 1] = self.landmark_flag
        self.nodes[:self.n_agents, 2] = np.logical_not(self.visited)
        obs = {"nodes": self.nodes.copy(), "edges": self.edges.copy(), "senders": self.senders.copy(),
               "receivers": self.receivers.copy(), "step": np.array([[self.step_counter]])}
        self.step_counter += 1
        new_sum = np.sum(self.visited[R:])
        done = self.step_counter == EPISODE_LENGTH or new_sum == self.T
        return obs, new_sum - old_sum, done


def generate_lattice(xmin, xmax, ymin, ymax, spacing=RES):
    """make_map.generate_lattice (make_map.py:30-67) for the axis-aligned square lattice
    that Coverage-v0 uses (lattice vectors (-spacing, 0), (0, -spacing))."""
    w, h = xmax - xmin, ymax - ymin
    nx, ny = w // spacing, h // spacing
    xs = np.arange(-nx, nx, dtype=float)[:, None]
    ys = np.arange(-ny, nx, dtype=float)[None, :]
    xl = -spacing * xs + 0.0 * ys
    yl = 0.0 * xs + -spacing * ys
    mask = (xl < w / 2.0) & (xl > -w / 2.0) & (yl < h / 2.0) & (yl > -h / 2.0)
    xl, yl = xl[mask] + (w // 2 + xmin), yl[mask] + (h // 2 + ymin)
    return np.stack([yl, xl], axis=1)


MAX_COST = 1000  # coverage.py:68
HORIZON = 10     # coverage.py:66


def time_matrix(n_targets, senders, receivers, horizon=HORIZON, edge_time=1.0):
    """construct_time_matrix(), coverage.py:621-653: per-source hop counts relaxed
    column-wise over the motion edges in list order (in place, Gauss-Seidel), sweeping
    while some entry changed and some entry is still infinite, at most horizon+1 sweeps.
    senders/receivers are target-local. Returns (cost with inf -> MAX_COST, prev)."""
    tm = np.full((n_targets, n_targets), np.inf)
    prev = -np.ones((n_targets, n_targets), dtype=int)
    np.fill_diagonal(tm, 0.0)
    changed, steps = True, 0
    while changed and np.sum(tm) == np.inf:
        changed = False
        for s, q in zip(senders, receivers):
            via = tm[:, s] + edge_time
            better = via < tm[:, q]
            prev[:, q] = np.where(better, s, prev[:, q])
            new = np.minimum(via, tm[:, q])
            changed = changed or not np.array_equal(new, tm[:, q])
            tm[:, q] = new
        steps += 1
        if steps > horizon > -1:
            break
    return np.nan_to_num(tm, posinf=MAX_COST), prev


def greedy_actions(cost, prev, cur, visited_targets, recv, n_robots):
    """controller(greedy=True), coverage.py:808-872 without its random fallback: for
    each robot the nearest (hop count, first index) unvisited target, and the action
    whose node is the next hop toward it. Returns (actions, needs_random) where
    needs_random marks robots the reference gives np_random.choice(4) instead."""
    R = n_robots
    c = cur - R
    r = cost[c, :].copy()
    vis = np.nonzero(visited_targets == 1)[0]
    r[:, vis] = MAX_COST
    # quirk (:818): the reference indexes with the (row, col) tuple of np.where on the
    # (T,1) visited column, so column 0 (the first target) is masked too whenever any
    # target is visited
    if len(vis):
        r[:, 0] = MAX_COST
    goal = np.argmin(r, axis=1)
    acts = np.zeros(R, np.int32)
    rand = np.zeros(R, bool)
    for i in range(R):
        if r[i, goal[i]] == MAX_COST or prev[goal[i], c[i]] == -1:
            rand[i] = True
            continue
        step = prev[goal[i], c[i]] + R
        acts[i] = int(np.nonzero(recv[i] == step)[0][0])
    return acts, rand


KEYS = ['nodes', 'edges', 'senders', 'receivers', 'step']  # coverage.py:90
N_GLOB_FEAT = 1   # coverage.py:59
MAX_EDGES = 4     # coverage.py:56


def flatten_obs(obs):
    """gym's FlattenDictWrapper.observation (used by the reference's test.py:33; gym
    itself is not vendored or installed, so this restates its published rule): ravel
    each value in key order and np.concatenate. The promotion of float32 nodes/edges,
    int32 senders/receivers and the int64 step gives float64."""
    return np.concatenate([np.asarray(obs[k]).ravel() for k in KEYS])


def unpack_obs(flat, dim_nodes=3):
    """unpack_obs, coverage.py:689-741, restated in NumPy (the reference needs
    TensorFlow, which is absent: parity unpinned beyond this restatement). flat is
    (B, L) float32, as the wrapper's Box declares. The senders are offset by the
    graph's first node BEFORE the padding test (:718-723), so only graph 0 loses its
    padded edges. Returns the graph tuple fields."""
    flat = np.asarray(flat, dtype=np.float32)
    B, L = flat.shape
    n_nodes = (L - N_GLOB_FEAT) // (MAX_EDGES * (2 + 1) + dim_nodes)
    max_n_edges = n_nodes * MAX_EDGES
    shapes = ((n_nodes, dim_nodes), (max_n_edges, 1), (max_n_edges, 1), (max_n_edges, 1), (1, N_GLOB_FEAT))
    sizes = [int(np.prod(s)) for s in shapes]
    parts = np.split(flat, np.cumsum(sizes)[:-1], axis=1)
    nodes, edges, senders, receivers, globs = [p.reshape((-1,) + s) for p, s in zip(parts, shapes)]
    nodes = nodes.reshape(-1, dim_nodes)
    n_node = np.full((B,), n_nodes)
    cum = (np.cumsum(n_node) - n_node).astype(np.float32).reshape(-1, 1, 1)
    senders = senders + cum
    receivers = receivers + cum
    mask = (senders != -1).reshape(B, -1)
    n_edge = mask.sum(axis=1)
    mask = mask.reshape(-1)
    edges = edges.reshape(-1, 1)[mask]
    senders = senders.reshape(-1)[mask]
    receivers = receivers.reshape(-1)[mask]
    return dict(n_node=n_node.astype(np.int32), nodes=nodes, n_edge=n_edge.astype(np.int32), edges=edges,
                senders=senders.astype(np.int32), receivers=receivers.astype(np.int32),
                globs=globs.reshape(B, N_GLOB_FEAT))

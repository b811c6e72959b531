"""Coverage-v0 on the MI355X engine — drop-in for gym_flock/envs/spatial/coverage.py.

Same constructor arguments, `keys`, spaces and methods as the reference
(`__init__` :83-164, `seed` :166-172, `step` :174-204, `reset` :366-425,
`closest_targets` :427-432, `controller` :800-872 with its random and greedy
branches, `construct_time_matrix` :621-653). The step — action
targets, collision-resolved moves, visited/reward and the padded graph observation —
and the per-graph setup (motion radius graph, static observation) run in
libgymflock.so (cov_* C-ABI). Host code keeps what the reference draws from its RNGs:
the target map (global np.random, maps.generate_targets) and reset()'s start and
unvisited draws (self.np_random), in the reference's call order.

Supported configuration: the module constants the reference ships with (PAD_ACTIONS,
COLLISION_CHECKS, PAD_NODES, distance edge features, HIDE_NODES False). Like the
reference, observations alias buffers that the next step overwrites only in the sense
that each call returns fresh host copies of the device arrays.
"""
import numpy as np

from ... import _native as nat
from ..._spaces import Box, Dict, Env, MultiDiscrete, np_random

N_NODE_FEAT = 3
N_EDGE_FEAT = 1
N_GLOB_FEAT = 1
MAX_NODES = 500
MAX_EDGES = 4
N_ACTIONS = 4
EPISODE_LENGTH = 75
HORIZON = 10
N_ROBOTS = 6
XMAX = 120
YMAX = 120
FRAC_ACTIVE = 0.5
NEARBY_STARTS = True
NEARBY_DENSITY = 5
DELTA = 5.5
N_CITIES = 12  # coverage.py:518
unvisited_regions = [(-100, 100, -100, 100)]
start_regions = [(-100, 100, -100, 100)]


MAX_COST = 1000  # coverage.py:68


class CoverageEnv(Env):
    def __init__(self, n_robots=N_ROBOTS, frac_active_targets=FRAC_ACTIVE, xmax=XMAX, ymax=YMAX,
                 starts=start_regions, unvisiteds=unvisited_regions, init_graph=True,
                 episode_length=EPISODE_LENGTH, res=DELTA, pad_nodes=True, max_nodes=MAX_NODES,
                 nearby_starts=NEARBY_STARTS, horizon=HORIZON, hide_nodes=False,
                 n_node_feat=N_NODE_FEAT, device=0):
        super(CoverageEnv, self).__init__()
        if hide_nodes or not pad_nodes or n_node_feat != N_NODE_FEAT:
            raise NotImplementedError("only the reference's shipped configuration (PAD_NODES, no hidden nodes, "
                                      "3 node features) is implemented")
        self.keys = ['nodes', 'edges', 'senders', 'receivers', 'step']
        self.n_node_feat = n_node_feat
        self.hide_nodes = hide_nodes
        self.horizon = horizon
        self.episode_length = episode_length
        self.nearby_starts = nearby_starts
        self.pad_nodes = pad_nodes
        self.max_nodes = max_nodes
        self.x_min, self.x_max, self.y_min, self.y_max = -xmax, xmax, -ymax, ymax
        self.res = res
        self.start_ranges = starts
        self.unvisited_ranges = unvisiteds
        self.np_random = None
        self.seed()
        self.nx = 2
        self.nu = 2
        self.n_robots = n_robots
        self.frac_active_targets = frac_active_targets
        self.comm_radius = 100.0
        self.motion_radius = self.res * 1.2
        self.obs_radius = self.res * 1.2
        self.n_actions = N_ACTIONS
        self.device = device
        self._h = nat.CoverageHandle(n_robots, 1, max_nodes, episode_length, res, self.motion_radius, device,
                                     horizon=horizon)
        self._map_cfg = nat.map_config_default(self.motion_radius, xmax, ymax, N_CITIES, DELTA)
        self.map_status = 0  # cov_generate_maps status bits of the current map
        if init_graph:
            try:
                targets, _ = self._generate_targets()
                self._initialize_graph(targets, on_device=True)
            except ValueError:
                # the reference builds this map's arrays and only fails when an observation
                # of it is taken (reset() draws a new map first)
                self.n_targets = None
        self.episode_reward = 0
        self.step_counter = 0
        self.last_loc = None
        self.fig = None
        # how step() runs: "direct" = one cov_step_host call (actions in the kernel
        # arguments, observation / reward / done / each robot's new node written by the
        # step into one pooled page-locked block, one wait); "getters" = cov_step, then
        # the observation and reward getters (a host round trip each)
        self.fetch_mode = "direct"
        self._closest = None       # robots' nodes after the last step (the next last_loc)
        self._want_greedy = False  # controller(greedy=True) in use: steps fuse the next one
        self._greedy_cache = None  # (actions, needs_random) of the current state, device-made
        self._motion_cache = None  # the motion graph's (senders, receivers), per graph
        self._abuf = None
        self._layout = None

    def seed(self, seed=None):
        self.np_random, seed = np_random(seed)
        return [seed]

    # --------------------------------------------------------------- graph setup
    def _generate_targets(self):
        """coverage.py:516-527. The 12 cities come from the global np.random here, drawn
        exactly as make_map.py:208 draws them; their Delaunay roads, the lattice points near
        them and the largest component of those points' radius graph are computed on the
        device, which then builds the motion graph too (cov_generate_maps). A map with more
        targets than max_nodes - n_robots raises (the reference's padded arrays cannot hold
        it either)."""
        cities = np.random.uniform(-self.x_max, self.x_max, size=(N_CITIES, 2))
        try:
            n, st, _ = self._h.generate_maps(cities=cities[None], env=0, map_config=self._map_cfg)
        except nat.GymFlockError as e:
            st = getattr(e, "status", None)
            if st is None or not st[0] & (nat.COV_MAP_TOO_MANY | nat.COV_MAP_TOO_FEW):
                raise
            self.map_status = int(st[0])
            # the reference fails here too, in _get_obs_reward (:325) with a ValueError: its
            # padded (max_nodes, 3) arrays cannot take n_targets + n_robots nodes
            raise ValueError("could not fit a map of %d targets and %d robots into max_nodes = %d (%s)"
                             % (int(e.n_targets[0]), self.n_robots, self.max_nodes, e)) from e
        self.map_status = int(st[0])
        return self._h.targets(0, int(n[0])), True

    def _initialize_graph(self, targets, on_device=False):
        """coverage.py:529-619; the motion graph itself is built on the device
        (on_device: it already was, by _generate_targets)."""
        self.targets = np.asarray(targets, dtype=np.float64)
        self.n_targets = self.targets.shape[0]
        self.n_agents = self.n_targets + self.n_robots
        self.max_edges = self.max_nodes * MAX_EDGES
        if not on_device:
            self._h.set_targets(self.targets, env=0)
        self._closest = self._greedy_cache = self._motion_cache = None
        self.n_motion_edges = int(self._h.n_motion()[0])
        if self.nearby_starts:
            n_nearest = self.get_n_nearest(self.np_random.choice(self.n_targets), self.n_robots * NEARBY_DENSITY)
            region = np.zeros(self.n_targets, bool)
            region[list(n_nearest)] = True
            self.start_region = region.tolist()  # [i in n_nearest for i in range(n_targets)]
        else:
            self.start_region = [True] * self.n_targets
        self.unvisited_region = [True] * self.n_targets
        self.action_space = MultiDiscrete([self.n_actions] * self.n_robots)
        self.observation_space = Dict([
            ("nodes", Box(shape=(self.max_nodes, self.n_node_feat), low=-np.inf, high=np.inf, dtype=np.float32)),
            ("edges", Box(shape=(self.max_edges, N_EDGE_FEAT), low=-np.inf, high=np.inf, dtype=np.float32)),
            ("senders", Box(shape=(self.max_edges, 1), low=0, high=self.n_agents, dtype=np.float32)),
            ("receivers", Box(shape=(self.max_edges, 1), low=0, high=self.n_agents, dtype=np.float32)),
            ("step", Box(shape=(1, 1), low=0, high=EPISODE_LENGTH, dtype=np.float32)),
        ])

    @property
    def motion_edges(self):
        """(senders, receivers) of the motion graph, global node indices (:572-594): read
        from the device once per graph (it only changes with the map), then the same arrays,
        as the reference's attribute."""
        if self._motion_cache is None:
            s, q = self._h.motion_edges(0, self.n_motion_edges)
            self._motion_cache = (s.astype(np.int64), q.astype(np.int64))
        return self._motion_cache

    def get_n_nearest(self, i, n):
        """coverage.py:655-673: grow a node set through the motion graph until it holds n."""
        s, q = self.motion_edges
        s, q = s - self.n_robots, q - self.n_robots
        n_nearest = {i}
        while len(n_nearest) < n:
            n_nearest = n_nearest.union(set(q[np.isin(s, list(n_nearest))].tolist()))
        return n_nearest

    # --------------------------------------------------------------------- API
    def reset(self):
        """coverage.py:366-425."""
        self.episode_reward = 0
        self.step_counter = 0
        self.last_loc = None
        targets, graph_changed = self._generate_targets()
        if graph_changed:
            self._initialize_graph(targets, on_device=True)
        starts = self.np_random.choice(np.arange(self.n_targets)[self.start_region], size=(self.n_robots,),
                                       replace=False)
        unvisited = np.arange(self.n_targets)[self.unvisited_region] + self.n_robots
        drop = self.np_random.choice(unvisited, size=(int(len(unvisited) * self.frac_active_targets),),
                                     replace=False)
        visited = np.ones((1, self._h.t_max), np.uint8)
        visited[0, drop - self.n_robots] = 0
        self._h.reset(starts[None], visited)
        self.step_counter = 1
        self._closest = starts.astype(np.int64) + self.n_robots  # robots sit on their start targets
        self._greedy_cache = None
        return self._h.obs(0)

    def step(self, action):
        """coverage.py:174-204 (with _get_obs_reward :234-364). In the default fetch mode
        ("direct") one library call with one wait (cov_step_host): the actions travel in
        the kernel arguments and the step writes the whole observation, reward, done flag
        and each robot's new node (the next step's last_loc) into one pooled page-locked
        block; once controller(greedy=True) is in use, the expert's actions for the
        resulting state are computed in the same launch."""
        if action is None:  # pragma: no cover (the reference skips the move)
            self._h.step(np.zeros((1, self.n_robots)))
            return self._obs_reward()
        a = np.asarray(action).reshape(-1)
        if a.shape[0] != self.n_robots or np.any((a < 0) | (a >= self.n_actions)):
            raise IndexError("each robot's action must be in [0, %d)" % self.n_actions)
        self.last_loc = self._closest if self._closest is not None else self.closest_targets
        if self.fetch_mode != "direct":
            self._h.step(a[None])
            self._closest = self._greedy_cache = None
            return self._obs_reward()
        R, M = self.n_robots, self.max_nodes
        if self._abuf is None:
            self._abuf = np.empty((1, R), np.int32)
        self._abuf[0] = a
        ng = self._want_greedy
        lay = self._layout
        if lay is None or lay[0] != ng:
            a64 = lambda b: (b + 63) & ~63  # noqa: E731
            o = [0]
            for nbytes in (12 * M, 16 * M, 16 * M, 16 * M, 8, 8, 1, 4 * R, 4 * R if ng else 0, R if ng else 0):
                o.append(o[-1] + a64(nbytes))
            lay = self._layout = (ng, o)
        o = lay[1]
        buf, base = nat.host_pool().block_addr(o[-1])
        if buf is None:  # not page-locked (pool cap): the library copies after the launch
            buf = np.empty(o[-1], np.uint8)
            base = buf.ctypes.data
        nodes = np.ndarray((M, 3), np.float32, buf, o[0])
        edges = np.ndarray((4 * M, 1), np.float32, buf, o[1])
        snd = np.ndarray((4 * M,), np.int32, buf, o[2])
        rcv = np.ndarray((4 * M,), np.int32, buf, o[3])
        stp = np.ndarray((1, 1), np.int64, buf, o[4])
        rw = np.ndarray((1,), np.float64, buf, o[5])
        dn = np.ndarray((1,), np.uint8, buf, o[6])
        cl = np.ndarray((R,), np.int32, buf, o[7])
        nxt = np.ndarray((R,), np.int32, buf, o[8]) if ng else None
        nrd = np.ndarray((R,), np.uint8, buf, o[9]) if ng else None
        self._h.step_host(self._abuf, base + o[0], base + o[1], base + o[2], base + o[3], base + o[4], base + o[5],
                          base + o[6], base + o[7], base + o[8] if ng else None, base + o[9] if ng else None)
        self._closest = cl.astype(np.int64)
        self._greedy_cache = (nxt.copy(), nrd.astype(bool)) if ng else None
        reward, done = float(rw[0]), bool(dn[0])
        self.step_counter += 1
        self.episode_reward += reward
        return {"nodes": nodes, "edges": edges, "senders": snd, "receivers": rcv, "step": stp}, reward, done, {}

    def _obs_reward(self):
        obs = self._h.obs(0)
        r, d = self._h.rewards()
        reward, done = float(r[0]), bool(d[0])
        self.step_counter += 1
        self.episode_reward += reward
        return obs, reward, done, {}

    def get_action_edges(self):
        """coverage.py:206-232: each robot's 4 action targets (its node's out-neighbours in
        ascending order, padded with its own node) as ((senders, receivers), dists, diff),
        read from the device observation's action-edge tail."""
        o = self._h.obs(0)
        R = self.n_robots
        base = self.max_edges - 4 * R
        senders = o["senders"][base:].astype(np.int64)
        receivers = o["receivers"][base:].astype(np.int64)
        x = self.x
        diff = x[senders, :] - x[receivers, :]
        return (senders, receivers), np.linalg.norm(diff, axis=1), diff

    @property
    def closest_targets(self):
        """coverage.py:427-432 (global node indices)."""
        return self._h.robots(0)[1].astype(np.int64)

    @property
    def x(self):
        xr, _ = self._h.robots(0)
        return np.vstack([xr, self.targets])

    @property
    def visited(self):
        return np.r_[np.ones(self.n_robots), self._h.visited(0)[:self.n_targets]].reshape(-1, 1)

    def controller(self, random=False, greedy=False, reset_solution=False):
        """coverage.py:800-872. random: np_random.choice over the 4 actions. greedy: the
        device expert (time matrix :621-653 built once per graph, nearest unvisited target,
        next hop from the predecessor matrix); robots it cannot route draw
        np_random.choice(4) here, in robot order, as the reference does (:863-864).
        The OR-Tools routing branch (greedy=False) is out of scope: it
        fails the way the reference does without OR-Tools installed."""
        if random:
            return self.np_random.choice(self.n_actions, size=(self.n_robots, 1))
        if not greedy:
            raise AssertionError("Vehicle routing controller is not available if OR-Tools is not imported.")
        self._want_greedy = True
        if self._greedy_cache is not None:  # computed by the step that made this state
            a, rnd = self._greedy_cache
            a = a.copy()
        else:
            a, rnd = self._h.controller_greedy()
            a, rnd = a[0].copy(), rnd[0]
        k = np.nonzero(rnd)[0]
        if len(k):  # one draw per robot in robot order: a batched draw is the same stream
            a[k] = self.np_random.choice(self.n_actions, size=len(k))
        return a.reshape(self.n_robots, 1).astype(np.int32)

    def construct_time_matrix(self, edge_time=1.0):
        """coverage.py:621-653 on the device: (time_matrix with inf -> MAX_COST, prev)."""
        if edge_time != 1.0:
            raise NotImplementedError("only the reference's uniform edge_time=1.0 is implemented")
        cost, prev = self._h.time_matrix(0, self.n_targets)
        return cost.astype(np.float64), prev.astype(np.int64)

    @property
    def graph_cost(self):
        return self.construct_time_matrix()[0]

    @property
    def graph_previous(self):
        return self.construct_time_matrix()[1]

    @property
    def graph_diameter(self):
        c = self.graph_cost
        return np.max(c[c < MAX_COST])

    @staticmethod
    def get_number_nodes(ob_space, n_node_feat=None):
        """coverage.py:675-680: node count of a flattened observation space."""
        if n_node_feat is None:
            n_node_feat = N_NODE_FEAT
        return (ob_space.shape[0] - N_GLOB_FEAT) // (MAX_EDGES * (2 + N_EDGE_FEAT) + n_node_feat)

    @staticmethod
    def get_node_features(n_node_feat=None):
        """coverage.py:682-687 (always N_NODE_FEAT)."""
        return N_NODE_FEAT

    @staticmethod
    def unpack_obs(obs, ob_space, dim_nodes=None):
        """coverage.py:689-741 without TensorFlow. obs is (B, L) flattened
        observations; it returns NumPy arrays in the reference's order (batch_size,
        n_node, nodes, n_edge, edges, senders, receivers, globs). Like the reference,
        the senders are offset by each graph's first node before the padding test, so
        only graph 0 drops its padded edges. For the device-side batch use
        VecCoverage.graphs_tuple()."""
        if dim_nodes is None:
            dim_nodes = N_NODE_FEAT
        obs = np.asarray(obs, dtype=np.float32)
        n_nodes = (ob_space.shape[0] - N_GLOB_FEAT) // (MAX_EDGES * (2 + N_EDGE_FEAT) + dim_nodes)
        max_n_edges = n_nodes * MAX_EDGES
        shapes = ((n_nodes, dim_nodes), (max_n_edges, N_EDGE_FEAT), (max_n_edges, 1), (max_n_edges, 1),
                  (1, N_GLOB_FEAT))
        sizes = [int(np.prod(sh)) for sh in shapes]
        parts = np.split(obs, np.cumsum(sizes)[:-1], axis=1)
        nodes, edges, senders, receivers, globs = [p.reshape((-1,) + sh) for p, sh in zip(parts, shapes)]
        batch_size = nodes.shape[0]
        nodes = nodes.reshape(-1, dim_nodes)
        n_node = np.full((batch_size,), n_nodes, dtype=np.int32)
        cum = (np.cumsum(n_node) - n_node).astype(np.float32).reshape(-1, 1, 1)
        senders = senders + cum
        receivers = receivers + cum
        mask = (senders != -1).reshape(batch_size, -1)
        n_edge = mask.sum(axis=1).astype(np.int32)
        mask = mask.reshape(-1)
        edges = edges.reshape(-1, N_EDGE_FEAT)[mask]
        senders = senders.reshape(-1)[mask].astype(np.int32)
        receivers = receivers.reshape(-1)[mask].astype(np.int32)
        return batch_size, n_node, nodes, n_edge, edges, senders, receivers, globs.reshape(batch_size, N_GLOB_FEAT)

    @staticmethod
    def unpack_obs_state(obs, ob_space, state, dim_state, dim_nodes=None):
        """coverage.py:744-798 without TensorFlow: unpack_obs plus the node features
        extended by each half of a (B*n_nodes, 2*dim_state) state, giving nodes1 and nodes2."""
        batch_size, n_node, nodes, n_edge, edges, senders, receivers, globs = CoverageEnv.unpack_obs(
            obs, ob_space, dim_nodes)
        st = np.asarray(state, dtype=np.float32).reshape(-1, dim_state * 2)
        nodes1 = np.concatenate([nodes, st[:, :dim_state]], axis=1)
        nodes2 = np.concatenate([nodes, st[:, dim_state:]], axis=1)
        return batch_size, n_node, nodes1, nodes2, n_edge, edges, senders, receivers, globs

    def render(self, mode='human'):
        pass

    def close(self):
        if self._h is not None:
            self._h.close()
            self._h = None

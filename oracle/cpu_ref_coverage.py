"""CPU baseline for bench.py's Coverage line (config 4): the reference's CoverageEnv.step
as its own sequence of Python loops and NumPy operations.

TEST/BENCH INFRASTRUCTURE ONLY (the `cpu_baseline` leg of bench.py's coverage_config4;
checked by scripts/check_cpu_ref.py and tests/test_oracle_coverage.py). The product
(gym-flock_amd/) never imports it.

oracle/coverage.py is the parity checker: it keeps a neighbour table and resolves the
claims with a set, which makes it several times faster than the reference and so a
flattering baseline. This module performs the reference's own operations, in its order,
so its time is the reference's time on the same host:

  step              coverage.py:174-204   closest_targets (R x T norm + argmin); per robot an
                                          np.where over the action-edge list; stay claims; a
                                          second per-robot loop with a second np.where and a
                                          list-membership collision test; position copies
  get_action_edges  :206-232              closest_targets again; per robot an np.where over
                                          the motion-edge list, np.append padding and
                                          concatenation; linalg.norm of the edge vectors
  _get_obs_reward   :234-364              doubled edge lists, a third closest_targets for the
                                          visited flags, the padded observation rewritten
                                          (senders/receivers tails, nodes.fill, node
                                          features), reward and done sums

The module configuration is the one the reference ships with (PAD_ACTIONS,
COLLISION_CHECKS, no comm edges, no node history, no hidden nodes, distance edge
features, coverage.py:38-62). The returned observation arrays alias the env's buffers,
as the reference's do (coverage.py:317-327, :353).
"""
import numpy as np

from oracle.coverage import EPISODE_LENGTH, MAX_EDGES, N_ACTIONS, RES

N_EDGE_FEAT = 1  # coverage.py:35
N_NODE_FEAT = 3  # coverage.py:34


class CpuCoverage:
    """One CoverageEnv's arrays (_initialize_graph, coverage.py:529-594) for a given target
    set; motion edges from _get_graph_edges(motion_radius, targets, self_loops=True)
    (utils.py:8-24: np.linalg.norm, r > rad -> 0, np.nonzero)."""

    def __init__(self, targets, n_robots, max_nodes, motion_radius=RES * 1.2):
        targets = np.asarray(targets, dtype=np.float64)
        self.n_robots = n_robots
        self.n_targets = targets.shape[0]
        self.n_agents = self.n_targets + n_robots
        self.max_nodes = max_nodes
        self.max_edges = max_nodes * MAX_EDGES
        self.res = RES
        self.x = np.zeros((self.n_agents, 2))
        self.x[n_robots:, 0:2] = targets
        self.robot_flag = np.vstack((np.ones((n_robots, 1)), np.zeros((self.n_targets, 1))))
        self.landmark_flag = np.vstack((np.zeros((n_robots, 1)), np.ones((self.n_targets, 1))))
        self.edges = np.zeros((self.max_edges, N_EDGE_FEAT), dtype=np.float32)
        self.nodes = np.zeros((self.max_nodes, N_NODE_FEAT), dtype=np.float32)
        self.senders = -1 * np.ones((self.max_edges,), dtype=np.int32)
        self.receivers = -1 * np.ones((self.max_edges,), dtype=np.int32)
        self.visited = np.ones((self.n_agents, 1))
        pos = self.x[n_robots:, 0:2]
        diff = pos.reshape((-1, 1, 2)) - pos.reshape((1, -1, 2))
        r = np.linalg.norm(diff, axis=2)
        r[r > motion_radius] = 0
        e = np.nonzero(r)
        self.motion_edges = (e[0] + n_robots, e[1] + n_robots)
        self.n_motion_edges = len(self.motion_edges[0])
        self.senders[:self.n_motion_edges] = self.motion_edges[0]
        self.receivers[:self.n_motion_edges] = self.motion_edges[1]
        self.edges[:self.n_motion_edges, 0] = r[e].reshape((-1,))
        self.step_counter = 0
        self.last_loc = None
        self.mov_edges = None

    def reset(self, start_targets, unvisited_targets):
        """reset() after its random draws (coverage.py:404-424): robots on start_targets
        (target-local indices), unvisited_targets (global indices) unvisited."""
        self.step_counter = 0
        self.last_loc = None
        self.x[:self.n_robots, 0:2] = self.x[np.asarray(start_targets) + self.n_robots, 0:2]
        self.visited.fill(1)
        self.visited[np.asarray(unvisited_targets)] = 0
        obs, _, _ = self._get_obs_reward()
        return obs

    # coverage.py:427-432
    @property
    def closest_targets(self):
        r = np.linalg.norm(self.x[:self.n_robots, 0:2].reshape((self.n_robots, 1, 2))
                           - self.x[self.n_robots:, 0:2].reshape((1, self.n_targets, 2)), axis=2)
        return np.argmin(r, axis=1) + self.n_robots

    # coverage.py:174-204
    def step(self, action):
        if type(action) == np.ndarray:
            action = action.flatten().tolist()
        self.last_loc = self.closest_targets
        next_locs = [-1] * len(action)
        for i in range(self.n_robots):
            cur_robot_edges = np.where(self.mov_edges[0] == i)
            next_loc = self.mov_edges[1][cur_robot_edges][action[i]]
            if next_loc == self.last_loc[i]:
                next_locs[i] = next_loc
        for i in range(self.n_robots):
            if next_locs[i] == -1:
                next_loc = self.mov_edges[1][np.where(self.mov_edges[0] == i)][action[i]]
                if next_loc not in next_locs:
                    next_locs[i] = next_loc
                    self.x[i, 0:2] = self.x[next_loc, 0:2]
                else:
                    next_locs[i] = self.last_loc[i]
        obs, reward, done = self._get_obs_reward()
        return obs, reward, done, {}

    # coverage.py:206-232
    def get_action_edges(self):
        senders = np.zeros((0,))
        receivers = np.zeros((0,))
        curr_nodes = self.closest_targets
        for i in range(self.n_robots):
            next_nodes = self.motion_edges[1][np.where(self.motion_edges[0] == curr_nodes[i])]
            n_next_nodes = np.shape(next_nodes)[0]
            if n_next_nodes < N_ACTIONS:
                next_nodes = np.append(next_nodes, [curr_nodes[i]] * (N_ACTIONS - n_next_nodes))
            senders = np.append(senders, [i] * 4)
            receivers = np.append(receivers, next_nodes)
        senders = senders.astype(int)
        receivers = receivers.astype(int)
        diff = self.x[senders, :] - self.x[receivers, :]
        dists = np.linalg.norm(self.x[senders, :] - self.x[receivers, :], axis=1)
        return (senders, receivers), dists, diff

    # coverage.py:234-364 (the branches the shipped module flags select)
    def _get_obs_reward(self):
        action_edges, action_dist, _ = self.get_action_edges()
        assert len(action_edges[0]) == N_ACTIONS * self.n_robots
        action_edges = (np.concatenate([action_edges[0], action_edges[1]], axis=0),
                        np.concatenate([action_edges[1], action_edges[0]], axis=0))
        action_dist = np.concatenate([action_dist, action_dist], axis=0)
        self.mov_edges = action_edges
        old_sum = np.sum(self.visited[self.n_robots:self.n_agents])
        self.visited[self.closest_targets] = 1
        senders = action_edges[1]
        receivers = action_edges[0]
        edges_dist = action_dist.reshape((-1, 1))
        assert len(senders) + self.n_motion_edges <= np.shape(self.senders)[0], "Increase MAX_EDGES"
        edges_dist = edges_dist / self.res
        edges = edges_dist.reshape((-1, 1))
        self.senders[self.n_motion_edges:] = -1
        self.receivers[self.n_motion_edges:] = -1
        self.nodes.fill(0)
        self.senders[-len(senders):] = senders
        self.receivers[-len(receivers):] = receivers
        self.edges[-len(senders):, :] = edges
        self.nodes[0:self.n_agents, 0] = self.robot_flag.flatten()
        self.nodes[0:self.n_agents, 1] = self.landmark_flag.flatten()
        self.nodes[0:self.n_agents, 2] = np.logical_not(self.visited).flatten()
        step_array = np.array([self.step_counter]).reshape((1, 1))
        obs = {'nodes': self.nodes, 'edges': self.edges, 'senders': self.senders, 'receivers': self.receivers,
               'step': step_array}
        self.step_counter += 1
        done = self.step_counter == EPISODE_LENGTH or np.sum(self.visited[self.n_robots:]) == self.n_targets
        reward = np.sum(self.visited[self.n_robots:]) - old_sum
        return obs, reward, done

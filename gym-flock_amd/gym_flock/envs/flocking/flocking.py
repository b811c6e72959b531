"""Flocking-v0 on the MI355X engine — drop-in for gym_flock/envs/flocking/flocking.py.

The observation is each agent's state relative to its n_neighbors (=7, :9) nearest
agents by r2 (:20-25), computed by the k-nearest HIP kernel. Ties between equal r2
resolve to the lower index (the reference's np.argsort is an unstable quicksort, so
its tie order is unspecified); indices are otherwise bit-exact.
"""
import numpy as np

from ... import _native as nat
from .flocking_relative import FlockingRelativeEnv


class FlockingEnv(FlockingRelativeEnv):

    def __init__(self, device=0):
        super(FlockingEnv, self).__init__(device)
        self.n_neighbors = 7
        self.n_f = self.nx_system * self.n_neighbors
        self.nearest = None

    def step(self, u):
        """:12-14."""
        u = np.asarray(u)
        assert u.shape == (self.n_agents, self.nu)
        self.u = u * self.action_scalar
        self._handle().step(u[None], flags=nat.FE_WITH_KNN)
        self._ctrl_cache = None
        self._fetch_obs()
        return (self.get_observation(), self.state_network), self.instant_cost(), False, {}

    def reset(self):
        """:16-18."""
        super(FlockingEnv, self).reset()
        return self.get_observation(), self.state_network

    def get_observation(self):
        """:20-25 — (N, 4*n_neighbors) float32: x_i - x_{nn_k(i)} for k < n_neighbors."""
        idx, obs = self._handle().knn(0)
        self.nearest = idx
        return obs

"""Module path of the reference's gym_flock/envs/flocking/flocking_stoch.py; the env is
implemented in variants.py on the shared step kernel."""
from gym_flock.envs.flocking.variants import FlockingStochasticEnv

__all__ = ["FlockingStochasticEnv"]

"""Module path of the reference's gym_flock/envs/flocking/flocking_leader.py; the env is
implemented in variants.py on the shared step kernel."""
from gym_flock.envs.flocking.variants import FlockingLeaderEnv

__all__ = ["FlockingLeaderEnv"]

"""Module path of the reference's gym_flock/envs/flocking/flocking_twoflocks.py; the env is
implemented in variants.py on the shared step kernel."""
from gym_flock.envs.flocking.variants import FlockingTwoFlocksEnv

__all__ = ["FlockingTwoFlocksEnv"]

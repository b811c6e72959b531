"""Flocking envs (reference: gym_flock/envs/flocking/__init__.py)."""
from gym_flock.envs.flocking.flocking_relative import FlockingRelativeEnv
from gym_flock.envs.flocking.flocking import FlockingEnv
from gym_flock.envs.flocking.variants import (FlockingLeaderEnv, FlockingObstacleEnv,
                                              FlockingStochasticEnv, FlockingTwoFlocksEnv)

__all__ = ["FlockingRelativeEnv", "FlockingEnv", "FlockingLeaderEnv", "FlockingObstacleEnv",
           "FlockingStochasticEnv", "FlockingTwoFlocksEnv"]

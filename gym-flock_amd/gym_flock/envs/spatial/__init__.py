"""Spatial (graph coverage) envs (reference: gym_flock/envs/spatial/__init__.py)."""
from gym_flock.envs.spatial.coverage import CoverageEnv

__all__ = ["CoverageEnv"]

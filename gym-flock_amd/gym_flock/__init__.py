"""gym_flock on MI355X: drop-in replacement for katetolstaya/gym-flock's env-step hot path.

Importing the package registers the env ids it implements with gym (when gym is
installed), using the reference's ids, entry points and episode limits
(reference gym_flock/__init__.py:40-94). The per-step work runs in libgymflock.so
(HIP, gfx950) through a ctypes C-ABI; see include/gymflock.h.
"""
from gym_flock._spaces import HAVE_GYM

__version__ = "0.1.0"

# id -> (entry point, max_episode_steps); reference gym_flock/__init__.py
ENV_IDS = {
    "FlockingRelative-v0": ("gym_flock.envs.flocking:FlockingRelativeEnv", 1000),  # :59-63
    "Flocking-v0": ("gym_flock.envs.flocking:FlockingEnv", 1000),                  # :53-57
    "Coverage-v0": ("gym_flock.envs.spatial:CoverageEnv", 75),                     # :40-44
    "FlockingLeader-v0": ("gym_flock.envs.flocking:FlockingLeaderEnv", 200),        # :65-69
    "FlockingObstacle-v0": ("gym_flock.envs.flocking:FlockingObstacleEnv", 200),    # :72-76
    "FlockingStochastic-v0": ("gym_flock.envs.flocking:FlockingStochasticEnv", 500),  # :84-88
    "FlockingTwoFlocks-v0": ("gym_flock.envs.flocking:FlockingTwoFlocksEnv", 500),  # :90-94
}

if HAVE_GYM:  # pragma: no cover - gym is not installed in the build image
    from gym.envs.registration import register

    for _id, (_ep, _steps) in ENV_IDS.items():
        try:
            register(id=_id, entry_point=_ep, max_episode_steps=_steps)
        except Exception:  # already registered (e.g. the reference package is also installed)
            pass


def make(env_id, **kwargs):
    """gym.make() equivalent that works without gym (no TimeLimit wrapper)."""
    import importlib
    mod, cls = ENV_IDS[env_id][0].split(":")
    return getattr(importlib.import_module(mod), cls)(**kwargs)

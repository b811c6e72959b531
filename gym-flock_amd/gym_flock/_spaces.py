"""gym.Env / gym.spaces when gym is installed, minimal stand-ins otherwise.

The reference depends on gym 0.11 (README.md:4); the engine itself does not, so the
env classes here subclass gym.Env only when it can be imported.
"""
import numpy as np

try:  # pragma: no cover - gym is not installed in the build image
    import gym as _gym
    from gym import spaces as _spaces

    Env = _gym.Env
    Box, MultiDiscrete, Dict = _spaces.Box, _spaces.MultiDiscrete, _spaces.Dict
    HAVE_GYM = True
except ImportError:
    HAVE_GYM = False

    class Env:
        """Stand-in for gym.Env (reset/step/render/close/seed)."""

        metadata = {"render.modes": ["human"]}

        def close(self):
            pass

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)

        def sample(self, rng=np.random):
            lo = np.broadcast_to(np.asarray(self.low, dtype=np.float64), self.shape)
            hi = np.broadcast_to(np.asarray(self.high, dtype=np.float64), self.shape)
            return rng.uniform(lo, hi).astype(self.dtype)

    class MultiDiscrete:
        def __init__(self, nvec):
            self.nvec = np.asarray(nvec)
            self.shape = self.nvec.shape

    class Dict:
        def __init__(self, spaces):
            self.spaces = dict(spaces)


def np_random(seed=None):
    """gym.utils.seeding.np_random equivalent: (RandomState, seed)."""
    return np.random.RandomState(seed), seed

"""Observation / action spaces.

Uses ``gym.spaces`` when gym is importable (so wrappers that type-check spaces work);
otherwise a minimal Box/Dict with gym's semantics: low/high cast to ``dtype`` (float32 by
default), ``sample`` = uniform(low, high).astype(dtype), ``contains`` = shape + bounds.
"""
import numpy as np

try:  # pragma: no cover - gym is not installed in the build image
    import gym as _gym
    Box = _gym.spaces.Box
    Dict = _gym.spaces.Dict
    GoalEnvBase = _gym.GoalEnv
except Exception:  # noqa: BLE001
    _gym = None

    class Box(object):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            low = np.asarray(low)
            high = np.asarray(high)
            if shape is None:
                shape = np.broadcast(low, high).shape
            self.shape = tuple(shape)
            self.low = np.broadcast_to(low, self.shape).astype(self.dtype)
            self.high = np.broadcast_to(high, self.shape).astype(self.dtype)
            self.np_random = np.random.RandomState()

        def seed(self, seed=None):
            self.np_random = np.random.RandomState(seed)
            return [seed]

        def sample(self):
            return self.np_random.uniform(low=self.low, high=self.high, size=self.shape).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

        def __repr__(self):
            return "Box(%s, %s)" % (self.shape, self.dtype)

    class Dict(object):
        def __init__(self, spaces):
            self.spaces = dict(spaces)

        def __getitem__(self, k):
            return self.spaces[k]

        def contains(self, x):
            return isinstance(x, dict) and all(k in x and s.contains(x[k]) for k, s in self.spaces.items())

    class GoalEnvBase(object):
        metadata = {"render.modes": []}

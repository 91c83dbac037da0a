"""Observation/action spaces of the Gym surface.

Uses gymnasium's spaces when gymnasium is installed (the reference depends on
it: block_blast_env.py:9-10, 79-98); otherwise small stand-ins with the
attributes the reference's callers read (``.spaces``, ``.n``, ``.shape``,
``.dtype``, ``.sample()``).
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - depends on the image
    import gymnasium as _gym
    from gymnasium import spaces as _spaces

    Env = _gym.Env
    Wrapper = _gym.Wrapper
    Box = _spaces.Box
    Discrete = _spaces.Discrete
    Dict = _spaces.Dict
    HAVE_GYMNASIUM = True
except Exception:  # gymnasium absent
    HAVE_GYMNASIUM = False

    class Env:  # minimal gym.Env stand-in
        metadata: dict = {}

        def reset(self, seed=None, options=None):
            return None

    class Wrapper(Env):  # minimal gym.Wrapper stand-in: delegate to the wrapped env
        def __init__(self, env):
            self.env = env
            self.observation_space = env.observation_space
            self.action_space = env.action_space

        def step(self, action):
            return self.env.step(action)

        def reset(self, **kwargs):
            return self.env.reset(**kwargs)

        def render(self):
            return self.env.render()

        def close(self):
            return self.env.close()

        @property
        def unwrapped(self):
            return getattr(self.env, "unwrapped", self.env)

        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(name)
            return getattr(self.env, name)

    class Box:
        def __init__(self, low, high, shape, dtype):
            self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)

        def sample(self):
            return np.random.uniform(self.low, self.high, self.shape).astype(self.dtype)

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"

    class Discrete:
        def __init__(self, n: int):
            self.n = int(n)
            self.shape = ()
            self.dtype = np.dtype(np.int64)

        def sample(self):
            return int(np.random.randint(self.n))

        def contains(self, x) -> bool:
            return 0 <= int(x) < self.n

        def __repr__(self):
            return f"Discrete({self.n})"

    class Dict:
        def __init__(self, spaces: dict):
            self.spaces = dict(spaces)

        def __getitem__(self, k):
            return self.spaces[k]

        def sample(self):
            return {k: s.sample() for k, s in self.spaces.items()}

        def __repr__(self):
            return f"Dict({self.spaces})"

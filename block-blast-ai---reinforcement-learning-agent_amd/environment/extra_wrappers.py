"""Host-side single-env wrappers of the reference (wrappers.py:144-309): reward
normalisation by the running variance of the discounted return, board frame
stacking, and the ``make_env`` factory.  They wrap the N=1 ``BlockBlastEnv``
and do no GPU work of their own, so they are plain numpy: a drop-in for the
reference's classes with the same constructor arguments, attributes
(``return_rms``, ``returns``, ``num_frames``) and arithmetic order."""
from __future__ import annotations

from collections import deque
from typing import Dict, Optional, Tuple

import numpy as np

from .block_blast_env import BlockBlastEnv
from .spaces import Box, Dict as DictSpace, Wrapper


class RunningMeanStd:
    """Running mean / variance merged batch by batch with Chan et al.'s
    parallel update in fp64 (wrappers.py:186-223); ``count`` starts at the
    pseudo-count ``epsilon`` of the prior moments (mean 0, variance 1)."""

    def __init__(self, epsilon: float = 1e-4, shape: Tuple[int, ...] = ()):
        self.mean = np.zeros(shape, dtype=np.float64)
        self.var = np.ones(shape, dtype=np.float64)
        self.count = epsilon

    def update(self, x: np.ndarray) -> None:
        batch = np.asarray(x)
        self.merge(batch.mean(axis=0), batch.var(axis=0), batch.shape[0])

    def merge(self, mean_b, var_b, n_b) -> None:
        """Fold in a batch of n_b samples with moments (mean_b, var_b)."""
        n_a = self.count
        n = n_a + n_b
        d = mean_b - self.mean
        # sum of squared deviations of the union, then the mean: the reference's operation order
        ss = self.var * n_a + var_b * n_b + np.square(d) * n_a * n_b / n
        self.mean, self.var, self.count = self.mean + d * n_b / n, ss / n, n

    _update_from_moments = merge  # the reference's name


class NormalizedRewardWrapper(Wrapper):
    """Rewards divided by sqrt(variance of the discounted return) + eps
    (wrappers.py:144-183); info['raw_reward'] keeps the unscaled reward and the
    return restarts at every episode end."""

    def __init__(self, env, gamma: float = 0.99, epsilon: float = 1e-8):
        super().__init__(env)
        self.gamma = gamma
        self.epsilon = epsilon
        self.return_rms = RunningMeanStd()
        self.returns = 0.0

    def reset(self, **kwargs):
        self.returns = 0.0
        return self.env.reset(**kwargs)

    def step(self, action):
        obs, reward, terminated, truncated, info = self.env.step(action)
        self.returns = self.returns * self.gamma + reward
        self.return_rms.update(np.array([self.returns]))
        scale = np.sqrt(self.return_rms.var) + self.epsilon
        if terminated or truncated:
            self.returns = 0.0
        info["raw_reward"] = reward
        return obs, reward / scale, terminated, truncated, info


class FrameStackWrapper(Wrapper):
    """The board planes of the last ``num_frames`` steps on a new leading axis
    (wrappers.py:226-279); pieces and action mask pass through.  A reset fills
    the window with the first board."""

    def __init__(self, env, num_frames: int = 4):
        super().__init__(env)
        self.num_frames = num_frames
        self._window: deque = deque(maxlen=num_frames)
        inner = env.observation_space
        board_shape = (num_frames,) + tuple(inner["board"].shape)
        self.observation_space = DictSpace({"board": Box(low=0.0, high=1.0, shape=board_shape, dtype=np.float32),
                                            "pieces": inner["pieces"], "action_mask": inner["action_mask"]})

    @property
    def frames(self):
        return list(self._window)

    def _observe(self, obs) -> Dict[str, np.ndarray]:
        return {"board": np.stack(tuple(self._window), axis=0), "pieces": obs["pieces"],
                "action_mask": obs["action_mask"]}

    def reset(self, **kwargs):
        obs, info = self.env.reset(**kwargs)
        self._window.clear()
        self._window.extend(obs["board"].copy() for _ in range(self.num_frames))
        return self._observe(obs), info

    def step(self, action):
        obs, reward, terminated, truncated, info = self.env.step(action)
        self._window.append(obs["board"].copy())  # the oldest frame drops out (maxlen)
        return self._observe(obs), reward, terminated, truncated, info


def make_env(seed: Optional[int] = None, reward_config: Optional[Dict[str, float]] = None,
             normalize_reward: bool = False, frame_stack: int = 1):
    """wrappers.py:282-309: a BlockBlastEnv, frame-stacked when frame_stack > 1,
    then reward-normalised when asked."""
    wrapped = BlockBlastEnv(seed=seed, reward_config=reward_config)
    wrapped = FrameStackWrapper(wrapped, num_frames=frame_stack) if frame_stack > 1 else wrapped
    return NormalizedRewardWrapper(wrapped) if normalize_reward else wrapped

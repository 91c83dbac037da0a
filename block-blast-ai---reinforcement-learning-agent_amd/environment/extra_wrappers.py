"""Host-side single-env wrappers of the reference (wrappers.py:144-309):
reward normalisation by a running return variance, board frame stacking, and
the ``make_env`` factory.  They wrap the N=1 ``BlockBlastEnv`` and hold no
GPU work of their own."""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np

from .block_blast_env import BlockBlastEnv
from .spaces import Box, Dict as DictSpace, Wrapper


class RunningMeanStd:
    """wrappers.py:186-223: parallel-moments running mean / variance (fp64)."""

    def __init__(self, epsilon: float = 1e-4, shape: Tuple[int, ...] = ()):
        self.mean = np.zeros(shape, dtype=np.float64)
        self.var = np.ones(shape, dtype=np.float64)
        self.count = epsilon

    def update(self, x: np.ndarray) -> None:
        x = np.asarray(x)
        self._update_from_moments(np.mean(x, axis=0), np.var(x, axis=0), x.shape[0])

    def _update_from_moments(self, batch_mean, batch_var, batch_count) -> None:
        delta = batch_mean - self.mean
        tot = self.count + batch_count
        m2 = self.var * self.count + batch_var * batch_count + np.square(delta) * self.count * batch_count / tot
        self.mean = self.mean + delta * batch_count / tot
        self.var = m2 / tot
        self.count = tot


class NormalizedRewardWrapper(Wrapper):
    """wrappers.py:144-183: reward / (sqrt(var of discounted return) + eps);
    the raw reward is kept in info['raw_reward']."""

    def __init__(self, env, gamma: float = 0.99, epsilon: float = 1e-8):
        super().__init__(env)
        self.gamma, self.epsilon = gamma, epsilon
        self.return_rms = RunningMeanStd()
        self.returns = 0.0

    def step(self, action):
        obs, reward, terminated, truncated, info = self.env.step(action)
        self.returns = self.returns * self.gamma + reward
        self.return_rms.update(np.array([self.returns]))
        normalized = reward / (np.sqrt(self.return_rms.var) + self.epsilon)
        if terminated or truncated:
            self.returns = 0.0
        info["raw_reward"] = reward
        return obs, normalized, terminated, truncated, info

    def reset(self, **kwargs):
        self.returns = 0.0
        return self.env.reset(**kwargs)


class FrameStackWrapper(Wrapper):
    """wrappers.py:226-279: the last ``num_frames`` boards stacked on axis 0
    (pieces and mask pass through)."""

    def __init__(self, env, num_frames: int = 4):
        super().__init__(env)
        self.num_frames = num_frames
        self.frames = None
        sp = env.observation_space
        self.observation_space = DictSpace({
            "board": Box(low=0.0, high=1.0, shape=(num_frames,) + tuple(sp["board"].shape), dtype=np.float32),
            "pieces": sp["pieces"],
            "action_mask": sp["action_mask"],
        })

    def _stacked(self, obs) -> Dict[str, np.ndarray]:
        return {"board": np.stack(self.frames, axis=0), "pieces": obs["pieces"], "action_mask": obs["action_mask"]}

    def reset(self, **kwargs):
        obs, info = self.env.reset(**kwargs)
        self.frames = [obs["board"].copy() for _ in range(self.num_frames)]
        return self._stacked(obs), info

    def step(self, action):
        obs, reward, terminated, truncated, info = self.env.step(action)
        self.frames.pop(0)
        self.frames.append(obs["board"].copy())
        return self._stacked(obs), reward, terminated, truncated, info


def make_env(seed: Optional[int] = None, reward_config: Optional[Dict[str, float]] = None,
             normalize_reward: bool = False, frame_stack: int = 1):
    """wrappers.py:282-309."""
    env = BlockBlastEnv(seed=seed, reward_config=reward_config)
    if frame_stack > 1:
        env = FrameStackWrapper(env, num_frames=frame_stack)
    if normalize_reward:
        env = NormalizedRewardWrapper(env)
    return env

"""Vectorised Block Blast env on the GPU.

Drop-in for the reference ``src/environment/wrappers.py::VectorizedBlockBlastEnv``
(wrappers.py:14-141): same constructor (env i seeded ``seed + i``), numpy
return types and shapes, auto-reset with ``terminal_observation`` /
``final_score`` in the terminated env's info.  Where the reference loops over
Python envs (wrappers.py:93) this class issues ONE ``bb_step`` launch for all
envs; ``step_device`` keeps everything on the GPU for training.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from runtime.device_env import DEFAULT_REWARDS, DeviceEnvBatch

from . import _host
from .spaces import Box, Dict as DictSpace, Discrete


class _EnvSlot:
    """Light view of env i (the reference exposes ``vec_env.envs[i]``)."""

    def __init__(self, vec: "VectorizedBlockBlastEnv", i: int):
        self._vec, self.index = vec, i

    @property
    def seed_value(self):
        return self._vec._seeds[self.index]

    @property
    def reward_config(self):
        return self._vec.reward_config

    def get_action_mask(self) -> np.ndarray:
        return self._vec.get_action_masks()[self.index]

    def close(self) -> None:
        pass


class VectorizedBlockBlastEnv:
    def __init__(
        self,
        num_envs: int,
        seed: Optional[int] = None,
        reward_config: Optional[Dict[str, float]] = None,
        device=None,
        env_offset: int = 0,
    ):
        self.num_envs = int(num_envs)
        self.env_offset = int(env_offset)
        self.reward_config = reward_config
        rw = dict(DEFAULT_REWARDS)
        if reward_config:
            rw.update(reward_config)
        self._seeds = self._seed_list(seed)
        self.dev = DeviceEnvBatch(self.num_envs, self._seeds, rw, autoreset=True, device=device,
                                  env_offset=self.env_offset)
        self.dev.reset()
        d = self.dev.device
        n = self.num_envs
        self._act = torch.zeros(n, dtype=torch.int32, device=d)
        self._x = torch.zeros((n, 4, 8, 8), dtype=torch.float32, device=d)
        self._mask = torch.zeros((n, 192), dtype=torch.int8, device=d)
        self._mask_bits = torch.zeros((n, 3), dtype=torch.int64, device=d)
        self.observation_space = DictSpace({
            "board": Box(low=0.0, high=1.0, shape=(8, 8), dtype=np.float32),
            "pieces": Box(low=0.0, high=1.0, shape=(3, 8, 8), dtype=np.float32),
            "action_mask": Box(low=0, high=1, shape=(192,), dtype=np.int8),
        })
        self.action_space = Discrete(192)
        self.single_action_space = self.action_space
        self.envs = [_EnvSlot(self, i) for i in range(n)] if n <= 4096 else _LazySlots(self)
        self._dones = np.zeros(n, dtype=bool)

    def _seed_list(self, seed: Optional[int]) -> List[Optional[int]]:
        # env i -> seed + i (wrappers.py:41); shards add their global offset
        if seed is None:
            return [None] * self.num_envs
        return [seed + self.env_offset + i for i in range(self.num_envs)]

    # ------------------------------------------------------------ numpy API
    def _host_obs(self) -> Dict[str, np.ndarray]:
        self.dev.obs(x=self._x, mask_i8=self._mask)
        x = self._x.cpu().numpy()
        return {
            "board": np.ascontiguousarray(x[:, 0]),
            "pieces": np.ascontiguousarray(x[:, 1:]),
            "action_mask": self._mask.cpu().numpy(),
        }

    def reset(self, seed: Optional[int] = None) -> Tuple[Dict[str, np.ndarray], List[Dict[str, Any]]]:
        """wrappers.py:53-73."""
        if seed is not None:
            self._seeds = self._seed_list(seed)
            self.dev.seed(self._seeds)
        self.dev.reset()
        self._dones.fill(False)
        return self._host_obs(), [_host.reset_info() for _ in range(self.num_envs)]

    def step(self, actions: np.ndarray):
        """wrappers.py:75-116, one kernel launch for every env."""
        a = np.asarray(actions).reshape(-1)
        if a.size != self.num_envs:
            raise ValueError(f"expected {self.num_envs} actions, got {a.size}")
        a64 = a.astype(np.int64)
        a64 = np.where((a64 >= -(2 ** 31)) & (a64 < 2 ** 31), a64, -1)
        self._act.copy_(torch.from_numpy(a64.astype(np.int32)))
        self.dev.step(self._act, want_info=True)
        obs = self._host_obs()
        rewards = self.dev.reward.cpu().numpy()
        terminated = self.dev.terminated.cpu().numpy().astype(bool)
        truncated = np.zeros(self.num_envs, dtype=bool)
        infos = _host.InfoList(self.dev.info_host().copy())
        return obs, rewards, terminated, truncated, infos

    def get_action_masks(self) -> np.ndarray:
        self.dev.obs(mask_i8=self._mask)
        return self._mask.cpu().numpy().astype(bool)

    def sample_valid_actions(self) -> np.ndarray:
        """Per-env uniform choice among legal actions with numpy's global RNG,
        like BlockBlastEnv.sample_valid_action (block_blast_env.py:318-323)."""
        masks = self.get_action_masks()
        out = np.zeros(self.num_envs, dtype=np.int64)
        for i in range(self.num_envs):
            valid = np.nonzero(masks[i])[0]
            out[i] = np.random.choice(valid) if valid.size else 0
        return out

    def close(self) -> None:
        self.dev.close()

    # ------------------------------------------------------------ device API
    def step_device(self, actions: torch.Tensor, **kw) -> Tuple[torch.Tensor, torch.Tensor]:
        """Step with int32 device actions; returns (reward f32, terminated u8)
        device tensors (valid until the next step)."""
        self.dev.step(actions, **kw)
        return self.dev.reward, self.dev.terminated

    def sample_valid_actions_device(self, out: torch.Tensor, seed: int = 0xB10C, step: int = 0) -> torch.Tensor:
        """Synthetic random policy (Philox) on the device."""
        self.dev.obs(mask_bits=self._mask_bits)
        self.dev.random_actions(self._mask_bits, out, seed=seed, step=step)
        return out


class _LazySlots:
    def __init__(self, vec):
        self._vec = vec

    def __len__(self):
        return self._vec.num_envs

    def __getitem__(self, i):
        if not 0 <= i < len(self):
            raise IndexError(i)
        return _EnvSlot(self._vec, i)

    def __iter__(self):
        return (self[i] for i in range(len(self)))

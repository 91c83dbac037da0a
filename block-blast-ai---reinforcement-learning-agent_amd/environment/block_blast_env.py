"""Gym surface of one Block Blast game, backed by the gfx950 vec-env (N = 1).

Drop-in for the reference ``src/environment/block_blast_env.py::BlockBlastEnv``
(block_blast_env.py:20-323): same constructor, constants, spaces, method names,
return types and reward/info semantics.  The game itself runs in ``bb_step``
on the GPU (no auto-reset for the single env: after game over every action is
invalid, as in the reference).  ``BlockBlastEnvFlat`` (326-389) is provided
for API completeness.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from game.pieces import NUM_PIECES
from runtime.device_env import DEFAULT_REWARDS, DeviceEnvBatch

from . import _host
from .spaces import Box, Dict as DictSpace, Discrete, Env


class BlockBlastEnv(Env):
    metadata = {"render_modes": ["human", "ansi"]}

    BOARD_SIZE = 8
    NUM_PIECES_PER_TURN = 3
    ACTION_SPACE_SIZE = NUM_PIECES_PER_TURN * BOARD_SIZE * BOARD_SIZE  # 192

    def __init__(
        self,
        render_mode: Optional[str] = None,
        reward_config: Optional[Dict[str, float]] = None,
        seed: Optional[int] = None,
        device=None,
    ):
        super().__init__()
        self.render_mode = render_mode
        self.seed_value = seed
        self.reward_config = dict(DEFAULT_REWARDS)
        if reward_config:
            self.reward_config.update(reward_config)
        self._dev = DeviceEnvBatch(1, [seed], self.reward_config, autoreset=False, device=device)
        self._dev.reset()  # GameEngine(seed) state == reset state (engine.py:99-125)
        d = self._dev.device
        self._act = torch.zeros(1, dtype=torch.int32, device=d)
        self._x = torch.zeros((1, 4, 8, 8), dtype=torch.float32, device=d)
        self._mask = torch.zeros((1, self.ACTION_SPACE_SIZE), dtype=torch.int8, device=d)
        self.observation_space = DictSpace({
            "board": Box(low=0.0, high=1.0, shape=(self.BOARD_SIZE, self.BOARD_SIZE), dtype=np.float32),
            "pieces": Box(low=0.0, high=1.0, shape=(self.NUM_PIECES_PER_TURN, self.BOARD_SIZE, self.BOARD_SIZE),
                          dtype=np.float32),
            "action_mask": Box(low=0, high=1, shape=(self.ACTION_SPACE_SIZE,), dtype=np.int8),
        })
        self.action_space = Discrete(self.ACTION_SPACE_SIZE)
        self._last_obs: Optional[Dict[str, np.ndarray]] = None

    # block_blast_env.py:104-132
    def _action_to_move(self, action: int) -> Tuple[int, int, int]:
        piece_idx = action // (self.BOARD_SIZE * self.BOARD_SIZE)
        remainder = action % (self.BOARD_SIZE * self.BOARD_SIZE)
        return piece_idx, remainder // self.BOARD_SIZE, remainder % self.BOARD_SIZE

    def _move_to_action(self, piece_idx: int, row: int, col: int) -> int:
        return piece_idx * self.BOARD_SIZE * self.BOARD_SIZE + row * self.BOARD_SIZE + col

    def _get_observation(self) -> Dict[str, np.ndarray]:
        self._dev.obs(x=self._x, mask_i8=self._mask)
        x = self._x.cpu().numpy()[0]
        obs = {
            "board": np.ascontiguousarray(x[0]),
            "pieces": np.ascontiguousarray(x[1:]),
            "action_mask": self._mask.cpu().numpy()[0].copy(),
        }
        self._last_obs = obs
        return obs

    def reset(self, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        """block_blast_env.py:195-222."""
        if seed is not None:
            self.seed_value = seed
            self._dev.seed([seed])
        self._dev.reset()
        return self._get_observation(), _host.reset_info()

    def step(self, action: int):
        """block_blast_env.py:224-264."""
        a = int(action)
        if not -(2 ** 31) <= a < 2 ** 31:
            a = -1  # outside the action space: invalid, like any piece_idx not in 0..2
        self._act.fill_(a)
        self._dev.step(self._act, want_info=True, want_f64=True)
        obs = self._get_observation()
        reward = float(self._dev.reward_f64.cpu().item())
        terminated = bool(self._dev.terminated.cpu().item())
        rec = self._dev.info_host()[0]
        info = _host.info_dict(rec, with_last_move=True)
        if rec["flags"] & 1:
            return obs, -10.0, False, False, info
        if self.render_mode == "human":
            self.render()
        return obs, reward, terminated, False, info

    def get_action_mask(self) -> np.ndarray:
        return self._get_observation()["action_mask"].astype(bool)

    def get_valid_actions(self) -> List[int]:
        return np.where(self.get_action_mask())[0].tolist()

    def sample_valid_action(self) -> int:
        valid = self.get_valid_actions()
        if not valid:
            return 0
        return np.random.choice(valid)

    def _state_text(self) -> str:
        s = self._dev.state()
        h = int(s["hand"][0])
        return _host.render_text(int(s["board"][0]), h, int(s["score"][0]), int(s["combo"][0]),
                                 int(s["moves"][0]), bool((h >> 21) & 1))

    def render(self) -> Optional[str]:
        if self.render_mode == "ansi":
            return self._state_text()
        if self.render_mode == "human":
            print("\033[2J\033[H")
            print(self._state_text())
        return None

    def close(self) -> None:
        pass


class BlockBlastEnvFlat(BlockBlastEnv):
    """178-d flat observation variant (block_blast_env.py:326-389): board 64 +
    3 x 37 piece one-hots (zeros for used slots) + 3 used flags."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        size = self.BOARD_SIZE * self.BOARD_SIZE + self.NUM_PIECES_PER_TURN * NUM_PIECES + self.NUM_PIECES_PER_TURN
        self.observation_space = DictSpace({
            "obs": Box(low=0.0, high=1.0, shape=(size,), dtype=np.float32),
            "action_mask": Box(low=0, high=1, shape=(self.ACTION_SPACE_SIZE,), dtype=np.int8),
        })

    def _get_observation(self) -> Dict[str, np.ndarray]:
        base = super()._get_observation()
        s = self._dev.state()
        h = int(s["hand"][0])
        onehots = np.zeros((self.NUM_PIECES_PER_TURN, NUM_PIECES), dtype=np.float32)
        used = _host.hand_used(h)
        for slot, pid in enumerate(_host.hand_ids(h)):
            if not used[slot]:
                onehots[slot, pid] = 1.0
        flat = np.concatenate([base["board"].reshape(-1), onehots.reshape(-1), np.array(used, dtype=np.float32)])
        return {"obs": flat, "action_mask": base["action_mask"]}

    def get_action_mask(self) -> np.ndarray:
        return self._get_observation()["action_mask"].astype(bool)

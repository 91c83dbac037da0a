"""ctypes binding of the C oracle (oracle/bb_oracle.c -> oracle/_build/libbboracle.so).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  ``CVecEnv`` mirrors
``bb_game.VecEnv`` (the reference's ``VectorizedBlockBlastEnv`` semantics,
wrappers.py:14-141) with array outputs, multi-threaded over envs, so parity
runs can cover BASELINE's full 65,536-env batch.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libbboracle.so")

_P = C.c_void_p
_U64 = C.c_uint64
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import subprocess

            from .build import build_oracle

            try:
                build_oracle()
            except (OSError, subprocess.CalledProcessError) as exc:  # no gcc / OpenMP here: the checker is absent
                import pytest

                pytest.skip(f"C oracle unavailable: {exc}")
        lib = C.CDLL(LIB_PATH)
        sig = {
            "bbo_abi_version": (C.c_int, []),
            "bbo_pcg64_seed": (None, [_U64, _P]),
            "bbo_rng_draws": (None, [_U64, C.c_uint32, C.c_int, _P]),
            "bbo_create": (_P, [C.c_int, _P, _P, _P, C.c_int]),
            "bbo_destroy": (None, [_P]),
            "bbo_reset": (None, [_P, C.c_int]),
            "bbo_step": (None, [_P, _P, _P, _P, _P, _P, _P, _P, C.c_int]),
            "bbo_rollout": (None, [_P, C.c_int, _P, _U64, _U64, _U64, _P, _P, _P, _P, _P, C.c_int]),
            "bbo_replay": (None, [_P, C.c_int, _P, _P, _P, _P, _P, _P, _P, _P, C.c_int]),
            "bbo_random_actions": (None, [_P, C.c_int, _U64, _U64, _U64, _P]),
            "bbo_state": (None, [_P] + [_P] * 12),
            "bbo_set_board_hand": (None, [_P, _P, _P]),
            "bbo_gen_hist": (None, [_P, _P]),
            "bbo_solvable_many": (None, [_P, _P, C.c_int, _P, C.c_int]),
            "bbo_play_random_game": (None, [_U64, _P, _P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_P)


REWARD_KEYS = ("line_clear_base", "block_placed", "game_over_penalty", "hole_penalty", "center_bonus",
               "combo_multiplier_bonus", "survival_bonus")


def pcg64_seed(seed: int):
    out = np.zeros(4, np.uint64)
    load().bbo_pcg64_seed(seed, _p(out))
    return [int(x) for x in out]


def rng_draws(seed: int, bound: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.uint32)
    load().bbo_rng_draws(seed, bound, n, _p(out))
    return out


def play_random_game(seed: int):
    out = np.zeros(8, np.int64)
    first = np.zeros(3, np.int32)
    load().bbo_play_random_game(seed, _p(out), _p(first))
    keys = ("score", "moves_made", "total_lines_cleared", "max_combo", "total_blocks_placed")
    st = {k: int(v) for k, v in zip(keys, out[:5])}
    st["board_fill_ratio"] = int(out[5]) / 64
    st["holes"] = int(out[6])
    st["center_openness"] = 1.0 - int(out[7]) / 16.0
    return st, [int(x) for x in first]


def solvable_many(boards: np.ndarray, hands: np.ndarray, threads: int = 0) -> np.ndarray:
    boards = np.ascontiguousarray(boards, np.uint64)
    hands = np.ascontiguousarray(hands, np.uint32)
    out = np.zeros(len(boards), np.uint8)
    load().bbo_solvable_many(_p(boards), _p(hands), len(boards), _p(out), threads)
    return out.astype(bool)


class CVecEnv:
    """N envs seeded ``seeds[i]`` (re-seeded every episode, block_blast_env.py:212-215)."""

    def __init__(self, seeds, reward_config=None, autoreset=True, has_seed=None):
        self.lib = load()
        self.seeds = np.ascontiguousarray(seeds, np.uint64)
        self.n = len(self.seeds)
        rw = None
        if reward_config is not None:
            from .bb_game import DEFAULT_REWARDS

            d = dict(DEFAULT_REWARDS)
            d.update(reward_config)
            rw = np.array([d[k] for k in REWARD_KEYS], np.float64)
        hs = None if has_seed is None else np.ascontiguousarray(has_seed, np.uint8)
        self.h = self.lib.bbo_create(self.n, _p(self.seeds), _p(hs), _p(rw), int(bool(autoreset)))
        self._keep = (rw, hs)

    def close(self):
        if self.h:
            self.lib.bbo_destroy(self.h)
            self.h = None

    __del__ = close

    def reset(self, threads: int = 0):
        self.lib.bbo_reset(self.h, threads)

    def step(self, actions, threads: int = 0):
        a = np.ascontiguousarray(actions, np.int32)
        n = self.n
        out = {"reward": np.zeros(n, np.float32), "reward_f64": np.zeros(n, np.float64),
               "terminated": np.zeros(n, np.uint8), "lines": np.zeros(n, np.uint8),
               "invalid": np.zeros(n, np.uint8), "mask": np.zeros((n, 3), np.uint64)}
        self.lib.bbo_step(self.h, _p(a), _p(out["reward"]), _p(out["reward_f64"]), _p(out["terminated"]),
                          _p(out["lines"]), _p(out["invalid"]), _p(out["mask"]), threads)
        return out

    def rollout(self, T, actions, policy_seed=0xB10C, policy_step0=0, env_offset=0, threads=0, mask=True):
        """T steps under the synthetic Philox policy (= bb_rollout); returns the
        [T][N] outputs and the next actions."""
        act = np.ascontiguousarray(actions, np.int32).copy()
        n = self.n
        out = {"reward": np.zeros((T, n), np.float32), "terminated": np.zeros((T, n), np.uint8),
               "lines": np.zeros((T, n), np.uint8), "actions": np.zeros((T, n), np.int32),
               "mask": np.zeros((T, n, 3), np.uint64) if mask else None}
        self.lib.bbo_rollout(self.h, T, _p(act), policy_seed, policy_step0, env_offset, _p(out["reward"]),
                             _p(out["terminated"]), _p(out["lines"]), _p(out["actions"]), _p(out["mask"]), threads)
        out["next_action"] = act
        return out

    def replay(self, actions, threads=0):
        """Step every env through recorded actions [T][N] (the training
        rollout, scripts/train.py:173-203 with wrappers.py:75-116): returns the
        pre-step snapshots (board bits, hand word, mask bits) and the outputs,
        with the final score / moves of each episode ending at (t, i) (0
        elsewhere; info['final_score'] / info['moves'], wrappers.py:97-101)."""
        a = np.ascontiguousarray(actions, np.int32)
        T, n = a.shape
        assert n == self.n
        out = {"board": np.zeros((T, n), np.uint64), "hand": np.zeros((T, n), np.uint32),
               "mask": np.zeros((T, n, 3), np.uint64), "reward": np.zeros((T, n), np.float32),
               "terminated": np.zeros((T, n), np.uint8), "ep_score": np.zeros((T, n), np.int64),
               "ep_moves": np.zeros((T, n), np.int32)}
        self.lib.bbo_replay(self.h, T, _p(a), _p(out["board"]), _p(out["hand"]), _p(out["mask"]),
                            _p(out["reward"]), _p(out["terminated"]), _p(out["ep_score"]), _p(out["ep_moves"]),
                            threads)
        return out

    def random_actions(self, mask, seed=0xB10C, step=0, env_offset=0):
        m = np.ascontiguousarray(mask, np.uint64)
        out = np.zeros(len(m), np.int32)
        self.lib.bbo_random_actions(_p(m), len(m), seed, step, env_offset, _p(out))
        return out

    def state(self):
        n = self.n
        s = {"board": np.zeros(n, np.uint64), "hand": np.zeros(n, np.uint32), "score": np.zeros(n, np.int64),
             "combo": np.zeros(n, np.int32), "max_combo": np.zeros(n, np.int32), "moves": np.zeros(n, np.int32),
             "lines": np.zeros(n, np.int32), "blocks": np.zeros(n, np.int32),
             "prev_holes": np.zeros(n, np.uint8), "prev_center": np.zeros(n, np.uint8),
             "rng": np.zeros((n, 3), np.uint64), "mask": np.zeros((n, 3), np.uint64)}
        self.lib.bbo_state(self.h, *(_p(s[k]) for k in ("board", "hand", "score", "combo", "max_combo", "moves",
                                                        "lines", "blocks", "prev_holes", "prev_center", "rng",
                                                        "mask")))
        return s

    def set_board_hand(self, board=None, hand=None):
        b = None if board is None else np.ascontiguousarray(board, np.uint64)
        h = None if hand is None else np.ascontiguousarray(hand, np.uint32)
        self.lib.bbo_set_board_hand(self.h, _p(b), _p(h))

    def gen_hist(self) -> np.ndarray:
        out = np.zeros(101, np.uint64)
        self.lib.bbo_gen_hist(self.h, _p(out))
        return out

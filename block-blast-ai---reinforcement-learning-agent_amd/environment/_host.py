"""Host-side formatting of device outputs into the reference's Python types.

Pure data formatting (bit unpacking, dict construction); every game rule ran
in ``bb_step`` on the GPU.
"""
from __future__ import annotations

from collections.abc import Sequence

import numpy as np

from game.pieces import PIECE_MASKS

BOARD = 8
HAND = 3
ACTIONS = 192

_SHIFTS = np.arange(64, dtype=np.uint64)


def board_planes(bits: np.ndarray) -> np.ndarray:
    """u64 [N] -> f32 [N, 8, 8] (bit r*8+c -> [r, c])."""
    b = np.asarray(bits, dtype=np.uint64).reshape(-1, 1)
    return ((b >> _SHIFTS) & np.uint64(1)).astype(np.float32).reshape(-1, BOARD, BOARD)


def piece_planes(hand: np.ndarray) -> np.ndarray:
    """packed hand word [N] -> f32 [N, 3, 8, 8] (zeros for used slots)."""
    h = np.asarray(hand, dtype=np.uint32).reshape(-1)
    out = np.zeros((h.size, HAND, BOARD, BOARD), dtype=np.float32)
    for s in range(HAND):
        ids = (h >> np.uint32(6 * s)) & np.uint32(63)
        used = (h >> np.uint32(18 + s)) & np.uint32(1)
        out[:, s] = PIECE_MASKS[ids] * (1.0 - used.astype(np.float32))[:, None, None]
    return out


def hand_ids(hand) -> list:
    h = int(hand)
    return [(h >> (6 * s)) & 63 for s in range(HAND)]


def hand_used(hand) -> list:
    h = int(hand)
    return [bool((h >> (18 + s)) & 1) for s in range(HAND)]


def terminal_observation(board_bits, hand) -> dict:
    """Observation of a terminal (game-over) state.  Game over is exactly "no
    unused piece has a legal anchor" (engine.py:382-388, 440-441), so its action
    mask is all zeros."""
    return {
        "board": board_planes(np.array([board_bits], dtype=np.uint64))[0],
        "pieces": piece_planes(np.array([hand], dtype=np.uint32))[0],
        "action_mask": np.zeros(ACTIONS, dtype=np.int8),
    }


def info_dict(rec, with_last_move: bool) -> dict:
    """One bb_info record -> block_blast_env.py:266-288 info dict."""
    info = {
        "score": int(rec["score"]),
        "moves": int(rec["moves"]),
        "lines_cleared": int(rec["lines"]),
        "max_combo": int(rec["max_combo"]),
        "blocks_placed": int(rec["blocks"]),
        "board_fill": int(rec["filled"]) / (BOARD ** 2),
        "holes": int(rec["holes"]),
        "invalid_action": bool(rec["flags"] & 1),
    }
    if with_last_move and (rec["flags"] & 4):
        info["last_move"] = {
            "blocks_placed": int(rec["last_blocks"]),
            "lines_cleared": int(rec["last_lines"]),
            "combo_multiplier": int(rec["last_cm"]),
            "score_gained": int(rec["score_gained"]),
        }
    return info


def reset_info() -> dict:
    """Info right after a reset (empty board, zero counters)."""
    return {
        "score": 0, "moves": 0, "lines_cleared": 0, "max_combo": 0, "blocks_placed": 0,
        "board_fill": 0.0, "holes": 0, "invalid_action": False,
    }


class InfoList(Sequence):
    """``infos`` of VectorizedBlockBlastEnv.step (wrappers.py:91-108) as a lazy
    sequence over the packed info records: the dict of env i is built only
    when it is read, so stepping 64k envs does not build 64k dicts."""

    def __init__(self, records: np.ndarray):
        self._rec = records
        self._cache = {}

    def __len__(self) -> int:
        return len(self._rec)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        d = self._cache.get(i)
        if d is None:
            r = self._rec[i]
            d = info_dict(r, with_last_move=True)
            if r["flags"] & 2:  # terminated -> wrappers.py:97-100
                d["terminal_observation"] = terminal_observation(r["term_board"], r["term_hand"])
                d["final_score"] = d["score"]
            self._cache[i] = d
        return d

    # vectorised accessors for callers that want arrays, not dicts
    @property
    def records(self) -> np.ndarray:
        return self._rec

    def terminated_indices(self) -> np.ndarray:
        return np.nonzero(self._rec["flags"] & 2)[0]


def render_text(board_bits, hand, score, combo, moves, over) -> str:
    """ASCII picture of one game (engine.py:526-535 / board.py:282-295 style)."""
    from game.pieces import PIECE_LIST

    g = board_planes(np.array([board_bits], dtype=np.uint64))[0]
    lines = ["  " + " ".join(str(i) for i in range(BOARD)), "  " + "-" * (BOARD * 2 - 1)]
    for r in range(BOARD):
        lines.append(f"{r}|" + " ".join("█" if g[r, c] else "·" for c in range(BOARD)))
    filled = int(g.sum())
    lines.append("  " + "-" * (BOARD * 2 - 1))
    lines.append(f"Blocks: {filled}, Empty: {BOARD * BOARD - filled}")
    lines.append(f"\nScore: {score} | Moves: {moves} | Combo: {combo} | Status: {'game_over' if over else 'playing'}")
    lines.append("\nAvailable pieces:")
    used = hand_used(hand)
    for s, pid in enumerate(hand_ids(hand)):
        lines.append(f"  [{s}] {PIECE_LIST[pid].name} ({'USED' if used[s] else 'available'})")
    return "\n".join(lines)

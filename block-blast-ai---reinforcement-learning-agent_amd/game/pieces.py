"""The 37 Block Blast pieces (host-side static table).

Same names, index order and cell sets as the reference ``src/game/pieces.py``
(shapes 78-236, dict order 244-318, helpers 321-368), but defined here as
64-bit bitboards (bit ``r*8+c``) -- the representation the gfx950 kernels use
(``csrc/bb_tables.cpp`` holds the identical table).  Cells, width/height and
masks are derived from the bits.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

# (name, bitboard) in reference index order.
_TABLE: Tuple[Tuple[str, int], ...] = (
    ("SINGLE", 0x1), ("DOMINO_H", 0x3), ("DOMINO_V", 0x101),
    ("DIAG2_TL_BR", 0x201), ("DIAG2_TR_BL", 0x102),
    ("TRIO_H", 0x7), ("TRIO_V", 0x10101),
    ("DIAG3_TL_BR", 0x40201), ("DIAG3_TR_BL", 0x10204),
    ("TRIO_L1", 0x301), ("TRIO_L2", 0x203), ("TRIO_L3", 0x103), ("TRIO_L4", 0x302),
    ("I_H", 0xF), ("I_V", 0x1010101), ("I5_H", 0x1F), ("I5_V", 0x101010101),
    ("O", 0x303),
    ("T_UP", 0x702), ("T_DOWN", 0x207), ("T_LEFT", 0x10301), ("T_RIGHT", 0x20302),
    ("S_H", 0x306), ("S_V", 0x20301), ("Z_H", 0x603), ("Z_V", 0x10302),
    ("L_1", 0x30101), ("L_2", 0x107), ("L_3", 0x20203), ("L_4", 0x704),
    ("J_1", 0x30202), ("J_2", 0x701), ("J_3", 0x10103), ("J_4", 0x407),
    ("RECT_2x3_H", 0x707), ("RECT_2x3_V", 0x30303), ("SQUARE_3x3", 0x70707),
)


class Piece:
    """Immutable piece: a name plus its cells anchored at (0, 0)."""

    __slots__ = ("_name", "_bits", "_blocks")

    def __init__(self, name: str, bits: int):
        object.__setattr__(self, "_name", name)
        object.__setattr__(self, "_bits", int(bits))
        cells = tuple((b // 8, b % 8) for b in range(64) if (bits >> b) & 1)
        object.__setattr__(self, "_blocks", cells)

    def __setattr__(self, key, value):  # frozen, like the reference dataclass
        raise AttributeError("Piece is immutable")

    @property
    def name(self) -> str:
        return self._name

    @property
    def bits(self) -> int:
        """Bitboard of the piece at origin (bit r*8+c)."""
        return self._bits

    @property
    def blocks(self) -> Tuple[Tuple[int, int], ...]:
        return self._blocks

    @property
    def num_blocks(self) -> int:
        return len(self._blocks)

    @property
    def width(self) -> int:
        return max(c for _, c in self._blocks) + 1

    @property
    def height(self) -> int:
        return max(r for r, _ in self._blocks) + 1

    def to_mask(self, board_size: int = 8) -> np.ndarray:
        m = np.zeros((board_size, board_size), dtype=np.float32)
        for r, c in self._blocks:
            if r < board_size and c < board_size:
                m[r, c] = 1.0
        return m

    def get_shape_array(self) -> np.ndarray:
        a = np.zeros((self.height, self.width), dtype=np.int8)
        for r, c in self._blocks:
            a[r, c] = 1
        return a

    def __eq__(self, other) -> bool:
        return isinstance(other, Piece) and other._name == self._name and other._bits == self._bits

    def __hash__(self) -> int:
        return hash((self._name, self._bits))

    def __repr__(self) -> str:
        return f"Piece({self._name}, {self.num_blocks} blocks)"


PIECES: Dict[str, Piece] = {name: Piece(name, bits) for name, bits in _TABLE}
PIECE_LIST: List[Piece] = list(PIECES.values())
PIECE_NAMES: List[str] = list(PIECES.keys())
NUM_PIECES: int = len(PIECE_LIST)
assert NUM_PIECES == 37

PIECE_BITS = np.array([p.bits for p in PIECE_LIST], dtype=np.uint64)
# f32 (37, 8, 8) shapes at origin: row id of the observation's piece planes.
PIECE_MASKS = np.stack([p.to_mask() for p in PIECE_LIST]).astype(np.float32)

globals().update(PIECES)  # SINGLE, DOMINO_H, ... SQUARE_3x3 as module attributes


def get_piece_by_name(name: str) -> Piece:
    if name not in PIECES:
        raise ValueError(f"Unknown piece: {name}. Valid pieces: {PIECE_NAMES}")
    return PIECES[name]


def get_piece_by_index(index: int) -> Piece:
    if not 0 <= index < NUM_PIECES:
        raise ValueError(f"Piece index must be 0-{NUM_PIECES - 1}, got {index}")
    return PIECE_LIST[index]


def get_piece_index(piece: Piece) -> int:
    return PIECE_LIST.index(piece)


def get_all_pieces() -> List[Piece]:
    return list(PIECE_LIST)


def get_random_pieces(n: int = 3, rng: np.random.Generator = None) -> List[Piece]:
    """Host-side draw with the reference's call (pieces.py:350-355); the
    vectorised env draws the same stream on the GPU."""
    rng = rng if rng is not None else np.random.default_rng()
    return [PIECE_LIST[int(i)] for i in rng.choice(NUM_PIECES, size=n, replace=True)]


def piece_to_one_hot(piece: Piece) -> np.ndarray:
    v = np.zeros(NUM_PIECES, dtype=np.float32)
    v[get_piece_index(piece)] = 1.0
    return v


def visualize_piece(piece: Piece) -> str:
    return "\n".join("".join("□" if x else " " for x in row) for row in piece.get_shape_array())

"""CPU facts the kernels rely on (checked with the oracle's reference DFS)."""
import itertools

import numpy as np
import pytest

from oracle import bb_game as O


@pytest.mark.slow
def test_every_hand_fits_an_empty_board():
    """engine.py:181-224 on an empty board is True for all 37^3 hands, so a
    reset draws exactly one attempt (the kernel's reset path relies on it)."""
    e = O.Engine(seed=0)
    grid = [[0] * 8 for _ in range(8)]
    for a, b, c in itertools.product(range(37), repeat=3):
        e.hand = [a, b, c]
        assert e._solvable([row[:] for row in grid], [False, False, False])


def test_pair_conflict_offsets():
    """|D(b,c)| = number of distinct linear offsets at which c collides with b
    -- the quick-accept bound of csrc/bb_solver.h -- equals the number of
    distinct relative positions where the two pieces overlap on a 15x15 plane
    (no wrap-around), i.e. linear offsets are exact for in-bounds anchors."""
    for b in range(37):
        for c in range(37):
            lin = {(rb * 8 + cb) - (rc * 8 + cc) for rb, cb in O.PIECE_CELLS[b] for rc, cc in O.PIECE_CELLS[c]}
            two_d = {(rb - rc, cb - cc) for rb, cb in O.PIECE_CELLS[b] for rc, cc in O.PIECE_CELLS[c]}
            assert len(lin) == len(two_d)

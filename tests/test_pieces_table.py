"""Product piece table (game/pieces.py) == oracle table == reference answers."""
import numpy as np
import pytest

import game.pieces as P
from oracle import bb_game as O


def test_same_table_as_oracle():
    assert P.PIECE_NAMES == O.PIECE_NAMES
    for p, cells in zip(P.PIECE_LIST, O.PIECE_CELLS):
        assert set(p.blocks) == set(cells)
        assert p.height == max(r for r, _ in cells) + 1 and p.width == max(c for _, c in cells) + 1


def test_reference_helpers():
    assert P.get_piece_by_name("O") == P.O and P.get_piece_by_name("SQUARE_3x3") == P.SQUARE_3x3
    with pytest.raises(ValueError):
        P.get_piece_by_name("INVALID")
    with pytest.raises(ValueError):
        P.get_piece_by_index(37)
    with pytest.raises(Exception):
        P.SINGLE.name = "x"
    assert P.get_all_pieces() is not P.PIECE_LIST
    assert P.piece_to_one_hot(P.SINGLE)[0] == 1 and P.piece_to_one_hot(P.SINGLE).sum() == 1
    assert P.O.to_mask(8).sum() == 4.0
    assert "□□" in P.visualize_piece(P.DOMINO_H)
    assert np.array_equal(P.O.get_shape_array(), [[1, 1], [1, 1]])
    r1, r2 = np.random.default_rng(42), np.random.default_rng(42)
    assert P.get_random_pieces(3, r1) == P.get_random_pieces(3, r2)
    assert [p.name for p in P.get_random_pieces(3, np.random.default_rng(42))] == ["DIAG2_TL_BR", "L_3", "Z_H"]

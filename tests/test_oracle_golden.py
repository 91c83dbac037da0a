"""Pin the CPU oracle (oracle/bb_game.py) before trusting it.

Golden vectors: tests/golden/golden_seed42.json holds the only outputs of the
reference itself observed here; the known answers of
the reference's own tests (tests/test_{pieces,board,engine}.py) are restated
below as data.
"""
import json
import os

import numpy as np
import pytest

from oracle import bb_game as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden_seed42.json")


def _g():
    with open(GOLDEN) as f:
        return json.load(f)


def test_seed42_initial_hand():
    g = _g()
    eng = O.Engine(seed=42)
    assert eng.hand == g["initial_hand_ids"]
    assert [O.PIECE_NAMES[i] for i in eng.hand] == g["initial_hand_names"]


def test_seed42_random_game_golden():
    g = _g()["play_random_game_42"]
    st = O.play_random_game(42)
    for k, v in g.items():
        assert st[k] == v, k


def test_random_game_deterministic():  # reference tests/test_engine.py:357-363
    for s in range(5):
        assert O.play_random_game(s) == O.play_random_game(s)


# ---- tests/test_pieces.py known answers -----------------------------------
BLOCK_COUNTS = {"SINGLE": 1, "DOMINO_H": 2, "DOMINO_V": 2, "DIAG2_TL_BR": 2, "DIAG2_TR_BL": 2, "TRIO_H": 3,
                "TRIO_V": 3, "DIAG3_TL_BR": 3, "DIAG3_TR_BL": 3, "TRIO_L1": 3, "TRIO_L2": 3, "TRIO_L3": 3,
                "TRIO_L4": 3, "I_H": 4, "I_V": 4, "I5_H": 5, "I5_V": 5, "O": 4, "T_UP": 4, "T_DOWN": 4, "T_LEFT": 4,
                "T_RIGHT": 4, "S_H": 4, "S_V": 4, "Z_H": 4, "Z_V": 4, "L_1": 4, "L_2": 4, "L_3": 4, "L_4": 4,
                "J_1": 4, "J_2": 4, "J_3": 4, "J_4": 4, "RECT_2x3_H": 6, "RECT_2x3_V": 6, "SQUARE_3x3": 9}
EXACT_SHAPES = {  # tests/test_pieces.py:138-182
    "SINGLE": {(0, 0)}, "DOMINO_H": {(0, 0), (0, 1)}, "DOMINO_V": {(0, 0), (1, 0)},
    "TRIO_H": {(0, 0), (0, 1), (0, 2)}, "TRIO_V": {(0, 0), (1, 0), (2, 0)},
    "I_H": {(0, 0), (0, 1), (0, 2), (0, 3)}, "I5_V": {(r, 0) for r in range(5)},
    "O": {(0, 0), (0, 1), (1, 0), (1, 1)}, "SQUARE_3x3": {(r, c) for r in range(3) for c in range(3)},
    "T_UP": {(0, 1), (1, 0), (1, 1), (1, 2)}, "L_1": {(0, 0), (1, 0), (2, 0), (2, 1)},
}


def test_piece_table_known_answers():
    assert O.NUM_PIECES == 37 and len(set(O.PIECE_NAMES)) == 37
    for name, cells in zip(O.PIECE_NAMES, O.PIECE_CELLS):
        assert len(cells) == BLOCK_COUNTS[name]
        assert min(r for r, _ in cells) == 0 and min(c for _, c in cells) == 0
        assert len(set(cells)) == len(cells)
    for name, cells in EXACT_SHAPES.items():
        assert set(O.PIECE_CELLS[O.PIECE_NAMES.index(name)]) == cells
    dims = {"SINGLE": (1, 1), "DOMINO_H": (2, 1), "DOMINO_V": (1, 2), "I_H": (4, 1), "I_V": (1, 4), "O": (2, 2),
            "SQUARE_3x3": (3, 3)}
    for name, (w, h) in dims.items():
        i = O.PIECE_NAMES.index(name)
        assert (O.PIECE_W[i], O.PIECE_H[i]) == (w, h)
    assert O.PIECE_NAMES[0] == "SINGLE"  # piece_to_one_hot(SINGLE)[0] == 1


def test_piece_table_bits_match_survey_appendix_b():
    g = _g()["piece_bits"]
    for i, cells in enumerate(O.PIECE_CELLS):
        bits = sum(1 << (r * 8 + c) for r, c in cells)
        assert bits == int(g[i], 16), O.PIECE_NAMES[i]


# ---- tests/test_board.py known answers ------------------------------------
def _grid():
    return [[0] * 8 for _ in range(8)]


def _pid(name):
    return O.PIECE_NAMES.index(name)


def test_board_placement_known_answers():
    g = _grid()
    assert O.can_place(g, _pid("SINGLE"), 0, 0) and O.can_place(g, _pid("SINGLE"), 7, 7)
    assert O.can_place(g, _pid("SQUARE_3x3"), 5, 5)
    assert not O.can_place(g, _pid("I_H"), 0, 6) and not O.can_place(g, _pid("SQUARE_3x3"), 6, 6)
    assert not O.can_place(g, _pid("SINGLE"), -1, 0) and not O.can_place(g, _pid("SINGLE"), 0, -1)
    cnt = lambda pid: sum(O.can_place(g, pid, r, c) for r in range(8) for c in range(8))  # noqa: E731
    assert cnt(_pid("SINGLE")) == 64 and cnt(_pid("I_H")) == 40
    O.place(g, _pid("SINGLE"), 4, 4)
    assert cnt(_pid("SINGLE")) == 63
    assert not O.can_place(g, _pid("SQUARE_3x3"), 3, 3)


def test_line_clears_known_answers():
    g = _grid()
    for c in range(8):
        g[0][c] = 1
    assert O.clear_lines(g) == (1, 0) and O.total_blocks(g) == 0
    g = _grid()
    for c in range(7):
        g[0][c] = 1
    assert O.clear_lines(g) == (0, 0) and O.total_blocks(g) == 7
    g = _grid()
    for c in range(8):
        g[4][c] = 1
    for r in range(8):
        g[r][4] = 1
    assert O.total_blocks(g) == 15
    assert O.clear_lines(g) == (1, 1) and O.total_blocks(g) == 0
    g = [[1] * 8 for _ in range(8)]
    assert O.clear_lines(g) == (8, 8) and O.total_blocks(g) == 0


def test_holes_and_center_known_answers():
    g = _grid()
    assert O.count_holes(g) == 0 and O.center_openness(g) == 1.0
    for r, c in [(0, 1), (2, 1), (1, 0), (1, 2)]:
        g[r][c] = 1
    assert O.count_holes(g) == 2  # tests/test_board.py:387-400
    g = _grid()
    for r in range(2, 6):
        for c in range(2, 6):
            g[r][c] = 1
    assert O.center_openness(g) == 0.0


# ---- tests/test_engine.py / test_environment.py known answers ------------
def test_engine_known_answers():
    e = O.Engine(seed=42)
    assert (e.score, e.moves, e.combo, e.over) == (0, 0, 0, False)
    assert not e.can_place_piece(-1, 0, 0) and not e.can_place_piece(3, 0, 0)
    assert e.make_move(0, -1, -1) is None and e.moves == 0
    mv = e.valid_moves()
    assert int(e.action_mask().sum()) == len(mv)
    p, r, c = mv[0]
    res = e.make_move(p, r, c)
    assert res is not None and res["blocks_placed"] > 0 and e.moves == 1
    assert not e.can_place_piece(p, r, c)
    assert e.action_mask()[p].sum() == 0


def test_env_action_encoding():
    assert O.Env.action_to_move(0) == (0, 0, 0)
    assert O.Env.action_to_move(64) == (1, 0, 0)
    assert O.Env.action_to_move(128) == (2, 0, 0)
    assert O.Env.action_to_move(63) == (0, 7, 7)


def test_env_invalid_action_and_termination():
    env = O.Env(seed=42)
    obs, info = env.reset()
    bad = int(np.where(obs["action_mask"] == 0)[0][0])
    _, r, t, tr, info = env.step(bad)
    assert r == -10.0 and info["invalid_action"] and not t and not tr
    rng = np.random.default_rng(0)
    for _ in range(1000):
        valid = np.nonzero(env.obs()["action_mask"])[0]
        _, r, t, _, _ = env.step(int(rng.choice(valid)))
        if t:
            break
    assert t
    assert env.obs()["action_mask"].sum() == 0  # game over <=> empty mask
    _, r, t, _, info = env.step(0)
    assert r == -10.0 and info["invalid_action"]


def test_vec_env_shapes():
    v = O.VecEnv(4, seed=1)
    obs, infos = v.reset()
    assert obs["board"].shape == (4, 8, 8) and obs["pieces"].shape == (4, 3, 8, 8)
    assert obs["action_mask"].shape == (4, 192) and len(infos) == 4

"""Crowded-board fixtures for the hand-generator stress tests (not a test module).

Start states where the env's next move uses the last unused slot of its hand, so that move triggers
_generate_new_pieces (engine.py:155-172) on a crowded board: random 45-95 % fills, boards with two
isolated holes per row and column, and the singles-only boards of _ISOLATED.  Optional Lemire
rejections at chosen PCG64 stream positions (pieces.py:350-355 -> numpy integers(0, 37)).
The oracle side is oracle.bb_game.Env set to the same state.
"""
import numpy as np

from oracle import bb_game as O

# 16 holes, two per row and per column, no two within one cell of each other (8-neighbourhood): every
# piece but SINGLE is 8-connected, so only singles fit.  After the step's own single, a hand is solvable
# only if it holds a single for the other hole of that row or column and the rest fits the cleared line
# (median 24 attempts, ~5% of the searches run all 100)
_ISOLATED = [(0, 1), (0, 3), (1, 5), (1, 7), (2, 1), (2, 3), (3, 5), (3, 7), (4, 0), (4, 2), (5, 4), (5, 6),
             (6, 0), (6, 2), (7, 4), (7, 6)]


def _case(rng, fill):
    if fill == -2.0:
        grid = np.ones((8, 8), dtype=np.int8)
        for r, c in _ISOLATED:
            grid[r, c] = 0
        if rng.integers(2):
            grid = grid.T
        grid = np.ascontiguousarray(grid[:: 1 - 2 * int(rng.integers(2)), :: 1 - 2 * int(rng.integers(2))])
        empties = np.argwhere(grid == 0)
        r, c = empties[rng.integers(len(empties))]
        return grid, int(r), int(c)
    if fill < 0:
        # two isolated holes per row/column: almost no hand fits -> attempts
        # run to the 100 limit (last hand kept) and most envs end the game
        while True:
            grid = np.ones((8, 8), dtype=np.int8)
            p1, p2 = rng.permutation(8), rng.permutation(8)
            if np.any(p1 == p2):
                continue
            grid[np.arange(8), p1] = 0
            grid[np.arange(8), p2] = 0
            if (grid.sum(axis=0) == 6).all():
                break
        empties = np.argwhere(grid == 0)
        r, c = empties[rng.integers(len(empties))]
        return grid, int(r), int(c)
    grid = (rng.random((8, 8)) < fill).astype(np.int8)
    # no full line on the start board (the reference never holds one)
    for r in range(8):
        if grid[r].all():
            grid[r, rng.integers(8)] = 0
    for c in range(8):
        if grid[:, c].all():
            grid[rng.integers(8), c] = 0
    empties = np.argwhere(grid == 0)
    r, c = empties[rng.integers(len(empties))]
    return grid, int(r), int(c)


_M = 0x2360ED051FC65DA44385DF649FCCF645  # PCG64 multiplier (numpy pcg64.h)
_MASK = (1 << 128) - 1


def _state_with_zero_draw(rng, inc, c, high):
    """A PCG64 state whose c-th 64-bit output (1-based; numpy steps, then
    outputs XSL-RR of the new state) has a zero low (high) 32-bit half: that
    32-bit draw is rejected by numpy's Lemire integers(0, 37) (0 * 37 < 2**32 % 37),
    so the attempts after it shift by one value.  p ~ 1.6e-9 per draw otherwise."""
    o = int(rng.integers(1, 1 << 32)) << 32 if not high else int(rng.integers(1, 1 << 32))
    hi = int(rng.integers(0, 1 << 63)) << 1 | 1
    rot = hi >> 58
    x = ((o << rot) | (o >> (64 - rot))) & ((1 << 64) - 1) if rot else o
    sc = (hi << 64) | (hi ^ x)
    a, sacc = 1, 0
    for _ in range(c):  # s_c = M^c s0 + S_c inc
        sacc = (sacc + a) & _MASK
        a = (a * _M) & _MASK
    return ((sc - sacc * inc) * pow(a, -1, 1 << 128)) & _MASK



def crowded_setup(fill, n, reject_at=None, seed_base=5000):
    """n start states (set_state arrays) and their oracle envs.  The action of the first step places SINGLE
    (slot 2, the last unused slot) on an empty cell.  reject_at: per env, the LCG output (1-based) whose low
    (even env) or high (odd env) half is a rejected draw; None: the streams of default_rng(seed_base + i)."""
    rng = np.random.default_rng(int(fill * 100) + 1000)
    boards = np.zeros(n, np.uint64)
    hands = np.zeros(n, np.uint32)
    acts = np.zeros(n, np.int32)
    refs = []
    for i in range(n):
        grid, r, c = _case(rng, fill)
        a, b = (int(x) for x in rng.integers(0, 37, 2))
        boards[i] = O.grid_to_u64(grid.tolist())
        hands[i] = a | (b << 6) | (0 << 12) | (0b011 << 18)
        acts[i] = 128 + r * 8 + c
        env = O.Env(seed=seed_base + i)
        env.engine.grid = grid.tolist()
        env.engine.hand = [a, b, 0]
        env.engine.used = [True, True, False]
        env.engine.rng = np.random.default_rng(seed_base + i)
        refs.append(env)
    state = dict(board=boards, hand=hands, prev_holes=np.zeros(n), prev_center=np.zeros(n))
    if reject_at is not None:
        st_rng = np.zeros((n, 3), np.uint64)
        for i, env in enumerate(refs):
            inc = env.engine.rng.bit_generator.state["state"]["inc"]
            s0 = _state_with_zero_draw(rng, inc, int(reject_at[i]), high=bool(i & 1))
            env.engine.rng.bit_generator.state = {"bit_generator": "PCG64", "state": {"state": s0, "inc": inc},
                                                  "has_uint32": 0, "uinteger": 0}
            st_rng[i] = (s0 >> 64, s0 & ((1 << 64) - 1), 0)
        state["rng"] = st_rng
    return state, acts, refs


def mask_bits(mask_bool):
    """(3, 8, 8) or (192,) bool -> the three u64 words of bbvec.h's mask layout."""
    m = np.asarray(mask_bool, dtype=bool).reshape(3, 64)
    return np.packbits(m, axis=1, bitorder="little").view("<u8").reshape(3)

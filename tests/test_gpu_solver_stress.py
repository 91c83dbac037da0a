"""GPU parity of the hand generator on crowded boards.

Random 45-80 % filled boards where the last unused slot holds SINGLE: placing
it triggers _generate_new_pieces (engine.py:155-172) on a crowded board, where
many 3-draw attempts fail (and some envs exhaust all 100 attempts and keep the
last hand).  The device result (hand, pcg state, score, reward, game over)
must equal the oracle's reference DFS exactly; this drives both the per-lane
solver and the wave-cooperative escalation kernel.
"""
import numpy as np
import pytest

from oracle import bb_game as O

pytestmark = pytest.mark.gpu


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


@pytest.mark.parametrize("fill", [0.45, 0.6, 0.7, 0.8, 0.9, 0.95, -1.0, -2.0])
@pytest.mark.parametrize("pack", ["1,0", "32,32", "3,7"])
def test_crowded_board_hand_generation(cuda, fill, pack, monkeypatch):
    """pack = escalation schedule (attempts per env in the first round, in
    later rounds; 0 = double the previous round's, capped at 32): every
    schedule must give the same hands."""
    _crowded(cuda, fill, pack, monkeypatch)


@pytest.mark.parametrize("fill", [0.6, 0.8, 0.95, -1.0])
def test_crowded_board_debug_fallback(cuda, fill, monkeypatch):
    """BB_DEBUG_MODE=2 (the solver counters) switches escalate_kernel to the
    one-env-at-a-time wave search (gen_hand_wave, bbvec.h bb_debug_counters):
    that path must stay bit-exact too."""
    monkeypatch.setenv("BB_DEBUG_MODE", "2")
    _crowded(cuda, fill, "8,32", monkeypatch)


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


def _crowded(cuda, fill, pack, monkeypatch, reject_at=None):
    """reject_at: per env, the LCG output (1-based) whose low or high half is a
    rejected draw (None: the streams of default_rng(seed))."""
    from runtime.device_env import DeviceEnvBatch

    first, nxt = pack.split(",")
    monkeypatch.setenv("BB_PACK_FIRST", first)
    monkeypatch.setenv("BB_PACK_NEXT", nxt)

    n = 512
    rng = np.random.default_rng(int(fill * 100) + 1000)
    dev = DeviceEnvBatch(n, seeds=[5000 + i for i in range(n)], device=cuda)
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
        env = O.Env(seed=5000 + i)
        env.engine.grid = grid.tolist()
        env.engine.hand = [a, b, 0]
        env.engine.used = [True, True, False]
        env.engine.rng = np.random.default_rng(5000 + i)
        refs.append(env)
    extra = {}
    if reject_at is not None:
        st_rng = np.zeros((n, 3), np.uint64)
        for i, env in enumerate(refs):
            inc = env.engine.rng.bit_generator.state["state"]["inc"]
            s0 = _state_with_zero_draw(rng, inc, int(reject_at[i]), high=bool(i & 1))
            env.engine.rng.bit_generator.state = {"bit_generator": "PCG64", "state": {"state": s0, "inc": inc},
                                                  "has_uint32": 0, "uinteger": 0}
            st_rng[i] = (s0 >> 64, s0 & ((1 << 64) - 1), 0)
        extra["rng"] = st_rng
    dev.set_state(board=boards, hand=hands, prev_holes=np.zeros(n), prev_center=np.zeros(n), **extra)
    import torch

    act_t = torch.from_numpy(acts).to(cuda)
    dev.step(act_t, want_f64=True, want_info=True)
    st = dev.state()
    rew = dev.reward_f64.cpu().numpy()
    term = dev.terminated.cpu().numpy()
    info = dev.info_host()
    attempts = []
    for i, env in enumerate(refs):
        _, r_ref, t_ref, _, inf = env.step(int(acts[i]))
        attempts.append(env.engine.attempts_last)
        assert rew[i] == r_ref, i
        assert bool(term[i]) == t_ref, i
        assert info[i]["score"] == inf["score"]
        if not t_ref:
            h = int(st["hand"][i])
            assert [(h >> (6 * s)) & 63 for s in range(3)] == env.engine.hand, i
            s = env.engine.rng.bit_generator.state
            assert (int(st["rng"][i, 0]) << 64 | int(st["rng"][i, 1])) == s["state"]["state"], i
            assert bool((h >> 22) & 1) == bool(s["has_uint32"]), i
            if s["has_uint32"]:
                assert int(st["rng"][i, 2]) == s["uinteger"], i
        else:  # terminated -> auto-reset happened; the terminal hand is in info
            h = int(info[i]["term_hand"])
            assert [(h >> (6 * s)) & 63 for s in range(3)] == env.engine.hand, i
    attempts = np.array(attempts)
    assert attempts.max() > 1  # the crowded boards really exercised rejection sampling
    dev.close()
    return attempts


@pytest.mark.parametrize("fill", [0.9, -2.0])
@pytest.mark.parametrize("pack", ["8,32", "1,0"])
def test_lemire_rejection_inside_hand_search(cuda, fill, pack, monkeypatch):
    """A rejected 32-bit draw at a chosen stream position (attempt 0 .. 99,
    low and high halves): the jump-ahead batches of the wave and workgroup
    searches assume three values per attempt and must fall back to the exact
    sequential stream from there on."""
    n = 512
    reject_at = 1 + (np.arange(n) * 37) % 60  # LCG outputs 1 .. 60 = attempts 0 .. 39
    attempts = _crowded(cuda, fill, pack, monkeypatch, reject_at=reject_at)
    reached = attempts > (2 * (reject_at - 1) + (np.arange(n) & 1)) // 3
    # searches that got past their rejected draw: ~60% on the singles-only boards, a few at fill 0.9
    assert reached.sum() > (n // 2 if fill == -2.0 else 4)

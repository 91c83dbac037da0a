"""Pure-Python CPU oracle of the Block Blast game + Gym surface.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Cell-grid restatement
of the reference algorithms, each function citing the reference file:line it
follows.  Deliberately written with per-cell loops like the reference (this is
also what makes it a faithful *speed* model of the reference's CPU path for the
``cpu_baseline`` leg of ``bench.py``).

The piece stream is ``numpy.random.default_rng(seed)`` exactly as the
reference uses it (``engine.py:109,138``, ``pieces.py:354``); numpy is a
dependency, not the reference.
"""
from __future__ import annotations

import numpy as np

BOARD = 8
HAND = 3
ACTIONS = HAND * BOARD * BOARD  # block_blast_env.py:38-40

# --------------------------------------------------------------------------
# Piece table: pieces.py:78-236 (shapes), 244-318 (dict order == index order).
# Written here as ASCII pictures ('#' = block) in index order.
# --------------------------------------------------------------------------
_PICTURES = [
    ("SINGLE", "#"),
    ("DOMINO_H", "##"),
    ("DOMINO_V", "#|#"),
    ("DIAG2_TL_BR", "#.|.#"),
    ("DIAG2_TR_BL", ".#|#."),
    ("TRIO_H", "###"),
    ("TRIO_V", "#|#|#"),
    ("DIAG3_TL_BR", "#..|.#.|..#"),
    ("DIAG3_TR_BL", "..#|.#.|#.."),
    ("TRIO_L1", "#.|##"),
    ("TRIO_L2", "##|.#"),
    ("TRIO_L3", "##|#."),
    ("TRIO_L4", ".#|##"),
    ("I_H", "####"),
    ("I_V", "#|#|#|#"),
    ("I5_H", "#####"),
    ("I5_V", "#|#|#|#|#"),
    ("O", "##|##"),
    ("T_UP", ".#.|###"),
    ("T_DOWN", "###|.#."),
    ("T_LEFT", "#.|##|#."),
    ("T_RIGHT", ".#|##|.#"),
    ("S_H", ".##|##."),
    ("S_V", "#.|##|.#"),
    ("Z_H", "##.|.##"),
    ("Z_V", ".#|##|#."),
    ("L_1", "#.|#.|##"),
    ("L_2", "###|#.."),
    ("L_3", "##|.#|.#"),
    ("L_4", "..#|###"),
    ("J_1", ".#|.#|##"),
    ("J_2", "#..|###"),
    ("J_3", "##|#.|#."),
    ("J_4", "###|..#"),
    ("RECT_2x3_H", "###|###"),
    ("RECT_2x3_V", "##|##|##"),
    ("SQUARE_3x3", "###|###|###"),
]


def _cells(picture: str):
    out = []
    for r, row in enumerate(picture.split("|")):
        for c, ch in enumerate(row):
            if ch == "#":
                out.append((r, c))
    return tuple(out)


PIECE_NAMES = [n for n, _ in _PICTURES]
PIECE_CELLS = [_cells(p) for _, p in _PICTURES]
NUM_PIECES = len(PIECE_CELLS)  # pieces.py:318
PIECE_H = [max(r for r, _ in cs) + 1 for cs in PIECE_CELLS]  # pieces.py:32-37
PIECE_W = [max(c for _, c in cs) + 1 for cs in PIECE_CELLS]  # pieces.py:24-30
assert NUM_PIECES == 37


def piece_mask(pid: int) -> np.ndarray:
    """pieces.py:39-45 ``Piece.to_mask``: f32 (8,8) with the shape at origin."""
    m = np.zeros((BOARD, BOARD), dtype=np.float32)
    for r, c in PIECE_CELLS[pid]:
        m[r, c] = 1.0
    return m


def draw_hand(rng: np.random.Generator):
    """pieces.py:350-355 ``get_random_pieces(3, rng)``."""
    return [int(x) for x in rng.choice(NUM_PIECES, size=HAND, replace=True)]


# --------------------------------------------------------------------------
# Board (board.py)
# --------------------------------------------------------------------------
def can_place(grid, pid, row, col) -> bool:
    """board.py:71-93: bounds + collision for every block."""
    for dr, dc in PIECE_CELLS[pid]:
        r, c = row + dr, col + dc
        if r < 0 or r >= BOARD or c < 0 or c >= BOARD:
            return False
        if grid[r][c] != 0:
            return False
    return True


def place(grid, pid, row, col) -> None:
    """board.py:110-113 (called only after a successful can_place)."""
    for dr, dc in PIECE_CELLS[pid]:
        grid[row + dr][col + dc] = 1


def clear_lines(grid):
    """board.py:144-193: full rows/cols found on the same grid, then all cleared.

    Returns (rows_cleared, cols_cleared).
    """
    rows = [r for r in range(BOARD) if all(grid[r][c] == 1 for c in range(BOARD))]
    cols = [c for c in range(BOARD) if all(grid[r][c] == 1 for r in range(BOARD))]
    for r in rows:
        for c in range(BOARD):
            grid[r][c] = 0
    for c in cols:
        for r in range(BOARD):
            grid[r][c] = 0
    return len(rows), len(cols)


def count_holes(grid) -> int:
    """board.py:195-216: empty cells whose 4 neighbours are filled or OOB."""
    holes = 0
    for r in range(BOARD):
        for c in range(BOARD):
            if grid[r][c] != 0:
                continue
            blocked = 0
            for dr, dc in ((-1, 0), (1, 0), (0, -1), (0, 1)):
                nr, nc = r + dr, c + dc
                if not (0 <= nr < BOARD and 0 <= nc < BOARD) or grid[nr][nc] == 1:
                    blocked += 1
            if blocked == 4:
                holes += 1
    return holes


def center_filled(grid) -> int:
    """Integer part of board.py:236-243 (``sum(grid[2:6,2:6])``)."""
    return sum(grid[r][c] for r in range(2, 6) for c in range(2, 6))


def center_openness(grid) -> float:
    """board.py:236-243."""
    return 1.0 - (center_filled(grid) / 16.0)


def total_blocks(grid) -> int:
    return sum(sum(row) for row in grid)


def grid_to_u64(grid) -> int:
    v = 0
    for r in range(BOARD):
        for c in range(BOARD):
            if grid[r][c]:
                v |= 1 << (r * BOARD + c)
    return v


def u64_to_grid(v: int):
    return [[(v >> (r * BOARD + c)) & 1 for c in range(BOARD)] for r in range(BOARD)]


# --------------------------------------------------------------------------
# Engine (engine.py)
# --------------------------------------------------------------------------
class Engine:
    """engine.py:81-535 ``GameEngine`` (state + rules)."""

    MAX_ATTEMPTS = 100  # engine.py:161

    def __init__(self, seed=None):
        # engine.py:99-125
        self.grid = [[0] * BOARD for _ in range(BOARD)]
        self.rng = np.random.default_rng(seed)
        self.hand = [0, 0, 0]
        self.used = [False, False, False]
        self.score = 0
        self.combo = 0
        self.moves = 0
        self.lines = 0
        self.over = False
        self.max_combo = 0
        self.blocks = 0
        self.attempts_last = 0  # diagnostics only
        self._generate()

    def reset(self, seed=None):
        """engine.py:127-153."""
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.grid = [[0] * BOARD for _ in range(BOARD)]
        self.used = [False, False, False]
        self.score = 0
        self.combo = 0
        self.moves = 0
        self.lines = 0
        self.over = False
        self.max_combo = 0
        self.blocks = 0
        self._generate()

    # engine.py:155-172
    def _generate(self):
        for attempt in range(self.MAX_ATTEMPTS):
            self.hand = draw_hand(self.rng)
            self.used = [False, False, False]
            self.attempts_last = attempt + 1
            if self._solvable([row[:] for row in self.grid], [False, False, False]):
                return

    # engine.py:181-224 (+ _simulate_line_clears 226-238)
    def _solvable(self, grid, used) -> bool:
        if all(used):
            return True
        for idx in range(HAND):
            if used[idx]:
                continue
            pid = self.hand[idx]
            for row in range(BOARD - PIECE_H[pid] + 1):
                for col in range(BOARD - PIECE_W[pid] + 1):
                    if not can_place(grid, pid, row, col):
                        continue
                    g2 = [r[:] for r in grid]
                    place(g2, pid, row, col)
                    clear_lines(g2)
                    u2 = list(used)
                    u2[idx] = True
                    if self._solvable(g2, u2):
                        return True
        return False

    def can_place_piece(self, p, row, col) -> bool:
        """engine.py:326-346."""
        if p < 0 or p >= HAND:
            return False
        if self.used[p]:
            return False
        if self.over:
            return False
        return can_place(self.grid, self.hand[p], row, col)

    def valid_moves(self):
        """engine.py:348-362 (piece-major, then row, col)."""
        out = []
        for p in range(HAND):
            if self.used[p]:
                continue
            for row in range(BOARD):
                for col in range(BOARD):
                    if can_place(self.grid, self.hand[p], row, col):
                        out.append((p, row, col))
        return out

    def action_mask(self) -> np.ndarray:
        """engine.py:364-380: bool (3,8,8); game-over status is NOT consulted."""
        m = np.zeros((HAND, BOARD, BOARD), dtype=bool)
        for p in range(HAND):
            if self.used[p]:
                continue
            for row in range(BOARD):
                for col in range(BOARD):
                    if can_place(self.grid, self.hand[p], row, col):
                        m[p, row, col] = True
        return m

    def has_valid_moves(self) -> bool:
        """engine.py:382-388 (+ board.py:134-142)."""
        for p in range(HAND):
            if self.used[p]:
                continue
            pid = self.hand[p]
            for row in range(BOARD - PIECE_H[pid] + 1):
                for col in range(BOARD - PIECE_W[pid] + 1):
                    if can_place(self.grid, pid, row, col):
                        return True
        return False

    def make_move(self, p, row, col):
        """engine.py:390-454.  Returns a dict mirroring ``MoveResult`` or None."""
        if not self.can_place_piece(p, row, col):
            return None
        pid = self.hand[p]
        n = len(PIECE_CELLS[pid])
        place(self.grid, pid, row, col)
        self.used[p] = True
        self.moves += 1
        self.blocks += n
        rows, cols = clear_lines(self.grid)
        lines = rows + cols
        if lines > 0:  # engine.py:419-424
            self.combo += 1
            self.max_combo = max(self.max_combo, self.combo)
            self.lines += lines
        else:
            self.combo = 0
        # engine.py:274-312 with blocks_in_lines = lines*8 (engine.py:427)
        gained = n
        if lines > 0:
            gained += (lines * BOARD * 10) * min(lines, 4) * min(self.combo + 1, 8)
        self.score += gained
        if all(self.used):  # engine.py:432-437
            self._generate()
        if not self.has_valid_moves():  # engine.py:440-441
            self.over = True
        return {
            "blocks_placed": n,
            "rows_cleared": rows,
            "cols_cleared": cols,
            "lines_cleared": lines,
            "combo_multiplier": min(lines, 4) if lines > 0 else 1,
            "score_gained": gained,
            "game_over": self.over,
        }

    def observation(self):
        """engine.py:478-507."""
        board = np.array(self.grid, dtype=np.float32)
        pieces = np.zeros((HAND, BOARD, BOARD), dtype=np.float32)
        for i in range(HAND):
            if not self.used[i]:
                pieces[i] = piece_mask(self.hand[i])
        return board, pieces, self.action_mask()

    def statistics(self):
        """engine.py:509-520."""
        return {
            "score": self.score,
            "moves_made": self.moves,
            "total_lines_cleared": self.lines,
            "max_combo": self.max_combo,
            "total_blocks_placed": self.blocks,
            "board_fill_ratio": total_blocks(self.grid) / (BOARD ** 2),
            "holes": count_holes(self.grid),
            "center_openness": center_openness(self.grid),
        }


def play_random_game(seed=None):
    """engine.py:538-576 (move choice interleaved with the piece stream)."""
    eng = Engine(seed=seed)
    while not eng.over:
        moves = eng.valid_moves()
        if not moves:
            break
        mv = moves[int(eng.rng.choice(len(moves)))]
        eng.make_move(*mv)
    return eng.statistics()


# --------------------------------------------------------------------------
# Gym surface (block_blast_env.py)
# --------------------------------------------------------------------------
DEFAULT_REWARDS = {  # block_blast_env.py:63-71
    "line_clear_base": 1.0,
    "block_placed": 0.01,
    "game_over_penalty": -1.0,
    "hole_penalty": -0.05,
    "center_bonus": 0.02,
    "combo_multiplier_bonus": 0.5,
    "survival_bonus": 0.001,
}


class Env:
    """block_blast_env.py:20-323 ``BlockBlastEnv`` (without gymnasium)."""

    def __init__(self, reward_config=None, seed=None):
        self.seed_value = seed
        self.rw = dict(DEFAULT_REWARDS)
        if reward_config:
            self.rw.update(reward_config)
        self.engine = Engine(seed=seed)
        self.prev_holes = 0
        self.prev_center = 1.0

    @staticmethod
    def action_to_move(a):
        """block_blast_env.py:104-118."""
        return a // 64, (a % 64) // 8, a % 8

    def obs(self):
        """block_blast_env.py:134-146."""
        b, p, m = self.engine.observation()
        return {"board": b, "pieces": p, "action_mask": m.flatten().astype(np.int8)}

    def _reward(self, res) -> float:
        """block_blast_env.py:148-193 (fp64, this exact order)."""
        rw = self.rw
        reward = 0.0
        reward += res["blocks_placed"] * rw["block_placed"]
        reward += rw["survival_bonus"]
        if res["lines_cleared"] > 0:
            line_reward = res["lines_cleared"] * rw["line_clear_base"]
            line_reward *= res["combo_multiplier"]
            reward += line_reward
            if res["combo_multiplier"] > 1:
                reward += (res["combo_multiplier"] - 1) * rw["combo_multiplier_bonus"]
        if res["game_over"]:
            reward += rw["game_over_penalty"]
        holes = count_holes(self.engine.grid)
        delta = holes - self.prev_holes
        if delta > 0:
            reward += delta * rw["hole_penalty"]
        self.prev_holes = holes
        center = center_openness(self.engine.grid)
        if center >= self.prev_center:
            reward += rw["center_bonus"] * 0.1
        self.prev_center = center
        return reward

    def info(self, res=None):
        """block_blast_env.py:266-288."""
        st = self.engine.statistics()
        info = {
            "score": st["score"],
            "moves": st["moves_made"],
            "lines_cleared": st["total_lines_cleared"],
            "max_combo": st["max_combo"],
            "blocks_placed": st["total_blocks_placed"],
            "board_fill": st["board_fill_ratio"],
            "holes": st["holes"],
            "invalid_action": False,
        }
        if res is not None:
            info["last_move"] = {
                "blocks_placed": res["blocks_placed"],
                "lines_cleared": res["lines_cleared"],
                "combo_multiplier": res["combo_multiplier"],
                "score_gained": res["score_gained"],
            }
        return info

    def reset(self, seed=None):
        """block_blast_env.py:195-222 (re-seeds with seed_value every episode)."""
        if seed is not None:
            self.seed_value = seed
        self.engine.reset(seed=self.seed_value)
        self.prev_holes = 0
        self.prev_center = 1.0
        return self.obs(), self.info()

    def step(self, action):
        """block_blast_env.py:224-264."""
        p, r, c = self.action_to_move(int(action))
        if not self.engine.can_place_piece(p, r, c):
            info = self.info()
            info["invalid_action"] = True
            return self.obs(), -10.0, False, False, info
        res = self.engine.make_move(p, r, c)
        reward = self._reward(res)
        terminated = bool(res["game_over"])
        return self.obs(), reward, terminated, False, self.info(res)


    def flat_obs(self):
        """block_blast_env.py:360-389 ``BlockBlastEnvFlat._get_observation``: board (64, row-major), then per
        hand slot a 37-wide one-hot of the piece id (all zeros for a used slot), then the 3 used flags as
        0/1 -- 178 float32 values -- and the int8 action mask."""
        g = self.engine
        vals = [float(g.grid[r][c]) for r in range(BOARD) for c in range(BOARD)]
        for slot in range(HAND):
            one_hot = [0.0] * len(_PICTURES)
            if not g.used[slot]:
                one_hot[g.hand[slot]] = 1.0
            vals += one_hot
        vals += [1.0 if u else 0.0 for u in g.used]
        return {"obs": np.array(vals, dtype=np.float32),
                "action_mask": g.action_mask().flatten().astype(np.int8)}


class ReturnNormalizer:
    """wrappers.py:144-184 ``NormalizedRewardWrapper`` restated with an independent variance: instead of
    the reference's incremental Chan update (wrappers.py:187-221) it keeps every discounted return and
    evaluates the pooled moments of the prior pseudo-sample (count 1e-4, mean 0, variance 1) and all
    returns from scratch in fp64 with ``math.fsum``.  Equal to the reference's arithmetic up to fp64
    rounding (tests compare within 1e-12 relative)."""

    PRIOR_COUNT = 1e-4

    def __init__(self, gamma=0.99, epsilon=1e-8):
        self.gamma, self.epsilon = gamma, epsilon
        self.returns = 0.0
        self.history = []

    def variance(self) -> float:
        import math

        c0, k = self.PRIOR_COUNT, len(self.history)
        n = c0 + k
        mean = math.fsum(self.history) / n  # the prior's mean is 0
        m2 = c0 * 1.0 + c0 * mean * mean + math.fsum((x - mean) ** 2 for x in self.history)
        return m2 / n

    def step(self, reward: float, done: bool) -> float:
        """wrappers.py:166-180: returns the normalised reward."""
        self.returns = self.returns * self.gamma + reward
        self.history.append(self.returns)
        out = reward / (self.variance() ** 0.5 + self.epsilon)
        if done:
            self.returns = 0.0
        return out

    def reset(self):
        self.returns = 0.0  # wrappers.py:182-184 (the statistics persist)


class FrameStack:
    """wrappers.py:224-280 ``FrameStackWrapper``: the last ``num_frames`` boards, oldest first; a reset
    fills the stack with copies of the first board."""

    def __init__(self, num_frames=4):
        self.num_frames = num_frames
        self.frames = None

    def reset(self, board):
        self.frames = [board.copy() for _ in range(self.num_frames)]
        return np.stack(self.frames, axis=0)

    def step(self, board):
        self.frames = self.frames[1:] + [board.copy()]
        return np.stack(self.frames, axis=0)


class VecEnv:
    """wrappers.py:14-141 ``VectorizedBlockBlastEnv`` (sequential loop)."""

    def __init__(self, num_envs, seed=None, reward_config=None):
        self.num_envs = num_envs
        self.envs = [
            Env(reward_config=reward_config, seed=(seed + i if seed is not None else None))
            for i in range(num_envs)
        ]

    @staticmethod
    def _stack(obs_list):
        return {
            "board": np.stack([o["board"] for o in obs_list]),
            "pieces": np.stack([o["pieces"] for o in obs_list]),
            "action_mask": np.stack([o["action_mask"] for o in obs_list]),
        }

    def reset(self, seed=None):
        obs, infos = [], []
        for i, e in enumerate(self.envs):
            o, inf = e.reset(seed=(seed + i if seed is not None else None))
            obs.append(o)
            infos.append(inf)
        return self._stack(obs), infos

    def step(self, actions):
        n = self.num_envs
        rewards = np.zeros(n, dtype=np.float32)
        term = np.zeros(n, dtype=bool)
        trunc = np.zeros(n, dtype=bool)
        obs, infos = [], []
        for i, (e, a) in enumerate(zip(self.envs, actions)):
            o, r, t, tr, inf = e.step(int(a))
            if t or tr:  # wrappers.py:97-102
                inf["terminal_observation"] = o
                inf["final_score"] = inf["score"]
                o, _ = e.reset()
            obs.append(o)
            rewards[i] = r
            term[i] = t
            trunc[i] = tr
            infos.append(inf)
        return self._stack(obs), rewards, term, trunc, infos

    def get_action_masks(self):
        return np.stack([e.obs()["action_mask"].astype(bool) for e in self.envs])

    # ---- packed views used by the parity tests -------------------------
    def packed_state(self):
        """(board u64, hand ids (N,3), used (N,3), score, moves, lines, combo,
        max_combo, blocks, prev_holes, prev_center_filled)."""
        out = {k: [] for k in ("board", "hand", "used", "score", "moves", "lines",
                               "combo", "max_combo", "blocks", "over")}
        for e in self.envs:
            g = e.engine
            out["board"].append(grid_to_u64(g.grid))
            out["hand"].append(list(g.hand))
            out["used"].append([bool(u) for u in g.used])
            out["score"].append(g.score)
            out["moves"].append(g.moves)
            out["lines"].append(g.lines)
            out["combo"].append(g.combo)
            out["max_combo"].append(g.max_combo)
            out["blocks"].append(g.blocks)
            out["over"].append(g.over)
        return {k: np.array(v, dtype=(np.uint64 if k == "board" else None)) for k, v in out.items()}

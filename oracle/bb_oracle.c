/*
 * bb_oracle.c -- C restatement of the Block Blast game, its Gym surface and
 * the vectorised env, for parity runs at BASELINE's full sizes and the timed
 * CPU baseline.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it, as the
 * checker or as the timed CPU baseline; the product library never links it.
 *
 * It restates the reference's ALGORITHMS, not the kernels' bitboard tricks:
 * the board is an 8x8 byte grid, placement tests are per-cell loops, line
 * clears scan rows and columns, holes look at four neighbours, and the hand
 * generator runs the reference's recursive DFS with board copies.  The only
 * 64-bit board words are the packed outputs (bit r*8+c = grid[r][c]), which is
 * the comparison format of the parity tests.
 *
 *   pieces      src/game/pieces.py:78-318 (shapes in dict order = index order),
 *               get_random_pieces pieces.py:350-355 (rng.choice(37, 3))
 *   board       src/game/board.py:71-93 can_place, 95-115 place_piece,
 *               144-193 find_complete_lines + clear_lines, 195-216 count_holes,
 *               236-243 get_center_openness
 *   engine      src/game/engine.py:127-153 reset, 155-172 _generate_new_pieces,
 *               174-238 _can_place_all_pieces / _can_place_remaining /
 *               _simulate_line_clears, 240-312 score, 364-388 mask and
 *               has_valid_moves, 390-454 make_move, 538-576 play_random_game
 *   env         src/environment/block_blast_env.py:104-118 _action_to_move,
 *               148-193 _calculate_reward, 195-222 reset, 224-264 step
 *   vec env     src/environment/wrappers.py:75-116 step (sequential, auto-reset
 *               re-seeds with the env's own seed_value, wrappers.py:97-102)
 *   numpy RNG   numpy SeedSequence (bit_generator.pyx: hashmix / mix /
 *               mix_entropy / generate_state), PCG64 set_seed + XSL-RR output
 *               (pcg64.h), next_uint32 buffering and bounded Lemire draws
 *               (distributions.c buffered_bounded_lemire_uint32) -- numpy is a
 *               dependency of the reference (requirements.txt:2), restated
 *               from its published algorithm and checked against numpy itself
 *   policy      Philox4x32-10 (Random123) synthetic random policy of BASELINE
 *               config 2 (no reference counterpart; matches oracle/philox.py)
 *
 * Build: oracle/build.py (gcc -O2 -fopenmp -ffp-contract=off -shared -fPIC).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BOARD 8
#define HAND 3
#define NPIECES 37
#define MAX_ATTEMPTS 100 /* engine.py:161 */

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------
 * piece table: pieces.py:78-236, index order of PIECES (pieces.py:244-318).
 * '#' = block, '|' = next row.
 * ---------------------------------------------------------------------- */
static const char* const kPictures[NPIECES] = {
    "#",           "##",          "#|#",         "#.|.#",       ".#|#.",       "###",
    "#|#|#",       "#..|.#.|..#", "..#|.#.|#..", "#.|##",       "##|.#",       "##|#.",
    ".#|##",       "####",        "#|#|#|#",     "#####",       "#|#|#|#|#",   "##|##",
    ".#.|###",     "###|.#.",     "#.|##|#.",    ".#|##|.#",    ".##|##.",     "#.|##|.#",
    "##.|.##",     ".#|##|#.",    "#.|#.|##",    "###|#..",     "##|.#|.#",    "..#|###",
    ".#|.#|##",    "#..|###",     "##|#.|#.",    "###|..#",     "###|###",     "##|##|##",
    "###|###|###",
};

typedef struct {
  int n;        /* num_blocks */
  int h, w;     /* height, width (pieces.py:24-37) */
  int dr[9], dc[9];
} Piece;

static Piece g_pieces[NPIECES];
static int g_init = 0;

static void init_pieces(void) {
  if (g_init) return;
  for (int p = 0; p < NPIECES; ++p) {
    Piece* pc = &g_pieces[p];
    int r = 0, c = 0, n = 0, h = 0, w = 0;
    for (const char* s = kPictures[p]; *s; ++s) {
      if (*s == '|') {
        ++r;
        c = 0;
        continue;
      }
      if (*s == '#') {
        pc->dr[n] = r;
        pc->dc[n] = c;
        ++n;
        if (r + 1 > h) h = r + 1;
        if (c + 1 > w) w = c + 1;
      }
      ++c;
    }
    pc->n = n;
    pc->h = h;
    pc->w = w;
  }
  g_init = 1;
}

/* ------------------------------------------------------------------------
 * numpy SeedSequence -> PCG64 (default_rng(seed)), next_uint32, Lemire
 * ---------------------------------------------------------------------- */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u
#define SS_XSHIFT 16
#define SS_POOL 4

static uint32_t ss_hashmix(uint32_t v, uint32_t* hc) {
  v ^= *hc;
  *hc *= SS_MULT_A;
  v *= *hc;
  v ^= v >> SS_XSHIFT;
  return v;
}

static uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
  r ^= r >> SS_XSHIFT;
  return r;
}

typedef struct {
  u128 state, inc;
  uint32_t buf;  /* numpy `uinteger` */
  int has;       /* numpy `has_uint32` */
} Pcg64;

static const u128 kPcgMult = (((u128)0x2360ED051FC65DA4ull) << 64) | 0x4385DF649FCCF645ull;

static void pcg_step(Pcg64* g) { g->state = g->state * kPcgMult + g->inc; }

/* SeedSequence(seed).generate_state(4, uint64) + PCG64 set_seed. */
static void pcg_seed(Pcg64* g, uint64_t seed) {
  uint32_t ent[2];
  int ne = 0;
  if (seed == 0) {
    ent[ne++] = 0;
  } else {
    while (seed) {
      ent[ne++] = (uint32_t)seed;
      seed >>= 32;
    }
  }
  uint32_t pool[SS_POOL];
  uint32_t hc = SS_INIT_A;
  for (int i = 0; i < SS_POOL; ++i) pool[i] = ss_hashmix(i < ne ? ent[i] : 0u, &hc);
  for (int s = 0; s < SS_POOL; ++s)
    for (int d = 0; d < SS_POOL; ++d)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
  /* entropy longer than the pool: never for a uint64 seed (at most 2 words) */
  uint32_t w[8];
  uint32_t hb = SS_INIT_B;
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i % SS_POOL];
    v ^= hb;
    hb *= SS_MULT_B;
    v *= hb;
    v ^= v >> SS_XSHIFT;
    w[i] = v;
  }
  uint64_t v0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  uint64_t v1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  uint64_t v2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32);
  uint64_t v3 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
  u128 initstate = ((u128)v0 << 64) | v1;
  u128 initseq = ((u128)v2 << 64) | v3;
  g->state = 0;
  g->inc = (initseq << 1) | 1u;
  pcg_step(g);
  g->state += initstate;
  pcg_step(g);
  g->has = 0;
  g->buf = 0;
}

static uint64_t pcg_next64(Pcg64* g) {
  pcg_step(g);
  uint64_t hi = (uint64_t)(g->state >> 64), lo = (uint64_t)g->state;
  uint64_t x = hi ^ lo;
  unsigned rot = (unsigned)(hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

static uint32_t pcg_next32(Pcg64* g) {
  if (g->has) {
    g->has = 0;
    return g->buf;
  }
  uint64_t v = pcg_next64(g);
  g->has = 1;
  g->buf = (uint32_t)(v >> 32);
  return (uint32_t)v;
}

/* Generator.integers(0, n) for 1 <= n <= 2^32 (int64 dtype): rng = n - 1;
 * rng == 0 consumes nothing; otherwise the bounded Lemire draw. */
static uint32_t draw_below(Pcg64* g, uint32_t n) {
  if (n <= 1) return 0;
  uint64_t m = (uint64_t)pcg_next32(g) * n;
  uint32_t left = (uint32_t)m;
  if (left < n) {
    uint32_t thr = (uint32_t)(0xFFFFFFFFu - (n - 1)) % n;
    while (left < thr) {
      m = (uint64_t)pcg_next32(g) * n;
      left = (uint32_t)m;
    }
  }
  return (uint32_t)(m >> 32);
}

/* ------------------------------------------------------------------------
 * board.py
 * ---------------------------------------------------------------------- */
typedef struct {
  uint8_t g[BOARD][BOARD];
} Grid;

static int can_place(const Grid* b, int pid, int row, int col) { /* board.py:71-93 */
  const Piece* p = &g_pieces[pid];
  for (int k = 0; k < p->n; ++k) {
    int r = row + p->dr[k], c = col + p->dc[k];
    if (r < 0 || r >= BOARD || c < 0 || c >= BOARD) return 0;
    if (b->g[r][c] != 0) return 0;
  }
  return 1;
}

static void place(Grid* b, int pid, int row, int col) { /* board.py:110-113 */
  const Piece* p = &g_pieces[pid];
  for (int k = 0; k < p->n; ++k) b->g[row + p->dr[k]][col + p->dc[k]] = 1;
}

/* board.py:144-193 (and engine.py:226-238): find on the same grid, then clear. */
static void clear_lines(Grid* b, int* nrows, int* ncols) {
  int rows[BOARD], cols[BOARD], nr = 0, nc = 0;
  for (int r = 0; r < BOARD; ++r) {
    int full = 1;
    for (int c = 0; c < BOARD; ++c) full &= b->g[r][c] == 1;
    if (full) rows[nr++] = r;
  }
  for (int c = 0; c < BOARD; ++c) {
    int full = 1;
    for (int r = 0; r < BOARD; ++r) full &= b->g[r][c] == 1;
    if (full) cols[nc++] = c;
  }
  for (int k = 0; k < nr; ++k)
    for (int c = 0; c < BOARD; ++c) b->g[rows[k]][c] = 0;
  for (int k = 0; k < nc; ++k)
    for (int r = 0; r < BOARD; ++r) b->g[r][cols[k]] = 0;
  if (nrows) *nrows = nr;
  if (ncols) *ncols = nc;
}

static int count_holes(const Grid* b) { /* board.py:195-216 */
  static const int D[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}};
  int holes = 0;
  for (int r = 0; r < BOARD; ++r)
    for (int c = 0; c < BOARD; ++c) {
      if (b->g[r][c] != 0) continue;
      int blocked = 0;
      for (int k = 0; k < 4; ++k) {
        int nr = r + D[k][0], nc = c + D[k][1];
        if (nr < 0 || nr >= BOARD || nc < 0 || nc >= BOARD || b->g[nr][nc] == 1) ++blocked;
      }
      if (blocked == 4) ++holes;
    }
  return holes;
}

static double center_openness(const Grid* b) { /* board.py:236-243 */
  int s = 0;
  for (int r = 2; r < 6; ++r)
    for (int c = 2; c < 6; ++c) s += b->g[r][c];
  return 1.0 - ((double)s / 16.0);
}

static uint64_t grid_bits(const Grid* b) {
  uint64_t v = 0;
  for (int r = 0; r < BOARD; ++r)
    for (int c = 0; c < BOARD; ++c)
      if (b->g[r][c]) v |= 1ull << (r * BOARD + c);
  return v;
}

static void grid_from_bits(Grid* b, uint64_t v) {
  for (int r = 0; r < BOARD; ++r)
    for (int c = 0; c < BOARD; ++c) b->g[r][c] = (uint8_t)((v >> (r * BOARD + c)) & 1u);
}

static int total_blocks(const Grid* b) {
  int s = 0;
  for (int r = 0; r < BOARD; ++r)
    for (int c = 0; c < BOARD; ++c) s += b->g[r][c];
  return s;
}

/* ------------------------------------------------------------------------
 * engine.py
 * ---------------------------------------------------------------------- */
typedef struct {
  Grid board;
  Pcg64 rng;
  int hand[HAND];
  int used[HAND];
  int64_t score;
  int combo, max_combo, moves, lines, blocks;
  int over;
  int last_attempts; /* attempts of the last _generate_new_pieces (diagnostics) */
} Engine;

/* engine.py:181-224 _can_place_remaining (recursive, board copies). */
static int can_place_remaining(const int hand[HAND], const Grid* b, int used_mask) {
  if (used_mask == 7) return 1;
  for (int idx = 0; idx < HAND; ++idx) {
    if (used_mask & (1 << idx)) continue;
    const int pid = hand[idx];
    const Piece* p = &g_pieces[pid];
    for (int row = 0; row < BOARD - p->h + 1; ++row)
      for (int col = 0; col < BOARD - p->w + 1; ++col) {
        if (!can_place(b, pid, row, col)) continue;
        Grid nb = *b;
        place(&nb, pid, row, col);
        clear_lines(&nb, NULL, NULL);
        if (can_place_remaining(hand, &nb, used_mask | (1 << idx))) return 1;
      }
  }
  return 0;
}

/* engine.py:155-172: up to 100 attempts of 3 draws; the last draw is kept. */
static void generate(Engine* e, uint64_t* hist) {
  for (int attempt = 0; attempt < MAX_ATTEMPTS; ++attempt) {
    for (int k = 0; k < HAND; ++k) e->hand[k] = (int)draw_below(&e->rng, NPIECES);
    e->used[0] = e->used[1] = e->used[2] = 0;
    e->last_attempts = attempt + 1;
    const int ok = can_place_remaining(e->hand, &e->board, 0);
#ifdef BBO_GEN_HOOK /* analysis builds only (tools/search_stats.c) */
    BBO_GEN_HOOK(e, attempt, ok);
#endif
    if (ok) {
      if (hist) hist[attempt] += 1;
      return;
    }
  }
  if (hist) hist[MAX_ATTEMPTS] += 1;
}

static void engine_reset(Engine* e, const Pcg64* seeded, uint64_t* hist) { /* engine.py:127-153 */
  if (seeded) e->rng = *seeded;
  memset(&e->board, 0, sizeof(e->board));
  e->used[0] = e->used[1] = e->used[2] = 0;
  e->score = 0;
  e->combo = e->max_combo = e->moves = e->lines = e->blocks = 0;
  e->over = 0;
  generate(e, hist);
}

static int has_valid_moves(const Engine* e) { /* engine.py:382-388, board.py:134-142 */
  for (int p = 0; p < HAND; ++p) {
    if (e->used[p]) continue;
    const int pid = e->hand[p];
    const Piece* pc = &g_pieces[pid];
    for (int r = 0; r < BOARD - pc->h + 1; ++r)
      for (int c = 0; c < BOARD - pc->w + 1; ++c)
        if (can_place(&e->board, pid, r, c)) return 1;
  }
  return 0;
}

static void action_mask(const Engine* e, uint64_t m[HAND]) { /* engine.py:364-380 (status not consulted) */
  for (int p = 0; p < HAND; ++p) {
    m[p] = 0;
    if (e->used[p]) continue;
    for (int r = 0; r < BOARD; ++r)
      for (int c = 0; c < BOARD; ++c)
        if (can_place(&e->board, e->hand[p], r, c)) m[p] |= 1ull << (r * BOARD + c);
  }
}

typedef struct {
  int blocks_placed, lines_cleared, combo_multiplier, game_over;
  int64_t score_gained;
} MoveResult;

/* engine.py:390-454; returns 0 for an illegal move (can_place_piece, 326-346). */
static int make_move(Engine* e, int p, int row, int col, MoveResult* res, uint64_t* hist) {
  if (p < 0 || p >= HAND || e->used[p] || e->over) return 0;
  const int pid = e->hand[p];
  if (!can_place(&e->board, pid, row, col)) return 0;
  const Piece* pc = &g_pieces[pid];
  place(&e->board, pid, row, col);
  e->used[p] = 1;
  e->moves += 1;
  e->blocks += pc->n;
  int rows, cols;
  clear_lines(&e->board, &rows, &cols);
  const int lines = rows + cols;
  if (lines > 0) { /* engine.py:419-424 */
    e->combo += 1;
    if (e->combo > e->max_combo) e->max_combo = e->combo;
    e->lines += lines;
  } else {
    e->combo = 0;
  }
  /* engine.py:240-312 with blocks_in_lines = lines * 8 (engine.py:427); the
   * streak multiplier reads the already incremented combo (engine.py:261) */
  int64_t gained = pc->n;
  if (lines > 0) {
    const int cm = lines < 4 ? lines : 4;
    const int streak = e->combo + 1 < 8 ? e->combo + 1 : 8;
    gained += (int64_t)(lines * BOARD * 10) * cm * streak;
  }
  e->score += gained;
  if (e->used[0] && e->used[1] && e->used[2]) generate(e, hist); /* engine.py:432-437 */
  if (!has_valid_moves(e)) e->over = 1;                           /* engine.py:440-441 */
  res->blocks_placed = pc->n;
  res->lines_cleared = lines;
  res->combo_multiplier = lines > 0 ? (lines < 4 ? lines : 4) : 1;
  res->score_gained = gained;
  res->game_over = e->over;
  return 1;
}

/* ------------------------------------------------------------------------
 * block_blast_env.py BlockBlastEnv + wrappers.py VectorizedBlockBlastEnv
 * ---------------------------------------------------------------------- */
typedef struct {
  double line_clear_base, block_placed, game_over_penalty, hole_penalty, center_bonus,
      combo_multiplier_bonus, survival_bonus;
} Rewards; /* block_blast_env.py:63-73 */

typedef struct {
  Engine eng;
  Pcg64 seeded; /* default_rng(seed_value) right after seeding */
  int has_seed;
  int prev_holes;
  double prev_center;
} Env;

typedef struct bbo_vec {
  int n;
  int autoreset;
  Rewards rw;
  Env* envs;
  uint64_t* hist_t;  /* per-thread histograms of generations by attempts used */
  int nthreads_hist;
} bbo_vec;

static double env_reward(const bbo_vec* v, Env* e, const MoveResult* r) { /* block_blast_env.py:148-193 */
  const Rewards* rw = &v->rw;
  double reward = 0.0;
  reward += r->blocks_placed * rw->block_placed;
  reward += rw->survival_bonus;
  if (r->lines_cleared > 0) {
    double line_reward = r->lines_cleared * rw->line_clear_base;
    line_reward *= r->combo_multiplier;
    reward += line_reward;
    if (r->combo_multiplier > 1) reward += (r->combo_multiplier - 1) * rw->combo_multiplier_bonus;
  }
  if (r->game_over) reward += rw->game_over_penalty;
  const int holes = count_holes(&e->eng.board);
  const int delta = holes - e->prev_holes;
  if (delta > 0) reward += delta * rw->hole_penalty;
  e->prev_holes = holes;
  const double center = center_openness(&e->eng.board);
  if (center >= e->prev_center) reward += rw->center_bonus * 0.1;
  e->prev_center = center;
  return reward;
}

static void env_reset(Env* e, uint64_t* hist) { /* block_blast_env.py:195-222 */
  engine_reset(&e->eng, e->has_seed ? &e->seeded : NULL, hist);
  e->prev_holes = 0;
  e->prev_center = 1.0;
}

typedef struct {
  double reward;
  int terminated, lines, invalid;
  int64_t score; /* info['score'] / info['moves'] after the move, before any auto-reset */
  int moves;
} StepOut;

/* block_blast_env.py:224-264 + the vec-env auto-reset of wrappers.py:97-102. */
static void env_step(const bbo_vec* v, Env* e, int action, StepOut* o, uint64_t* hist) {
  const int p = action / 64, r = (action % 64) / 8, c = action % 8; /* block_blast_env.py:104-118 */
  MoveResult res;
  o->lines = 0;
  o->invalid = 0;
  o->score = e->eng.score;
  o->moves = e->eng.moves;
  if (action < 0 || !make_move(&e->eng, p, r, c, &res, hist)) { /* block_blast_env.py:240-245 */
    o->reward = -10.0;
    o->terminated = 0;
    o->invalid = 1;
    return;
  }
  o->reward = env_reward(v, e, &res);
  o->terminated = res.game_over;
  o->lines = res.lines_cleared;
  o->score = e->eng.score; /* wrappers.py:97-101: final_score = info['score'], read before env.reset() */
  o->moves = e->eng.moves;
  if (o->terminated && v->autoreset) env_reset(e, hist);
}

/* ---------------- Philox4x32-10 synthetic policy (oracle/philox.py) ------ */
static uint32_t philox_w0(uint64_t seed, uint64_t idx, uint64_t step) {
  uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32), c2 = (uint32_t)step, c3 = (uint32_t)(step >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  return c0;
}

static int32_t policy_action(const uint64_t m[HAND], uint32_t u) {
  int cnt = 0;
  for (int p = 0; p < HAND; ++p) cnt += __builtin_popcountll(m[p]);
  if (cnt == 0) return 0;
  uint32_t k = (uint32_t)(((uint64_t)u * (uint32_t)cnt) >> 32);
  for (int a = 0; a < HAND * 64; ++a)
    if ((m[a >> 6] >> (a & 63)) & 1u) {
      if (k == 0) return a;
      --k;
    }
  return 0;
}

/* ------------------------------------------------------------------------
 * C-ABI (ctypes, tests only)
 * ---------------------------------------------------------------------- */
int bbo_abi_version(void) { return 1; }

void bbo_pcg64_seed(uint64_t seed, uint64_t out[4]) {
  Pcg64 g;
  pcg_seed(&g, seed);
  out[0] = (uint64_t)(g.state >> 64);
  out[1] = (uint64_t)g.state;
  out[2] = (uint64_t)(g.inc >> 64);
  out[3] = (uint64_t)g.inc;
}

/* n draws of integers(0, bound) after default_rng(seed) (bound 0: raw next_uint32). */
void bbo_rng_draws(uint64_t seed, uint32_t bound, int n, uint32_t* out) {
  Pcg64 g;
  pcg_seed(&g, seed);
  for (int i = 0; i < n; ++i) out[i] = bound ? draw_below(&g, bound) : pcg_next32(&g);
}

/* rewards: 7 doubles in bb_reward_cfg order, or NULL for the defaults.
 * has_seed NULL: every env seeded; has_seed[i] == 0: seed_value None, the
 * stream (default_rng(seeds[i]) here) continues across resets. */
bbo_vec* bbo_create(int n, const uint64_t* seeds, const uint8_t* has_seed, const double* rewards, int autoreset) {
  init_pieces();
  bbo_vec* v = (bbo_vec*)calloc(1, sizeof(bbo_vec));
  v->n = n;
  v->autoreset = autoreset;
  static const double kDefaults[7] = {1.0, 0.01, -1.0, -0.05, 0.02, 0.5, 0.001};
  const double* r = rewards ? rewards : kDefaults;
  v->rw.line_clear_base = r[0];
  v->rw.block_placed = r[1];
  v->rw.game_over_penalty = r[2];
  v->rw.hole_penalty = r[3];
  v->rw.center_bonus = r[4];
  v->rw.combo_multiplier_bonus = r[5];
  v->rw.survival_bonus = r[6];
  v->envs = (Env*)calloc((size_t)n, sizeof(Env));
  for (int i = 0; i < n; ++i) {
    Env* e = &v->envs[i];
    e->has_seed = has_seed ? has_seed[i] != 0 : 1;
    pcg_seed(&e->seeded, seeds[i]);
    e->eng.rng = e->seeded;
  }
  return v;
}

void bbo_destroy(bbo_vec* v) {
  if (!v) return;
  free(v->envs);
  free(v->hist_t);
  free(v);
}

static int set_threads(int threads) {
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
  return threads;
#else
  (void)threads;
  return 1;
#endif
}

static uint64_t* thread_hist(bbo_vec* v, int nt) {
  if (v->nthreads_hist < nt) {
    uint64_t* h = (uint64_t*)calloc((size_t)nt * (MAX_ATTEMPTS + 1), sizeof(uint64_t));
    if (v->hist_t) memcpy(h, v->hist_t, (size_t)v->nthreads_hist * (MAX_ATTEMPTS + 1) * sizeof(uint64_t));
    free(v->hist_t);
    v->hist_t = h;
    v->nthreads_hist = nt;
  }
  return v->hist_t;
}

static int my_thread(void) {
#ifdef _OPENMP
  return omp_get_thread_num();
#else
  return 0;
#endif
}

/* env.reset() of every env (wrappers.py:53-73). */
void bbo_reset(bbo_vec* v, int threads) {
  const int nt = set_threads(threads);
  uint64_t* H = thread_hist(v, nt);
#pragma omp parallel for num_threads(nt) schedule(dynamic, 64)
  for (int i = 0; i < v->n; ++i) env_reset(&v->envs[i], H + (size_t)my_thread() * (MAX_ATTEMPTS + 1));
}

/* One vec step (wrappers.py:75-116).  Any output may be NULL.
 * mask: post-step (post-reset) [n][3] bits. */
void bbo_step(bbo_vec* v, const int32_t* actions, float* reward, double* reward64, uint8_t* term, uint8_t* lines,
              uint8_t* invalid, uint64_t* mask, int threads) {
  const int nt = set_threads(threads);
  uint64_t* H = thread_hist(v, nt);
#pragma omp parallel for num_threads(nt) schedule(dynamic, 64)
  for (int i = 0; i < v->n; ++i) {
    StepOut o;
    env_step(v, &v->envs[i], actions[i], &o, H + (size_t)my_thread() * (MAX_ATTEMPTS + 1));
    if (reward) reward[i] = (float)o.reward;
    if (reward64) reward64[i] = o.reward;
    if (term) term[i] = (uint8_t)o.terminated;
    if (lines) lines[i] = (uint8_t)o.lines;
    if (invalid) invalid[i] = (uint8_t)o.invalid;
    if (mask) action_mask(&v->envs[i].eng, &mask[3 * (size_t)i]);
  }
}

/* T steps under the synthetic random policy, equal to bb_rollout: act_io[n]
 * holds the first step's actions and receives the action after the last
 * step; step t draws the NEXT action with policy step policy_step0 + t + 1.
 * Outputs are [T][n] (mask [T][n][3]); any may be NULL. */
void bbo_rollout(bbo_vec* v, int T, int32_t* act_io, uint64_t policy_seed, uint64_t policy_step0,
                 uint64_t env_offset, float* reward, uint8_t* term, uint8_t* lines, int32_t* actions,
                 uint64_t* mask, int threads) {
  const int nt = set_threads(threads);
  uint64_t* H = thread_hist(v, nt);
  const size_t n = (size_t)v->n;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 16)
  for (int i = 0; i < v->n; ++i) {
    uint64_t* hist = H + (size_t)my_thread() * (MAX_ATTEMPTS + 1);
    Env* e = &v->envs[i];
    int32_t a = act_io[i];
    for (int t = 0; t < T; ++t) {
      StepOut o;
      env_step(v, e, a, &o, hist);
      const size_t k = (size_t)t * n + (size_t)i;
      if (reward) reward[k] = (float)o.reward;
      if (term) term[k] = (uint8_t)o.terminated;
      if (lines) lines[k] = (uint8_t)o.lines;
      if (actions) actions[k] = a;
      uint64_t m[HAND];
      action_mask(&e->eng, m);
      if (mask) memcpy(&mask[3 * k], m, sizeof(m));
      a = policy_action(m, philox_w0(policy_seed, env_offset + (uint64_t)i, policy_step0 + (uint64_t)t + 1));
    }
    act_io[i] = a;
  }
}

static uint32_t hand_word(const Engine* g) {
  return (uint32_t)g->hand[0] | ((uint32_t)g->hand[1] << 6) | ((uint32_t)g->hand[2] << 12) |
         ((uint32_t)g->used[0] << 18) | ((uint32_t)g->used[1] << 19) | ((uint32_t)g->used[2] << 20) |
         ((uint32_t)g->over << 21) | ((uint32_t)g->rng.has << 22);
}

/* Replay of a training rollout (scripts/train.py:173-203): T vec steps with
 * recorded actions [T][n].  Per (t, i): the pre-step state snapshot (board
 * bits, packed hand word, mask bits -- what the rollout buffer stores before
 * the step), the step's f32 reward and terminated flag, and on termination the
 * episode's final score and moves (info['final_score'] / info['moves'],
 * wrappers.py:97-101; 0 elsewhere).  Any output may be NULL. */
void bbo_replay(bbo_vec* v, int T, const int32_t* actions, uint64_t* board, uint32_t* hand, uint64_t* mask,
                float* reward, uint8_t* term, int64_t* ep_score, int32_t* ep_moves, int threads) {
  const int nt = set_threads(threads);
  uint64_t* H = thread_hist(v, nt);
  const size_t n = (size_t)v->n;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 16)
  for (int i = 0; i < v->n; ++i) {
    uint64_t* hist = H + (size_t)my_thread() * (MAX_ATTEMPTS + 1);
    Env* e = &v->envs[i];
    for (int t = 0; t < T; ++t) {
      const size_t k = (size_t)t * n + (size_t)i;
      if (board) board[k] = grid_bits(&e->eng.board);
      if (hand) hand[k] = hand_word(&e->eng);
      if (mask) action_mask(&e->eng, &mask[3 * k]);
      StepOut o;
      env_step(v, e, actions[k], &o, hist);
      if (reward) reward[k] = (float)o.reward;
      if (term) term[k] = (uint8_t)o.terminated;
      if (ep_score) ep_score[k] = o.terminated ? o.score : 0;
      if (ep_moves) ep_moves[k] = o.terminated ? o.moves : 0;
    }
  }
}

/* The synthetic policy on given masks (bb_random_actions). */
void bbo_random_actions(const uint64_t* mask, int n, uint64_t seed, uint64_t step, uint64_t env_offset,
                        int32_t* out) {
  for (int i = 0; i < n; ++i)
    out[i] = policy_action(&mask[3 * (size_t)i], philox_w0(seed, env_offset + (uint64_t)i, step));
}

/* Packed state (bbvec.h bb_state_view layout).  hand word: 3 x 6-bit ids,
 * used bits 18-20, game over 21, has_uint32 22.  Any pointer may be NULL. */
void bbo_state(const bbo_vec* v, uint64_t* board, uint32_t* hand, int64_t* score, int32_t* combo, int32_t* max_combo,
               int32_t* moves, int32_t* lines, int32_t* blocks, uint8_t* prev_holes, uint8_t* prev_center,
               uint64_t* rng, uint64_t* mask) {
  for (int i = 0; i < v->n; ++i) {
    const Env* e = &v->envs[i];
    const Engine* g = &e->eng;
    if (board) board[i] = grid_bits(&g->board);
    if (hand)
      hand[i] = (uint32_t)g->hand[0] | ((uint32_t)g->hand[1] << 6) | ((uint32_t)g->hand[2] << 12) |
                ((uint32_t)g->used[0] << 18) | ((uint32_t)g->used[1] << 19) | ((uint32_t)g->used[2] << 20) |
                ((uint32_t)g->over << 21) | ((uint32_t)g->rng.has << 22);
    if (score) score[i] = g->score;
    if (combo) combo[i] = g->combo;
    if (max_combo) max_combo[i] = g->max_combo;
    if (moves) moves[i] = g->moves;
    if (lines) lines[i] = g->lines;
    if (blocks) blocks[i] = g->blocks;
    if (prev_holes) prev_holes[i] = (uint8_t)e->prev_holes;
    if (prev_center) prev_center[i] = (uint8_t)(int)((1.0 - e->prev_center) * 16.0 + 0.5);
    if (rng) {
      rng[3 * (size_t)i + 0] = (uint64_t)(g->rng.state >> 64);
      rng[3 * (size_t)i + 1] = (uint64_t)g->rng.state;
      rng[3 * (size_t)i + 2] = g->rng.buf;
    }
    if (mask) action_mask(g, &mask[3 * (size_t)i]);
  }
}

/* Overwrite board / hand of every env (the pcg stream is kept); crowded-board
 * tests.  hand uses the packed word above (has_uint32 ignored). */
void bbo_set_board_hand(bbo_vec* v, const uint64_t* board, const uint32_t* hand) {
  for (int i = 0; i < v->n; ++i) {
    Engine* g = &v->envs[i].eng;
    if (board) grid_from_bits(&g->board, board[i]);
    if (hand) {
      for (int k = 0; k < HAND; ++k) {
        g->hand[k] = (int)((hand[i] >> (6 * k)) & 63u);
        g->used[k] = (int)((hand[i] >> (18 + k)) & 1u);
      }
      g->over = (int)((hand[i] >> 21) & 1u);
    }
  }
}

/* Generations by number of attempts used: out[k] = generations settled by
 * attempt k+1 (k < 100), out[100] = all 100 attempts failed (last draw kept). */
void bbo_gen_hist(const bbo_vec* v, uint64_t* out) {
  memset(out, 0, (MAX_ATTEMPTS + 1) * sizeof(uint64_t));
  for (int t = 0; t < v->nthreads_hist; ++t)
    for (int k = 0; k <= MAX_ATTEMPTS; ++k) out[k] += v->hist_t[(size_t)t * (MAX_ATTEMPTS + 1) + k];
}

/* The reference DFS verdict (engine.py:174-224) for many (board, hand) pairs. */
void bbo_solvable_many(const uint64_t* boards, const uint32_t* hands, int n, uint8_t* out, int threads) {
  init_pieces();
  const int nt = set_threads(threads);
#pragma omp parallel for num_threads(nt) schedule(dynamic, 64)
  for (int i = 0; i < n; ++i) {
    Grid g;
    grid_from_bits(&g, boards[i]);
    const int hand[HAND] = {(int)(hands[i] & 63u), (int)((hands[i] >> 6) & 63u), (int)((hands[i] >> 12) & 63u)};
    out[i] = (uint8_t)can_place_remaining(hand, &g, 0);
  }
}

/* engine.py:538-576 play_random_game(seed): out = {score, moves, lines,
 * max_combo, blocks, filled cells, holes, centre cells filled}; first_hand[3]. */
void bbo_play_random_game(uint64_t seed, int64_t out[8], int32_t first_hand[3]) {
  init_pieces();
  Engine e;
  memset(&e, 0, sizeof(e));
  pcg_seed(&e.rng, seed);
  generate(&e, NULL);
  if (first_hand)
    for (int k = 0; k < HAND; ++k) first_hand[k] = e.hand[k];
  int mv[HAND * 64][3];
  while (!e.over) {
    int nm = 0; /* engine.py:348-362 get_valid_moves order */
    for (int p = 0; p < HAND; ++p) {
      if (e.used[p]) continue;
      for (int r = 0; r < BOARD; ++r)
        for (int c = 0; c < BOARD; ++c)
          if (can_place(&e.board, e.hand[p], r, c)) {
            mv[nm][0] = p;
            mv[nm][1] = r;
            mv[nm][2] = c;
            ++nm;
          }
    }
    if (!nm) break;
    const int k = (int)draw_below(&e.rng, (uint32_t)nm); /* engine.rng.choice(len(valid_moves)) */
    MoveResult res;
    make_move(&e, mv[k][0], mv[k][1], mv[k][2], &res, NULL);
  }
  out[0] = e.score;
  out[1] = e.moves;
  out[2] = e.lines;
  out[3] = e.max_combo;
  out[4] = e.blocks;
  out[5] = total_blocks(&e.board);
  out[6] = count_holes(&e.board);
  int s = 0;
  for (int r = 2; r < 6; ++r)
    for (int c = 2; c < 6; ++c) s += e.board.g[r][c];
  out[7] = s;
}

/*
 * dead_piece.c -- diagnostics (not product, not test): how many of the hands that
 * _generate_new_pieces (engine.py:155-172) rejects are rejected for a cheap reason:
 * a piece with no legal anchor on the board can only be placed after a line clear,
 * and the first clear must come from the pieces that do have anchors; if no row or
 * column has at most (their cells) empty cells, no clear can ever happen first, so
 * the hand is unsolvable.  Counts every attempt of the bench workload's random play.
 *   gcc -O2 -o /tmp/dead_piece tools/dead_piece.c && /tmp/dead_piece [N] [T]
 */
#include <stdio.h>

struct Engine;
static void gen_hook(const struct Engine* e, int attempt, int ok);
#define BBO_GEN_HOOK(e, attempt, ok) gen_hook((const struct Engine*)(e), attempt, ok)
#include "../oracle/bb_oracle.c"

static uint64_t g_anch[NPIECES];
static int g_offs[NPIECES][9];

static void init_bits(void) {
  init_pieces();
  for (int p = 0; p < NPIECES; ++p) {
    const Piece* pc = &g_pieces[p];
    for (int k = 0; k < pc->n; ++k) g_offs[p][k] = pc->dr[k] * 8 + pc->dc[k];
    uint64_t a = 0;
    for (int r = 0; r <= 8 - pc->h; ++r)
      for (int c = 0; c <= 8 - pc->w; ++c) a |= 1ull << (r * 8 + c);
    g_anch[p] = a;
  }
}

static uint64_t anchors_of(int p, uint64_t B) {
  uint64_t acc = 0;
  for (int k = 0; k < g_pieces[p].n; ++k) acc |= B >> g_offs[p][k];
  return g_anch[p] & ~acc;
}

static int min_line_empty(uint64_t B) {
  int m = 8;
  for (int r = 0; r < 8; ++r) {
    int e = 8 - __builtin_popcountll((B >> (8 * r)) & 0xFFull);
    if (e < m) m = e;
  }
  for (int c = 0; c < 8; ++c) {
    int e = 0;
    for (int r = 0; r < 8; ++r) e += !((B >> (8 * r + c)) & 1ull);
    if (e < m) m = e;
  }
  return m;
}

static uint64_t slots_all, slots_unsolv, slots_dead1, slots_dead2;
static uint64_t n_att, n_unsolv, n_caught, n_unsound, n_first_unsolv, n_first_caught, n_caught2, n_unsound2;

static int full_line(uint64_t B) {
  for (int r = 0; r < 8; ++r) if (((B >> (8 * r)) & 0xFFull) == 0xFFull) return 1;
  for (int c = 0; c < 8; ++c) {
    int f = 1;
    for (int r = 0; r < 8; ++r) f &= (int)((B >> (8 * r + c)) & 1ull);
    if (f) return 1;
  }
  return 0;
}

static uint64_t shape_of(int p) {
  uint64_t s = 0;
  for (int k = 0; k < g_pieces[p].n; ++k) s |= 1ull << g_offs[p][k];
  return s;
}

/* stronger: with one placeable piece, does any of its anchors complete a line? */
static int dead2(const int h[3], uint64_t B) {
  int nz[3], k = 0, zero = 0, cells = 0;
  for (int i = 0; i < 3; ++i) {
    if (anchors_of(h[i], B)) { nz[k++] = h[i]; cells += g_pieces[h[i]].n; }
    else zero++;
  }
  if (!zero) return 0;
  if (zero == 3) return 1;
  if (min_line_empty(B) > cells) return 1;
  if (k == 1) {
    for (uint64_t A = anchors_of(nz[0], B); A; A &= A - 1)
      if (full_line(B | (shape_of(nz[0]) << __builtin_ctzll(A)))) return 0;
    return 1;
  }
  return 0;
}

static void gen_hook(const struct Engine* ee, int attempt, int ok) {
  const Engine* e = (const Engine*)ee;
  uint64_t B = grid_bits(&e->board);
  if (B == 0) return;
  const int* h = e->hand;
  n_att++;
  int zero = 0, cells = 0;
  for (int i = 0; i < 3; ++i) {
    if (anchors_of(h[i], B)) cells += g_pieces[h[i]].n;
    else zero++;
  }
  const int dead = zero > 0 && (zero == 3 || min_line_empty(B) > cells);
  const int d2 = dead2(h, B);
  uint64_t S = 0;
  for (int i = 0; i < 3; ++i) S += __builtin_popcountll(anchors_of(h[i], B));
  slots_all += S;
  if (!ok) { slots_unsolv += S; slots_dead1 += dead ? S : 0; slots_dead2 += d2 ? S : 0; }
  if (!ok) n_caught2 += d2;
  else if (d2) n_unsound2++;
  if (!ok) {
    n_unsolv++;
    n_caught += dead;
    if (attempt == 0) { n_first_unsolv++; n_first_caught += dead; }
  } else if (dead) {
    n_unsound++;
  }
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 8192;
  int T = argc > 2 ? atoi(argv[2]) : 128;
  init_bits();
  uint64_t* seeds = malloc(sizeof(uint64_t) * n);
  for (int i = 0; i < n; ++i) seeds[i] = 42 + (uint64_t)i;
  bbo_vec* v = bbo_create(n, seeds, NULL, NULL, 1);
  bbo_reset(v, 1);
  uint64_t* m = malloc(sizeof(uint64_t) * 3 * n);
  int32_t* a = malloc(sizeof(int32_t) * n);
  bbo_state(v, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, m);
  bbo_random_actions(m, n, 0xB10C, 0, 0, a);
  bbo_rollout(v, T, a, 0xB10C, 0, 0, NULL, NULL, NULL, NULL, NULL, 1);
  printf("attempts %llu, unsolvable %llu (%.4f); caught by the dead-piece rule %llu (%.4f of unsolvable); "
         "first attempts unsolvable %llu, caught %.4f; UNSOUND %llu\n",
         (unsigned long long)n_att, (unsigned long long)n_unsolv, (double)n_unsolv / n_att,
         (unsigned long long)n_caught, (double)n_caught / n_unsolv, (unsigned long long)n_first_unsolv,
         (double)n_first_caught / n_first_unsolv, (unsigned long long)n_unsound);
  printf("level-1 slots: all attempts %llu, unsolvable %llu, dead rule %llu, + exact one-piece %llu\n",
         (unsigned long long)slots_all, (unsigned long long)slots_unsolv, (unsigned long long)slots_dead1,
         (unsigned long long)slots_dead2);
  printf("with the exact one-placeable-piece test: caught %.4f of unsolvable; UNSOUND %llu\n",
         (double)n_caught2 / n_unsolv, (unsigned long long)n_unsound2);
  return n_unsound != 0;
}

/*
 * search_stats.c -- diagnostics (not product, not test): statistics of the
 * hand generator (engine.py:155-238) on the bench workload, to size the GPU
 * hand search.  Compiles the C oracle with a hook on every attempt of
 * _generate_new_pieces and classifies it with the bitboard tests the kernels
 * use (csrc/bb_solver.h quick_slots / pair_quick).
 *
 *   gcc -O2 -fopenmp -o /tmp/search_stats tools/search_stats.c && /tmp/search_stats [N] [T]
 */
#include <stdio.h>

struct Engine;
static void gen_hook(const struct Engine* e, int attempt, int ok);
#define BBO_GEN_HOOK(e, attempt, ok) gen_hook((const struct Engine*)(e), attempt, ok)
#include "../oracle/bb_oracle.c"

static uint64_t g_shape[NPIECES], g_anch[NPIECES];
static int g_offs[NPIECES][9];
static int g_dtab[NPIECES][NPIECES];

static void init_bits(void) {
  init_pieces();
  for (int p = 0; p < NPIECES; ++p) {
    const Piece* pc = &g_pieces[p];
    uint64_t s = 0;
    for (int k = 0; k < pc->n; ++k) {
      s |= 1ull << (pc->dr[k] * 8 + pc->dc[k]);
      g_offs[p][k] = pc->dr[k] * 8 + pc->dc[k];
    }
    g_shape[p] = s;
    uint64_t a = 0;
    for (int r = 0; r <= 8 - pc->h; ++r)
      for (int c = 0; c <= 8 - pc->w; ++c) a |= 1ull << (r * 8 + c);
    g_anch[p] = a;
  }
  for (int b = 0; b < NPIECES; ++b)
    for (int c = 0; c < NPIECES; ++c) {
      int seen[128] = {0}, cnt = 0;
      for (int i = 0; i < g_pieces[b].n; ++i)
        for (int j = 0; j < g_pieces[c].n; ++j) {
          int d = g_offs[b][i] - g_offs[c][j] + 64;
          if (!seen[d]) seen[d] = 1, ++cnt;
        }
      g_dtab[b][c] = cnt;
    }
}

static uint64_t anchors_of(int p, uint64_t B) {
  uint64_t acc = 0;
  for (int k = 0; k < g_pieces[p].n; ++k) acc |= B >> g_offs[p][k];
  return g_anch[p] & ~acc;
}

static uint64_t clear_full(uint64_t B) {
  uint64_t r = B & (B >> 1);
  r &= r >> 2;
  r &= r >> 4;
  r &= 0x0101010101010101ull;
  uint64_t c = B & (B >> 8);
  c &= c >> 16;
  c &= c >> 32;
  c &= 0xFFull;
  uint64_t rm = (r << 8) - r, cm = c | (c << 8);
  cm |= cm << 16;
  cm |= cm << 32;
  return B & ~(rm | cm);
}

static int pair_quick(uint64_t B1, int b, int c) {
  uint64_t A2 = anchors_of(b, B1), A3 = anchors_of(c, B1);
  if (!(A2 | A3)) return 0;
  if (A2 && __builtin_popcountll(A3) > g_dtab[b][c]) return 1;
  if (A3 && __builtin_popcountll(A2) > g_dtab[b][c]) return 1;
  if (A2 && anchors_of(c, clear_full(B1 | (g_shape[b] << __builtin_ctzll(A2))))) return 1;
  if (A3 && anchors_of(b, clear_full(B1 | (g_shape[c] << __builtin_ctzll(A3))))) return 1;
  return 2;
}

/* exact pair test (both orders, every anchor) */
static int pair_exact(uint64_t B1, int b, int c) {
  uint64_t A2 = anchors_of(b, B1), A3 = anchors_of(c, B1);
  for (uint64_t it = A2; it; it &= it - 1)
    if (anchors_of(c, clear_full(B1 | (g_shape[b] << __builtin_ctzll(it))))) return 1;
  for (uint64_t it = A3; it; it &= it - 1)
    if (anchors_of(b, clear_full(B1 | (g_shape[c] << __builtin_ctzll(it))))) return 1;
  return 0;
}

/* quick slot k: first piece f = k % 3 at its lowest (k < 3) / highest anchor */
static int quick_slot(uint64_t B, const int h[3], int k) {
  int f = k % 3, b = f == 0 ? 1 : 0, c = f == 2 ? 1 : 2;
  uint64_t A = anchors_of(h[f], B);
  if (!A) return 0;
  int p = k < 3 ? __builtin_ctzll(A) : 63 - __builtin_clzll(A);
  return pair_quick(clear_full(B | (g_shape[h[f]] << p)), h[b], h[c]) == 1;
}

enum {
  S_ATT,            /* attempts */
  S_ATT1,           /* first attempts */
  S_ATT1_OK,        /* first attempts solvable */
  S_Q0,             /* first attempt accepted by quick slot 0 */
  S_Q01,            /* ... by slot 0 or 1 (the rollout kernel's two copies) */
  S_Q012,           /* ... by slots 0..2 */
  S_Q0_5,           /* ... by slots 0..5 */
  S_ANYQ,           /* ... by pair_quick on some level-1 slot */
  S_OK_NOQUICK,     /* solvable, no level-1 slot quick-accepts */
  S_FAIL,           /* attempts not solvable */
  S_FAIL_NOANCH3,   /* ... no piece fits at all */
  S_FAIL_SOME0,     /* ... some piece has no anchor on B */
  S_FAIL_PAIRS,     /* ... level-1 slots (total) */
  S_FAIL_PQREJ,     /* ... level-1 slots pair_quick rejects outright (A2|A3 == 0) */
  S_OK_SLOTS,       /* solvable: level-1 slots before the first exact success (f-major) */
  S_LATER,          /* attempts after the first */
  S_LATER_OK,
  S_LATER_Q01,
  S_GEN_MULTI,      /* generations needing more than one attempt */
  S_N
};
static uint64_t S[S_N];

/* rows / columns a pair of pieces (y, z) could complete together: a line
 * with more empty cells than the two pieces' extents along it cannot fill */
static int line_reachable2(uint64_t B, int y, int z) {
  int wmax = g_pieces[y].w + g_pieces[z].w, hmax = g_pieces[y].h + g_pieces[z].h;
  for (int r = 0; r < 8; ++r)
    if (8 - __builtin_popcountll((B >> (8 * r)) & 0xFF) <= wmax) return 1;
  for (int c = 0; c < 8; ++c)
    if (8 - __builtin_popcountll(B & (0x0101010101010101ull << c)) <= hmax) return 1;
  return 0;
}

/* 1 = provably unsolvable (sound), 0 = unknown */
static int quick_reject(uint64_t B, const int h[3], const uint64_t A[3]) {
  if (!(A[0] | A[1] | A[2])) return 1;
  for (int x = 0; x < 3; ++x) {
    if (A[x]) continue;
    int y = x == 0 ? 1 : 0, z = x == 2 ? 1 : 2;
    if (!line_reachable2(B, h[y], h[z])) return 1;
  }
  return 0;
}

/* in-lane policy over one generation: per attempt, accept on quick slots
 * 0|1, reject on quick_reject, else park.  Counted per generation. */
enum { P_GEN, P_PARK1, P_PARK2, P_PARK3, P_PARK4, P_REJ_FIRE, P_UNSOLV, P_N };
static uint64_t P[P_N];
static int g_state = 0; /* 0 = deciding in-lane, >0 parked at attempt g_state */
static uint64_t fill_hist[65];

static void gen_hook(const struct Engine* ee, int attempt, int ok) {
  const Engine* e = (const Engine*)ee;
  uint64_t B = grid_bits(&e->board);
  if (B == 0) return; /* resets: every hand fits an empty board */
  const int* h = e->hand;
  S[S_ATT]++;
  {
    uint64_t A_[3] = {anchors_of(h[0], B), anchors_of(h[1], B), anchors_of(h[2], B)};
    int acc = quick_slot(B, h, 0) | quick_slot(B, h, 1);
    int rej = quick_reject(B, h, A_);
    if (!ok) P[P_UNSOLV]++;
    if (rej) {
      P[P_REJ_FIRE]++;
      if (ok) { fprintf(stderr, "UNSOUND reject\n"); exit(1); }
    }
    if (attempt == 0) { P[P_GEN]++; g_state = 0; }
    if (g_state == 0 && !acc && !rej) {
      g_state = attempt + 1;
      if (attempt < 4) P[P_PARK1 + attempt]++;
    }
  }
  int q0 = quick_slot(B, h, 0), q1 = quick_slot(B, h, 1);
  if (attempt == 0) {
    S[S_ATT1]++;
    fill_hist[__builtin_popcountll(B)]++;
    if (ok) S[S_ATT1_OK]++;
    S[S_Q0] += q0;
    S[S_Q01] += q0 | q1;
    int q2 = quick_slot(B, h, 2), q35 = quick_slot(B, h, 3) | quick_slot(B, h, 4) | quick_slot(B, h, 5);
    S[S_Q012] += q0 | q1 | q2;
    S[S_Q0_5] += q0 | q1 | q2 | q35;
  } else {
    S[S_LATER]++;
    S[S_LATER_OK] += ok;
    S[S_LATER_Q01] += q0 | q1;
    if (attempt == 1) S[S_GEN_MULTI]++;
  }
  uint64_t A[3] = {anchors_of(h[0], B), anchors_of(h[1], B), anchors_of(h[2], B)};
  int anyq = 0, slots = 0, found = 0;
  for (int f = 0; f < 3; ++f) {
    int b = f == 0 ? 1 : 0, c = f == 2 ? 1 : 2;
    for (uint64_t it = A[f]; it; it &= it - 1) {
      uint64_t B1 = clear_full(B | (g_shape[h[f]] << __builtin_ctzll(it)));
      int q = pair_quick(B1, h[b], h[c]);
      if (q == 1) anyq = 1;
      if (!ok) {
        S[S_FAIL_PAIRS]++;
        if (q == 0) S[S_FAIL_PQREJ]++;
      } else if (!found) {
        ++slots;
        if (q == 1 || pair_exact(B1, h[b], h[c])) found = 1;
      }
    }
  }
  if (ok) {
    S[S_OK_SLOTS] += slots;
    if (!anyq) S[S_OK_NOQUICK]++;
    if (attempt == 0) S[S_ANYQ] += anyq;
  } else {
    S[S_FAIL]++;
    if (!(A[0] | A[1] | A[2])) S[S_FAIL_NOANCH3]++;
    if (!A[0] || !A[1] || !A[2]) S[S_FAIL_SOME0]++;
  }
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 8192;
  int T = argc > 2 ? atoi(argv[2]) : 256;
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
  const double env_steps = (double)n * T;
  printf("envs %d x steps %d = %.0f env-steps\n", n, T, env_steps);
  printf("non-empty generations (first attempts): %llu  = %.4f per env-step\n", (unsigned long long)S[S_ATT1],
         S[S_ATT1] / env_steps);
  printf("attempts total %llu (%.3f per generation)\n", (unsigned long long)S[S_ATT], (double)S[S_ATT] / S[S_ATT1]);
  printf("first attempt solvable      %.4f\n", (double)S[S_ATT1_OK] / S[S_ATT1]);
  printf("quick slot 0 accepts        %.4f\n", (double)S[S_Q0] / S[S_ATT1]);
  printf("quick slots 0|1 accept      %.4f   (rollout kernel in-lane test)\n", (double)S[S_Q01] / S[S_ATT1]);
  printf("quick slots 0..2 accept     %.4f\n", (double)S[S_Q012] / S[S_ATT1]);
  printf("quick slots 0..5 accept     %.4f\n", (double)S[S_Q0_5] / S[S_ATT1]);
  printf("some level-1 slot quick-acc %.4f\n", (double)S[S_ANYQ] / S[S_ATT1]);
  printf("generations needing >1 attempt %.4f\n", (double)S[S_GEN_MULTI] / S[S_ATT1]);
  printf("later attempts %llu: solvable %.4f, quick 0|1 %.4f\n", (unsigned long long)S[S_LATER],
         (double)S[S_LATER_OK] / S[S_LATER], (double)S[S_LATER_Q01] / S[S_LATER]);
  printf("unsolvable attempts %llu: no piece fits %.4f, some piece without anchor %.4f, level-1 slots %.1f each "
         "(pair_quick rejects %.3f of them)\n",
         (unsigned long long)S[S_FAIL], (double)S[S_FAIL_NOANCH3] / S[S_FAIL], (double)S[S_FAIL_SOME0] / S[S_FAIL],
         (double)S[S_FAIL_PAIRS] / S[S_FAIL], (double)S[S_FAIL_PQREJ] / S[S_FAIL_PAIRS]);
  uint64_t nok = S[S_ATT] - S[S_FAIL];
  printf("solvable attempts %llu: slots to first success %.2f, none quick-accepted %.4f\n", (unsigned long long)nok,
         (double)S[S_OK_SLOTS] / nok, (double)S[S_OK_NOQUICK] / nok);
  printf("in-lane policy (accept quick 0|1, reject R1/R2, else park): generations %llu, park at attempt 1: %.4f, 2: %.4f, 3: %.4f, 4: %.4f; reject fires on %.4f of unsolvable attempts\n",
         (unsigned long long)P[P_GEN], (double)P[P_PARK1] / P[P_GEN], (double)P[P_PARK2] / P[P_GEN],
         (double)P[P_PARK3] / P[P_GEN], (double)P[P_PARK4] / P[P_GEN], (double)P[P_REJ_FIRE] / P[P_UNSOLV]);
  printf("board fill at first attempts (cells: share):");
  for (int k = 0; k <= 64; k += 4) {
    uint64_t s = 0;
    for (int j = k; j < k + 4 && j <= 64; ++j) s += fill_hist[j];
    printf(" %d:%.3f", k, (double)s / S[S_ATT1]);
  }
  printf("\n");
  bbo_destroy(v);
  return 0;
}

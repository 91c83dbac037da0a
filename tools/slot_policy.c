/*
 * slot_policy.c -- diagnostics (not product, not test): which two in-lane
 * quick tests (one per env copy of the rollout kernel) settle most first
 * attempts of _generate_new_pieces (engine.py:155-238) on the bench workload.
 *   gcc -O2 -fopenmp -o /tmp/slot_policy tools/slot_policy.c && /tmp/slot_policy [N] [T]
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

static int lowbit(uint64_t x) { return __builtin_ctzll(x); }
static int highbit(uint64_t x) { return 63 - __builtin_clzll(x); }

/* pair_quick variants: mode 0 = shipped (|D| bound + first leaf each order);
 * mode 1 = + last leaf each order */
static int pair_quick(uint64_t B1, int b, int c, int mode) {
  uint64_t A2 = anchors_of(b, B1), A3 = anchors_of(c, B1);
  if (!(A2 | A3)) return 0;
  if (A2 && __builtin_popcountll(A3) > g_dtab[b][c]) return 1;
  if (A3 && __builtin_popcountll(A2) > g_dtab[b][c]) return 1;
  if (mode == -1) return 2;
  if (mode == -3) {  /* leaves as "z fits on B1 | y@q" (no clear): A_z & ~conflict */
    if (A2 && anchors_of(c, B1 | (g_shape[b] << lowbit(A2)))) return 1;
    if (A3 && anchors_of(b, B1 | (g_shape[c] << lowbit(A3)))) return 1;
    return 2;
  }
  if (A2 && anchors_of(c, clear_full(B1 | (g_shape[b] << lowbit(A2))))) return 1;
  if (mode == -2) return 2;
  if (A3 && anchors_of(b, clear_full(B1 | (g_shape[c] << lowbit(A3))))) return 1;
  if (mode >= 1) {
    if (A2 && anchors_of(c, clear_full(B1 | (g_shape[b] << highbit(A2))))) return 1;
    if (A3 && anchors_of(b, clear_full(B1 | (g_shape[c] << highbit(A3))))) return 1;
  }
  return 2;
}

/* slot (f, which anchor): which 0 lowest, 1 highest */
static int slot_test(uint64_t B, const int h[3], int f, int which, int mode) {
  int b = f == 0 ? 1 : 0, c = f == 2 ? 1 : 2;
  uint64_t A = anchors_of(h[f], B);
  if (!A) return 0;
  int p = which ? highbit(A) : lowbit(A);
  return pair_quick(clear_full(B | (g_shape[h[f]] << p)), h[b], h[c], mode) == 1;
}

/* order pieces by anchor count ascending (ties by slot), ignoring pieces without anchors */
static void order_by_anchors(uint64_t B, const int h[3], int ord[3], int* nz) {
  int cnt[3];
  for (int i = 0; i < 3; ++i) cnt[i] = __builtin_popcountll(anchors_of(h[i], B)), ord[i] = i;
  for (int i = 0; i < 3; ++i)
    for (int j = i + 1; j < 3; ++j)
      if (cnt[ord[j]] < cnt[ord[i]]) { int t = ord[i]; ord[i] = ord[j]; ord[j] = t; }
  *nz = 0;
  int o2[3], k = 0;
  for (int i = 0; i < 3; ++i) if (cnt[ord[i]]) o2[k++] = ord[i];
  for (int i = 0; i < 3; ++i) if (!cnt[ord[i]]) o2[k++] = ord[i];
  *nz = 0;
  for (int i = 0; i < 3; ++i) { ord[i] = o2[i]; if (cnt[o2[i]]) (*nz)++; }
}

enum { NPOL = 24 };
static const char* pol_names[NPOL] = {
  "shipped: f0 low | f1 low",
  "f0 low | f0 high",
  "f0 low | f1 low, +last leaf",
  "least-anchors piece low | 2nd least low",
  "least-anchors low | least-anchors high",
  "least low | 2nd least low, +last leaf",
  "most-anchors low | 2nd most low",
  "f0 low | f1 low | f2 low (3 slots)",
  "least low | 2nd low | 3rd low (3 slots)",
  "least low|high, 2nd low|high (4 slots)",
  "f0 low | f1 high",
  "least low | 2nd least high",
  "shipped slots, |D| bound only",
  "shipped slots, |D| + first order leaf",
  "shipped slots, leaves without clears",
  "most cells low | 2nd most cells low",
  "most cells low | most cells high",
  "1 slot: f0 low",
  "1 slot: f0 high",
  "1 slot: least-anchors low",
  "1 slot: most cells low",
  "1 slot: most-anchors low",
  "1 slot: f0 low, +last leaf",
  "1 slot: most cells low, +last leaf",
};
static uint64_t acc_cnt[NPOL], n_first, n_ok;
enum { KMAX = 16 };
static uint64_t acc_k_fixed[KMAX + 1], acc_k_dfs[KMAX + 1], acc_k_rr[KMAX + 1];

/* k-th anchor (rank) of A from the low end, or from the high end when neg */
static int rank_bit(uint64_t A, int r, int high) {
  for (int i = 0; i < r; ++i) {
    if (!A) return -1;
    if (high) A &= ~(1ull << (63 - __builtin_clzll(A))); else A &= A - 1;
  }
  if (!A) return -1;
  return high ? 63 - __builtin_clzll(A) : lowbit(A);
}

static int slot_at(uint64_t B, const int h[3], int f, int p) {
  int b = f == 0 ? 1 : 0, c = f == 2 ? 1 : 2;
  return pair_quick(clear_full(B | (g_shape[h[f]] << p)), h[b], h[c], 0) == 1;
}

static void gen_hook(const struct Engine* ee, int attempt, int ok) {
  const Engine* e = (const Engine*)ee;
  uint64_t B = grid_bits(&e->board);
  if (B == 0 || attempt != 0) return;
  const int* h = e->hand;
  n_first++;
  n_ok += ok;
  int ord[3], nz;
  order_by_anchors(B, h, ord, &nz);
  int r[NPOL];
  r[0] = slot_test(B, h, 0, 0, 0) | slot_test(B, h, 1, 0, 0);
  r[1] = slot_test(B, h, 0, 0, 0) | slot_test(B, h, 0, 1, 0);
  r[2] = slot_test(B, h, 0, 0, 1) | slot_test(B, h, 1, 0, 1);
  r[3] = slot_test(B, h, ord[0], 0, 0) | slot_test(B, h, ord[1], 0, 0);
  r[4] = slot_test(B, h, ord[0], 0, 0) | slot_test(B, h, ord[0], 1, 0);
  r[5] = slot_test(B, h, ord[0], 0, 1) | slot_test(B, h, ord[1], 0, 1);
  r[6] = slot_test(B, h, ord[2], 0, 0) | slot_test(B, h, ord[1], 0, 0);
  r[7] = r[0] | slot_test(B, h, 2, 0, 0);
  r[8] = r[3] | slot_test(B, h, ord[2], 0, 0);
  r[9] = r[4] | slot_test(B, h, ord[1], 0, 0) | slot_test(B, h, ord[1], 1, 0);
  r[10] = slot_test(B, h, 0, 0, 0) | slot_test(B, h, 1, 1, 0);
  r[11] = slot_test(B, h, ord[0], 0, 0) | slot_test(B, h, ord[1], 1, 0);
  r[12] = slot_test(B, h, 0, 0, -1) | slot_test(B, h, 1, 0, -1);
  r[13] = slot_test(B, h, 0, 0, -2) | slot_test(B, h, 1, 0, -2);
  r[14] = slot_test(B, h, 0, 0, -3) | slot_test(B, h, 1, 0, -3);
  {
    int oc[3] = {0, 1, 2};
    for (int i = 0; i < 3; ++i)
      for (int j = i + 1; j < 3; ++j)
        if (g_pieces[h[oc[j]]].n > g_pieces[h[oc[i]]].n) { int t = oc[i]; oc[i] = oc[j]; oc[j] = t; }
    r[15] = slot_test(B, h, oc[0], 0, 0) | slot_test(B, h, oc[1], 0, 0);
    r[16] = slot_test(B, h, oc[0], 0, 0) | slot_test(B, h, oc[0], 1, 0);
    r[17] = slot_test(B, h, 0, 0, 0);
    r[18] = slot_test(B, h, 0, 1, 0);
    r[19] = slot_test(B, h, ord[0], 0, 0);
    r[20] = slot_test(B, h, oc[0], 0, 0);
    r[21] = slot_test(B, h, nz ? ord[nz - 1] : 0, 0, 0);
    r[22] = slot_test(B, h, 0, 0, 1);
    r[23] = slot_test(B, h, oc[0], 0, 1);
  }
  {
    /* fixed list: round j covers (f0,f1,f2) at the j/2-th anchor from the low (even j) or high (odd j) end */
    uint64_t A[3] = {anchors_of(h[0], B), anchors_of(h[1], B), anchors_of(h[2], B)};
    int hit = 0;
    for (int k = 0; k < KMAX; ++k) {
      const int f = k % 3, round = k / 3, high = round & 1, rank = round / 2;
      const int p = rank_bit(A[f], rank, high);
      if (p >= 0 && slot_at(B, h, f, p)) hit = 1;
      acc_k_fixed[k + 1] += hit;
    }
    /* DFS order: f-major, anchors ascending */
    hit = 0;
    int k = 0;
    for (int f = 0; f < 3 && k < KMAX; ++f)
      for (uint64_t it = A[f]; it && k < KMAX; it &= it - 1, ++k) {
        if (slot_at(B, h, f, lowbit(it))) hit = 1;
        acc_k_dfs[k + 1] += hit;
      }
    for (; k < KMAX; ++k) acc_k_dfs[k + 1] += hit;
    /* round-robin over f, anchors ascending within f */
    hit = 0;
    k = 0;
    uint64_t it[3] = {A[0], A[1], A[2]};
    while (k < KMAX && (it[0] | it[1] | it[2])) {
      for (int f = 0; f < 3 && k < KMAX; ++f) {
        if (!it[f]) continue;
        const int p = lowbit(it[f]);
        it[f] &= it[f] - 1;
        if (slot_at(B, h, f, p)) hit = 1;
        acc_k_rr[++k] += hit;
      }
    }
    for (; k < KMAX; ++k) acc_k_rr[k + 1] += hit;
  }
  for (int k = 0; k < NPOL; ++k) {
    if (r[k] && !ok) { fprintf(stderr, "UNSOUND %d\n", k); exit(1); }
    acc_cnt[k] += r[k];
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
  printf("first attempts %llu, solvable %.4f\n", (unsigned long long)n_first, (double)n_ok / n_first);
  for (int k = 0; k < NPOL; ++k)
    printf("%-45s accept %.4f  park %.4f\n", pol_names[k], (double)acc_cnt[k] / n_first,
           1.0 - (double)acc_cnt[k] / n_first);
  printf("k slots per drawing env:  fixed(f-rotating, low/high)  DFS(f-major)  round-robin\n");
  for (int k = 1; k <= KMAX; ++k)
    printf("  k=%2d  accept %.4f  %.4f  %.4f\n", k, (double)acc_k_fixed[k] / n_first, (double)acc_k_dfs[k] / n_first,
           (double)acc_k_rr[k] / n_first);
  return 0;
}

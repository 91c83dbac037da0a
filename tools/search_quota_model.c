/*
 * search_quota_model.c -- diagnostics (not product, not test): the rollout kernel's search calls
 * (csrc/bb_solver.h gen_hands_multi, called by rollout_async_kernel's search waves on the envs that the
 * in-lane fewest-anchor quick test posted) replayed on the C oracle's bench workload, comparing the pass
 * schedule of round 4 (every slot of the leading attempts, packed f-major up to 3 passes of 64) with a
 * quota schedule (every active attempt gets at most Q slots per pass, so the first pass tests the leading
 * slots of many attempts: a solvable attempt succeeds on its first ~1.3 slots).
 *   gcc -O2 -o /tmp/sqm tools/search_quota_model.c && /tmp/sqm [N] [T] [E] [Q] [Qnext]
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

static int g_noleaf = 0;  /* pass quick test without the two leaf tests */
static int pair_quick(uint64_t B1, int b, int c, uint64_t* A2o, uint64_t* A3o) {
  uint64_t A2 = anchors_of(b, B1), A3 = anchors_of(c, B1);
  *A2o = A2, *A3o = A3;
  if (!(A2 | A3)) return 0;
  if (A2 && __builtin_popcountll(A3) > g_dtab[b][c]) return 1;
  if (A3 && __builtin_popcountll(A2) > g_dtab[b][c]) return 1;
  if (g_noleaf == 1) return 2;
  if (g_noleaf == 3) {  /* 4 leaves: lowest and highest anchor of each order */
    if (A2 && anchors_of(c, clear_full(B1 | (g_shape[b] << lowbit(A2))))) return 1;
    if (A3 && anchors_of(b, clear_full(B1 | (g_shape[c] << lowbit(A3))))) return 1;
    if (A2 && anchors_of(c, clear_full(B1 | (g_shape[b] << (63 - __builtin_clzll(A2)))))) return 1;
    if (A3 && anchors_of(b, clear_full(B1 | (g_shape[c] << (63 - __builtin_clzll(A3)))))) return 1;
    return 2;
  }
  if (g_noleaf == 2) {  /* sound clear-free leaves: "z fits on B1 | y@q" */
    if (A2 && anchors_of(c, B1 | (g_shape[b] << lowbit(A2)))) return 1;
    if (A3 && anchors_of(b, B1 | (g_shape[c] << lowbit(A3)))) return 1;
    return 2;
  }
  if (A2 && anchors_of(c, clear_full(B1 | (g_shape[b] << lowbit(A2))))) return 1;
  if (A3 && anchors_of(b, clear_full(B1 | (g_shape[c] << lowbit(A3))))) return 1;
  return 2;
}

static int pair_exact(uint64_t B1, int b, int c) {
  uint64_t A2 = anchors_of(b, B1), A3 = anchors_of(c, B1);
  for (uint64_t it = A2; it; it &= it - 1)
    if (anchors_of(c, clear_full(B1 | (g_shape[b] << lowbit(it))))) return 1;
  for (uint64_t it = A3; it; it &= it - 1)
    if (anchors_of(b, clear_full(B1 | (g_shape[c] << lowbit(it))))) return 1;
  return 0;
}

static int quick_slot(uint64_t B, const int h[3], int k) {
  int f = k % 3, b = f == 0 ? 1 : 0, c = f == 2 ? 1 : 2;
  uint64_t A = anchors_of(h[f], B);
  if (!A) return 0;
  int p = k < 3 ? lowbit(A) : 63 - __builtin_clzll(A);
  uint64_t a2, a3;
  return pair_quick(clear_full(B | (g_shape[h[f]] << p)), h[b], h[c], &a2, &a3) == 1;
}

/* ---- replay: every generation with its pre-draw stream state ---------- */
typedef struct {
  int t, i;
  uint64_t B;
  Pcg64 pre;
} Gen;
static Gen* g_gens;
static size_t g_ngen, g_capgen;
static bbo_vec* g_v;
static Pcg64* g_pre;
static int g_t;

static void gen_hook(const struct Engine* ee, int attempt, int ok) {
  (void)ok;
  const Engine* e = (const Engine*)ee;
  if (attempt != 0) return;
  uint64_t B = grid_bits(&e->board);
  if (B == 0) return;
  const int i = (int)((const Env*)e - g_v->envs);
  if (g_ngen == g_capgen) {
    g_capgen = g_capgen ? 2 * g_capgen : 1 << 16;
    g_gens = realloc(g_gens, g_capgen * sizeof(Gen));
  }
  g_gens[g_ngen++] = (Gen){g_t, i, B, g_pre[i]};
}

static void draw_hand(Pcg64* s, int h[3]) {
  for (int k = 0; k < 3; ++k) h[k] = (int)draw_below(s, NPIECES);
}


/* the in-lane test of the rollout kernel: the fewest-anchor piece at its lowest anchor (quick_rank_bf) */
static int quick_rank0(uint64_t B, const int h[3]) {
  uint64_t A[3];
  unsigned c[3];
  for (int f = 0; f < 3; ++f) A[f] = anchors_of(h[f], B), c[f] = A[f] ? __builtin_popcountll(A[f]) : 65u;
  const int r1 = (c[0] <= c[1]) + (c[2] < c[1]), r2 = (c[0] <= c[2]) + (c[1] <= c[2]);
  const int f = r2 == 0 ? 2 : (r1 == 0 ? 1 : 0);
  const int b = f == 0 ? 1 : 0, cc = f == 2 ? 1 : 2;
  if (!A[f]) return 0;
  uint64_t a2, a3;
  return pair_quick(clear_full(B | (g_shape[h[f]] << lowbit(A[f]))), h[b], h[cc], &a2, &a3) == 1;
}

typedef struct {
  double calls, rounds, passes, slots, slow_rounds, slow_tasks, envs;
} Stats;

static int g_P = 3;

/* mode 0: round-4 packing; mode 1: quota Q per active attempt per pass (Qn in later passes) */
static void model_call(Gen** par, int E0, int pack_first, int pack_next, int mode, int Q, int Qn, Stats* st) {
  int att[64], todo[64];
  Pcg64 s[64];
  for (int e = 0; e < E0; ++e) att[e] = 0, s[e] = par[e]->pre, todo[e] = 1;
  int E = E0, pk = pack_first;
  st->calls += 1;
  st->envs += E0;
  while (E > 0) {
    int idx[64], m = 0;
    for (int e = 0; e < E0; ++e)
      if (todo[e]) idx[m++] = e;
    int K = 64 / E;
    if (K > pk) K = pk;
    if (K > 32) K = 32;
    if (K < 1) K = 1;
    const int nl = E * K;
    int hands[64][3], S[64], valid[64];
    Pcg64 after[64];
    uint64_t A[64][3];
    for (int L = 0; L < nl; ++L) {
      const int k = L / E, e = idx[L % E];
      valid[L] = att[e] + k < MAX_ATTEMPTS;
      Pcg64 c = s[e];
      for (int q = 0; q <= k; ++q) draw_hand(&c, hands[L]);
      after[L] = c;
      S[L] = 0;
      if (valid[L])
        for (int f = 0; f < 3; ++f) A[L][f] = anchors_of(hands[L][f], par[e]->B), S[L] += __builtin_popcountll(A[L][f]);
    }
    st->rounds += 1;
    /* slot lists per lane, f-major */
    static int sf[64][200], sp[64][200];
    for (int L = 0; L < nl; ++L) {
      int n = 0;
      if (valid[L])
        for (int f = 0; f < 3; ++f)
          for (uint64_t it = A[L][f]; it; it &= it - 1) sf[L][n] = f, sp[L][n] = lowbit(it), ++n;
    }
    int done[64] = {0}, ok[64] = {0}, packed = nl;
    if (mode == 0) {  /* leading lanes whose slots fit g_P passes */
      int incl = 0;
      packed = 0;
      for (int L = 0; L < nl; ++L) {
        incl += valid[L] ? S[L] : 0;
        if (incl <= 64 * g_P) packed = L + 1; else break;
      }
      if (packed == 0) packed = 1;
    }
    for (int pass = 0;; ++pass) {
      /* env decisions */
      int undecided = 0;
      int dec[64] = {0};
      for (int es = 0; es < E; ++es) {
        int d = 0, all = 1;
        for (int L = es; L < packed; L += E) {
          if (!valid[L]) continue;
          if (ok[L]) { d = 1; break; }
          if (done[L] < S[L]) { all = 0; break; }
        }
        dec[es] = d || all;
        undecided += !dec[es];
      }
      if (!undecided) break;
      /* build the pass */
      int cnt = 0, lane_of[64], slot_of[64];
      for (int L = 0; L < packed && cnt < 64; ++L) {
        const int es = L % E;
        if (dec[es] || !valid[L] || ok[L] || done[L] >= S[L]) continue;
        int blocked = 0;
        for (int j = es; j < L; j += E) blocked |= ok[j];
        if (blocked) continue;
        int q = S[L] - done[L];
        if (mode == 1) {
          const int cap = pass == 0 ? Q : Qn;
          if (q > cap) q = cap;
        }
        for (int k2 = 0; k2 < q && cnt < 64; ++k2) lane_of[cnt] = L, slot_of[cnt] = done[L] + k2, ++cnt;
      }
      if (!cnt) break;
      st->passes += 1;
      st->slots += cnt;
      int qq[64];
      uint64_t A2s[64], A3s[64], B1s[64];
      for (int x = 0; x < cnt; ++x) {
        const int L = lane_of[x], f = sf[L][slot_of[x]], b = f == 0 ? 1 : 0, c = f == 2 ? 1 : 2;
        B1s[x] = clear_full(par[idx[L % E]]->B | (g_shape[hands[L][f]] << sp[L][slot_of[x]]));
        qq[x] = pair_quick(B1s[x], hands[L][b], hands[L][c], &A2s[x], &A3s[x]);
        if (qq[x] == 1) ok[L] = 1;
      }
      int tasks = 0;
      for (int x = 0; x < cnt; ++x) {
        const int L = lane_of[x];
        int blocked = 0;
        for (int j = L % E; j <= L; j += E) blocked |= ok[j];
        if (qq[x] == 2 && !blocked) {
          tasks += __builtin_popcountll(A2s[x]) + __builtin_popcountll(A3s[x]);
          const int f = sf[L][slot_of[x]], b = f == 0 ? 1 : 0, c = f == 2 ? 1 : 2;
          if (pair_exact(B1s[x], hands[L][b], hands[L][c])) ok[L] = 1;
        }
      }
      if (tasks) st->slow_tasks += tasks, st->slow_rounds += (tasks + 63) / 64;
      for (int x = 0; x < cnt; ++x) done[lane_of[x]] = slot_of[x] + 1 > done[lane_of[x]] ? slot_of[x] + 1 : done[lane_of[x]];
    }
    for (int es = 0; es < E; ++es) {
      const int e = idx[es];
      int hit = -1, last = -1, npk = 0;
      for (int L = es; L < packed; L += E) {
        if (!valid[L]) continue;
        if (ok[L]) { hit = L; break; }
        if (done[L] < S[L]) break;
        ++npk, last = L;
      }
      if (hit >= 0) s[e] = after[hit], todo[e] = 0;
      else if (last >= 0) {
        s[e] = after[last];
        att[e] += npk;
        if (att[e] >= MAX_ATTEMPTS) todo[e] = 0;
      }
    }
    E = 0;
    for (int e = 0; e < E0; ++e) E += todo[e];
    pk = pack_next > 0 ? pack_next : 2 * pk;
    if (pk > 32) pk = 32;
  }
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 8192;
  int T = argc > 2 ? atoi(argv[2]) : 128;
  int Ecall = argc > 3 ? atoi(argv[3]) : 7;
  int Q = argc > 4 ? atoi(argv[4]) : 8;
  int Qn = argc > 5 ? atoi(argv[5]) : 64;
  if (argc > 6) g_noleaf = atoi(argv[6]);
  init_bits();
  uint64_t* seeds = malloc(sizeof(uint64_t) * n);
  for (int i = 0; i < n; ++i) seeds[i] = 42 + (uint64_t)i;
  bbo_vec* v = bbo_create(n, seeds, NULL, NULL, 1);
  g_v = v;
  g_pre = malloc(sizeof(Pcg64) * n);
  bbo_reset(v, 1);
  uint64_t* m = malloc(sizeof(uint64_t) * 3 * n);
  int32_t* a = malloc(sizeof(int32_t) * n);
  bbo_state(v, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, m);
  bbo_random_actions(m, n, 0xB10C, 0, 0, a);
  for (int t = 0; t < T; ++t) {
    g_t = t;
    for (int i = 0; i < n; ++i) g_pre[i] = v->envs[i].eng.rng;
    for (int i = 0; i < n; ++i) {
      StepOut o;
      env_step(v, &v->envs[i], a[i], &o, NULL);
      uint64_t mm[HAND];
      action_mask(&v->envs[i].eng, mm);
      a[i] = policy_action(mm, philox_w0(0xB10C, (uint64_t)i, (uint64_t)t + 1));
    }
  }
  Gen** posted = malloc(sizeof(Gen*) * g_ngen);
  size_t np = 0;
  for (size_t gi = 0; gi < g_ngen; ++gi) {
    Pcg64 c = g_gens[gi].pre;
    int h[3];
    draw_hand(&c, h);
    if (!quick_rank0(g_gens[gi].B, h)) posted[np++] = &g_gens[gi];
  }
  for (int mode = 0; mode < 2; ++mode) {
    Stats st = {0};
    for (size_t k = 0; k < np; k += Ecall) {
      const int E = np - k < (size_t)Ecall ? (int)(np - k) : Ecall;
      model_call(posted + k, E, 8, 32, mode, Q, Qn, &st);
    }
    const double cyc = 3.63 * st.rounds + 3.83 * st.passes + 1.57 * st.slow_rounds;
    printf("%s: generations %zu posted %zu (%.3f); calls %.0f envs/call %.2f rounds/call %.2f passes/call %.2f "
           "slots/pass %.1f slow rounds/call %.2f -> modelled %.2fk cycles/call, %.1f per posted env\n",
           mode ? "quota" : "round-4", g_ngen, np, (double)np / g_ngen, st.calls, st.envs / st.calls,
           st.rounds / st.calls, st.passes / st.calls, st.slots / st.passes, st.slow_rounds / st.calls,
           cyc / st.calls, cyc * 1000 / st.envs);
  }
  return 0;
}

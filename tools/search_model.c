/*
 * search_model.c -- diagnostics (not product, not test): replays the bench
 * workload on the C oracle and models the rollout kernel's wave search
 * (csrc/bb_solver.h gen_hands_multi) on every wave-step's parked envs:
 * rounds, passes, slot and exact-phase task counts, so that search designs
 * can be compared on the CPU before they are built.
 *   gcc -O2 -o /tmp/search_model tools/search_model.c -lm && /tmp/search_model [N] [T] [pack_first] [pack_next]
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

/* ---- model of gen_hands_multi -------------------------------------------- */
typedef struct {
  double calls, rounds, passes, slots, slow_rounds, slow_tasks, lanes_drawn, lanes_packed, envs;
} Stats;

static int g_P = 1;
static double* g_wave_cyc;  /* modelled search cycles per wave */
static double g_call_max, g_heavy_cyc;
static long g_heavy_n;
static double g_cls[2][2], g_cls_n[2][2];  /* slow tasks by slot class: [one-sided][line reachable] */  /* passes (64 slots each) an attempt batch may span */

static void model_call(Gen** par, int E0, int pack_first, int pack_next, Stats* st) {
  int att[64];
  Pcg64 s[64];
  int todo[64];
  int E = E0;
  for (int e = 0; e < E0; ++e) att[e] = 0, s[e] = par[e]->pre, todo[e] = 1;
  int pk = pack_first;
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
      const int k = L / E, es = L % E, e = idx[es];
      valid[L] = att[e] + k < MAX_ATTEMPTS;
      Pcg64 c = s[e];
      for (int q = 0; q <= k; ++q) draw_hand(&c, hands[L]);
      after[L] = c;
      S[L] = 0;
      if (valid[L])
        for (int f = 0; f < 3; ++f) A[L][f] = anchors_of(hands[L][f], par[e]->B), S[L] += __builtin_popcountll(A[L][f]);
    }
    int incl = 0, nb = 0, lane_end[64];
    for (int L = 0; L < nl; ++L) {
      incl += valid[L] ? S[L] : 0;
      lane_end[L] = incl;
      if (incl <= 64 * g_P) nb = L + 1; else break;
    }
    if (nb == 0) nb = 1;
    int total = lane_end[nb - 1];
    st->rounds += 1;
    st->lanes_drawn += nl;
    st->lanes_packed += nb;
    int ok_lane[64] = {0};
    int slot_lane[4096], slot_f[4096], slot_p[4096], ns = 0;
    for (int L = 0; L < nb; ++L) {
      if (!valid[L]) continue;
      for (int f = 0; f < 3; ++f)
        for (uint64_t it = A[L][f]; it; it &= it - 1)
          if (ns < 4096) slot_lane[ns] = L, slot_f[ns] = f, slot_p[ns] = lowbit(it), ++ns;
    }
    int base = 0;
    for (;;) {
      st->passes += 1;
      const int hi = base + 64 < total ? base + 64 : total;
      st->slots += hi - base;
      int q[64];
      uint64_t A2s[64], A3s[64];
      for (int x = base; x < hi; ++x) {
        const int L = slot_lane[x], f = slot_f[x], b = f == 0 ? 1 : 0, c = f == 2 ? 1 : 2;
        const uint64_t B1 = clear_full(par[idx[L % E]]->B | (g_shape[hands[L][f]] << slot_p[x]));
        q[x - base] = pair_quick(B1, hands[L][b], hands[L][c], &A2s[x - base], &A3s[x - base]);
        if (q[x - base] == 1) ok_lane[L] = 1;
      }
      int tasks = 0;
      for (int x = base; x < hi; ++x) {
        const int L = slot_lane[x];
        int blocked = 0;  /* an attempt lane of the same env up to L has succeeded */
        for (int j = L % E; j <= L; j += E) blocked |= ok_lane[j];
        if (q[x - base] == 2 && !blocked) {
          const int t2 = __builtin_popcountll(A2s[x - base]) + __builtin_popcountll(A3s[x - base]);
          tasks += t2;
          {
            const uint64_t a2 = A2s[x - base], a3 = A3s[x - base];
            const int fl = slot_f[x], bb = fl == 0 ? 1 : 0, cc = fl == 2 ? 1 : 2;
            const uint64_t B1x = clear_full(par[idx[L % E]]->B | (g_shape[hands[L][fl]] << slot_p[x]));
            int cls = (a2 && a3) ? 0 : 1;
            /* one-sided: only the piece with anchors can go first, and it must complete a line */
            int reach = 1;
            if (cls) {
              const int y = a2 ? hands[L][bb] : hands[L][cc];
              int r2 = 0;
              for (int r = 0; r < 8; ++r) if (8 - __builtin_popcountll((B1x >> (8 * r)) & 0xFF) <= g_pieces[y].w) r2 = 1;
              for (int c = 0; c < 8; ++c) if (8 - __builtin_popcountll(B1x & (0x0101010101010101ull << c)) <= g_pieces[y].h) r2 = 1;
              reach = r2;
            }
            g_cls[cls][reach] += t2;
            g_cls_n[cls][reach] += 1;
          }
          const int f = slot_f[x], b = f == 0 ? 1 : 0, c = f == 2 ? 1 : 2;
          const uint64_t B1 = clear_full(par[idx[L % E]]->B | (g_shape[hands[L][f]] << slot_p[x]));
          if (pair_exact(B1, hands[L][b], hands[L][c])) ok_lane[L] = 1;
        }
      }
      if (tasks) {
        st->slow_tasks += tasks;
        st->slow_rounds += (tasks + 63) / 64;
      }
      base += 64;
      if (base >= total) break;
      /* every env decided?  (its earliest ok lane has only complete lanes before it, or all its lanes complete) */
      int undecided = 0;
      for (int es = 0; es < E; ++es) {
        int dec = 0;
        for (int L = es; L < nb; L += E) {
          if (!valid[L]) continue;
          if (ok_lane[L]) { dec = 1; break; }
          if (lane_end[L] > base) break;  /* not complete, no success yet */
        }
        if (!dec) {
          int last = -1;
          for (int L = es; L < nb; L += E) if (valid[L]) last = L;
          if (last < 0 || lane_end[last] <= base) dec = 1;  /* all complete: exhausted */
        }
        undecided += !dec;
      }
      if (!undecided) break;
    }
    /* resolve */
    for (int es = 0; es < E; ++es) {
      const int e = idx[es];
      int hit = -1, last = -1, npk = 0;
      for (int L = es; L < nb; L += E) {
        if (!valid[L]) continue;
        if (lane_end[L] - S[L] >= base && !ok_lane[L]) break;  /* never tested */
        if (ok_lane[L]) { hit = L; break; }
        if (lane_end[L] > base) break;  /* partially tested, no success: undecided */
        ++npk;
        last = L;
      }
      if (hit >= 0) {
        s[e] = after[hit];
        todo[e] = 0;
      } else if (last >= 0) {
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
  int pack_first = argc > 3 ? atoi(argv[3]) : 8;
  int pack_next = argc > 4 ? atoi(argv[4]) : 32;
  int epw = 32;
  if (argc > 5) g_P = atoi(argv[5]);
  if (argc > 6) epw = atoi(argv[6]);
  if (argc > 7) g_noleaf = atoi(argv[7]);
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
  /* group parked generations by (t, wave) */
  Stats st = {0};
  size_t parked = 0;
  Gen** grp = malloc(sizeof(Gen*) * 64);
  g_wave_cyc = calloc(n / epw + 1, sizeof(double));
  size_t gi = 0;
  /* g_gens is in (t, i) order already (single-threaded replay) */
  while (gi < g_ngen) {
    const int t = g_gens[gi].t, w = g_gens[gi].i / epw;
    int E = 0;
    for (; gi < g_ngen && g_gens[gi].t == t && g_gens[gi].i / epw == w; ++gi) {
      Pcg64 c = g_gens[gi].pre;
      int h[3];
      draw_hand(&c, h);
      const int nl_save = g_noleaf;
      g_noleaf = 0;
      const int acc = quick_slot(g_gens[gi].B, h, 0) | quick_slot(g_gens[gi].B, h, 1);
      g_noleaf = nl_save;
      if (acc) continue;
      grp[E++] = &g_gens[gi];
    }
    if (E) {
      parked += E;
      const Stats before = st;
      model_call(grp, E, pack_first, pack_next, &st);
      const double cyc = 3.63 * (st.rounds - before.rounds) + 3.83 * (st.passes - before.passes) +
                         1.57 * (st.slow_rounds - before.slow_rounds);
      g_wave_cyc[w] += cyc;
      if (cyc > g_call_max) g_call_max = cyc;
      if (cyc > 40.0) {
        g_heavy_n++;
        g_heavy_cyc += cyc;
        if (g_heavy_n <= 8)
          printf("heavy call: E=%d rounds %.0f passes %.0f slow %.0f -> %.0fk\n", E, st.rounds - before.rounds,
                 st.passes - before.passes, st.slow_rounds - before.slow_rounds, cyc);
      }
    }
  }
  const double wave_steps = (double)(n / epw) * T;
  printf("envs %d x %d steps, pack %d,%d: generations %zu, parked %zu (%.4f per wave-step)\n", n, T, pack_first,
         pack_next, g_ngen, parked, parked / wave_steps);
  printf("calls/wave-step %.3f  envs/call %.2f  rounds/call %.2f  passes/round %.2f  slots/pass %.1f  "
         "lanes drawn/round %.1f packed/round %.1f  slow rounds/round %.2f  slow tasks/round %.1f\n",
         st.calls / wave_steps, st.envs / st.calls, st.rounds / st.calls, st.passes / st.rounds,
         st.slots / st.passes, st.lanes_drawn / st.rounds, st.lanes_packed / st.rounds, st.slow_rounds / st.rounds,
         st.slow_tasks / st.rounds);
  const double cr = 3.63, cp = 3.83, cs = 1.57;  /* k-cycles per round / pass / slow round (GPU diag, round 2) */
  printf("per wave-step: rounds %.3f passes %.3f slow rounds %.3f  -> modelled search %.2fk cycles\n",
         st.rounds / wave_steps, st.passes / wave_steps, st.slow_rounds / wave_steps,
         (cr * st.rounds + cp * st.passes + cs * st.slow_rounds) / wave_steps);
  printf("slow tasks by slot class: both-sided %.0f (%.0f slots), one-sided reachable %.0f (%.0f), one-sided unreachable %.0f (%.0f)\n",
         g_cls[0][1], g_cls_n[0][1], g_cls[1][1], g_cls_n[1][1], g_cls[1][0], g_cls_n[1][0]);
  {
    const int nw = n / epw;
    double mx = 0, mean = 0;
    for (int w = 0; w < nw; ++w) { mean += g_wave_cyc[w]; if (g_wave_cyc[w] > mx) mx = g_wave_cyc[w]; }
    mean /= nw;
    const double base = 7.3 * T;  /* k-cycles of in-lane work per wave over T steps (GPU diag) */
    printf("per wave over %d steps: search mean %.0fk max %.0fk; with in-lane base: max/mean %.3f; heaviest call %.1fk\n",
           T, mean, mx, (mx + base) / (mean + base), g_call_max);
  }
  printf("calls above 40k cycles: %ld, %.1f%% of search cycles\n", g_heavy_n, 100.0 * g_heavy_cyc / (3.63 * st.rounds + 3.83 * st.passes + 1.57 * st.slow_rounds));
  printf("per env-step: modelled search %.1f cycles\n", (cr * st.rounds + cp * st.passes + cs * st.slow_rounds) * 1000 / wave_steps / epw);
  return 0;
}

// bb_solver.h -- exact "can all three pieces be placed in some order" test
// (engine.py:155-238 _generate_new_pieces / _can_place_remaining /
// _simulate_line_clears) on bitboards, plus the rejection-sampling hand draw.
//
// Only the boolean of the reference's DFS matters (it decides how many
// 3-draw attempts consume the PCG64 stream), so any exact algorithm is
// allowed.  Structure:
//   level 1: every legal anchor p of the first piece f (all 3 choices of f),
//            B1 = clear(B | f<<p);
//   level 2: can the remaining pair (y, z) both be placed on B1?
//     * quick accept: with D(y,z) = {oy_i - oz_j} (linear cell offsets), a
//       y-anchor conflicts with at most |D| z-anchors, so |A_z| > |D| and
//       A_y != 0 => a disjoint pair exists (clears only ever remove cells);
//     * order y then z, set algebra instead of a placement loop:
//         G = AND_{r in A_z} (r - D)   = y-anchors at which EVERY z-anchor
//                                         collides (computed as one 128-bit
//                                         shift + AND per z-anchor);
//       any q in A_y \ G leaves a z-anchor free => yes.  A q in G can only
//       succeed if y at q completes a line (the clear may free room for z):
//       those few q are checked explicitly.  Same for order z then y.
//   level 3 is the anchors_of() != 0 test.
// The per-lane search runs under a work budget; a board that exceeds it is
// finished by a whole wave (solve_wave: lane l takes level-1 anchor l) in the
// escalation kernel, so one hard board never serialises a wave of easy ones.
#pragma once
#include "bb_device.h"

namespace bb {

constexpr int kUnlimited = 1 << 30;

// Work-budget ticks (roughly proportional to instruction counts).
constexpr int kTickAnchors = 4;
constexpr int kTickG = 1;
constexpr int kTickQ = 1;

__device__ __forceinline__ bool has_full_line(uint64_t B) {
  uint64_t r = B & (B >> 1);
  r &= r >> 2;
  r &= r >> 4;
  uint64_t c = B & (B >> 8);
  c &= c >> 16;
  c &= c >> 32;
  return ((r & kCol0) | (c & 0xFFull)) != 0ull;
}

// High 64 bits of a 128-bit value shifted left by s (0 <= s < 64).
__device__ __forceinline__ uint64_t hi_shl(uint64_t lo, uint64_t hi, int s) {
  return s ? (hi << s) | (lo >> (64 - s)) : hi;
}

// 128-bit mask with bit (64 - d) for every d in D(y,z) = {oy_i - oz_j}.
__device__ __forceinline__ void pair_conflict_mask(const PieceRow& y, const PieceRow& z, uint64_t& lo,
                                                   uint64_t& hi) {
  lo = 0;
  hi = 0;
  uint64_t offs = z.offs;
  for (uint32_t j = 0; j < z.ncells; ++j) {
    const int o = (int)(offs & 63u);
    offs >>= 6;
    lo |= y.ym_lo << o;
    hi |= hi_shl(y.ym_lo, y.ym_hi, o);
  }
}

// Order "y then z" on B1 (Ay, Az: anchors of y, z on B1; Ay != 0).
// 1 yes, 0 no, -1 budget exhausted.
__device__ __forceinline__ int one_order(uint64_t B1, const PieceRow& y, const PieceRow& z, uint64_t Ay,
                                         uint64_t Az, int& budget) {
  uint64_t mlo, mhi;
  pair_conflict_mask(y, z, mlo, mhi);
  uint64_t G = ~0ull;
  uint64_t it = Az;
  while (it) {
    const int r = __ffsll((unsigned long long)it) - 1;
    it &= it - 1;
    G &= hi_shl(mlo, mhi, r);
    budget -= kTickG;
    if (Ay & ~G) return 1;
  }
  if (Ay & ~G) return 1;
  // every y-anchor blocks every z-anchor: only a line clear by y can help
  it = Ay;
  while (it) {
    if (budget <= 0) return -1;
    const int q = __ffsll((unsigned long long)it) - 1;
    it &= it - 1;
    const uint64_t B2 = B1 | (y.shape << q);
    budget -= kTickQ;
    if (has_full_line(B2)) {
      budget -= kTickAnchors;
      if (anchors_of(z, clear_full(B2))) return 1;
    }
  }
  return 0;
}

// Level 2: can pieces b and c both still be placed (either order) on B1?
__device__ __forceinline__ int solve_pair(uint64_t B1, const PieceRow& pb, const PieceRow& pc, uint32_t dbc,
                                          int& budget) {
  const uint64_t A2 = anchors_of(pb, B1);
  const uint64_t A3 = anchors_of(pc, B1);
  budget -= 2 * kTickAnchors;
  if ((A2 | A3) == 0) return 0;
  if (A2 && (uint32_t)__popcll(A3) > dbc) return 1;
  if (A3 && (uint32_t)__popcll(A2) > dbc) return 1;
  if (budget <= 0) return -1;
  int r = 0;
  if (A2) r = one_order(B1, pb, pc, A2, A3, budget);
  if (r != 0) return r;
  if (A3) r = one_order(B1, pc, pb, A3, A2, budget);
  return r;
}

// Full single-lane test.  1 solvable, 0 not, -1 budget exhausted.
__device__ __forceinline__ int solve_lane(uint64_t B, const PieceRow* tbl, const uint8_t* dtab, uint32_t i0,
                                          uint32_t i1, uint32_t i2, int& budget) {
  const uint32_t ids[3] = {i0, i1, i2};
#pragma unroll 1
  for (int f = 0; f < 3; ++f) {
    const uint32_t fi = ids[f];
    const uint32_t bi = ids[f == 0 ? 1 : 0];
    const uint32_t ci = ids[f == 2 ? 1 : 2];
    const PieceRow pf = tbl[fi];
    const PieceRow pb = tbl[bi];
    const PieceRow pc = tbl[ci];
    const uint32_t dbc = dtab[bi * kPieces + ci];
    uint64_t A1 = anchors_of(pf, B);
    budget -= kTickAnchors;
    while (A1) {
      if (budget <= 0) return -1;
      const int p = __ffsll((unsigned long long)A1) - 1;
      A1 &= A1 - 1;
      const uint64_t B1 = clear_full(B | (pf.shape << p));
      const int r = solve_pair(B1, pb, pc, dbc, budget);
      if (r != 0) return r;
    }
  }
  return 0;
}

// Whole-wave test of one board (all 64 lanes call it with identical
// arguments).  Lane l owns level-1 anchor l.
__device__ __forceinline__ bool solve_wave(uint64_t B, const PieceRow* tbl, const uint8_t* dtab, uint32_t i0,
                                           uint32_t i1, uint32_t i2, int lane) {
  const uint32_t ids[3] = {i0, i1, i2};
#pragma unroll 1
  for (int f = 0; f < 3; ++f) {
    const uint32_t fi = ids[f];
    const uint32_t bi = ids[f == 0 ? 1 : 0];
    const uint32_t ci = ids[f == 2 ? 1 : 2];
    const PieceRow pf = tbl[fi];
    const uint64_t A1 = anchors_of(pf, B);
    bool ok = false;
    if ((A1 >> lane) & 1ull) {
      const PieceRow pb = tbl[bi];
      const PieceRow pc = tbl[ci];
      int budget = kUnlimited;
      const uint64_t B1 = clear_full(B | (pf.shape << lane));
      ok = solve_pair(B1, pb, pc, dtab[bi * kPieces + ci], budget) == 1;
    }
    if (__ballot(ok)) return true;
  }
  return false;
}

// _generate_new_pieces (engine.py:155-172) for one lane, under a budget.
// attempt: attempts already used (in/out).  Returns true when the hand is
// final (solvable, or 100 attempts exhausted -> last draw kept).  Returns false
// when the budget ran out: rng is rolled back to just before the unfinished
// attempt's three draws so the wave can replay it.
__device__ __forceinline__ bool gen_hand_lane(uint64_t B, Pcg& rng, uint32_t& ids, int& attempt,
                                              const PieceRow* tbl, const uint8_t* dtab, int budget) {
#pragma unroll 1
  for (; attempt < kMaxAttempts; ++attempt) {
    const Pcg save = rng;
    const uint32_t a = draw_piece(rng);
    const uint32_t b = draw_piece(rng);
    const uint32_t c = draw_piece(rng);
    ids = a | (b << 6) | (c << 12);
    const int r = solve_lane(B, tbl, dtab, a, b, c, budget);
    if (r == 1) return true;
    if (r < 0) {
      rng = save;
      return false;
    }
  }
  return true;
}

// Wave-cooperative continuation of gen_hand_lane for one env (all 64 lanes
// call it with identical arguments; on return ids/rng are the final hand and
// stream state, identical in every lane).
//
// Level-1 tasks of an attempt are its (f, p) pairs, f in {0,1,2}, p in
// anchors(f, B), laid out f-major.  Consecutive attempts are drawn ahead
// (the PCG stream does not depend on the verdicts) and packed while their
// tasks fit one wave: a crowded board that fails attempt after attempt has
// few anchors, so up to kPack attempts are tested in one pass.  Slots are in
// attempt order, hence the lowest successful lane names the first attempt
// that the reference's sequential loop would have accepted.  An attempt
// with more than 64 tasks is processed alone in passes of 64 slots.
// The batch starts at one attempt and doubles after every fully failed
// batch, so the common case (attempt accepted at once) never draws ahead.
// Each pass first runs only the O(1) quick test of every slot; the slot's
// exact level-2 search (one_order loops) runs only when no quick accept
// decides the pass, so lanes stuck in long loops never hold up an easy win.
constexpr int kPack = 8;

// Quick part of solve_pair: 1 accept, 0 reject, 2 undecided (A2/A3 returned).
__device__ __forceinline__ int pair_quick(uint64_t B1, const PieceRow& pb, const PieceRow& pc, uint32_t dbc,
                                          uint64_t& A2, uint64_t& A3) {
  A2 = anchors_of(pb, B1);
  A3 = anchors_of(pc, B1);
  if ((A2 | A3) == 0) return 0;
  if (A2 && (uint32_t)__popcll(A3) > dbc) return 1;
  if (A3 && (uint32_t)__popcll(A2) > dbc) return 1;
  // the reference DFS's own first leaf of each order (an exact success)
  if (A2) {
    const int q = __ffsll((unsigned long long)A2) - 1;
    if (anchors_of(pc, clear_full(B1 | (pb.shape << q)))) return 1;
  }
  if (A3) {
    const int r = __ffsll((unsigned long long)A3) - 1;
    if (anchors_of(pb, clear_full(B1 | (pc.shape << r)))) return 1;
  }
  return 2;
}

__device__ __forceinline__ bool pair_slow(uint64_t B1, const PieceRow& pb, const PieceRow& pc, uint64_t A2,
                                          uint64_t A3) {
  int budget = kUnlimited;
  if (A2 && one_order(B1, pb, pc, A2, A3, budget) == 1) return true;
  if (A3 && one_order(B1, pc, pb, A3, A2, budget) == 1) return true;
  return false;
}

// ---------------------------------------------------------------------------
// Load-balanced exact level-2 search for every undecided slot of a pass.
// The per-slot loops of one_order (G = AND over z-anchors, then the line-
// completing y-anchors) become flat task lists -- (slot, z-anchor) and
// (slot, y-anchor) -- dealt round-robin to the 64 lanes; per-slot results
// are combined with LDS atomics.  Cost ~ total tasks / 64 instead of the
// longest slot's loop.
// ---------------------------------------------------------------------------
struct SlowLds {
  uint64_t B1[64];
  uint64_t Af[64];   // anchors of the piece placed first in the current order
  uint64_t As[64];   // anchors of the piece placed second
  uint64_t G[64];    // AND-accumulator
  uint64_t Mlo[64], Mhi[64];
  uint32_t pre[64];  // exclusive prefix of task counts
  uint32_t ok[64];
  uint8_t first[64], second[64];
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, int lane, uint32_t& total) {
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(x, o);
    if (lane >= o) x += u;
  }
  total = __shfl(x, 63);
  return x - v;
}

// last slot s < U with pre[s] <= t
__device__ __forceinline__ int find_slot(const volatile SlowLds* L, int U, uint32_t t) {
  int lo = 0, hi = U - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L->pre[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// need: this lane owns an undecided slot.  Returns the slot's verdict.
__device__ __forceinline__ bool pair_slow_wave(SlowLds* L, const PieceRow* tbl, bool need, uint64_t B1,
                                               uint32_t bi, uint32_t ci, uint64_t A2, uint64_t A3, int lane) {
  const uint64_t needs = __ballot(need);
  const int U = __popcll(needs);
  const int s = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(needs >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needs, 0u));
  volatile SlowLds* V = L;
  bool ok = false;
#pragma unroll 1
  for (int order = 0; order < 2; ++order) {
    const uint32_t fid = order == 0 ? bi : ci;
    const uint32_t sid = order == 0 ? ci : bi;
    const uint64_t Af = order == 0 ? A2 : A3;
    const uint64_t As = order == 0 ? A3 : A2;
    const bool active = need && !ok && Af != 0ull;
    if (!__ballot(active)) continue;
    // ---- phase G: G[s] = AND_{r in As} (r - D(first, second)) ----------
    uint32_t cnt = 0;
    if (active) {
      uint64_t mlo, mhi;
      pair_conflict_mask(tbl[fid], tbl[sid], mlo, mhi);
      V->B1[s] = B1;
      V->Af[s] = Af;
      V->As[s] = As;
      V->G[s] = ~0ull;
      V->Mlo[s] = mlo;
      V->Mhi[s] = mhi;
      V->ok[s] = 0u;
      V->first[s] = (uint8_t)fid;
      V->second[s] = (uint8_t)sid;
      cnt = (uint32_t)__popcll(As);
    }
    uint32_t T;
    const uint32_t pre = wave_excl_scan(cnt, lane, T);
    // zero-count slots share the next slot's prefix; find_slot takes the last
    // slot with pre <= t, which is always one that owns task t
    if (need) V->pre[s] = pre;
    wave_sync();
    for (uint32_t t = (uint32_t)lane; t < T; t += 64) {
      const int k = find_slot(V, U, t);
      const uint32_t idx = t - V->pre[k];
      const int r = select_bit(V->As[k], idx);
      atomicAnd((unsigned long long*)&L->G[k], (unsigned long long)hi_shl(V->Mlo[k], V->Mhi[k], r));
    }
    wave_sync();
    bool undecided = false;
    if (active) {
      if (Af & ~V->G[s]) ok = true;
      else undecided = true;
    }
    // ---- phase Q: y-anchors that complete a line (all of Af lies in G) --
    cnt = undecided ? (uint32_t)__popcll(Af) : 0u;
    const uint32_t pre2 = wave_excl_scan(cnt, lane, T);
    if (T == 0) continue;
    if (need) V->pre[s] = pre2;
    wave_sync();
    for (uint32_t t = (uint32_t)lane; t < T; t += 64) {
      const int k = find_slot(V, U, t);
      const uint32_t idx = t - V->pre[k];
      const int q = select_bit(V->Af[k], idx);
      const uint64_t B2 = V->B1[k] | (tbl[V->first[k]].shape << q);
      if (has_full_line(B2) && anchors_of(tbl[V->second[k]], clear_full(B2))) V->ok[k] = 1u;
    }
    wave_sync();
    if (undecided && V->ok[s]) ok = true;
  }
  return ok;
}

// stats (diagnostics, may be null): [0] attempts consumed, [1] passes,
// [2] passes that ran the slow path, [3] max slots of a pass.
__device__ __forceinline__ void gen_hand_wave(uint64_t B, Pcg& rng, uint32_t& ids, int attempt,
                                              const PieceRow* tbl, const uint8_t* dtab, int lane,
                                              SlowLds* slow, uint32_t* stats = nullptr) {
  const int attempt0 = attempt;
  // batch entry j lives in lane j's registers
  uint32_t e_ids = 0;
  uint64_t e_A0 = 0, e_A1 = 0, e_A2 = 0;
  int e_off = 0;
  uint64_t e_hi = 0, e_lo = 0;
  uint32_t e_buf = 0;
  int e_has = 0;
  uint32_t last_ids = ids;
  int pack = 1;
#pragma unroll 1
  while (attempt < kMaxAttempts) {
    // ---- build a batch -------------------------------------------------
    int nb = 0, total = 0;
#pragma unroll 1
    while (nb < pack && attempt + nb < kMaxAttempts) {
      const Pcg before = rng;
      const uint32_t a = draw_piece(rng);
      const uint32_t b = draw_piece(rng);
      const uint32_t c = draw_piece(rng);
      const uint64_t A0 = anchors_of(tbl[a], B);
      const uint64_t A1 = anchors_of(tbl[b], B);
      const uint64_t A2 = anchors_of(tbl[c], B);
      const int S = __popcll(A0) + __popcll(A1) + __popcll(A2);
      if (nb > 0 && total + S > 64) {
        rng = before;  // does not fit: redrawn as the first attempt of the next batch
        break;
      }
      if (lane == nb) {
        e_ids = a | (b << 6) | (c << 12);
        e_A0 = A0;
        e_A1 = A1;
        e_A2 = A2;
        e_off = total;
        e_hi = rng.hi;
        e_lo = rng.lo;
        e_buf = rng.buf;
        e_has = rng.has;
      }
      total += S;
      ++nb;
      if (total >= 64) break;
    }
    // ---- test it: passes of 64 slots ------------------------------------
#pragma unroll 1
    for (int base = 0; base < total; base += 64) {
      const int slot = base + lane;
      int j = 0;
      for (int k = 1; k < nb; ++k)
        if (__shfl(e_off, k) <= slot) j = k;
      // cross-lane reads stay outside divergent code: ds_bpermute returns
      // garbage for source lanes that are inactive
      const uint32_t jid = __shfl(e_ids, j);
      const uint64_t jA0 = __shfl(e_A0, j), jA1 = __shfl(e_A1, j), jA2 = __shfl(e_A2, j);
      const int joff = __shfl(e_off, j);
      int q = 0;
      uint64_t B1 = 0, A2 = 0, A3 = 0;
      uint32_t bi = 0, ci = 0;
      if (slot < total) {
        int rem = slot - joff;
        const int c0 = __popcll(jA0), c1 = __popcll(jA1);
        int f;
        uint64_t Af;
        if (rem < c0) {
          f = 0;
          Af = jA0;
        } else if (rem < c0 + c1) {
          f = 1;
          Af = jA1;
          rem -= c0;
        } else {
          f = 2;
          Af = jA2;
          rem -= c0 + c1;
        }
        const int p = select_bit(Af, (uint32_t)rem);
        const uint32_t fi = hand_id(jid, f);
        bi = hand_id(jid, f == 0 ? 1 : 0);
        ci = hand_id(jid, f == 2 ? 1 : 2);
        const PieceRow pf = tbl[fi];
        B1 = clear_full(B | (pf.shape << p));
        q = pair_quick(B1, tbl[bi], tbl[ci], dtab[bi * kPieces + ci], A2, A3);
      }
      // quick accepts decide the pass unless an EARLIER attempt of it is
      // still undecided (its exact search must run first)
      const uint64_t qhit = __ballot(q == 1);
      const int jq = qhit ? __shfl(j, __ffsll((unsigned long long)qhit) - 1) : kPack;
      bool ok = q == 1;
      const bool need = q == 2 && j < jq;
      const uint64_t needs = __ballot(need);
      if (stats) {
        stats[1] += 1;
        stats[2] += needs ? 1u : 0u;
        const uint32_t sl = (uint32_t)(total - base < 64 ? total - base : 64);
        stats[3] = stats[3] > sl ? stats[3] : sl;
      }
      if (needs) {
        const bool r = pair_slow_wave(slow, tbl, need, B1, bi, ci, A2, A3, lane);
        if (need) ok = r;
      }
      const uint64_t hit = __ballot(ok);
      if (hit) {
        const int winner = __ffsll((unsigned long long)hit) - 1;
        const int jw = __shfl(j, winner);
        ids = __shfl(e_ids, jw);
        rng.hi = __shfl(e_hi, jw);
        rng.lo = __shfl(e_lo, jw);
        rng.buf = __shfl(e_buf, jw);
        rng.has = __shfl(e_has, jw) != 0;
        if (stats) stats[0] = (uint32_t)(attempt + jw + 1 - attempt0);
        return;
      }
    }
    // every attempt of the batch failed: continue after its last one
    const int jl = nb - 1;
    last_ids = __shfl(e_ids, jl);
    rng.hi = __shfl(e_hi, jl);
    rng.lo = __shfl(e_lo, jl);
    rng.buf = __shfl(e_buf, jl);
    rng.has = __shfl(e_has, jl) != 0;
    attempt += nb;
    pack = pack * 2 < kPack ? pack * 2 : kPack;
  }
  ids = last_ids;  // 100 failures: the last hand is kept (engine.py:171-172)
  if (stats) stats[0] = (uint32_t)(attempt - attempt0);
}

}  // namespace bb

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
// gen_hands_multi (bottom) runs the searches of several envs with a whole
// wave; gen_hand_wave (one env per wave) serves the solver-counter diagnostic
// mode (BB_DEBUG_MODE=2), the per-lane gen_hand_lane (budgeted) the in-lane
// mode (BB_LANE_BUDGET > 0); the parity tests exercise all three.
#pragma once
#include "bb_device.h"


namespace bb {

// Work-budget ticks (roughly proportional to instruction counts).
constexpr int kTickAnchors = 4;
constexpr int kTickG = 1;
constexpr int kTickQ = 1;

__device__ __forceinline__ bool has_full_line(uint64_t B) {
  const uint32_t lo = (uint32_t)B, hi = (uint32_t)(B >> 32);
  uint32_t a = lo & hi;
  a &= a >> 16;
  a &= a >> 8;
  return ((full_row_bytes(lo) | full_row_bytes(hi)) | (a & 0xFFu)) != 0u;
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
  for (uint32_t j = 0, nz = ncells_of(z); j < nz; ++j) {
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

// pair_quick without branches: 0 reject, 1 accept, 2 undecided, A2 / A3 out.
__device__ __forceinline__ int pair_quick_bf(uint64_t B1, const PieceRow& pb, const PieceRow& pc, uint32_t dbc,
                                             uint64_t& A2, uint64_t& A3) {
  A2 = anchors_of(pb, B1);
  A3 = anchors_of(pc, B1);
  const bool dacc = (A2 && (uint32_t)__popcll(A3) > dbc) || (A3 && (uint32_t)__popcll(A2) > dbc);
  const int q = __ffsll((unsigned long long)A2) - 1;
  const int r = __ffsll((unsigned long long)A3) - 1;
  const bool leaf2 = A2 && anchors_of(pc, clear_full(B1 | (pb.shape << (q & 63)))) != 0ull;
  const bool leaf3 = A3 && anchors_of(pb, clear_full(B1 | (pc.shape << (r & 63)))) != 0ull;
  return (A2 | A3) == 0ull ? 0 : ((dacc || leaf2 || leaf3) ? 1 : 2);
}

// In-lane quick test of fixed level-1 slot k of the drawn hand (x0, x1, x2) on
// B, without branches (the rollout and fused step kernels): the first piece
// f = k mod 3 at its lowest (k < 3) or highest anchor, then pair_quick's |D|
// tests and both leaves, all computed and combined, so the whole test is one
// basic block (SIMT runs the leaves anyway whenever any lane of the wave needs
// them).  True on an accept (an exact success).
__device__ __forceinline__ bool quick_slot_bf(uint64_t B, uint32_t x0, uint32_t x1, uint32_t x2, const PieceRow* tbl,
                                              const uint8_t* dtab, int k) {
  const int f = k % 3;
  const uint32_t fi = f == 0 ? x0 : (f == 1 ? x1 : x2);
  const uint32_t bi = f == 0 ? x1 : x0;
  const uint32_t ci = f == 2 ? x1 : x2;
  const PieceRow& pf = tbl[fi];
  const PieceRow& pb = tbl[bi];
  const PieceRow& pc = tbl[ci];
  const uint32_t dbc = dtab[bi * kPieces + ci];
  const uint64_t Af = anchors_of(pf, B);
  const int p = k < 3 ? __ffsll((unsigned long long)Af) - 1 : 63 - __clzll((long long)(Af | 1ull));
  const uint64_t B1 = clear_full(B | (pf.shape << (p & 63)));
  const uint64_t A2 = anchors_of(pb, B1);
  const uint64_t A3 = anchors_of(pc, B1);
  const bool dacc = (A2 && (uint32_t)__popcll(A3) > dbc) || (A3 && (uint32_t)__popcll(A2) > dbc);
  const int q = __ffsll((unsigned long long)A2) - 1;
  const int r = __ffsll((unsigned long long)A3) - 1;
  const bool leaf2 = A2 && anchors_of(pc, clear_full(B1 | (pb.shape << (q & 63)))) != 0ull;
  const bool leaf3 = A3 && anchors_of(pb, clear_full(B1 | (pc.shape << (r & 63)))) != 0ull;
  return Af != 0ull && (dacc || leaf2 || leaf3);
}

// quick_slot_bf's test on the level-1 slot whose first piece is the hand's
// piece of anchor-count rank `rank` on B (0: the fewest anchors, 1: the
// second fewest; ties: the lower hand slot first), at its lowest anchor.  The
// tightest piece placed first leaves the freest pair behind: on the bench
// workload rank 0 alone settles 78.6% of first attempts against 74.3% for
// slot 0, ranks 0 + 1 80.5% against 79.0% for slots 0 + 1
// (tools/slot_policy.c), so fewer hands go to the search.
__device__ __forceinline__ bool quick_rank_bf(uint64_t B, uint32_t x0, uint32_t x1, uint32_t x2, const PieceRow* tbl,
                                              const uint8_t* dtab, int rank) {
  const uint64_t A0 = anchors_of(tbl[x0], B), A1 = anchors_of(tbl[x1], B), A2x = anchors_of(tbl[x2], B);
  const uint32_t c0 = A0 ? (uint32_t)__popcll(A0) : 65u;
  const uint32_t c1 = A1 ? (uint32_t)__popcll(A1) : 65u;
  const uint32_t c2 = A2x ? (uint32_t)__popcll(A2x) : 65u;
  // rank of each slot in (count, slot) order
  const int r1 = (c0 <= c1) + (c2 < c1);
  const int r2 = (c0 <= c2) + (c1 <= c2);
  const bool f1 = r1 == rank, f2 = r2 == rank;
  const uint32_t fi = f2 ? x2 : (f1 ? x1 : x0);
  const uint32_t bi = (f1 || f2) ? x0 : x1;
  const uint32_t ci = f2 ? x1 : x2;
  const uint64_t Af = f2 ? A2x : (f1 ? A1 : A0);
  const PieceRow& pb = tbl[bi];
  const PieceRow& pc = tbl[ci];
  const uint32_t dbc = dtab[bi * kPieces + ci];
  const int p = __ffsll((unsigned long long)Af) - 1;
  const uint64_t B1 = clear_full(B | (tbl[fi].shape << (p & 63)));
  const uint64_t A2 = anchors_of(pb, B1);
  const uint64_t A3 = anchors_of(pc, B1);
  const bool dacc = (A2 && (uint32_t)__popcll(A3) > dbc) || (A3 && (uint32_t)__popcll(A2) > dbc);
  const int q = __ffsll((unsigned long long)A2) - 1;
  const int r = __ffsll((unsigned long long)A3) - 1;
  const bool leaf2 = A2 && anchors_of(pc, clear_full(B1 | (pb.shape << (q & 63)))) != 0ull;
  const bool leaf3 = A3 && anchors_of(pb, clear_full(B1 | (pc.shape << (r & 63)))) != 0ull;
  return Af != 0ull && (dacc || leaf2 || leaf3);
}

// In-lane quick test of the first attempt (step_kernel): draw its three
// pieces and test up to `slots` fixed level-1 slots -- first piece f = k mod 3
// at its lowest (k < 3) or highest anchor -- with pair_quick.  Straight-line
// work, no budget loop.  Settles only on an accept (an exact success); else
// rolls the stream back so the wave search redraws the attempt.
__device__ __forceinline__ bool quick_hand(uint64_t B, Pcg& rng, uint32_t& ids, const PieceRow* tbl,
                                           const uint8_t* dtab, int slots) {
  const Pcg save = rng;
  uint32_t x0, x1, x2;
  draw3(rng, x0, x1, x2);
  ids = x0 | (x1 << 6) | (x2 << 12);
  uint64_t A[3];
  A[0] = anchors_of(tbl[x0], B);
  A[1] = anchors_of(tbl[x1], B);
  A[2] = anchors_of(tbl[x2], B);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    if (k >= slots) break;
    const int f = k % 3;
    const uint64_t Af = A[f];
    if (!Af) continue;
    const uint32_t fi = f == 0 ? x0 : (f == 1 ? x1 : x2);
    const uint32_t bi = f == 0 ? x1 : x0;
    const uint32_t ci = f == 2 ? x1 : x2;
    const int p = k < 3 ? __ffsll((unsigned long long)Af) - 1 : 63 - __clzll((long long)Af);
    const uint64_t B1 = clear_full(B | (tbl[fi].shape << p));
    uint64_t A2, A3;
    if (pair_quick(B1, tbl[bi], tbl[ci], dtab[bi * kPieces + ci], A2, A3) == 1) return true;
  }
  rng = save;
  return false;
}

// Some row or column has at most 5 empty cells (>= 3 filled): a prerequisite
// for any single placement to complete a line.
__device__ __forceinline__ bool line_within_reach(uint64_t B) {
  uint64_t x = B - ((B >> 1) & 0x5555555555555555ull);
  x = (x & 0x3333333333333333ull) + ((x >> 2) & 0x3333333333333333ull);
  x = (x + (x >> 4)) & 0x0F0F0F0F0F0F0F0Full;  // per-row popcounts, one byte each
  if ((x + 0x7D7D7D7D7D7D7D7Dull) & 0x8080808080808080ull) return true;
#pragma unroll
  for (int c = 0; c < 8; ++c)
    if (__popcll(B & (kCol0 << c)) >= 3) return true;
  return false;
}

// ---------------------------------------------------------------------------
// Wave64 cross-lane helpers on DPP (gfx9 row_shr / row_bcast): VALU-only, no
// LDS round trip per step, unlike __shfl_up (ds_bpermute).
// ---------------------------------------------------------------------------
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_zero(uint32_t x) {  // lanes out of range / in masked rows read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, true);
}
// Inclusive prefix sum over the 64 lanes.
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
  x += dpp_zero<0x111, 0xF>(x);  // row_shr:1
  x += dpp_zero<0x112, 0xF>(x);  // row_shr:2
  x += dpp_zero<0x114, 0xF>(x);  // row_shr:4
  x += dpp_zero<0x118, 0xF>(x);  // row_shr:8
  x += dpp_zero<0x142, 0xA>(x);  // row_bcast:15 into rows 1, 3
  x += dpp_zero<0x143, 0xC>(x);  // row_bcast:31 into rows 2, 3
  return x;
}
// Inclusive prefix max over the 64 lanes (values >= 0).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  x = max(x, dpp_zero<0x111, 0xF>(x));
  x = max(x, dpp_zero<0x112, 0xF>(x));
  x = max(x, dpp_zero<0x114, 0xF>(x));
  x = max(x, dpp_zero<0x118, 0xF>(x));
  x = max(x, dpp_zero<0x142, 0xA>(x));
  x = max(x, dpp_zero<0x143, 0xC>(x));
  return x;
}
// Order this wave's LDS accesses across lanes (one wave's DS instructions
// execute in order; this only stops the compiler from moving them).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Hand-off flags between the waves of one workgroup (rollout_async_kernel's records): the payload travels
// through LDS only, so the release / acquire fences order LDS accesses alone (workgroup scope, local
// address space: one s_waitcnt lgkmcnt(0), no wait on the wave's outstanding global stores).
__device__ __forceinline__ void lds_flag_store_release(uint32_t* f, uint32_t v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_flag_load_acquire(uint32_t* f) {
  const uint32_t v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  return v;
}

// Exact level 2 of the undecided slots, flattened over the wave: the
// reference DFS's own leaf tests (engine.py:196-224 _can_place_remaining),
// one per lane -- for every undecided slot, every anchor q of b (then c must
// fit on clear(B1 | b@q)) and every anchor r of c (then b must fit on
// clear(B1 | c@r)).  The tasks of all slots are dealt out 64 at a time; a
// task's owner slot is found by scattering each slot's first task index to
// LDS and taking a prefix max (DPP).  Returns this lane's slot verdict.
// lds: 64 words of wave-private LDS scratch.  All lanes call it.
//
// key (1): env << 8 | attempt order of this lane's slot.  A success
// decides its env's attempt, so it settles every slot of the same env at the
// same or a later attempt (those verdicts can no longer change the earliest
// success); the scan stops once every needed slot is settled or has had all
// of its tasks.  An attempt that is solvable usually succeeds on its first
// tasks, so this ends the flattened scan long before its last task.
//
// 1: one order's leaves suffice where the first placement
// clears nothing.  If c at r completes no line and b then fits, b's anchor is
// disjoint from c@r on B1, so placing b there first (a clear only frees cells)
// leaves c@r legal: that b-first leaf succeeds too.  So every leaf of the order
// whose first piece has fewer anchors is tested, and of the other order only
// the first placements that complete a line.
// The filter is a per-lane loop over anchors: it pays only for long task lists
// (more than BB_SLOW_LINE_MIN tasks over the wave) and only where one long list
// sets the launch time -- bb_step's single step (kLineOnly); in the rollout
// kernel the same code measured -2% (its exact phases are short and the tail
// averages out over the steps).
#ifndef BB_SLOW_LINE_MIN
#define BB_SLOW_LINE_MIN 512
#endif
template <bool kLineOnly = false>
__device__ __forceinline__ bool slow_phase_wave(bool need, uint64_t B1, uint32_t bi, uint32_t ci, uint64_t A2,
                                                uint64_t A3, const PieceRow* tbl, int lane, uint32_t* lds,
                                                uint32_t key) {
  if constexpr (kLineOnly && 1) {
  const uint32_t all = need ? (uint32_t)(__popcll(A2) + __popcll(A3)) : 0u;
  const uint32_t all_tot = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_add(all), 63);  // every lane
  if (all_tot > (uint32_t)BB_SLOW_LINE_MIN && need) {
    if (__popcll(A3) < __popcll(A2)) {  // c first in full, b first only where b completes a line
      const uint32_t ti = bi;
      bi = ci;
      ci = ti;
      const uint64_t tA = A2;
      A2 = A3;
      A3 = tA;
    }
    uint64_t line = 0ull;  // anchors of ci (second order's first piece) that complete a line on B1
    if (A3 && line_within_reach(B1)) {
      const uint64_t cs = tbl[ci].shape;
      uint64_t x = A3;
#pragma unroll 1
      while (x) {
        const uint64_t bit = x & (0ull - x);
        x ^= bit;
        if (has_full_line(B1 | (cs << (__ffsll((unsigned long long)bit) - 1)))) line |= bit;
      }
    }
    A3 = line;
  }
  }
  const uint32_t n2 = need ? (uint32_t)__popcll(A2) : 0u;
  const uint32_t cnt = n2 + (need ? (uint32_t)__popcll(A3) : 0u);
  const uint32_t incl = wave_incl_add(cnt);
  const uint32_t off = incl - cnt;
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  uint64_t won_mask = 0ull;  // bit o: slot o has a successful leaf
  uint64_t pending = __ballot(need);  // needed slots not settled yet
#pragma unroll 1
  for (uint32_t base = 0; base < total; base += 64u) {
    // owner of task base+lane: the last slot whose first task is <= it
    wave_lds_fence();
    lds[lane] = 0u;
    wave_lds_fence();
    if (cnt && off < base + 64u && incl > base) atomicMax(&lds[off > base ? off - base : 0u], (uint32_t)lane);
    wave_lds_fence();
    const int o = (int)wave_incl_max(lds[lane]);
    const uint32_t t = base + (uint32_t)lane;
    const uint64_t oB = __shfl(B1, o);
    const uint64_t oA2 = __shfl(A2, o), oA3 = __shfl(A3, o);
    const uint32_t oid = __shfl(bi | (ci << 8), o);
    const uint32_t k = t - __shfl(off, o);
    const uint32_t on2 = __shfl(n2, o);
    bool hit = false;
    if (t < total) {
      const bool bfirst = k < on2;
      const PieceRow& first = tbl[bfirst ? (oid & 0xFFu) : (oid >> 8)];
      const PieceRow& second = tbl[bfirst ? (oid >> 8) : (oid & 0xFFu)];
      const int pos = select_bit(bfirst ? oA2 : oA3, bfirst ? k : k - on2);
      hit = anchors_of(second, clear_full(oB | (first.shape << pos))) != 0ull;
    }
    // owners with a hit: a wave-uniform mask (hits are rare; one readlane each)
    uint64_t hits = __ballot(hit);
    while (hits) {
      const int l = __ffsll((unsigned long long)hits) - 1;
      hits &= hits - 1;
      const int ol = __builtin_amdgcn_readlane(o, l);
      won_mask |= 1ull << ol;
      const uint32_t ko = (uint32_t)__builtin_amdgcn_readlane((int)key, ol);
      pending &= ~__ballot((key >> 8) == (ko >> 8) && (key & 0xFFu) >= (ko & 0xFFu));
    }
    pending &= ~__ballot(need && incl <= base + 64u);  // every task of the slot done
    if (!pending) break;
  }
  return (won_mask >> lane) & 1ull;
}

// ---------------------------------------------------------------------------
// Wave-cooperative _generate_new_pieces (engine.py:155-172) for one env: all
// 64 lanes call it with identical arguments; on return ids/rng are the final
// hand and stream state, identical in every lane.
//
//  * anchors of all 37 pieces on B are computed once, lane x = piece x;
//  * a batch of attempts is drawn in parallel, lane k = attempt k, by PCG64
//    jump-ahead (state after c steps = A^c s + inc * S_c, host-built table):
//    the stream position of every draw is known because each attempt eats
//    exactly three 32-bit values unless a Lemire rejection occurs (p ~ 5e-9
//    per draw) -- any rejection in the batch falls back to sequential draws;
//  * level-1 tasks of an attempt are its (f, p) pairs, f-major; consecutive
//    attempts are packed while their tasks fit 64 lanes.  Slots are in attempt
//    order, so the lowest successful lane names the first attempt the
//    reference's sequential loop would have accepted.  An attempt with more
//    than 64 tasks is processed alone in passes of 64 slots;
//  * each pass first runs the O(1) quick test of every slot (quick accept +
//    the reference DFS's first leaf); the exact level-2 search runs only
//    for slots of attempts that the quick tests leave undecided;
//  * the batch starts at one attempt and doubles after each failed batch.
// ---------------------------------------------------------------------------
constexpr int kPack = 32;
#ifndef BB_MULTI_PASSES
#define BB_MULTI_PASSES 3  // gen_hands_multi: a round packs attempts for up to this many 64-slot passes
#endif
constexpr int kMultiPasses = BB_MULTI_PASSES;
static_assert(3 * kPack / 2 + 2 <= kJumpMax, "jump table too short for the batch size");

__device__ __forceinline__ void mul128(uint64_t alo, uint64_t ahi, uint64_t blo, uint64_t bhi, uint64_t& lo,
                                       uint64_t& hi) {
  lo = alo * blo;
  hi = __umul64hi(alo, blo) + alo * bhi + ahi * blo;
}

__device__ __forceinline__ uint64_t xsl_rr(uint64_t hi, uint64_t lo) {
  const uint64_t x = hi ^ lo;
  const unsigned rot = (unsigned)(hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

// Draw attempt k of a batch starting at stream state s0 without touching s0.
// Returns true when a Lemire rejection would have shifted the stream.
__device__ __forceinline__ bool draw_attempt_jump(const Pcg& s0, const JumpRow* J, int k, uint32_t& ids,
                                                  Pcg& after) {
  constexpr uint64_t ML = 0x4385DF649FCCF645ull, MH = 0x2360ED051FC65DA4ull;
  const int h = s0.has ? 1 : 0;
  const int v0 = 3 * k;
  const int cfirst = v0 >= h ? (v0 - h) / 2 + 1 : 1;
  const JumpRow j = J[cfirst];
  uint64_t l1, h1, l2, h2;
  mul128(j.a_lo, j.a_hi, s0.lo, s0.hi, l1, h1);
  mul128(j.s_lo, j.s_hi, s0.inc_lo, s0.inc_hi, l2, h2);
  const uint64_t c_lo = l1 + l2;
  const uint64_t c_hi = h1 + h2 + (c_lo < l1 ? 1ull : 0ull);
  uint64_t n_lo, n_hi;  // one more LCG step
  mul128(c_lo, c_hi, ML, MH, n_lo, n_hi);
  n_lo += s0.inc_lo;
  n_hi += s0.inc_hi + (n_lo < s0.inc_lo ? 1ull : 0ull);
  const uint64_t o1 = xsl_rr(c_hi, c_lo);
  const uint64_t o2 = xsl_rr(n_hi, n_lo);
  bool rej = false;
  ids = 0;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int v = v0 + d;
    uint32_t val;
    if (v < h) {
      val = s0.buf;
    } else {
      const int c = (v - h) / 2 + 1;
      const uint64_t o = c == cfirst ? o1 : o2;
      val = ((v - h) & 1) ? (uint32_t)(o >> 32) : (uint32_t)o;
    }
    const uint64_t m = (uint64_t)val * 37ull;
    rej |= (uint32_t)m < 7u;
    ids |= (uint32_t)(m >> 32) << (6 * d);
  }
  const int used = v0 + 3 - h;           // values taken from LCG outputs
  const int calls = (used + 1) / 2;      // == cfirst or cfirst + 1
  after = s0;
  const bool second = calls != cfirst;
  after.lo = second ? n_lo : c_lo;
  after.hi = second ? n_hi : c_hi;
  after.has = (used & 1) != 0;
  after.buf = after.has ? (uint32_t)((second ? o2 : o1) >> 32) : 0u;
  return rej;
}

__device__ __forceinline__ void gen_hand_wave(uint64_t B, Pcg& rng, uint32_t& ids, int attempt,
                                              const PieceRow* tbl, const uint8_t* dtab, const JumpRow* J,
                                              int lane, int pack_first, int pack_next, uint32_t* lds,
                                              uint32_t* stats = nullptr) {  // diagnostics: [12] counters
  const int attempt0 = attempt;
  // anchors of every piece on B: lane x holds piece x
  const uint64_t acache = lane < kPieces ? anchors_of(tbl[lane], B) : 0ull;
  uint32_t last_ids = ids;
  int pack = pack_first < kPack ? pack_first : kPack;
#pragma unroll 1
  while (attempt < kMaxAttempts) {
    // ---- draw a batch: lane k = attempt k --------------------------------
    const int kb = pack < kMaxAttempts - attempt ? pack : kMaxAttempts - attempt;
    uint32_t e_ids = 0;
    Pcg e_after = rng;
    bool rej = false;
    if (lane < kb) rej = draw_attempt_jump(rng, J, lane, e_ids, e_after);
    int nb_draw = kb;
    if (__ballot(rej)) {  // rare: redo one attempt with sequential draws
      Pcg s = rng;
      const uint32_t a = draw_piece(s), b = draw_piece(s), c = draw_piece(s);
      if (lane == 0) {
        e_ids = a | (b << 6) | (c << 12);
        e_after = s;
      }
      nb_draw = 1;
    }
    const uint64_t eA0 = __shfl(acache, (int)hand_id(e_ids, 0));
    const uint64_t eA1 = __shfl(acache, (int)hand_id(e_ids, 1));
    const uint64_t eA2 = __shfl(acache, (int)hand_id(e_ids, 2));
    const uint32_t S = lane < nb_draw ? (uint32_t)(__popcll(eA0) + __popcll(eA1) + __popcll(eA2)) : 0u;
    const uint32_t incl = wave_incl_add(S);
    const int e_off = (int)(incl - S);
    // attempts packed into this pass: the leading ones whose tasks fit 64
    int nb = __popcll(__ballot(lane < nb_draw && incl <= 64u));
    if (nb == 0) nb = 1;
    const int total = (int)__shfl(incl, nb - 1);
    // ---- test the batch: passes of 64 slots ------------------------------
#pragma unroll 1
    for (int base = 0; base < total; base += 64) {
      const uint64_t tq0 = stats ? __builtin_amdgcn_s_memtime() : 0;
      const int slot = base + lane;
      // j = the packed attempt that owns this slot: each attempt marks its
      // first slot of the pass in LDS, then a prefix max over the lanes
      int j = 0;
      if (nb > 1) {
        wave_lds_fence();
        lds[lane] = 0u;
        wave_lds_fence();
        if (lane < nb && S && e_off < base + 64 && e_off + (int)S > base)
          atomicMax(&lds[e_off > base ? e_off - base : 0], (uint32_t)lane);
        wave_lds_fence();
        j = (int)wave_incl_max(lds[lane]);
      }
      const uint32_t jid = __shfl(e_ids, j);
      const uint64_t jA0 = __shfl(eA0, j), jA1 = __shfl(eA1, j), jA2 = __shfl(eA2, j);
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
        bi = hand_id(jid, f == 0 ? 1 : 0);
        ci = hand_id(jid, f == 2 ? 1 : 2);
        B1 = clear_full(B | (tbl[hand_id(jid, f)].shape << p));
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
        stats[8] += sl;
        stats[9] += (uint32_t)__popcll(needs);
      }
      const uint64_t tq1 = stats ? __builtin_amdgcn_s_memtime() : 0;
      if (stats) stats[4] += (uint32_t)(tq1 - tq0);
      if (needs) {
        const uint64_t tq2 = stats ? __builtin_amdgcn_s_memtime() : 0;
        ok |= slow_phase_wave(need, B1, bi, ci, A2, A3, tbl, lane, lds, (uint32_t)j);  // one env: attempt j
        if (stats) {
          const uint64_t tq3 = __builtin_amdgcn_s_memtime();
          stats[5] += (uint32_t)(tq2 - tq1);
          stats[6] += (uint32_t)(tq3 - tq2);
        }
      }
      const uint64_t hit = __ballot(ok);
      if (hit) {
        const int jw = __shfl(j, __ffsll((unsigned long long)hit) - 1);
        ids = __shfl(e_ids, jw);
        rng.hi = __shfl(e_after.hi, jw);
        rng.lo = __shfl(e_after.lo, jw);
        rng.buf = __shfl(e_after.buf, jw);
        rng.has = __shfl((int)e_after.has, jw) != 0;
        if (stats) {
          stats[0] = (uint32_t)(attempt + jw + 1 - attempt0);
          stats[10] = needs ? 1u : 0u;  // decided by a pass that needed the exact search
        }
        return;
      }
    }
    // every packed attempt failed: continue after the last one
    const int jl = nb - 1;
    last_ids = __shfl(e_ids, jl);
    rng.hi = __shfl(e_after.hi, jl);
    rng.lo = __shfl(e_after.lo, jl);
    rng.buf = __shfl(e_after.buf, jl);
    rng.has = __shfl((int)e_after.has, jl) != 0;
    attempt += nb;
    pack = pack_next > 0 ? pack_next : pack * 2;
    pack = pack < kPack ? pack : kPack;
  }
  ids = last_ids;  // 100 failures: the last hand is kept (engine.py:171-172)
  if (stats) stats[0] = (uint32_t)(attempt - attempt0);
}

// ---------------------------------------------------------------------------
// Wave-cooperative _generate_new_pieces for SEVERAL envs at once: the envs
// parked in one rollout step.  Env e is held by lane e (and its copies in
// lanes e + kEnvs, ...): board eB, stream rng; parked has bit e set for every
// env to solve (e < kEnvs).  On return those lanes hold the final hand ids and stream state,
// exactly the result of each env's own sequential loop.
//
// Each round draws a batch of attempts for every unsolved env by jump-ahead,
// ATTEMPT-major (lane L = env slot L mod E, attempt L / E), so the leading
// attempts -- the ones that usually decide -- of all envs share the first
// pass.  Slots of the leading attempts that fit 64 lanes are tested as in
// gen_hand_wave; an env accepts its earliest attempt with a successful slot
// once every earlier attempt of its own is decided, else it advances past its
// packed (all failed) attempts.  The first attempt lane is always packed, so
// every round makes progress.
// ---------------------------------------------------------------------------
struct NoRelease {
  __device__ void operator()(bool) const {}
};

// release(done): called after every round with done set in the lanes of the envs that round decided (their
// rng / ids are final), so a caller can hand them on before the other envs' later rounds
template <int kEnvs, bool kLineOnly = false, typename Release = NoRelease>
__device__ __forceinline__ void gen_hands_multi(uint64_t parked, uint64_t eB, Pcg& rng, uint32_t& ids,
                                                const PieceRow* tbl, const uint8_t* dtab, const JumpRow* J,
                                                int lane, int pack_first, int pack_next, uint32_t* lds,
                                                uint64_t* prof = nullptr,  // diagnostics: [6] cycle sums
                                                int att0 = 0,  // attempts an earlier pass consumed (env lanes)
                                                const Release& release = Release()) {
#define BB_MT(x) const uint64_t x = prof ? __builtin_amdgcn_s_memtime() : 0
  const int me = lane % kEnvs;  // env index held by this lane
  int att = att0;             // attempts consumed so far (env lanes)
  uint32_t last_ids = 0;      // last drawn hand, kept after 100 failures (engine.py:171-172)
  uint64_t todo = parked;
  // attempts per env in this round: pack_first, then pack_next (0: double the
  // previous round's, as gen_hand_wave does), capped at kPack
  int pk = pack_first < kPack ? pack_first : kPack;
#pragma unroll 1
  while (todo) {
    BB_MT(p0);
    const int E = __popcll(todo);
    int K = 64 / E;
    K = K < pk ? K : pk;
    K = K < kPack ? K : kPack;
    K = K > 1 ? K : 1;
    const int nl = E * K;
    // env slot, attempt offset of this lane: lane / E through the f32 reciprocal
    // ((lane + 0.5) / E is >= 1/64 away from an integer, far above its error)
    const int k = (int)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)E));
    const int es = lane - k * E;
    const int e = select_bit(todo, (uint32_t)es);
    Pcg s0;
    s0.hi = __shfl(rng.hi, e);
    s0.lo = __shfl(rng.lo, e);
    s0.inc_hi = __shfl(rng.inc_hi, e);
    s0.inc_lo = __shfl(rng.inc_lo, e);
    s0.buf = __shfl(rng.buf, e);
    s0.has = __shfl((int)rng.has, e) != 0;
    const uint64_t B = __shfl(eB, e);
    const int a0 = __shfl(att, e);
    const bool valid = lane < nl && a0 + k < kMaxAttempts;
    uint32_t e_ids = 0;
    Pcg e_after = s0;
    bool rej = false;
    if (valid) rej = draw_attempt_jump(s0, J, k, e_ids, e_after);
    if (__ballot(rej)) {
      // rare Lemire rejection: the lowest env on the exact sequential path
      const int e0 = __ffsll((unsigned long long)todo) - 1;
      Pcg w;
      w.hi = __shfl(rng.hi, e0);
      w.lo = __shfl(rng.lo, e0);
      w.inc_hi = __shfl(rng.inc_hi, e0);
      w.inc_lo = __shfl(rng.inc_lo, e0);
      w.buf = __shfl(rng.buf, e0);
      w.has = __shfl((int)rng.has, e0) != 0;
      uint32_t wids = (uint32_t)__shfl((int)last_ids, e0);
      gen_hand_wave(__shfl(eB, e0), w, wids, __shfl(att, e0), tbl, dtab, J, lane, pk, pack_next, lds);
      if (me == e0) {
        rng = w;
        ids = wids;
      }
      release(me == e0);
      todo &= todo - 1;
      continue;
    }
    BB_MT(p1);
    uint64_t eA0 = 0ull, eA1 = 0ull, eA2 = 0ull;
    if (valid) {
      eA0 = anchors_of(tbl[hand_id(e_ids, 0)], B);
      eA1 = anchors_of(tbl[hand_id(e_ids, 1)], B);
      eA2 = anchors_of(tbl[hand_id(e_ids, 2)], B);
    }
    const uint32_t S = valid ? (uint32_t)(__popcll(eA0) + __popcll(eA1) + __popcll(eA2)) : 0u;
    const uint32_t incl = wave_incl_add(S);
    const int e_off = (int)(incl - S);
    // leading attempt lanes whose slots fit kMultiPasses passes of 64
    int nb = __popcll(__ballot(lane < nl && incl <= 64u * kMultiPasses));
    if (nb == 0) nb = 1;
    const uint64_t packed = (nb >= 64 ? ~0ull : ((1ull << nb) - 1ull)) & __ballot(valid);
    const int total = __builtin_amdgcn_readlane((int)incl, nb - 1);
    uint64_t every = 1ull;  // bits 0, E, 2E, ...: the lanes of env slot 0
    for (int w = E; w < 64; w <<= 1) every |= every << w;
    uint64_t okm = 0ull;  // attempt lanes with a successful slot
    BB_MT(p2);
    uint64_t pq = 0, ps = 0;
#pragma unroll 1
    for (int base = 0; base < total; base += 64) {
      BB_MT(q0);
      const int slot = base + lane;
      int j = 0;
      if (nb > 1) {
        wave_lds_fence();
        lds[lane] = 0u;
        wave_lds_fence();
        if (lane < nb && S && e_off < base + 64 && e_off + (int)S > base)
          atomicMax(&lds[e_off > base ? e_off - base : 0], (uint32_t)lane);
        wave_lds_fence();
        j = (int)wave_incl_max(lds[lane]);
      }
      const uint32_t jid = __shfl(e_ids, j);
      const uint64_t jA0 = __shfl(eA0, j), jA1 = __shfl(eA1, j), jA2 = __shfl(eA2, j);
      const uint64_t jB = __shfl(B, j);
      const int joff = __shfl(e_off, j);
      int q = 0;
      uint64_t B1 = 0, A2 = 0, A3 = 0;
      uint32_t bi = 0, ci = 0;
      {  // every lane computes its slot (lanes past `total` a dummy one) and drops it by select
        const int rem0 = slot - joff;
        const int c0 = __popcll(jA0), c1 = __popcll(jA1);
        const int f = rem0 < c0 ? 0 : (rem0 < c0 + c1 ? 1 : 2);
        const uint64_t Af = f == 0 ? jA0 : (f == 1 ? jA1 : jA2);
        const int rem = rem0 - (f == 0 ? 0 : (f == 1 ? c0 : c0 + c1));
        const int p = select_bit(Af, (uint32_t)rem) & 63;
        bi = hand_id(jid, f == 0 ? 1 : 0);
        ci = hand_id(jid, f == 2 ? 1 : 2);
        B1 = clear_full(jB | (tbl[hand_id(jid, f)].shape << p));
        q = pair_quick_bf(B1, tbl[bi], tbl[ci], dtab[bi * kPieces + ci], A2, A3);
        if (slot >= total) q = 0;
      }
      // attempt lanes with a quick accept: attempt lane L owns the pass's slot
      // bits [lo, hi) of any slot ballot
      const int lo = e_off > base ? e_off - base : 0;
      const int hi = e_off + (int)S - base < 64 ? e_off + (int)S - base : 64;
      const uint64_t own = (lane < nb && hi > lo) ? ((hi - lo == 64 ? ~0ull : ((1ull << (hi - lo)) - 1ull)) << lo)
                                                  : 0ull;
      const uint64_t qam = __ballot((__ballot(q == 1) & own) != 0ull);
      // exact search only where no attempt of the same env up to this one accepted already
      const uint64_t jenv = every << (j % E);
      bool ok = q == 1;
      const bool need = q == 2 && !((qam | okm) & jenv & ((2ull << j) - 1ull));
      BB_MT(q1);
      if (__ballot(need))  // attempt lane j = env slot j % E, its attempt j / E
        ok |= slow_phase_wave<kLineOnly>(need, B1, bi, ci, A2, A3, tbl, lane, lds,
                                         (uint32_t)((j % E) << 8 | (j / E)));
      BB_MT(q2);
      pq += q1 - q0;
      ps += q2 - q1;
      okm |= __ballot((__ballot(ok) & own) != 0ull);
      // stop once every env is decided: it has a successful attempt lane (its
      // earlier lanes' slots came first, so they are complete and failed), or
      // all of its packed lanes are complete
      if (base + 64 >= total) break;
      const uint64_t complete = __ballot(lane < nb && incl <= (uint32_t)(base + 64));
      bool undecided = false;
      if (lane < E) {
        const uint64_t envl = (every << lane) & packed;
        undecided = !(okm & envl) && (envl & ~complete) != 0ull;
      }
      if (!__ballot(undecided)) break;
    }
    BB_MT(p3);
    // resolve every env of the round in its own lanes
    const bool mine = (todo >> me) & 1ull;
    const int my_es = __popcll(todo & ((1ull << me) - 1ull));
    const uint64_t em = mine ? (every << my_es) & packed : 0ull;  // my env's packed attempt lanes
    const uint64_t hit = em & okm;
    int src = -1;
    if (hit) src = __ffsll((unsigned long long)hit) - 1;  // earliest successful attempt
    else if (em) src = 63 - __clzll((long long)em);        // last packed (all failed)
    const int from = src < 0 ? lane : src;
    const uint32_t f_ids = __shfl(e_ids, from);
    Pcg fa;
    fa.hi = __shfl(e_after.hi, from);
    fa.lo = __shfl(e_after.lo, from);
    fa.buf = __shfl(e_after.buf, from);
    fa.has = __shfl((int)e_after.has, from) != 0;
    bool done = false;
    if (src >= 0) {
      rng.hi = fa.hi;
      rng.lo = fa.lo;
      rng.buf = fa.buf;
      rng.has = fa.has;
      if (hit) {
        ids = f_ids;
        done = true;
      } else {
        att += __popcll(em);
        last_ids = f_ids;
        if (att >= kMaxAttempts) {
          ids = last_ids;
          done = true;
        }
      }
    }
    todo &= ~(__ballot(done && lane < kEnvs) & (kEnvs >= 64 ? ~0ull : ((1ull << (kEnvs & 63)) - 1ull)));
    release(done && lane < kEnvs);
    pk = pack_next > 0 ? pack_next : 2 * pk;
    pk = pk < kPack ? pk : kPack;
    if (prof) {
      BB_MT(p4);
      prof[0] += p1 - p0;  // batch setup + jump draws
      prof[1] += p2 - p1;  // anchors, prefix scan, packing
      prof[2] += pq;       // pass: quick tests + flags
      prof[3] += ps;       // pass: exact phase
      prof[4] += (p3 - p2) - pq - ps;  // pass overhead (owner flags of ok)
      prof[5] += p4 - p3;  // resolve
    }
  }
#undef BB_MT
}

// ---------------------------------------------------------------------------
// gen_hands_multi with a quota pass schedule (round 5).  Same contract and same result (the earliest
// successful attempt of every env, every earlier attempt of it proven unsolvable; 100 attempts -> the
// last draw), different order of work.  gen_hands_multi packs the leading attempt lanes whose level-1
// slots fit kMultiPasses passes and tests all of their slots: a solvable attempt has ~50-75 slots but
// succeeds on its first ~1.3 (tools/search_stats.c), so a pass was spent on one attempt's slots while
// other envs' first attempts waited for the next round's draws.  Here every pass deals each ACTIVE
// attempt lane (valid, not yet successful, slots left, its env undecided and no earlier attempt of its
// env successful) at most `quota` of its next untested slots (kQuota in the round's first pass, then up
// to 64), attempt-major, until the 64 slot lanes are full; an env is decided once it has a successful
// attempt whose earlier attempts are all complete, or all of its attempts are complete.  Every round
// ends with every env decided, so it advances either to its accepted attempt or past all its drawn
// ones.  tools/search_quota_model.c (bench workload, 7 envs per call): 1.04 rounds and 2.2 passes per
// call against 1.68 and 3.0 for the packed schedule, -23% modelled search cycles.
// ---------------------------------------------------------------------------
#ifndef BB_QUOTA_FIRST
#define BB_QUOTA_FIRST 4
#endif
#ifndef BB_QUOTA_NEXT
#define BB_QUOTA_NEXT 64
#endif

template <int kEnvs, bool kLineOnly = false, typename Release = NoRelease>
__device__ __forceinline__ void gen_hands_quota(uint64_t parked, uint64_t eB, Pcg& rng, uint32_t& ids,
                                                const PieceRow* tbl, const uint8_t* dtab, const JumpRow* J,
                                                int lane, int pack_first, int pack_next, uint32_t* lds,
                                                uint64_t* prof = nullptr, int att0 = 0,
                                                const Release& release = Release()) {
#define BB_MT(x) const uint64_t x = prof ? __builtin_amdgcn_s_memtime() : 0
  const int me = lane % kEnvs;
  int att = att0;
  uint32_t last_ids = 0;
  uint64_t todo = parked;
  int pk = pack_first < kPack ? pack_first : kPack;
#pragma unroll 1
  while (todo) {
    BB_MT(p0);
    const int E = __popcll(todo);
    int K = 64 / E;
    K = K < pk ? K : pk;
    K = K < kPack ? K : kPack;
    K = K > 1 ? K : 1;
    const int nl = E * K;
    const int k = (int)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)E));
    const int es = lane - k * E;
    const int e = select_bit(todo, (uint32_t)es);
    Pcg s0;
    s0.hi = __shfl(rng.hi, e);
    s0.lo = __shfl(rng.lo, e);
    s0.inc_hi = __shfl(rng.inc_hi, e);
    s0.inc_lo = __shfl(rng.inc_lo, e);
    s0.buf = __shfl(rng.buf, e);
    s0.has = __shfl((int)rng.has, e) != 0;
    const uint64_t B = __shfl(eB, e);
    const int a0 = __shfl(att, e);
    const bool valid = lane < nl && a0 + k < kMaxAttempts;
    uint32_t e_ids = 0;
    Pcg e_after = s0;
    bool rej = false;
    if (valid) rej = draw_attempt_jump(s0, J, k, e_ids, e_after);
    if (__ballot(rej)) {  // rare Lemire rejection: the lowest env on the exact sequential path
      const int e0 = __ffsll((unsigned long long)todo) - 1;
      Pcg w;
      w.hi = __shfl(rng.hi, e0);
      w.lo = __shfl(rng.lo, e0);
      w.inc_hi = __shfl(rng.inc_hi, e0);
      w.inc_lo = __shfl(rng.inc_lo, e0);
      w.buf = __shfl(rng.buf, e0);
      w.has = __shfl((int)rng.has, e0) != 0;
      uint32_t wids = (uint32_t)__shfl((int)last_ids, e0);
      gen_hand_wave(__shfl(eB, e0), w, wids, __shfl(att, e0), tbl, dtab, J, lane, pk, pack_next, lds);
      if (me == e0) {
        rng = w;
        ids = wids;
      }
      release(me == e0);
      todo &= todo - 1;
      continue;
    }
    BB_MT(p1);
    uint64_t eA0 = 0ull, eA1 = 0ull, eA2 = 0ull;
    if (valid) {
      eA0 = anchors_of(tbl[hand_id(e_ids, 0)], B);
      eA1 = anchors_of(tbl[hand_id(e_ids, 1)], B);
      eA2 = anchors_of(tbl[hand_id(e_ids, 2)], B);
    }
    const int S = valid ? __popcll(eA0) + __popcll(eA1) + __popcll(eA2) : 0;
    const uint64_t vmask = __ballot(valid);
    uint64_t every = 1ull;  // bits 0, E, 2E, ...: the attempt lanes of env slot 0
    for (int w = E; w < 64; w <<= 1) every |= every << w;
    const uint64_t envl = lane < E ? (every << lane) & vmask : 0ull;  // lanes of env slot `lane` (lane < E)
    int done = 0;           // this attempt lane's slots tested so far
    uint64_t okm = 0ull;    // attempt lanes with a successful slot
    BB_MT(p2);
    uint64_t pq = 0, ps = 0;
#pragma unroll 1
    for (int pass = 0;; ++pass) {
      // env decisions (lanes < E, env slot = lane): decided by its earliest success with every earlier
      // attempt complete, or by all of its attempts complete
      const uint64_t complete = __ballot(valid && done >= S) | ~vmask;
      bool undecided = false;
      if (lane < E) {
        const uint64_t okl = okm & envl;
        const uint64_t prior = okl ? envl & ((okl & (0ull - okl)) - 1ull) : envl;
        undecided = (prior & ~complete) != 0ull;
      }
      const uint64_t und = __ballot(undecided);  // bit es: env slot es undecided
      if (!und) break;
      BB_MT(q0);
      // this attempt lane's share of the pass: its env undecided, no success of its env at or before it
      const uint64_t jenv_all = every << es;  // lanes of my env slot
      const bool blocked = (okm & jenv_all & ((2ull << lane) - 1ull)) != 0ull;
      const bool act = valid && done < S && ((und >> es) & 1ull) && !blocked;
      const int cap = pass == 0 ? BB_QUOTA_FIRST : BB_QUOTA_NEXT;
      int c = act ? (S - done < cap ? S - done : cap) : 0;
      const int incl0 = (int)wave_incl_add((uint32_t)c);
      const int off = incl0 - c;
      c = off >= 64 ? 0 : (off + c > 64 ? 64 - off : c);  // the pass holds 64 slots
      const int total = __builtin_amdgcn_readlane(incl0, 63) < 64 ? __builtin_amdgcn_readlane(incl0, 63) : 64;
      // owner j of slot lane `lane`: the last attempt lane whose first slot of the pass is <= it
      wave_lds_fence();
      lds[lane] = 0u;
      wave_lds_fence();
      if (c > 0) atomicMax(&lds[off], (uint32_t)lane);
      wave_lds_fence();
      const int j = (int)wave_incl_max(lds[lane]);
      const uint32_t jid = __shfl(e_ids, j);
      const uint64_t jA0 = __shfl(eA0, j), jA1 = __shfl(eA1, j), jA2 = __shfl(eA2, j);
      const uint64_t jB = __shfl(B, j);
      const int jrem0 = __shfl(done - off, j) + lane;  // slot index within attempt j
      int q = 0;
      uint64_t B1 = 0, A2 = 0, A3 = 0;
      uint32_t bi = 0, ci = 0;
      {  // every lane computes its slot (lanes past `total` a dummy one) and drops it by select
        const int c0 = __popcll(jA0), c1 = __popcll(jA1);
        const int f = jrem0 < c0 ? 0 : (jrem0 < c0 + c1 ? 1 : 2);
        const uint64_t Af = f == 0 ? jA0 : (f == 1 ? jA1 : jA2);
        const int rem = jrem0 - (f == 0 ? 0 : (f == 1 ? c0 : c0 + c1));
        const int p = select_bit(Af, (uint32_t)rem) & 63;
        bi = hand_id(jid, f == 0 ? 1 : 0);
        ci = hand_id(jid, f == 2 ? 1 : 2);
        B1 = clear_full(jB | (tbl[hand_id(jid, f)].shape << p));
        q = pair_quick_bf(B1, tbl[bi], tbl[ci], dtab[bi * kPieces + ci], A2, A3);
        if (lane >= total) q = 0;
      }
      // attempt lane L owns the pass's slot bits [off, off + c)
      const uint64_t own = c > 0 ? (c == 64 ? ~0ull : ((1ull << c) - 1ull)) << off : 0ull;
      const uint64_t qam = __ballot((__ballot(q == 1) & own) != 0ull);
      const uint64_t jenv = every << (j % E);
      bool ok = q == 1;
      const bool need = q == 2 && !((qam | okm) & jenv & ((2ull << j) - 1ull));
      BB_MT(q1);
      if (__ballot(need))
        ok |= slow_phase_wave<kLineOnly>(need, B1, bi, ci, A2, A3, tbl, lane, lds,
                                         (uint32_t)((j % E) << 8 | (j / E)));
      BB_MT(q2);
      pq += q1 - q0;
      ps += q2 - q1;
      okm |= __ballot((__ballot(ok) & own) != 0ull);
      done += c;
    }
    BB_MT(p3);
    // resolve every env of the round in its own lanes: its earliest successful attempt, else past all
    // of its (complete, failed) attempts
    const bool mine = (todo >> me) & 1ull;
    const int my_es = __popcll(todo & ((1ull << me) - 1ull));
    const uint64_t em = mine ? (every << my_es) & vmask : 0ull;
    const uint64_t hit = em & okm;
    int src = -1;
    if (hit) src = __ffsll((unsigned long long)hit) - 1;
    else if (em) src = 63 - __clzll((long long)em);
    const int from = src < 0 ? lane : src;
    const uint32_t f_ids = __shfl(e_ids, from);
    Pcg fa;
    fa.hi = __shfl(e_after.hi, from);
    fa.lo = __shfl(e_after.lo, from);
    fa.buf = __shfl(e_after.buf, from);
    fa.has = __shfl((int)e_after.has, from) != 0;
    bool fin = false;
    if (src >= 0) {
      rng.hi = fa.hi;
      rng.lo = fa.lo;
      rng.buf = fa.buf;
      rng.has = fa.has;
      if (hit) {
        ids = f_ids;
        fin = true;
      } else {
        att += __popcll(em);
        last_ids = f_ids;
        if (att >= kMaxAttempts) {
          ids = last_ids;
          fin = true;
        }
      }
    }
    todo &= ~(__ballot(fin && lane < kEnvs) & (kEnvs >= 64 ? ~0ull : ((1ull << (kEnvs & 63)) - 1ull)));
    release(fin && lane < kEnvs);
    pk = pack_next > 0 ? pack_next : 2 * pk;
    pk = pk < kPack ? pk : kPack;
    if (prof) {
      BB_MT(p4);
      prof[0] += p1 - p0;
      prof[1] += p2 - p1;
      prof[2] += pq;
      prof[3] += ps;
      prof[4] += (p3 - p2) - pq - ps;
      prof[5] += p4 - p3;
    }
  }
#undef BB_MT
}

}  // namespace bb

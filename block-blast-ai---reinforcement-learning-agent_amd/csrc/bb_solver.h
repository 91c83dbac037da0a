// bb_solver.h -- exact "can all three pieces be placed in some order" test
// (engine.py:155-238 _generate_new_pieces / _can_place_remaining /
// _simulate_line_clears) on bitboards, plus the rejection-sampling hand draw.
//
// Only the boolean of the reference's DFS matters (it decides how many
// 3-draw attempts consume the PCG64 stream), so any exact algorithm is
// allowed.  Structure:
//   level 1: every legal anchor p of the first piece f (all 3 choices of f);
//   level 2: the remaining pair (b, c) on B1 = clear(B | f<<p):
//     quick accept (exact sufficient condition, no search): with D(b,c) the
//     set of linear offsets ob_i - oc_j, a b-anchor q conflicts with at most
//     |D| c-anchors, so popcount(anchors(c,B1)) > |D| and some b-anchor
//     exist => a disjoint pair exists => placeable in order b, c (line clears
//     only remove cells, so they can never invalidate it);
//     otherwise exhaustive: every b-anchor q then "c has any anchor on
//     clear(B1 | b<<q)", and the symmetric order.
//   level 3 is the anchors_of() != 0 test.
// Per-lane search runs under a work budget; an env that exceeds it is handed
// to the whole wave (solve_wave: lane l takes level-1 anchor l), so one hard
// board never serialises 64 lanes.
#pragma once
#include "bb_device.h"

namespace bb {

constexpr int kUnlimited = 1 << 30;

// Level 2: can pieces b and c both still be placed (either order) on B1?
// Returns 1 yes, 0 no, -1 budget exhausted.  Budget unit = one anchors_of().
__device__ __forceinline__ int solve_pair(uint64_t B1, const PieceRow& pb, const PieceRow& pc, uint32_t dbc,
                                          int& budget) {
  uint64_t A2 = anchors_of(pb, B1);
  uint64_t A3 = anchors_of(pc, B1);
  budget -= 2;
  if ((A2 | A3) == 0) return 0;
  if (A2 && (uint32_t)__popcll(A3) > dbc) return 1;
  if (A3 && (uint32_t)__popcll(A2) > dbc) return 1;
  // order b then c
  uint64_t it = A2;
  while (it) {
    if (budget <= 0) return -1;
    int q = __ffsll((unsigned long long)it) - 1;
    it &= it - 1;
    uint64_t B2 = clear_full(B1 | (pb.shape << q));
    --budget;
    if (anchors_of(pc, B2)) return 1;
  }
  // order c then b
  it = A3;
  while (it) {
    if (budget <= 0) return -1;
    int q = __ffsll((unsigned long long)it) - 1;
    it &= it - 1;
    uint64_t B2 = clear_full(B1 | (pc.shape << q));
    --budget;
    if (anchors_of(pb, B2)) return 1;
  }
  return 0;
}

// Full single-lane test.  1 solvable, 0 not, -1 budget exhausted.
__device__ __forceinline__ int solve_lane(uint64_t B, const PieceRow* tbl, const uint8_t* dtab,
                                          uint32_t i0, uint32_t i1, uint32_t i2, int& budget) {
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
    --budget;
    while (A1) {
      if (budget <= 0) return -1;
      int p = __ffsll((unsigned long long)A1) - 1;
      A1 &= A1 - 1;
      uint64_t B1 = clear_full(B | (pf.shape << p));
      int r = solve_pair(B1, pb, pc, dbc, budget);
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
      uint64_t B1 = clear_full(B | (pf.shape << lane));
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
    uint32_t a = draw_piece(rng);
    uint32_t b = draw_piece(rng);
    uint32_t c = draw_piece(rng);
    ids = a | (b << 6) | (c << 12);
    int r = solve_lane(B, tbl, dtab, a, b, c, budget);
    if (r == 1) return true;
    if (r < 0) {
      rng = save;
      return false;
    }
  }
  return true;
}

// Wave-cooperative continuation of gen_hand_lane for one env.
__device__ __forceinline__ void gen_hand_wave(uint64_t B, Pcg& rng, uint32_t& ids, int attempt,
                                              const PieceRow* tbl, const uint8_t* dtab, int lane) {
#pragma unroll 1
  for (; attempt < kMaxAttempts; ++attempt) {
    uint32_t a = draw_piece(rng);
    uint32_t b = draw_piece(rng);
    uint32_t c = draw_piece(rng);
    ids = a | (b << 6) | (c << 12);
    if (solve_wave(B, tbl, dtab, a, b, c, lane)) return;
  }
}

}  // namespace bb

// bb_device.h -- device-side building blocks of the Block Blast vec-env (gfx950).
//
// Everything here works on one 8x8 board held as a uint64 bitboard in VGPRs
// (bit r*8+c == grid[r][c], reference board.py:30).  Each helper names the
// reference function whose semantics it reproduces.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bb {

constexpr int kPieces = 37;
constexpr int kHand = 3;
constexpr int kMaxAttempts = 100;  // engine.py:161

constexpr uint64_t kRow0 = 0x00000000000000FFull;
constexpr uint64_t kRow7 = 0xFF00000000000000ull;
constexpr uint64_t kCol0 = 0x0101010101010101ull;
constexpr uint64_t kCol7 = 0x8080808080808080ull;
constexpr uint64_t kCenter = 0x00003C3C3C3C0000ull;  // rows 2-5 x cols 2-5 (board.py:242)

// One row of the piece table, staged into LDS by every kernel.
//   shape   : cells of the piece anchored at (0,0)
//   anchors : legal anchor squares on an empty board (r <= 8-h, c <= 8-w)
//   offs    : 9 packed 6-bit cell offsets (padded by repetition) so that the
//             blocked-anchor dilation is a fixed 9-step OR chain with no branch
//   ym      : 128-bit "mirror" with bit (64 - o) for every cell offset o, the
//             seed of the pair-conflict masks of bb_solver.h
//   sh      : the cell offsets as a Minkowski program S = X + {0,s1} + {0,s2}
//             with |X| <= 4 (linear offsets; built on the host and checked
//             exact there): sh[0..3] the offsets of X (repeated to fill),
//             sh[4] = s1, sh[5] = s2 (0 = no step) | cell count << 8.  One
//             word per shift, so each is a 64-bit shift's amount operand as
//             is (the hardware reads bits 5:0).  anchors_of costs 6 shifts
//             for every piece instead of one per cell (9 for SQUARE_3x3 =
//             {0,1,2} + {0,8} + {0,8}).
#ifndef BB_ROW_PAD
// bytes of padding per PieceRow: a 72-byte stride (an odd number of 8-byte words) spreads the lanes'
// per-piece LDS reads over every bank (64-byte rows: 5.2x the bank-conflict cycles and -4% on the rollout;
// 80 / 88 / 104 bytes: -1.3% / -0.4% / +0.1%; profiles/r04/p2_*)
#define BB_ROW_PAD 8
#endif
struct PieceRow {
  uint64_t shape;
  uint64_t anchors;
  uint64_t offs;
  uint64_t ym_lo;
  uint64_t ym_hi;
  uint32_t sh[6];
#if BB_ROW_PAD
  uint8_t pad[BB_ROW_PAD];
#endif
};

__host__ __device__ inline uint32_t ncells_of(const PieceRow& p) { return (p.sh[5] >> 8) & 0xFFu; }

// PCG64 jump-ahead table row c: A^c and S_c = sum_{i<c} A^i (mod 2^128), so
// the state after c steps is A^c * s + inc * S_c (built on the host).
constexpr int kJumpMax = 64;
struct JumpRow {
  uint64_t a_lo, a_hi, s_lo, s_hi;
};

// Board.can_place over all anchors at once (board.py:71-93 x engine.py:364-380):
// anchor a is blocked iff some cell a+off is filled, i.e. bit a of (B >> off).
// The OR over the cell offsets runs as the row's Minkowski program (PieceRow
// sh): 4 shifts for X, then x |= x >> s for each step.  Every bit a term
// reads at a legal anchor a is a cell of the piece placed at a, so nothing
// wraps or leaves the board there; other anchors are masked off.
__host__ __device__ inline uint64_t dilate(const PieceRow& p, uint64_t B) {
  // sh[0..4] < 64 by construction (no mask needed); sh[5] carries the cell count above bit 7
  uint64_t x = (B >> p.sh[0]) | (B >> p.sh[1]);
  x |= (B >> p.sh[2]) | (B >> p.sh[3]);
  x |= x >> p.sh[4];
  x |= x >> (p.sh[5] & 63u);
  return x;
}

// Packed hand word (also the host-visible layout, see bbvec.h bb_state_view).
__host__ __device__ inline uint32_t hand_id(uint32_t h, int slot) { return (h >> (6 * slot)) & 63u; }
__host__ __device__ inline uint32_t hand_used(uint32_t h) { return (h >> 18) & 7u; }
__host__ __device__ inline bool hand_over(uint32_t h) { return (h >> 21) & 1u; }
__host__ __device__ inline bool hand_has32(uint32_t h) { return (h >> 22) & 1u; }
__host__ __device__ inline uint32_t hand_pack(uint32_t a, uint32_t b, uint32_t c, uint32_t used,
                                              bool over, bool has32) {
  return a | (b << 6) | (c << 12) | (used << 18) | ((uint32_t)over << 21) | ((uint32_t)has32 << 22);
}

// --------------------------------------------------------------------------
// Bitboard rules
// --------------------------------------------------------------------------

__device__ __forceinline__ uint64_t anchors_of(const PieceRow& p, uint64_t B) { return p.anchors & ~dilate(p, B); }

// Board.find_complete_lines + clear_lines (board.py:144-193), and the DFS's
// _simulate_line_clears (engine.py:226-238): full rows/cols are found on the
// same board, then their union is cleared.  Worked on the two 32-bit halves
// (rows 0-3 / 4-7): a row byte is full iff its low 7 bits carry into bit 7
// and bit 7 is set; the columns are the AND of all eight row bytes.
__device__ __forceinline__ uint32_t full_row_bytes(uint32_t h) {  // 0x80 in every 0xFF byte
  return ((h & 0x7F7F7F7Fu) + 0x01010101u) & h & 0x80808080u;
}

__device__ __forceinline__ uint64_t clear_full(uint64_t B, int& rows, int& cols) {
  const uint32_t lo = (uint32_t)B, hi = (uint32_t)(B >> 32);
  const uint32_t flo = full_row_bytes(lo), fhi = full_row_bytes(hi);
  uint32_t a = lo & hi;
  a &= a >> 16;
  a &= a >> 8;                                          // byte 0: the full columns
  const uint32_t cs = __builtin_amdgcn_perm(a, a, 0u);  // byte 0 broadcast to all four bytes
  rows = __popc(flo) + __popc(fhi);
  cols = __popc(a & 0xFFu);
  const uint32_t rlo = (flo >> 7) * 0xFFu, rhi = (fhi >> 7) * 0xFFu;  // full rows spread over their bytes
  return ((uint64_t)(hi & ~(rhi | cs)) << 32) | (lo & ~(rlo | cs));
}

__device__ __forceinline__ uint64_t clear_full(uint64_t B) {
  int r, c;
  return clear_full(B, r, c);
}

// Board.count_holes (board.py:195-216): empty cells whose four neighbours are
// all filled or off-board.
__device__ __forceinline__ int count_holes(uint64_t B) {
  uint64_t n = (B << 8) | kRow0;
  uint64_t s = (B >> 8) | kRow7;
  uint64_t w = ((B << 1) & ~kCol0) | kCol0;
  uint64_t e = ((B >> 1) & ~kCol7) | kCol7;
  return __popcll(~B & n & s & w & e);
}

// --------------------------------------------------------------------------
// numpy PCG64 (XSL-RR 128/64) + Generator.integers(0, 37) Lemire draw.
// Stream-exact with np.random.default_rng (engine.py:109,138; pieces.py:354).
// --------------------------------------------------------------------------
struct Pcg {
  uint64_t hi, lo;        // 128-bit LCG state
  uint64_t inc_hi, inc_lo;
  uint32_t buf;           // buffered upper 32-bit half (numpy `uinteger`)
  uint32_t has;           // numpy `has_uint32` (0/1); a full word: no padding bytes, which the
                          // compiler otherwise round-trips through scratch on every struct copy
};

__device__ __forceinline__ uint64_t pcg_next64(Pcg& s) {
  constexpr uint64_t MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
  uint64_t lo = s.lo * ML;
  uint64_t hi = __umul64hi(s.lo, ML) + s.lo * MH + s.hi * ML;
  lo += s.inc_lo;
  hi += s.inc_hi + (lo < s.inc_lo ? 1ull : 0ull);
  s.lo = lo;
  s.hi = hi;
  uint64_t x = hi ^ lo;
  unsigned rot = (unsigned)(hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

__device__ __forceinline__ uint32_t pcg_next32(Pcg& s) {
  if (s.has) {
    s.has = 0u;
    return s.buf;
  }
  uint64_t v = pcg_next64(s);
  s.has = 1u;
  s.buf = (uint32_t)(v >> 32);
  return (uint32_t)v;
}

// buffered_bounded_lemire_uint32 with rng_excl = 37; threshold (2^32-37) % 37 = 7.
__device__ __forceinline__ uint32_t draw_piece(Pcg& s) {
  uint64_t m = (uint64_t)pcg_next32(s) * 37ull;
  uint32_t left = (uint32_t)m;
  if (left < 37u) {
    while (left < 7u) {
      m = (uint64_t)pcg_next32(s) * 37ull;
      left = (uint32_t)m;
    }
  }
  return (uint32_t)(m >> 32);
}

// get_random_pieces(3, rng) (pieces.py:350-355): three draws without a
// branch on has_uint32 -- the two LCG outputs the three 32-bit values can need
// are computed unconditionally and the values picked by select, so a wave
// with mixed has_uint32 runs two LCG steps instead of three masked ones.  A
// Lemire rejection (p ~ 5e-9 per draw) redoes the draws sequentially.
__device__ __forceinline__ void draw3(Pcg& s, uint32_t& a, uint32_t& b, uint32_t& c) {
  const Pcg s0 = s;
  const uint64_t o1 = pcg_next64(s);
  const uint64_t h1 = s.hi, l1 = s.lo;
  const uint64_t o2 = pcg_next64(s);
  const bool has = s0.has != 0u;
  const uint32_t v0 = has ? s0.buf : (uint32_t)o1;
  const uint32_t v1 = has ? (uint32_t)o1 : (uint32_t)(o1 >> 32);
  const uint32_t v2 = has ? (uint32_t)(o1 >> 32) : (uint32_t)o2;
  const uint64_t m0 = (uint64_t)v0 * 37ull, m1 = (uint64_t)v1 * 37ull, m2 = (uint64_t)v2 * 37ull;
  if ((uint32_t)m0 < 7u || (uint32_t)m1 < 7u || (uint32_t)m2 < 7u) {  // rare: numpy's rejection loop
    s = s0;
    a = draw_piece(s);
    b = draw_piece(s);
    c = draw_piece(s);
    return;
  }
  a = (uint32_t)(m0 >> 32);
  b = (uint32_t)(m1 >> 32);
  c = (uint32_t)(m2 >> 32);
  if (has) {  // one LCG output used, its upper half consumed (numpy keeps the stale value in `uinteger`)
    s.hi = h1;
    s.lo = l1;
    s.has = 0u;
    s.buf = (uint32_t)(o1 >> 32);
  } else {    // two used, the upper half of the second one buffered
    s.has = 1u;
    s.buf = (uint32_t)(o2 >> 32);
  }
}

// --------------------------------------------------------------------------
// Philox4x32-10 (Random123) -- synthetic policy / sampling uniforms.
// --------------------------------------------------------------------------
__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += W0;
      k1 += W1;
    }
    uint64_t p0 = (uint64_t)M0 * c[0];
    uint64_t p1 = (uint64_t)M1 * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
  }
}

__device__ __forceinline__ void philox_words(uint64_t seed, uint64_t idx, uint64_t step, uint32_t out[4]) {
  out[0] = (uint32_t)idx;
  out[1] = (uint32_t)(idx >> 32);
  out[2] = (uint32_t)step;
  out[3] = (uint32_t)(step >> 32);
  philox4x32_10(out, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// Index of the k-th (0-based) set bit of x (k < popcount(x)).
__device__ __forceinline__ int select_bit(uint64_t x, uint32_t k) {
  int pos = 0;
  uint32_t c = __popc((uint32_t)x);
  if (k >= c) { k -= c; x >>= 32; pos += 32; }
  c = __popc((uint32_t)x & 0xFFFFu);
  if (k >= c) { k -= c; x >>= 16; pos += 16; }
  c = __popc((uint32_t)x & 0xFFu);
  if (k >= c) { k -= c; x >>= 8; pos += 8; }
  c = __popc((uint32_t)x & 0xFu);
  if (k >= c) { k -= c; x >>= 4; pos += 4; }
  c = __popc((uint32_t)x & 0x3u);
  if (k >= c) { k -= c; x >>= 2; pos += 2; }
  c = (uint32_t)x & 1u;
  if (k >= c) { pos += 1; }
  return pos;
}

// Synthetic random policy: the k-th legal action, k = (u * popcount) >> 32,
// u = word 0 of Philox4x32-10 at counter (idx, step) under key seed.
__device__ __forceinline__ uint32_t policy_uniform(uint64_t seed, uint64_t idx, uint64_t step) {
  uint32_t w[4];
  philox_words(seed, idx, step, w);
  return w[0];
}

__device__ __forceinline__ int32_t random_policy_u(uint64_t m0, uint64_t m1, uint64_t m2, uint32_t u) {
  const uint32_t c0 = __popcll(m0), c1 = __popcll(m1), c2 = __popcll(m2);
  const uint32_t tot = c0 + c1 + c2;
  uint32_t k = (uint32_t)(((uint64_t)u * tot) >> 32);
  // the word holding the k-th set bit, picked by select: one select_bit, no divergent paths
  const bool in0 = k < c0, in1 = k < c0 + c1;
  const uint64_t w = in0 ? m0 : (in1 ? m1 : m2);
  k -= in0 ? 0u : (in1 ? c0 : c0 + c1);
  const int base = in0 ? 0 : (in1 ? 64 : 128);
  return tot == 0 ? 0 : base + select_bit(w, k);
}

__device__ __forceinline__ int32_t random_policy(uint64_t m0, uint64_t m1, uint64_t m2, uint64_t seed,
                                                 uint64_t idx, uint64_t step) {
  return random_policy_u(m0, m1, m2, policy_uniform(seed, idx, step));
}

}  // namespace bb

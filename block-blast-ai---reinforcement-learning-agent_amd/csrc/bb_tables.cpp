// bb_tables.cpp -- host-side static tables and numpy-exact PCG64 seeding.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bb_env_internal.h"
#include "bb_seed.h"

namespace bb {

using seed::kShapes;  // bb_seed.h: the 37 shapes of src/game/pieces.py:78-236 (bit r*8+c)
static_assert(seed::kNumPieces == kPieces, "piece count");

// S (k linear cell offsets) as X + {0,s1} + {0,s2} (Minkowski sums, |X| <= 4):
// the anchors_of program of PieceRow.  Pieces of <= 4 cells take X = S and no
// steps.  Returns false if no such program exists (none of the 37 shapes).
static bool minkowski_program(const int* S, int k, uint32_t sh[6]) {
  uint64_t sset[2] = {0, 0};
  for (int i = 0; i < k; ++i) sset[S[i] >> 6] |= 1ull << (S[i] & 63);
  auto in = [&](int v) { return v >= 0 && v < 128 && ((sset[v >> 6] >> (v & 63)) & 1ull); };
  for (int s1 = 0; s1 < 64; ++s1) {
    for (int s2 = 0; s2 <= (s1 ? s1 : 0); ++s2) {
      const int T[4] = {0, s1, s2, s1 + s2};
      // X = every cell x with x + T inside S; the program is exact iff X + T == S
      int X[9], nx = 0;
      for (int i = 0; i < k; ++i) {
        bool ok = true;
        for (int t = 0; t < 4; ++t) ok = ok && in(S[i] + T[t]);
        if (ok) X[nx++] = S[i];
      }
      if (nx == 0) continue;
      uint64_t cover[2] = {0, 0};
      for (int i = 0; i < nx; ++i)
        for (int t = 0; t < 4; ++t) cover[(X[i] + T[t]) >> 6] |= 1ull << ((X[i] + T[t]) & 63);
      if (cover[0] != sset[0] || cover[1] != sset[1]) continue;
      // drop members of X whose cells the others already cover, down to 4
      for (int i = 0; i < nx && nx > 4;) {
        uint64_t c2[2] = {0, 0};
        for (int j = 0; j < nx; ++j)
          if (j != i)
            for (int t = 0; t < 4; ++t) c2[(X[j] + T[t]) >> 6] |= 1ull << ((X[j] + T[t]) & 63);
        if (c2[0] == sset[0] && c2[1] == sset[1]) {
          X[i] = X[--nx];
        } else {
          ++i;
        }
      }
      if (nx > 4) continue;
      for (int j = 0; j < 4; ++j) sh[j] = (uint32_t)X[j < nx ? j : 0];
      sh[4] = (uint32_t)s1;
      sh[5] = (uint32_t)s2;
      return true;
    }
  }
  return false;
}

void build_piece_tables(PieceRow rows[kPieces], uint8_t dtab[kPieces * kPieces]) {
  int offs[kPieces][9];
  int n[kPieces];
  for (int p = 0; p < kPieces; ++p) {
    const uint64_t s = kShapes[p];
    int h = 0, w = 0, k = 0;
    for (int b = 0; b < 64; ++b) {
      if ((s >> b) & 1ull) {
        offs[p][k++] = b;
        if (b / 8 + 1 > h) h = b / 8 + 1;
        if (b % 8 + 1 > w) w = b % 8 + 1;
      }
    }
    n[p] = k;
    uint64_t anchors = 0;
    for (int r = 0; r <= 8 - h; ++r)
      for (int c = 0; c <= 8 - w; ++c) anchors |= 1ull << (r * 8 + c);
    uint64_t packed = 0;
    for (int j = 0; j < 9; ++j) packed |= (uint64_t)offs[p][j < k ? j : 0] << (6 * j);
    uint64_t ylo = 0, yhi = 0;
    for (int j = 0; j < k; ++j) {
      const int bit = 64 - offs[p][j];
      if (bit >= 64) yhi |= 1ull << (bit - 64);
      else ylo |= 1ull << bit;
    }
    rows[p].ym_lo = ylo;
    rows[p].ym_hi = yhi;
    rows[p].shape = s;
    rows[p].anchors = anchors;
    rows[p].offs = packed;
    if (!minkowski_program(offs[p], k, rows[p].sh)) abort();  // every one of the 37 shapes has one
    rows[p].sh[5] |= (uint32_t)k << 8;
    // the program's dilation equals the per-cell one on the legal anchors (self-check)
    uint64_t r = 0x9E3779B97F4A7C15ull ^ (uint64_t)p;
    for (int t = 0; t < 64; ++t) {
      r ^= r << 13, r ^= r >> 7, r ^= r << 17;
      const uint64_t B = r & (r >> 3);  // ~1/4 filled .. varied
      uint64_t direct = 0;
      for (int j = 0; j < k; ++j) direct |= B >> offs[p][j];
      const uint64_t x = dilate(rows[p], B);
      if ((anchors & ~x) != (anchors & ~direct)) abort();
    }
  }
  // |{ob_i - oc_j}|: distinct linear offsets at which piece c collides with b.
  for (int b = 0; b < kPieces; ++b) {
    for (int c = 0; c < kPieces; ++c) {
      bool seen[128];
      memset(seen, 0, sizeof(seen));
      int cnt = 0;
      for (int i = 0; i < n[b]; ++i)
        for (int j = 0; j < n[c]; ++j) {
          int d = offs[b][i] - offs[c][j] + 64;
          if (!seen[d]) {
            seen[d] = true;
            ++cnt;
          }
        }
      dtab[b * kPieces + c] = (uint8_t)cnt;
    }
  }
}

void build_jump_table(JumpRow rows[kJumpMax + 1]) {
  typedef unsigned __int128 u128;
  const u128 mult = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
  u128 a = 1, s = 0;  // A^0, S_0
  for (int c = 0; c <= kJumpMax; ++c) {
    rows[c].a_lo = (uint64_t)a;
    rows[c].a_hi = (uint64_t)(a >> 64);
    rows[c].s_lo = (uint64_t)s;
    rows[c].s_hi = (uint64_t)(s >> 64);
    s += a;
    a *= mult;
  }
}

// numpy default_rng(seed) initialisation (engine.py:109,138): bb_seed.h, shared with the host backend
void pcg64_seed_numpy(uint64_t seed, uint64_t out[4]) { seed::pcg64_seed_numpy(seed, out); }

}  // namespace bb

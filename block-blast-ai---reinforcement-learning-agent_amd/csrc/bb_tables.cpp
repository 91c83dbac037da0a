// bb_tables.cpp -- host-side static tables and numpy-exact PCG64 seeding.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bb_env_internal.h"

namespace bb {

// The 37 shapes of src/game/pieces.py:78-236 as bitboards anchored at (0,0),
// in PIECES dict order (pieces.py:244-318) == piece index.  Bit r*8+c.
static const uint64_t kShapes[kPieces] = {
    0x1ull,          0x3ull,           0x101ull,     0x201ull,     0x102ull,     0x7ull,     0x10101ull,
    0x40201ull,      0x10204ull,       0x301ull,     0x203ull,     0x103ull,     0x302ull,   0xFull,
    0x1010101ull,    0x1Full,          0x101010101ull, 0x303ull,   0x702ull,     0x207ull,   0x10301ull,
    0x20302ull,      0x306ull,         0x20301ull,   0x603ull,     0x10302ull,   0x30101ull, 0x107ull,
    0x20203ull,      0x704ull,         0x30202ull,   0x701ull,     0x10103ull,   0x407ull,   0x707ull,
    0x30303ull,      0x70707ull,
};

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

// ---------------------------------------------------------------------------
// numpy SeedSequence(seed).generate_state(4, uint64) + PCG64 set_seed:
// the exact initialisation behind np.random.default_rng(seed)
// (engine.py:109,138).  Verified against numpy in tests/.
// ---------------------------------------------------------------------------
namespace {
constexpr uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u;
constexpr uint32_t INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
constexpr uint32_t MIX_L = 0xca01f9ddu, MIX_R = 0x4973f715u;

inline uint32_t hashmix(uint32_t v, uint32_t& hc) {
  v ^= hc;
  hc *= MULT_A;
  v *= hc;
  v ^= v >> 16;
  return v;
}
inline uint32_t mixw(uint32_t x, uint32_t y) {
  uint32_t r = MIX_L * x - MIX_R * y;
  r ^= r >> 16;
  return r;
}
}  // namespace

void pcg64_seed_numpy(uint64_t seed, uint64_t out[4]) {
  // entropy -> little-endian uint32 words (at least one word)
  uint32_t ent[2];
  int nent = 0;
  ent[nent++] = (uint32_t)seed;
  if (seed >> 32) ent[nent++] = (uint32_t)(seed >> 32);
  uint32_t pool[4];
  uint32_t hc = INIT_A;
  for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < nent ? ent[i] : 0u, hc);
  for (int s = 0; s < 4; ++s)
    for (int d = 0; d < 4; ++d)
      if (s != d) pool[d] = mixw(pool[d], hashmix(pool[s], hc));
  for (int s = 4; s < nent; ++s)
    for (int d = 0; d < 4; ++d) pool[d] = mixw(pool[d], hashmix(ent[s], hc));
  uint32_t st[8];
  uint32_t hb = INIT_B;
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i % 4];
    v ^= hb;
    hb *= MULT_B;
    v *= hb;
    v ^= v >> 16;
    st[i] = v;
  }
  uint64_t w[4];
  for (int i = 0; i < 4; ++i) w[i] = (uint64_t)st[2 * i] | ((uint64_t)st[2 * i + 1] << 32);
  typedef unsigned __int128 u128;
  const u128 mult = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
  const u128 initstate = ((u128)w[0] << 64) | w[1];
  const u128 initseq = ((u128)w[2] << 64) | w[3];
  u128 inc = (initseq << 1) | 1u;
  u128 state = 0;
  state = state * mult + inc;
  state += initstate;
  state = state * mult + inc;
  out[0] = (uint64_t)(state >> 64);
  out[1] = (uint64_t)state;
  out[2] = (uint64_t)(inc >> 64);
  out[3] = (uint64_t)inc;
}

}  // namespace bb

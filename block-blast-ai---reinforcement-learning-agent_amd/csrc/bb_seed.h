// bb_seed.h -- HIP-free pieces shared by the gfx950 library (bb_tables.cpp)
// and the host backend (bb_host.cpp): the 37 piece shapes and numpy's exact
// default_rng(seed) initialisation.
#pragma once
#include <stdint.h>

namespace bb {
namespace seed {

// The 37 shapes of src/game/pieces.py:78-236 as bitboards anchored at (0,0),
// in PIECES dict order (pieces.py:244-318) == piece index.  Bit r*8+c.
constexpr int kNumPieces = 37;
constexpr uint64_t kShapes[kNumPieces] = {
    0x1ull,          0x3ull,           0x101ull,     0x201ull,     0x102ull,     0x7ull,     0x10101ull,
    0x40201ull,      0x10204ull,       0x301ull,     0x203ull,     0x103ull,     0x302ull,   0xFull,
    0x1010101ull,    0x1Full,          0x101010101ull, 0x303ull,   0x702ull,     0x207ull,   0x10301ull,
    0x20302ull,      0x306ull,         0x20301ull,   0x603ull,     0x10302ull,   0x30101ull, 0x107ull,
    0x20203ull,      0x704ull,         0x30202ull,   0x701ull,     0x10103ull,   0x407ull,   0x707ull,
    0x30303ull,      0x70707ull,
};

typedef unsigned __int128 u128;
constexpr u128 kPcgMult = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;

// numpy SeedSequence(seed).generate_state(4, uint64) + PCG64 set_seed: the
// exact initialisation behind np.random.default_rng(seed) (engine.py:109,138).
// out = {state_hi, state_lo, inc_hi, inc_lo}.  Verified against numpy in tests/.
inline void pcg64_seed_numpy(uint64_t seed, uint64_t out[4]) {
  constexpr uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u;
  constexpr uint32_t INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
  constexpr uint32_t MIX_L = 0xca01f9ddu, MIX_R = 0x4973f715u;
  auto hashmix = [](uint32_t v, uint32_t& hc) {
    v ^= hc;
    hc *= MULT_A;
    v *= hc;
    v ^= v >> 16;
    return v;
  };
  auto mixw = [](uint32_t x, uint32_t y) {
    uint32_t r = MIX_L * x - MIX_R * y;
    r ^= r >> 16;
    return r;
  };
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
  const u128 initstate = ((u128)w[0] << 64) | w[1];
  const u128 initseq = ((u128)w[2] << 64) | w[3];
  const u128 inc = (initseq << 1) | 1u;
  u128 state = 0;
  state = state * kPcgMult + inc;
  state += initstate;
  state = state * kPcgMult + inc;
  out[0] = (uint64_t)(state >> 64);
  out[1] = (uint64_t)state;
  out[2] = (uint64_t)(inc >> 64);
  out[3] = (uint64_t)inc;
}

}  // namespace seed
}  // namespace bb

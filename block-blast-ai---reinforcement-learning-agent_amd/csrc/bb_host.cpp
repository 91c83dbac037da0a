// bb_host.cpp -- host (CPU) backend of the env half of include/bbvec.h.
//
// A second implementation of the same C-ABI for machines without the MI355X,
// built by g++ into libbbvec_host.so (runtime/build.py build_host_lib).  It is
// selected explicitly (DeviceEnvBatch / VectorizedBlockBlastEnv with
// device="cpu"); nothing ever falls back to it: libbbvec.so still fails
// loudly without a HIP device, and the GPU tests never load this library.
// All "d_" pointers are host memory here and `stream` is ignored.
//
// Same semantics as the gfx950 kernels, bit for bit: uint64 bitboards (bit
// r*8+c), numpy-exact PCG64 piece streams, the reference's fp64 reward order,
// the vec-env auto-reset with its re-seed, the Philox synthetic policy.  The
// hand search is the reference DFS itself (engine.py:174-238) on bitboards, one
// env per thread (OpenMP over envs).  Parity: tests/test_host_backend.py runs it
// against the C oracle (oracle/bb_oracle.c) step for step.
//
// Reference: src/environment/wrappers.py:75-116 (vec step, auto-reset) ->
// block_blast_env.py:224-264 (step, reward 148-193) -> engine.py:390-454.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/bbvec.h"
#include "bb_seed.h"

namespace {

using bb::seed::u128;
constexpr int kPieces = 37;
constexpr uint64_t kRow0 = 0xFFull, kRow7 = 0xFF00000000000000ull;
constexpr uint64_t kCol0 = 0x0101010101010101ull, kCol7 = 0x8080808080808080ull;
constexpr uint64_t kCenter = 0x00003C3C3C3C0000ull;  // rows 2-5 x cols 2-5 (board.py:242)

struct Piece {
  uint64_t shape, anchors;
  int n, off[9];
};

struct Tables {
  Piece p[kPieces];
  Tables() {
    for (int k = 0; k < kPieces; ++k) {
      Piece& q = p[k];
      q.shape = bb::seed::kShapes[k];
      q.n = 0;
      int h = 0, w = 0;
      for (int b = 0; b < 64; ++b)
        if ((q.shape >> b) & 1ull) {
          q.off[q.n++] = b;
          h = b / 8 + 1 > h ? b / 8 + 1 : h;
          w = b % 8 + 1 > w ? b % 8 + 1 : w;
        }
      q.anchors = 0;
      for (int r = 0; r <= 8 - h; ++r)
        for (int c = 0; c <= 8 - w; ++c) q.anchors |= 1ull << (r * 8 + c);
    }
  }
};
const Tables& T() {
  static const Tables t;
  return t;
}

// engine.py:364-380 / board.py:71-93 over all anchors: anchor a is blocked iff
// some cell a + off is filled
inline uint64_t anchors_of(int pid, uint64_t B) {
  const Piece& q = T().p[pid];
  uint64_t x = 0;
  for (int j = 0; j < q.n; ++j) x |= B >> q.off[j];
  return q.anchors & ~x;
}

// board.py:144-193: full rows / cols of the same board, union cleared
inline uint64_t clear_full(uint64_t B, int& rows, int& cols) {
  uint64_t rm = 0, cm = 0;
  rows = cols = 0;
  for (int r = 0; r < 8; ++r)
    if (((B >> (8 * r)) & 0xFFull) == 0xFFull) rm |= 0xFFull << (8 * r), ++rows;
  for (int c = 0; c < 8; ++c)
    if ((B & (kCol0 << c)) == (kCol0 << c)) cm |= kCol0 << c, ++cols;
  return B & ~(rm | cm);
}
inline uint64_t clear_full(uint64_t B) {
  int r, c;
  return clear_full(B, r, c);
}

// board.py:195-216: empty cells whose four neighbours are filled or off-board
inline int count_holes(uint64_t B) {
  const uint64_t n = (B << 8) | kRow0, s = (B >> 8) | kRow7;
  const uint64_t w = ((B << 1) & ~kCol0) | kCol0, e = ((B >> 1) & ~kCol7) | kCol7;
  return __builtin_popcountll(~B & n & s & w & e);
}

// numpy PCG64 (XSL-RR) + Generator.integers(0, 37) buffered Lemire draw
struct Pcg {
  u128 state, inc;
  uint32_t buf;
  bool has;
};
inline uint64_t next64(Pcg& g) {
  g.state = g.state * bb::seed::kPcgMult + g.inc;
  const uint64_t hi = (uint64_t)(g.state >> 64), lo = (uint64_t)g.state;
  const uint64_t x = hi ^ lo;
  const unsigned rot = (unsigned)(hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
inline uint32_t next32(Pcg& g) {
  if (g.has) {
    g.has = false;
    return g.buf;
  }
  const uint64_t v = next64(g);
  g.has = true;
  g.buf = (uint32_t)(v >> 32);
  return (uint32_t)v;
}
inline uint32_t draw_piece(Pcg& g) {  // pieces.py:350-355, rng_excl 37: threshold (2^32 - 37) % 37 = 7
  uint64_t m = (uint64_t)next32(g) * 37ull;
  uint32_t left = (uint32_t)m;
  if (left < 37u)
    while (left < 7u) {
      m = (uint64_t)next32(g) * 37ull;
      left = (uint32_t)m;
    }
  return (uint32_t)(m >> 32);
}

// engine.py:174-238: can all three pieces be placed in some order, with the
// line clears in between?  (Only the boolean matters.)
bool solvable(uint64_t B, const uint32_t id[3]) {
  for (int f = 0; f < 3; ++f) {
    const int y = f == 0 ? 1 : 0, z = f == 2 ? 1 : 2;
    for (uint64_t a1 = anchors_of(id[f], B); a1; a1 &= a1 - 1) {
      const uint64_t B1 = clear_full(B | (T().p[id[f]].shape << __builtin_ctzll(a1)));
      for (int o = 0; o < 2; ++o) {
        const uint32_t py = id[o ? z : y], pz = id[o ? y : z];
        for (uint64_t a2 = anchors_of(py, B1); a2; a2 &= a2 - 1) {
          const uint64_t B2 = clear_full(B1 | (T().p[py].shape << __builtin_ctzll(a2)));
          if (anchors_of(pz, B2)) return true;
        }
      }
    }
  }
  return false;
}

// Philox4x32-10 word 0 at counter (idx, step) under key seed; the synthetic policy
uint32_t philox_w0(uint64_t seed, uint64_t idx, uint64_t step) {
  uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32), c2 = (uint32_t)step, c3 = (uint32_t)(step >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  return c0;
}
int32_t policy_action(const uint64_t m[3], uint32_t u) {
  const uint32_t tot = (uint32_t)(__builtin_popcountll(m[0]) + __builtin_popcountll(m[1]) + __builtin_popcountll(m[2]));
  if (tot == 0) return 0;
  uint32_t k = (uint32_t)(((uint64_t)u * tot) >> 32);
  for (int s = 0; s < 3; ++s) {
    const uint32_t c = (uint32_t)__builtin_popcountll(m[s]);
    if (k < c) {
      uint64_t x = m[s];
      for (uint32_t q = 0; q < k; ++q) x &= x - 1;
      return 64 * s + __builtin_ctzll(x);
    }
    k -= c;
  }
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------
// handle: structure-of-arrays state like the device slab (bb_device_ptrs)
// ---------------------------------------------------------------------------
struct bb_env {
  int n = 0;
  int autoreset = 1;
  bb_reward_cfg cfg{};
  std::vector<uint64_t> board, mask, seed_hi, seed_lo;
  std::vector<uint32_t> hand;  // 3 x 6-bit ids | used << 18 | over << 21 | has_uint32 << 22
  std::vector<int64_t> score;
  std::vector<int32_t> combo, max_combo, moves, lines, blocks;
  std::vector<uint16_t> prev;  // _prev_holes | filled centre cells << 8
  std::vector<Pcg> rng;
  std::vector<uint8_t> has_seed;
  std::string err;
};

static thread_local std::string g_create_err;

namespace {

int fail(bb_env* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  else g_create_err = msg;
  return code;
}

inline uint32_t hand_id(uint32_t h, int s) { return (h >> (6 * s)) & 63u; }

void masks_of(uint64_t B, uint32_t hand, uint64_t m[3]) {  // engine.py:364-380 (status not consulted)
  for (int s = 0; s < 3; ++s) m[s] = ((hand >> (18 + s)) & 1u) ? 0ull : anchors_of(hand_id(hand, s), B);
}

// block_blast_env.py:195-222 -> engine.py:127-153: re-seed with seed_value when
// there is one, clear, first hand (every hand fits an empty board: no search)
void reset_env(bb_env* e, int i) {
  Pcg& g = e->rng[i];
  if (e->has_seed[i]) {
    g.state = ((u128)e->seed_hi[i] << 64) | e->seed_lo[i];
    g.buf = 0;
    g.has = false;
  }
  const uint32_t a = draw_piece(g), b = draw_piece(g), c = draw_piece(g);
  e->board[i] = 0;
  e->hand[i] = a | (b << 6) | (c << 12) | ((uint32_t)g.has << 22);
  e->score[i] = 0;
  e->combo[i] = e->max_combo[i] = e->moves[i] = e->lines[i] = e->blocks[i] = 0;
  e->prev[i] = 0;  // _prev_holes = 0, _prev_center_openness = 1.0
  masks_of(0, e->hand[i], &e->mask[3 * (size_t)i]);
}

struct Out {
  double reward;
  bool term, valid;
  int lines;
};

// One env step (block_blast_env.py:224-264 with engine.make_move,
// engine.py:390-454) plus the vec env's auto-reset (wrappers.py:97-102).
Out step_env(bb_env* e, int i, int act, bb_info* info, int64_t* final_score, int32_t* final_moves) {
  Out o{-10.0, false, false, 0};  // invalid action (block_blast_env.py:240-245): no state change
  uint64_t B = e->board[i];
  uint32_t hand = e->hand[i];
  const int p = act >> 6, cell = act & 63;
  const uint32_t used = (hand >> 18) & 7u;
  bool valid = act >= 0 && act < 192 && !((hand >> 21) & 1u) && !((used >> p) & 1u);
  const Piece* pc = nullptr;
  if (valid) {
    pc = &T().p[hand_id(hand, p)];
    valid = ((pc->anchors >> cell) & 1ull) && ((pc->shape << cell) & B) == 0;
  }
  int nblk = 0, lines = 0, cm = 1, holes = 0;
  int64_t gained = 0;
  if (valid) {
    nblk = pc->n;
    e->moves[i] += 1;
    e->blocks[i] += nblk;
    int rows, cols;
    B = clear_full(B | (pc->shape << cell), rows, cols);
    lines = rows + cols;
    if (lines > 0) {
      e->combo[i] += 1;
      if (e->combo[i] > e->max_combo[i]) e->max_combo[i] = e->combo[i];
      e->lines[i] += lines;
      cm = lines < 4 ? lines : 4;
      const int streak = e->combo[i] + 1 < 8 ? e->combo[i] + 1 : 8;  // post-increment combo (engine.py:261)
      gained = nblk + (int64_t)(lines * 8 * 10) * cm * streak;         // blocks_in_lines = lines*8 (engine.py:427)
    } else {
      e->combo[i] = 0;
      gained = nblk;
    }
    e->score[i] += gained;
    const uint32_t nu = used | (1u << p);
    if (nu == 7u) {  // engine.py:432-437 -> _generate_new_pieces (155-172)
      Pcg& g = e->rng[i];
      uint32_t id[3] = {0, 0, 0};
      for (int attempt = 0; attempt < 100; ++attempt) {
        id[0] = draw_piece(g);
        id[1] = draw_piece(g);
        id[2] = draw_piece(g);
        if (solvable(B, id)) break;  // after 100 failures the last draw stays (engine.py:171-172)
      }
      hand = id[0] | (id[1] << 6) | (id[2] << 12) | ((uint32_t)g.has << 22);
    } else {
      hand = (hand & 0x3FFFFu) | (nu << 18) | (hand & (1u << 22));
    }
    uint64_t m[3];
    masks_of(B, hand, m);
    const bool over = (m[0] | m[1] | m[2]) == 0ull;  // engine.py:440-441
    if (over) hand |= 1u << 21;
    // _calculate_reward (block_blast_env.py:158-193), fp64 in the reference's order
    const bb_reward_cfg& c = e->cfg;
    double R = 0.0;
    R += (double)nblk * c.block_placed;
    R += c.survival_bonus;
    if (lines > 0) {
      double lr = (double)lines * c.line_clear_base;
      lr *= (double)cm;
      R += lr;
      if (cm > 1) R += (double)(cm - 1) * c.combo_multiplier_bonus;
    }
    if (over) R += c.game_over_penalty;
    holes = count_holes(B);
    const int dh = holes - (int)(e->prev[i] & 0xFFu);
    if (dh > 0) R += (double)dh * c.hole_penalty;
    const int center = __builtin_popcountll(B & kCenter);
    if (center <= (int)(e->prev[i] >> 8)) R += c.center_bonus * 0.1;  // openness >= previous
    e->prev[i] = (uint16_t)(holes | (center << 8));
    e->board[i] = B;
    e->hand[i] = hand;
    memcpy(&e->mask[3 * (size_t)i], m, sizeof(m));
    o = Out{R, over, true, lines};
  } else if (info) {
    holes = count_holes(B);
  }
  if (info) {  // block_blast_env.py:266-288: after the move, before any auto-reset
    bb_info& f = info[i];
    f.score = e->score[i];
    f.score_gained = gained;
    f.term_board = e->board[i];
    f.moves = e->moves[i];
    f.lines = e->lines[i];
    f.max_combo = e->max_combo[i];
    f.blocks = e->blocks[i];
    f.term_hand = e->hand[i];
    f.holes = (uint8_t)holes;
    f.filled = (uint8_t)__builtin_popcountll(e->board[i]);
    f.flags = (uint8_t)((valid ? 4u : 1u) | (o.term ? 2u : 0u));
    f.last_blocks = (uint8_t)nblk;
    f.last_lines = (uint8_t)lines;
    f.last_cm = (uint8_t)cm;
    f.pad[0] = f.pad[1] = 0;
  }
  if (o.term) {
    if (final_score) final_score[i] = e->score[i];
    if (final_moves) final_moves[i] = e->moves[i];
    if (e->autoreset) reset_env(e, i);
  }
  return o;
}

}  // namespace

#ifndef BB_BUILD_ID
#define BB_BUILD_ID "unhashed"
#endif
static const char kBuildIdMarker[] = "bbvec-build-id:" BB_BUILD_ID;  // runtime/build.py host_source_id

extern "C" {

int bb_abi_version(void) { return BB_ABI_VERSION; }

const char* bb_build_id(void) { return kBuildIdMarker + 15; }

const char* bb_last_error(const bb_env* env) { return env ? env->err.c_str() : g_create_err.c_str(); }

int32_t bb_num_envs(const bb_env* env) { return env ? env->n : 0; }

int bb_pcg64_seed(uint64_t seed, uint64_t out[4]) {
  if (!out) return BB_ERR_ARG;
  bb::seed::pcg64_seed_numpy(seed, out);
  return BB_OK;
}

int bb_create(int32_t num_envs, int32_t device, const bb_reward_cfg* cfg, int32_t autoreset, bb_env** out) {
  (void)device;  // the host backend has no devices
  if (!out) return fail(nullptr, BB_ERR_ARG, "bb_create: out is NULL");
  *out = nullptr;
  if (num_envs <= 0) return fail(nullptr, BB_ERR_ARG, "bb_create: num_envs must be positive");
  if (!cfg) return fail(nullptr, BB_ERR_ARG, "bb_create: reward config is NULL");
  bb_env* e = new bb_env();
  const size_t n = (size_t)num_envs;
  e->n = num_envs;
  e->autoreset = autoreset ? 1 : 0;
  e->cfg = *cfg;
  e->board.assign(n, 0);
  e->mask.assign(3 * n, 0);
  e->seed_hi.assign(n, 0);
  e->seed_lo.assign(n, 0);
  e->hand.assign(n, 0);
  e->score.assign(n, 0);
  e->combo.assign(n, 0);
  e->max_combo.assign(n, 0);
  e->moves.assign(n, 0);
  e->lines.assign(n, 0);
  e->blocks.assign(n, 0);
  e->prev.assign(n, 0);
  e->rng.assign(n, Pcg{0, 1, 0, false});
  e->has_seed.assign(n, 0);
  *out = e;
  return BB_OK;
}

void bb_destroy(bb_env* env) { delete env; }

int bb_seed(bb_env* env, const uint64_t* h_seeds, const uint8_t* h_has_seed, const uint64_t* h_raw) {
  if (!env) return BB_ERR_ARG;
  if (!h_has_seed) return fail(env, BB_ERR_ARG, "bb_seed: has_seed is NULL");
  for (int i = 0; i < env->n; ++i) {
    uint64_t w[4];
    if (h_has_seed[i] == 1) {
      if (!h_seeds) return fail(env, BB_ERR_ARG, "bb_seed: seeds is NULL");
      bb::seed::pcg64_seed_numpy(h_seeds[i], w);
    } else {
      if (!h_raw) return fail(env, BB_ERR_ARG, "bb_seed: raw state is NULL");
      for (int k = 0; k < 4; ++k) w[k] = h_raw[4 * (size_t)i + k];
      w[3] |= 1ull;  // PCG increments are odd
    }
    env->has_seed[i] = h_has_seed[i] ? 1 : 0;
    env->seed_hi[i] = w[0];
    env->seed_lo[i] = w[1];
    env->rng[i] = Pcg{((u128)w[0] << 64) | w[1], ((u128)w[2] << 64) | w[3], 0, false};
    env->hand[i] = 0;
  }
  return BB_OK;
}

int bb_reset(bb_env* env, const uint8_t* d_env_mask, void* stream) {
  (void)stream;
  if (!env) return BB_ERR_ARG;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < env->n; ++i) {
    if (d_env_mask && !d_env_mask[i]) continue;
    env->rng[i].has = (env->hand[i] >> 22) & 1u;
    reset_env(env, i);
  }
  return BB_OK;
}

int bb_step(bb_env* env, const int32_t* d_actions, const bb_step_out* out, void* stream) {
  (void)stream;
  if (!env) return BB_ERR_ARG;
  if (!d_actions || !out || !out->reward || !out->terminated)
    return fail(env, BB_ERR_ARG, "bb_step: actions, reward and terminated are required");
#pragma omp parallel for schedule(dynamic, 256)
  for (int i = 0; i < env->n; ++i) {
    const Out o = step_env(env, i, d_actions[i], out->info, out->final_score, out->final_moves);
    out->reward[i] = (float)o.reward;
    out->terminated[i] = o.term ? 1 : 0;
    if (out->reward_f64) out->reward_f64[i] = o.reward;
    if (out->lines) out->lines[i] = (uint8_t)o.lines;
    const uint64_t* m = &env->mask[3 * (size_t)i];
    if (out->mask) memcpy(&out->mask[3 * (size_t)i], m, 24);
    if (out->next_action)
      out->next_action[i] = policy_action(m, philox_w0(out->policy_seed, out->env_offset + (uint64_t)i, out->policy_step));
  }
  return BB_OK;
}

int bb_rollout(bb_env* env, int32_t steps, const int32_t* d_actions, const bb_rollout_out* out, void* stream) {
  (void)stream;
  if (!env) return BB_ERR_ARG;
  if (steps < 0) return fail(env, BB_ERR_ARG, "bb_rollout: steps must be >= 0");
  if (!d_actions || !out || !out->reward || !out->terminated)
    return fail(env, BB_ERR_ARG, "bb_rollout: actions, reward and terminated are required");
  const size_t n = (size_t)env->n;
#pragma omp parallel for schedule(dynamic, 64)
  for (int i = 0; i < env->n; ++i) {
    int32_t a = d_actions[i];
    for (int t = 0; t < steps; ++t) {
      const Out o = step_env(env, i, a, nullptr, nullptr, nullptr);
      const size_t k = (size_t)t * n + (size_t)i;
      out->reward[k] = (float)o.reward;
      out->terminated[k] = o.term ? 1 : 0;
      if (out->lines) out->lines[k] = (uint8_t)o.lines;
      if (out->actions) out->actions[k] = a;
      const uint64_t* m = &env->mask[3 * (size_t)i];
      if (out->mask) memcpy(&out->mask[3 * k], m, 24);
      a = policy_action(m, philox_w0(out->policy_seed, out->env_offset + (uint64_t)i,
                                     out->policy_step0 + (uint64_t)t + 1));
    }
    if (out->next_action && steps > 0) out->next_action[i] = a;
  }
  return BB_OK;
}

// every call runs to completion on the calling thread, and no loop here is bounded by a cap: nothing to report
int bb_sync(bb_env* env, void* stream) {
  (void)stream;
  return env ? BB_OK : BB_ERR_ARG;
}

// engine.py:478-507 / wrappers.py:118-126: board plane + unused pieces' shapes at
// the origin, f32 [N][4][8][8]; masks as int8 / f32 [N][192] and bits [N][3]
int bb_obs(bb_env* env, float* d_x, int8_t* d_mask_i8, float* d_mask_f32, uint64_t* d_mask_bits, void* stream) {
  (void)stream;
  if (!env) return BB_ERR_ARG;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < env->n; ++i) {
    const uint64_t* m = &env->mask[3 * (size_t)i];
    if (d_x) {
      float* x = d_x + (size_t)i * 256;
      const uint32_t h = env->hand[i];
      for (int pl = 0; pl < 4; ++pl) {
        const uint64_t v = pl == 0 ? env->board[i]
                                   : (((h >> (17 + pl)) & 1u) ? 0ull : T().p[hand_id(h, pl - 1)].shape);
        for (int b = 0; b < 64; ++b) x[64 * pl + b] = (float)((v >> b) & 1ull);
      }
    }
    for (int a = 0; a < 192; ++a) {
      const int bit = (int)((m[a >> 6] >> (a & 63)) & 1ull);
      if (d_mask_i8) d_mask_i8[(size_t)i * 192 + a] = (int8_t)bit;
      if (d_mask_f32) d_mask_f32[(size_t)i * 192 + a] = (float)bit;
    }
    if (d_mask_bits) memcpy(&d_mask_bits[3 * (size_t)i], m, 24);
  }
  return BB_OK;
}

int bb_device_ptrs(bb_env* env, uint64_t** d_board, uint32_t** d_hand, uint64_t** d_mask) {
  if (!env) return BB_ERR_ARG;
  if (d_board) *d_board = env->board.data();
  if (d_hand) *d_hand = env->hand.data();
  if (d_mask) *d_mask = env->mask.data();
  return BB_OK;
}

int bb_snapshot(bb_env* env, uint64_t* d_board, uint32_t* d_hand, uint64_t* d_mask_bits, void* stream) {
  (void)stream;
  if (!env) return BB_ERR_ARG;
  const size_t n = (size_t)env->n;
  if (d_board) memcpy(d_board, env->board.data(), n * 8);
  if (d_hand) memcpy(d_hand, env->hand.data(), n * 4);
  if (d_mask_bits) memcpy(d_mask_bits, env->mask.data(), n * 24);
  return BB_OK;
}

int bb_get_state(bb_env* env, const bb_state_view* v) {
  if (!env || !v) return BB_ERR_ARG;
  const size_t n = (size_t)env->n;
  if (v->board) memcpy(v->board, env->board.data(), n * 8);
  if (v->hand) memcpy(v->hand, env->hand.data(), n * 4);
  if (v->score) memcpy(v->score, env->score.data(), n * 8);
  if (v->combo) memcpy(v->combo, env->combo.data(), n * 4);
  if (v->max_combo) memcpy(v->max_combo, env->max_combo.data(), n * 4);
  if (v->moves) memcpy(v->moves, env->moves.data(), n * 4);
  if (v->lines) memcpy(v->lines, env->lines.data(), n * 4);
  if (v->blocks) memcpy(v->blocks, env->blocks.data(), n * 4);
  for (size_t i = 0; i < n; ++i) {
    if (v->prev_holes) v->prev_holes[i] = (uint8_t)(env->prev[i] & 0xFF);
    if (v->prev_center) v->prev_center[i] = (uint8_t)(env->prev[i] >> 8);
    if (v->rng) {
      v->rng[3 * i] = (uint64_t)(env->rng[i].state >> 64);
      v->rng[3 * i + 1] = (uint64_t)env->rng[i].state;
      v->rng[3 * i + 2] = env->rng[i].buf;
    }
  }
  return BB_OK;
}

int bb_set_state(bb_env* env, const bb_state_view* v) {
  if (!env || !v) return BB_ERR_ARG;
  const size_t n = (size_t)env->n;
  if (v->board) memcpy(env->board.data(), v->board, n * 8);
  if (v->hand) memcpy(env->hand.data(), v->hand, n * 4);
  if (v->score) memcpy(env->score.data(), v->score, n * 8);
  if (v->combo) memcpy(env->combo.data(), v->combo, n * 4);
  if (v->max_combo) memcpy(env->max_combo.data(), v->max_combo, n * 4);
  if (v->moves) memcpy(env->moves.data(), v->moves, n * 4);
  if (v->lines) memcpy(env->lines.data(), v->lines, n * 4);
  if (v->blocks) memcpy(env->blocks.data(), v->blocks, n * 4);
  for (size_t i = 0; i < n; ++i) {
    const uint16_t h = v->prev_holes ? v->prev_holes[i] : (uint16_t)(env->prev[i] & 0xFF);
    const uint16_t c = v->prev_center ? v->prev_center[i] : (uint16_t)(env->prev[i] >> 8);
    env->prev[i] = (uint16_t)(h | (c << 8));
    if (v->rng) {
      env->rng[i].state = ((u128)v->rng[3 * i] << 64) | v->rng[3 * i + 1];
      env->rng[i].buf = (uint32_t)v->rng[3 * i + 2];
    }
    env->rng[i].has = (env->hand[i] >> 22) & 1u;
    masks_of(env->board[i], env->hand[i], &env->mask[3 * i]);  // derived state
  }
  return BB_OK;
}

int bb_random_actions(const uint64_t* d_mask_bits, int32_t n, uint64_t seed, uint64_t step, uint64_t env_offset,
                      int32_t* d_actions, void* stream) {
  (void)stream;
  if (!d_mask_bits || !d_actions || n < 0) return fail(nullptr, BB_ERR_ARG, "bb_random_actions: bad arguments");
  for (int32_t i = 0; i < n; ++i)
    d_actions[i] = policy_action(&d_mask_bits[3 * (size_t)i], philox_w0(seed, env_offset + (uint64_t)i, step));
  return BB_OK;
}

}  // extern "C"

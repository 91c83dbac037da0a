// bb_env.hip -- MI355X (gfx950) vectorised Block Blast environment.
//
// Per-env state lives in HBM as structure-of-arrays (coalesced 2/4/8-byte
// columns); the 37-piece table, the |D| pair table and the PCG64 jump-ahead
// table are staged into LDS once per workgroup.  The kernels:
//   rollout_async_kernel -- bb_rollout (T >= 2 steps per launch, the bench and
//                      BASELINE config 2): env waves step 64 envs each, one per
//                      lane, with the state in VGPRs; search waves of the same
//                      workgroup run the hand searches the in-lane quick test
//                      leaves open.
//   step_fused_kernel -- bb_step in one launch (two lanes per env, searches in
//                      the wave): the path under the Gym surface and the
//                      trainer's rollout (one step between CNN forwards).
//   step_kernel + escalate_kernel -- the same step as two launches (per-lane
//                      step, then wave-cooperative searches of the parked
//                      envs): BB_STEP_KERNELS=2 and the diagnostic modes
//                      (BB_DEBUG_MODE, BB_LANE_BUDGET, BB_LANE_QUICK).
//   reset / observation expansion / mask refresh / random policy kernels.
//
// Reference semantics: src/environment/wrappers.py:75-116 (vec step, auto-reset)
// -> src/environment/block_blast_env.py:224-264 (step, invalid action, reward
// 148-193) -> src/game/engine.py:390-454 (make_move) and board.py.
#include <hip/hip_runtime.h>

#include "bb_device.h"
#include "bb_env_internal.h"
#include "bb_solver.h"

namespace bb {

#ifndef BB_STEP_BLOCK
#define BB_STEP_BLOCK 128
#endif
constexpr int kStepBlock = BB_STEP_BLOCK;
#ifndef BB_ESC_BLOCK
#define BB_ESC_BLOCK 256
#endif
constexpr int kEscBlock = BB_ESC_BLOCK;
#ifndef BB_ESC_GROUP
#define BB_ESC_GROUP 32  // with the multi-env search: 8 -> 32 took the step tail from 71 to 68 us
#endif
constexpr int kEscGroup = BB_ESC_GROUP;  // envs owned by one escalation wave (< 64)
static_assert(kEscGroup > 0 && kEscGroup < 64, "gen_hands_multi masks (1 << kEnvs) - 1");

constexpr int kDPad = (kPieces * kPieces + 15) / 16 * 16;  // |D| table padded to whole 16-byte vectors

struct alignas(16) Tables {
  PieceRow row[kPieces];
  alignas(16) uint8_t d[kDPad];
};
static_assert(sizeof(PieceRow) % 8 == 0, "PieceRow staged as 8-byte vectors");

// Global -> LDS copy of the piece rows (8-byte vectors: a row stride of an odd number of 8-byte words
// spreads the lanes' per-piece reads over every LDS bank) and of the |D| table (and, for the kernels that
// run hand searches, the PCG64 jump-ahead table) as 16-byte vectors: every load of a thread is issued
// before its first LDS store, so the staging costs one memory latency (byte-wise copying cost ~22 serial
// ones).  The device buffers are padded (slab carving rounds to 256 bytes).
constexpr int kJumpVec = (kJumpMax + 1) * (int)sizeof(JumpRow) / 16;
static_assert(sizeof(JumpRow) % 16 == 0, "JumpRow staged as 16-byte vectors");

template <bool kWithJump = false>
__device__ __forceinline__ void stage_tables(Tables& t, const PieceRow* g_rows, const uint8_t* g_d,
                                             JumpRow* jt = nullptr, const JumpRow* g_jump = nullptr) {
  constexpr int kRow8 = kPieces * (int)sizeof(PieceRow) / 8;
  constexpr int kTabVec = kDPad / 16;
  constexpr int kTot = kTabVec + (kWithJump ? kJumpVec : 0);
  constexpr int kPer = (kTot + 63) / 64;
  constexpr int kPer8 = (kRow8 + 63) / 64;
  const int tid = threadIdx.x;
  const int nthr = (int)blockDim.x;
  // one source / destination address per vector (a single select each), so the
  // staged values stay in registers (a pointer select per load put them in scratch)
  uint2 w[kPer8];
#pragma unroll
  for (int k = 0; k < kPer8; ++k) {
    const int idx = tid + k * nthr;
    w[k] = reinterpret_cast<const uint2*>(g_rows)[idx < kRow8 ? idx : 0];
  }
  uint4 v[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int idx = tid + k * nthr;
    const int j = idx < kTot ? idx : 0;
    const char* src = j < kTabVec ? reinterpret_cast<const char*>(g_d) + 16 * j
                                  : reinterpret_cast<const char*>(g_jump) + 16 * (j - kTabVec);
    v[k] = *reinterpret_cast<const uint4*>(src);
  }
#pragma unroll
  for (int k = 0; k < kPer8; ++k) {
    const int idx = tid + k * nthr;
    if (idx < kRow8) reinterpret_cast<uint2*>(t.row)[idx] = w[k];
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int idx = tid + k * nthr;
    if (idx < kTot) {
      char* dst = idx < kTabVec ? reinterpret_cast<char*>(t.d) + 16 * idx
                                : reinterpret_cast<char*>(jt) + 16 * (idx - kTabVec);
      *reinterpret_cast<uint4*>(dst) = v[k];
    }
  }
  __syncthreads();
}

// Every lane gets lane (l mod 32)'s value: v_permlane32_swap(x, x) moves lanes 0-31 of the source into
// lanes 32-63 of the destination and leaves lanes 0-31 in place.
__device__ __forceinline__ uint32_t lower_half_bcast(uint32_t x) {
  return __builtin_amdgcn_permlane32_swap(x, x, false, false)[0];
}


__device__ __forceinline__ void masks_of(const Tables& t, uint64_t B, uint32_t hand, uint64_t m[3]) {
  const uint32_t used = hand_used(hand);
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    m[s] = (used >> s) & 1u ? 0ull : anchors_of(t.row[hand_id(hand, s)], B);
  }
}

// Everything the finalisation of one env's step needs.
struct StepCtx {
  int i;
  bool valid;
  bool drew;
  uint64_t B;
  uint32_t hand;  // ids | used | has_uint32 (over bit set by finalize)
  int64_t score;
  int32_t combo, max_combo, moves, lines_tot, blocks;
  uint32_t prev;
  int nblk, lines, cm;
  int64_t gained;
  Pcg rng;  // inc always valid; state valid when drew (or loaded for reset)
  uint64_t seed_hi, seed_lo;
  bool has_seed;
};

// pending-record packing: attempt | nblk << 8 | lines << 16 | cm << 24 | gained << 32
__device__ __forceinline__ uint64_t pack_pending(int attempt, int nblk, int lines, int cm, int64_t gained) {
  return (uint64_t)attempt | ((uint64_t)nblk << 8) | ((uint64_t)lines << 16) | ((uint64_t)cm << 24) |
         ((uint64_t)(uint32_t)gained << 32);
}

// Validity check and make_move of one lane's action (block_blast_env.py:237-245
// -> engine.py:326-346 can_place_piece, 406-429 place / clear / score).  On a
// legal move that used the last slot, returns true with s.drew set and the
// used bits cleared: the caller draws the new hand (engine.py:432-437).
__device__ __forceinline__ bool apply_move(const Tables& t, StepCtx& s, int act) {
  s.drew = false;
  s.nblk = 0;
  s.lines = 0;
  s.cm = 1;
  s.gained = 0;
  const int p = act >> 6;     // a // 64 for a >= 0
  const int cell = act & 63;  // r*8 + c
  uint32_t used = hand_used(s.hand);
  bool valid = act >= 0 && act < 192 && !hand_over(s.hand) && !((used >> p) & 1u);
  PieceRow pr{};
  if (valid) {
    pr = t.row[hand_id(s.hand, p)];
    valid = ((pr.anchors >> cell) & 1ull) && ((pr.shape << cell) & s.B) == 0;
  }
  s.valid = valid;
  if (!valid) return false;
  s.nblk = (int)ncells_of(pr);
  used |= 1u << p;
  s.moves += 1;
  s.blocks += s.nblk;
  int rows, cols;
  s.B = clear_full(s.B | (pr.shape << cell), rows, cols);
  s.lines = rows + cols;
  if (s.lines > 0) {
    s.combo += 1;
    s.max_combo = s.combo > s.max_combo ? s.combo : s.max_combo;
    s.lines_tot += s.lines;
    s.cm = s.lines < 4 ? s.lines : 4;
    const int streak = s.combo + 1 < 8 ? s.combo + 1 : 8;  // post-increment combo (engine.py:261)
    s.gained = s.nblk + (int64_t)(s.lines * 8 * 10) * s.cm * streak;  // blocks_in_lines = lines*8 (engine.py:427)
  } else {
    s.combo = 0;
    s.gained = s.nblk;
  }
  s.score += s.gained;
  if (used == 7u) {
    s.drew = true;
    s.hand &= ~(7u << 18);
    return true;
  }
  s.hand = (s.hand & 0x3FFFFu) | (used << 18) | (s.hand & (1u << 22));
  return false;
}

// apply_move without branches (the rollout kernel): every quantity is computed
// for the lane's action and committed by select, so the move is one basic
// block the scheduler can interleave with the step's other independent work.
// Same results as apply_move for every action, legal or not.
__device__ __forceinline__ bool apply_move_bf(const Tables& t, StepCtx& s, int act) {
  const bool inrange = (unsigned)act < 192u;
  const int p = inrange ? (act >> 6) : 0;
  const int cell = act & 63;
  const uint32_t used0 = hand_used(s.hand);
  const PieceRow& pr = t.row[hand_id(s.hand, p)];
  const uint64_t placed = pr.shape << cell;
  const bool valid = inrange && !hand_over(s.hand) && !((used0 >> p) & 1u) && ((pr.anchors >> cell) & 1ull) &&
                     (placed & s.B) == 0ull;
  const int nblk = (int)ncells_of(pr);
  int rows, cols;
  const uint64_t B2 = clear_full(s.B | placed, rows, cols);
  const int lines = rows + cols;
  const int combo1 = s.combo + 1;
  const int cm = lines < 4 ? lines : 4;
  const int streak = combo1 + 1 < 8 ? combo1 + 1 : 8;  // post-increment combo (engine.py:261)
  const int64_t gained = lines > 0 ? nblk + (int64_t)(lines * 8 * 10) * cm * streak : (int64_t)nblk;
  const bool clr = valid && lines > 0;
  s.valid = valid;
  s.nblk = valid ? nblk : 0;
  s.lines = valid ? lines : 0;
  s.cm = clr ? cm : 1;
  s.gained = valid ? gained : 0;
  s.B = valid ? B2 : s.B;
  s.moves += valid ? 1 : 0;
  s.blocks += valid ? nblk : 0;
  s.max_combo = clr && combo1 > s.max_combo ? combo1 : s.max_combo;
  s.combo = valid ? (lines > 0 ? combo1 : 0) : s.combo;
  s.lines_tot += valid ? lines : 0;
  s.score += valid ? gained : 0;
  const uint32_t used = used0 | (1u << p);
  const bool drew = valid && used == 7u;
  s.drew = drew;
  s.hand = !valid ? s.hand
                  : (drew ? (s.hand & ~(7u << 18)) : ((s.hand & 0x3FFFFu) | (used << 18) | (s.hand & (1u << 22))));
  return drew;
}

// ---------------------------------------------------------------------------
// reset: engine.py:127-153 + block_blast_env.py:210-217
// ---------------------------------------------------------------------------
__device__ __forceinline__ void reset_lane(const Tables& t, bool has_seed, uint64_t seed_hi, uint64_t seed_lo,
                                           Pcg& rng, uint64_t& B, uint32_t& hand, uint64_t m[3]) {
  if (has_seed) {  // re-seed with seed_value every episode
    rng.hi = seed_hi;
    rng.lo = seed_lo;
    rng.buf = 0;
    rng.has = 0u;
  }
  B = 0;
  // Every one of the 37^3 hands fits an empty board (checked exhaustively
  // against the reference DFS in tests/test_solver_bounds.py), so the first
  // attempt of _generate_new_pieces always succeeds: three draws, no search.
  const uint32_t a0 = draw_piece(rng);
  const uint32_t a1 = draw_piece(rng);
  const uint32_t a2 = draw_piece(rng);
  hand = hand_pack(a0, a1, a2, 0u, false, rng.has);
  masks_of(t, B, hand, m);
}

__device__ __forceinline__ void store_reset(const EnvDev& e, int i, const Pcg& rng, uint32_t hand,
                                            const uint64_t m[3]) {
  e.board[i] = 0ull;
  e.hand[i] = hand;
  e.rng_hi[i] = rng.hi;
  e.rng_lo[i] = rng.lo;
  e.rng_buf[i] = rng.buf;
  e.score[i] = 0;
  e.combo[i] = 0;
  e.max_combo[i] = 0;
  e.moves[i] = 0;
  e.lines[i] = 0;
  e.blocks[i] = 0;
  e.prev[i] = 0;  // _prev_holes = 0, _prev_center_openness = 1.0 (0 centre cells filled)
  e.mask[3 * i + 0] = m[0];
  e.mask[3 * i + 1] = m[1];
  e.mask[3 * i + 2] = m[2];
}

// _calculate_reward of a legal move (block_blast_env.py:158-193): fp64 in the
// reference's exact operation order.  holes / center: the post-move values
// that become _prev_holes / the filled-centre count.
__device__ __forceinline__ double move_reward(const StepCtx& s, const StepArgs& a, bool over, int& holes,
                                              int& center) {
  double R = 0.0;
  R = __dadd_rn(R, __dmul_rn((double)s.nblk, a.cfg.block_placed));
  R = __dadd_rn(R, a.cfg.survival_bonus);
  if (s.lines > 0) {
    double lr = __dmul_rn((double)s.lines, a.cfg.line_clear_base);
    lr = __dmul_rn(lr, (double)s.cm);
    R = __dadd_rn(R, lr);
    if (s.cm > 1) R = __dadd_rn(R, __dmul_rn((double)(s.cm - 1), a.cfg.combo_multiplier_bonus));
  }
  if (over) R = __dadd_rn(R, a.cfg.game_over_penalty);
  holes = count_holes(s.B);
  const int dh = holes - (int)(s.prev & 0xFFu);
  if (dh > 0) R = __dadd_rn(R, __dmul_rn((double)dh, a.cfg.hole_penalty));
  center = __popcll(s.B & kCenter);
  if (center <= (int)(s.prev >> 8)) R = __dadd_rn(R, a.center_tenth);  // openness >= previous
  return R;
}

// ---------------------------------------------------------------------------
// finalize: game over, shaped reward, info, auto-reset, mask, policy, stores
// ---------------------------------------------------------------------------
__device__ __forceinline__ void finalize(const Tables& t, const EnvDev& e, StepCtx& s, const StepArgs& a) {
  const int i = s.i;
  const bool fprof = (a.dbg & 8) != 0;  // diagnostics: finalize sub-phase timestamps
  const uint64_t F0 = fprof ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t m[3];
  masks_of(t, s.B, s.hand, m);
  const uint64_t F1 = fprof ? __builtin_amdgcn_s_memtime() : 0;
  double rew = -10.0;  // invalid action (block_blast_env.py:240-245)
  bool term = false;
  int holes = 0, center = 0;
  if (s.valid) {
    const bool over = (m[0] | m[1] | m[2]) == 0ull;  // engine.py:440-441
    if (over) s.hand |= 1u << 21;
    rew = move_reward(s, a, over, holes, center);
    term = over;
  } else if (a.info) {
    holes = count_holes(s.B);
  }

  const uint64_t F2 = fprof ? __builtin_amdgcn_s_memtime() : 0;
  if (a.info) {
    bb_info inf;
    inf.score = s.score;
    inf.score_gained = s.gained;
    inf.term_board = s.B;
    inf.moves = s.moves;
    inf.lines = s.lines_tot;
    inf.max_combo = s.max_combo;
    inf.blocks = s.blocks;
    inf.term_hand = s.hand;
    inf.holes = (uint8_t)holes;
    inf.filled = (uint8_t)__popcll(s.B);
    inf.flags = (uint8_t)((s.valid ? 4u : 1u) | (term ? 2u : 0u));
    inf.last_blocks = (uint8_t)s.nblk;
    inf.last_lines = (uint8_t)s.lines;
    inf.last_cm = (uint8_t)s.cm;
    inf.pad[0] = inf.pad[1] = 0;
    a.info[i] = inf;
  }
  a.reward[i] = (float)rew;
  a.terminated[i] = term ? 1 : 0;
  if (a.reward_f64) a.reward_f64[i] = rew;
  if (a.lines) a.lines[i] = (uint8_t)s.lines;
  if (term) {  // info['final_score'] / info['moves'] of the ending episode (wrappers.py:97-101)
    if (a.final_score) a.final_score[i] = s.score;
    if (a.final_moves) a.final_moves[i] = s.moves;
  }

  const uint64_t F3 = fprof ? __builtin_amdgcn_s_memtime() : 0;
  if (term && a.autoreset) {
    // wrappers.py:97-102: env.reset() with the stored seed_value
    uint64_t B;
    uint32_t hand;
    reset_lane(t, s.has_seed, s.seed_hi, s.seed_lo, s.rng, B, hand, m);
    store_reset(e, i, s.rng, hand, m);
  } else if (s.valid) {
    e.board[i] = s.B;
    e.hand[i] = s.hand;
    if (s.drew) {
      e.rng_hi[i] = s.rng.hi;
      e.rng_lo[i] = s.rng.lo;
      e.rng_buf[i] = s.rng.buf;
    }
    e.score[i] = s.score;
    e.combo[i] = s.combo;
    e.max_combo[i] = s.max_combo;
    e.moves[i] = s.moves;
    e.lines[i] = s.lines_tot;
    e.blocks[i] = s.blocks;
    e.prev[i] = (uint16_t)(holes | (center << 8));
    e.mask[3 * i + 0] = m[0];
    e.mask[3 * i + 1] = m[1];
    e.mask[3 * i + 2] = m[2];
  }
  const uint64_t F4 = fprof ? __builtin_amdgcn_s_memtime() : 0;
  if (a.mask_out) {
    a.mask_out[3 * i + 0] = m[0];
    a.mask_out[3 * i + 1] = m[1];
    a.mask_out[3 * i + 2] = m[2];
  }
  if (a.next_action) {
    a.next_action[i] = random_policy(m[0], m[1], m[2], a.policy_seed, a.env_offset + (uint64_t)i, a.policy_step);
  }
  if (fprof) {
    const uint64_t F5 = __builtin_amdgcn_s_memtime();
    a.dbg_out[4 * i + 2] = (F1 - F0) | ((F2 - F1) << 16) | ((F3 - F2) << 32) | ((F4 - F3) << 48);
    a.dbg_out[4 * i + 3] = (F5 - F4) | ((uint64_t)(term ? 1 : 0) << 32);
  }
}

__global__ void __launch_bounds__(kStepBlock) reset_kernel(EnvDev e, const PieceRow* g_rows, const uint8_t* g_d,
                                                           const uint8_t* sel) {
  __shared__ Tables t;
  stage_tables(t, g_rows, g_d);
  const int i = blockIdx.x * kStepBlock + threadIdx.x;
  if (i >= e.n) return;
  if (sel && !sel[i]) return;
  const uint32_t h0 = e.hand[i];
  Pcg rng;
  rng.hi = e.rng_hi[i];
  rng.lo = e.rng_lo[i];
  rng.inc_hi = e.inc_hi[i];
  rng.inc_lo = e.inc_lo[i];
  rng.buf = e.rng_buf[i];
  rng.has = hand_has32(h0);
  uint64_t B;
  uint32_t hand;
  uint64_t m[3];
  reset_lane(t, e.has_seed[i] != 0, e.seed_hi[i], e.seed_lo[i], rng, B, hand, m);
  store_reset(e, i, rng, hand, m);
  e.pend[i] = 0;
}

// ---------------------------------------------------------------------------
// step
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kStepBlock) step_kernel(EnvDev e, const PieceRow* g_rows, const uint8_t* g_d,
                                                          const int32_t* __restrict__ actions, StepArgs a) {
  __shared__ Tables t;
  const bool prof = (a.dbg & 4) != 0;  // diagnostics: phase timestamps
  const uint64_t T0 = prof ? __builtin_amdgcn_s_memtime() : 0;
  const int i = blockIdx.x * kStepBlock + threadIdx.x;
  const bool live = i < e.n;
  // ---- every column up front (in flight while the tables are staged) ------
  StepCtx s;
  int act = -1;
  if (live) {
    s.i = i;
    act = actions[i];
    s.B = e.board[i];
    s.hand = e.hand[i];
    s.score = e.score[i];
    s.combo = e.combo[i];
    s.max_combo = e.max_combo[i];
    s.moves = e.moves[i];
    s.lines_tot = e.lines[i];
    s.blocks = e.blocks[i];
    s.prev = e.prev[i];
    s.rng.hi = e.rng_hi[i];
    s.rng.lo = e.rng_lo[i];
    s.rng.buf = e.rng_buf[i];
    s.rng.inc_hi = e.inc_hi[i];
    s.rng.inc_lo = e.inc_lo[i];
    s.seed_hi = e.seed_hi[i];
    s.seed_lo = e.seed_lo[i];
    s.has_seed = e.has_seed[i] != 0;
  }
  stage_tables(t, g_rows, g_d);
  const uint64_t T1 = prof ? __builtin_amdgcn_s_memtime() : 0;
  if (!live) return;
  s.rng.has = hand_has32(s.hand);

  // ---- validity + make_move: block_blast_env.py:237-245, engine.py:326-429
  const bool draw = apply_move(t, s, act);
  const bool valid = s.valid;
  const uint64_t T2 = prof ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t T3 = T2;

  if (valid) {
    uint32_t ids = s.hand & 0x3FFFFu;
    if (prof) T3 = __builtin_amdgcn_s_memtime();
    if (draw) {
      // ---- all three used -> new hand (engine.py:432-437) ---------------
      int attempt = 0;
      bool done;
      if (a.dbg & 1) {  // diagnostics only: first draw, no solvability test (NOT reference semantics)
        ids = draw_piece(s.rng);
        ids |= draw_piece(s.rng) << 6;
        ids |= draw_piece(s.rng) << 12;
        done = true;
      } else if (a.lane_quick > 0) {
        done = quick_hand(s.B, s.rng, ids, t.row, t.d, a.lane_quick);
      } else if (a.lane_budget <= 0) {
        done = false;  // every search runs wave-cooperatively in escalate_kernel
      } else {
        const uint64_t c0 = (a.dbg & 2) ? __builtin_amdgcn_s_memtime() : 0;
        done = gen_hand_lane(s.B, s.rng, ids, attempt, t.row, t.d, a.lane_budget);
        if (a.dbg & 2) {
          a.dbg_out[4 * i + 0] = __builtin_amdgcn_s_memtime() - c0;
          a.dbg_out[4 * i + 1] = (uint64_t)attempt | ((uint64_t)(!done) << 32);
          a.dbg_out[4 * i + 2] = 0;
          a.dbg_out[4 * i + 3] = s.B;
        }
      }
      s.hand = ids | ((uint32_t)s.rng.has << 22);
      if (!done) {
        // park: post-move state + the unfinished attempt for escalate_kernel
        e.board[i] = s.B;
        e.hand[i] = s.hand;
        e.rng_hi[i] = s.rng.hi;
        e.rng_lo[i] = s.rng.lo;
        e.rng_buf[i] = s.rng.buf;
        e.score[i] = s.score;
        e.combo[i] = s.combo;
        e.max_combo[i] = s.max_combo;
        e.moves[i] = s.moves;
        e.lines[i] = s.lines_tot;
        e.blocks[i] = s.blocks;
        e.pscratch[i] = pack_pending(attempt, s.nblk, s.lines, s.cm, s.gained);
        e.pend[i] = 1;
        if (prof) {
          const uint64_t T4 = __builtin_amdgcn_s_memtime();
          a.dbg_out[4 * i + 0] = (T1 - T0) | ((T2 - T1) << 16) | ((T3 - T2) << 32) | ((T4 - T3) << 48);
          a.dbg_out[4 * i + 1] = 1;
        }
        return;
      }
    }
  }
  const uint64_t T4 = prof ? __builtin_amdgcn_s_memtime() : 0;
  finalize(t, e, s, a);
  if (prof) {
    const uint64_t T5 = __builtin_amdgcn_s_memtime();
    a.dbg_out[4 * i + 0] = (T1 - T0) | ((T2 - T1) << 16) | ((T3 - T2) << 32) | ((T4 - T3) << 48);
    a.dbg_out[4 * i + 1] = 2 | ((T5 - T4) << 16) | ((uint64_t)s.drew << 8);
  }
}

// ---------------------------------------------------------------------------
// escalation: finish parked envs with a whole wave each
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kEscBlock) escalate_kernel(EnvDev e, const PieceRow* g_rows, const uint8_t* g_d,
                                                             StepArgs a) {
  __shared__ Tables t;
  __shared__ uint32_t scratch[kEscBlock];  // 64 words per wave (slow_phase_wave)
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * kEscBlock + threadIdx.x) >> 6;
  const int base = wave * kEscGroup;
  const int mine = base + lane;
  const bool flagged = lane < kEscGroup && mine < e.n && e.pend[mine] != 0;
  const uint64_t parked = __ballot(flagged);
  // owner lane k holds env base+k: all of its columns in one round trip,
  // in flight while the tables are staged (every thread stages its share)
  StepCtx s;
  uint64_t pr = 0;
  if (flagged) {
    s.i = mine;
    s.valid = true;
    s.drew = true;
    s.B = e.board[mine];
    const uint32_t h = e.hand[mine];
    s.rng.hi = e.rng_hi[mine];
    s.rng.lo = e.rng_lo[mine];
    s.rng.buf = e.rng_buf[mine];
    s.rng.inc_hi = e.inc_hi[mine];
    s.rng.inc_lo = e.inc_lo[mine];
    s.rng.has = hand_has32(h);
    pr = e.pscratch[mine];
    s.score = e.score[mine];
    s.combo = e.combo[mine];
    s.max_combo = e.max_combo[mine];
    s.moves = e.moves[mine];
    s.lines_tot = e.lines[mine];
    s.blocks = e.blocks[mine];
    s.prev = e.prev[mine];
    s.seed_hi = e.seed_hi[mine];
    s.seed_lo = e.seed_lo[mine];
    s.has_seed = e.has_seed[mine] != 0;
    s.nblk = (int)((pr >> 8) & 0xFFu);
    s.lines = (int)((pr >> 16) & 0xFFu);
    s.cm = (int)((pr >> 24) & 0xFFu);
    s.gained = (int64_t)(uint32_t)(pr >> 32);
  }
  stage_tables(t, g_rows, g_d);  // small groups mostly find nothing parked: no jump table in LDS
  const JumpRow* J = a.jump;
  if (!parked) return;
  uint32_t my_ids = 0;
  // the parked envs of this wave searched together, attempts of several envs
  // packed into one pass (gen_hands_multi, as in rollout_kernel); the step
  // kernel's attempts count against each env's 100 (engine.py:159-172)
  if (!(a.dbg & 2)) {
    gen_hands_multi<kEscGroup, true>(parked, s.B, s.rng, my_ids, t.row, t.d, J, lane, a.pack_first, a.pack_next,
                               scratch + (threadIdx.x & ~63), nullptr, (int)(pr & 0xFFu));
    if (flagged) {
      s.hand = my_ids | ((uint32_t)s.rng.has << 22);
      finalize(t, e, s, a);
      e.pend[mine] = 0;
    }
    return;
  }
  // one parked env at a time, searched by the whole wave (register broadcast)
  uint64_t it = parked;
  while (it) {
    const int k = __ffsll((unsigned long long)it) - 1;
    it &= it - 1;
    Pcg w;
    w.hi = __shfl(s.rng.hi, k);
    w.lo = __shfl(s.rng.lo, k);
    w.inc_hi = __shfl(s.rng.inc_hi, k);
    w.inc_lo = __shfl(s.rng.inc_lo, k);
    w.buf = __shfl(s.rng.buf, k);
    w.has = __shfl((int)s.rng.has, k) != 0;
    const uint64_t wB = __shfl(s.B, k);
    const int watt = __shfl((int)(pr & 0xFFu), k);
    uint32_t ids = 0;
    const uint64_t c0 = (a.dbg & 2) ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t st[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    gen_hand_wave(wB, w, ids, watt, t.row, t.d, a.jump, lane, a.pack_first, a.pack_next,
                  scratch + (threadIdx.x & ~63), (a.dbg & 2) ? st : nullptr);
    if ((a.dbg & 2) && lane == 0) {
      a.dbg_out[4 * (base + k) + 2] = __builtin_amdgcn_s_memtime() - c0;
      a.dbg_out[4 * (base + k) + 1] = (uint64_t)st[0] | ((uint64_t)st[1] << 16) | ((uint64_t)st[2] << 32) |
                                      ((uint64_t)st[3] << 48);
      a.dbg_out[4 * (base + k) + 0] = (uint64_t)st[4] | ((uint64_t)st[5] << 32);
      a.dbg_out[4 * (base + k) + 3] = (uint64_t)st[6] | ((uint64_t)st[7] << 32);
    }
    if (lane == k) {
      s.rng = w;
      my_ids = ids;
    }
  }
  // finalise every parked env in parallel (its owner lane)
  if (flagged) {
    s.hand = my_ids | ((uint32_t)s.rng.has << 22);
    finalize(t, e, s, a);
    e.pend[mine] = 0;
  }
}

// ---------------------------------------------------------------------------
#ifndef BB_STEP_QUOTA
// bb_step's in-wave searches (step_fused_kernel): the quota pass schedule too (0: packed passes; 3.08e9 vs
// 2.945e9 env-steps/s, three interleaved repeats, profiles/r05/ab/r05s_*)
#define BB_STEP_QUOTA 1
#endif
// bb_step in one launch: step_fused_kernel.  Two lanes per env (32 envs per
// wave): lanes l and l + 32 both hold env l.  Copy 1 idles through the move
// and the finalize and takes the post-move board and the drawn pieces from
// copy 0 (one v_permlane32_swap per dword) for its own in-lane quick-test slot
// (copy c tests slot c), so a drawn hand gets two slots; the hands both slots
// leave open are searched by the whole wave (gen_hands_multi: attempts of the
// wave's parked envs packed into 64-lane passes).  At 65,536 envs this is two
// waves per SIMD, which hides the LDS / dependent-ALU latency of the searches.
// Output for output identical to the step + escalate kernel pair
// (tests/test_gpu_env_parity.py runs both) and to one step of bb_rollout.
// ---------------------------------------------------------------------------
constexpr int kStepEnvs = 32;  // envs per wave (two copies per env)
#ifndef BB_STEP_ROLL_BLOCK
#define BB_STEP_ROLL_BLOCK 512  // threads per workgroup (8 waves: the SIMD partners in one workgroup)
#endif
constexpr int kStepRollBlock = BB_STEP_ROLL_BLOCK;
#ifndef BB_STEP_QPICK
#define BB_STEP_QPICK 0  // 0: copy c tests slot c (first piece = hand slot c); 1: the hand's piece of anchor-count
                         // rank c (quick_rank_bf): 2.90e9 vs 2.94e9 env-steps/s, the extra anchors cost more here
                         // than the fewer wave searches save (profiles/r04/ab/q2_*)
#endif

// kStepOut: the bb_step info record and fp64 reward are written when asked for.  The seeded-reset state
// (seed words, has_seed) is read and expanded only by the envs that terminate, and the PCG64 columns are
// written back only where the stream moved (a draw or a reset).
template <bool kStepOut>
__global__ void __launch_bounds__(kStepRollBlock, 1) step_fused_kernel(EnvDev e, const PieceRow* g_rows,
                                                                      const uint8_t* g_d, StepArgs a, RollArgs r) {
  constexpr int kE = kStepEnvs;
  constexpr int kBlock = kStepRollBlock;
  constexpr uint64_t kEnvMask = (1ull << kE) - 1ull;
  __shared__ Tables t;
  __shared__ uint32_t scratch[kBlock];  // 64 words per wave (slow_phase_wave)
  uint32_t* lds = scratch + (threadIdx.x & ~63);
  __shared__ JumpRow jt[kJumpMax + 1];
  const int lane = threadIdx.x & 63;
  const int half = lane / kE;  // copy index; 0 = primary copy of the env (stores)
  const int wave = (blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int i = wave * kE + (lane % kE);
  const bool live = i < e.n;
  const bool primary = live && half == 0;
  StepCtx s;
  s.seed_hi = s.seed_lo = 0ull;
  s.has_seed = false;
  int act = 0;
  // the action mask is recomputed from board + hand: the stored column is never read
  uint64_t m[3] = {0ull, 0ull, 0ull};
  if (live) {
    s.i = i;
    act = r.first_action[i];
    s.B = e.board[i];
    s.hand = e.hand[i];
    s.score = e.score[i];
    s.combo = e.combo[i];
    s.max_combo = e.max_combo[i];
    s.moves = e.moves[i];
    s.lines_tot = e.lines[i];
    s.blocks = e.blocks[i];
    s.prev = e.prev[i];
    s.rng.hi = e.rng_hi[i];
    s.rng.lo = e.rng_lo[i];
    s.rng.buf = e.rng_buf[i];
    s.rng.inc_hi = e.inc_hi[i];
    s.rng.inc_lo = e.inc_lo[i];
  }
  bool rng_moved = false;  // the stream advanced (a draw or a reset): its columns are written back
  // The two waves on a SIMD issue by priority, then age: with equal priority the older one runs nearly
  // unimpeded and the younger one finishes up to 1.3x later, which sets the launch time.  Of two SIMD
  // partners (same workgroup, same SIMD, found from HW_ID) the lower-numbered takes priority 1.
  constexpr int kWaves = kBlock / 64;
  __shared__ uint32_t wave_simd[kWaves];
  const int wv = threadIdx.x >> 6;
  if (lane == 0) wave_simd[wv] = ((uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3u;  // HW_ID.SIMD_ID
  stage_tables<true>(t, g_rows, g_d, jt, a.jump);  // ends with __syncthreads
  int pw = wv;  // partner wave: the other wave of this workgroup on this SIMD (itself if none)
#pragma unroll
  for (int k = 0; k < kWaves; ++k)
    if (k != wv && wave_simd[k] == wave_simd[wv]) pw = k;
  if (__ballot(live) == 0ull) return;  // wave-uniform
  if (wv < pw) __builtin_amdgcn_s_setprio(1);
  if (live) s.rng.has = hand_has32(s.hand);

  // ---- the move (copy 0) and attempt 1's draws: block_blast_env.py:237-245, engine.py:326-437
  bool park = false;
  Pcg after = s.rng;  // stream state after attempt 1's draws
  uint32_t ids0 = 0;
  bool drew0 = false;
  if (live && half == 0) {
    drew0 = apply_move_bf(t, s, act);
    if (drew0) {
      const Pcg save = s.rng;
      uint32_t x0, x1, x2;
      draw3(s.rng, x0, x1, x2);
      ids0 = x0 | (x1 << 6) | (x2 << 12);
      after = s.rng;
      s.rng = save;
      s.hand = ids0;
    }
  }
  // ---- in-lane quick test of attempt 1, slot `half` of each copy
  const uint32_t idq = lower_half_bcast((uint32_t)ids0 | ((uint32_t)drew0 << 31));
  const uint64_t Bq = ((uint64_t)lower_half_bcast((uint32_t)(s.B >> 32)) << 32) | lower_half_bcast((uint32_t)s.B);
#if BB_STEP_QPICK
  if (live && (idq >> 31)) park = !quick_rank_bf(Bq, idq & 63u, (idq >> 6) & 63u, (idq >> 12) & 63u, t.row, t.d, half);
#else
  if (live && (idq >> 31)) park = !quick_slot_bf(Bq, idq & 63u, (idq >> 6) & 63u, (idq >> 12) & 63u, t.row, t.d, half);
#endif
  // accept if either copy accepted; else roll back for the wave search
  uint64_t drew_bits = __ballot(live && half == 0 && s.drew);  // copy 1 did not move: copy 0's flags
  drew_bits |= drew_bits << kE;
  uint64_t acc = ~__ballot(park) & drew_bits;
  acc |= (acc >> kE) | (acc << kE);  // every copy sees the other's verdict
  const bool accepted = (acc >> lane) & 1ull;
  if (live && s.drew && half == 0) {
    rng_moved = true;
    if (accepted) s.rng = after;
    park = !accepted;
    s.hand = (s.hand & 0x3FFFFu) | ((uint32_t)s.rng.has << 22);
  }
  // ---- hand searches the in-lane test left open (engine.py:155-172): the whole wave
  const uint64_t parked = __ballot(park) & kEnvMask;
  if (parked) {
    uint32_t ids = 0;
#if BB_STEP_QUOTA
    gen_hands_quota<kE, true>(parked, s.B, s.rng, ids, t.row, t.d, jt, lane, a.pack_first, a.pack_next, lds);
#else
    gen_hands_multi<kE, true>(parked, s.B, s.rng, ids, t.row, t.d, jt, lane, a.pack_first, a.pack_next, lds);
#endif
    if ((parked >> (lane % kE)) & 1ull) s.hand = ids | ((uint32_t)s.rng.has << 22);
  }
  // ---- finalize (copy 0): game over, reward, outputs, auto-reset, mask, policy
  const uint32_t u_next = policy_uniform(a.policy_seed, a.env_offset + (uint64_t)i, r.policy_step0 + 1);
  if (primary) {
    masks_of(t, s.B, s.hand, m);
    double rew = -10.0;  // invalid action (block_blast_env.py:240-245)
    bool term = false;
    int holes = 0;
    if (s.valid) {
      const bool over = (m[0] | m[1] | m[2]) == 0ull;  // engine.py:440-441
      if (over) s.hand |= 1u << 21;
      int center;
      rew = move_reward(s, a, over, holes, center);
      s.prev = (uint32_t)(holes | (center << 8));
      term = over;
    } else if (kStepOut && r.info) {
      holes = count_holes(s.B);
    }
    r.reward[i] = (float)rew;
    r.terminated[i] = term ? 1 : 0;
    if (r.lines) r.lines[i] = (uint8_t)s.lines;
    if (r.actions) r.actions[i] = act;
    if (kStepOut && r.reward_f64) r.reward_f64[i] = rew;
    if (kStepOut && r.info) {  // block_blast_env.py:266-288, values after the move, before the auto-reset
      bb_info inf;
      inf.score = s.score;
      inf.score_gained = s.gained;
      inf.term_board = s.B;
      inf.moves = s.moves;
      inf.lines = s.lines_tot;
      inf.max_combo = s.max_combo;
      inf.blocks = s.blocks;
      inf.term_hand = s.hand;
      inf.holes = (uint8_t)holes;
      inf.filled = (uint8_t)__popcll(s.B);
      inf.flags = (uint8_t)((s.valid ? 4u : 1u) | (term ? 2u : 0u));
      inf.last_blocks = (uint8_t)s.nblk;
      inf.last_lines = (uint8_t)s.lines;
      inf.last_cm = (uint8_t)s.cm;
      inf.pad[0] = inf.pad[1] = 0;
      r.info[i] = inf;
    }
    if (term) {  // info['final_score'] / info['moves'] of the ending episode (wrappers.py:97-101)
      if (r.final_score) r.final_score[i] = s.score;
      if (r.final_moves) r.final_moves[i] = s.moves;
    }
    if (term && a.autoreset) {  // wrappers.py:97-102: env.reset() with the stored seed_value
      rng_moved = true;
      s.has_seed = e.has_seed[i] != 0;
      if (s.has_seed) {
        s.seed_hi = e.seed_hi[i];
        s.seed_lo = e.seed_lo[i];
      }
      reset_lane(t, s.has_seed, s.seed_hi, s.seed_lo, s.rng, s.B, s.hand, m);
      s.score = 0;
      s.combo = 0;
      s.max_combo = 0;
      s.moves = 0;
      s.lines_tot = 0;
      s.blocks = 0;
      s.prev = 0;
    }
    if (r.mask) {
      r.mask[3 * i + 0] = m[0];
      r.mask[3 * i + 1] = m[1];
      r.mask[3 * i + 2] = m[2];
    }
    act = random_policy_u(m[0], m[1], m[2], u_next);  // Philox (seed, env, policy_step)
    e.board[i] = s.B;
    e.hand[i] = s.hand;
    if (rng_moved) {
      e.rng_hi[i] = s.rng.hi;
      e.rng_lo[i] = s.rng.lo;
      e.rng_buf[i] = s.rng.buf;
    }
    e.score[i] = s.score;
    e.combo[i] = s.combo;
    e.max_combo[i] = s.max_combo;
    e.moves[i] = s.moves;
    e.lines[i] = s.lines_tot;
    e.blocks[i] = s.blocks;
    e.prev[i] = (uint16_t)s.prev;
    e.mask[3 * i + 0] = m[0];
    e.mask[3 * i + 1] = m[1];
    e.mask[3 * i + 2] = m[2];
    if (r.next_action) r.next_action[i] = act;
  }
}

// ---------------------------------------------------------------------------
// bb_rollout: T steps of every env in one launch under the fused random
// policy (BASELINE config 2), with the hand searches taken off the step loop.
//
// A workgroup (one per CU at 65,536 envs) holds kAEW = 4 env waves of 64 envs,
// one lane per env, whose state stays in VGPRs for the whole launch, and
// kASW search waves (one env wave and one search wave per SIMD).  An env whose
// new hand the in-lane quick test (two fixed slots) leaves open posts its
// post-move board and rolled-back stream to an LDS record and is blocked; its
// wave goes on stepping its other envs (each env keeps its own step counter,
// outputs go to [its step][N]).  A search wave claims posted records of the
// whole workgroup (compare-and-swap), runs gen_hands_multi over every env it
// claimed and hands each env back -- stream + hand -- as soon as the round
// that decides it ends; the env finalizes that step in the env wave's next
// poll.  Each env's trajectory is exactly the one T chained bb_step calls
// compute (the same draws, the same tests, the same Philox keys); only the
// order in which a wave's envs advance changes.
//
// Termination: an env wave ends when each of its envs has done T steps (it
// never waits: blocked envs are polled once per iteration), and raises its
// flag; a search wave ends when the flags of all env waves are up (a wave
// raises it only after every request it posted was answered).  Iteration
// caps on the env waves bound the kernel even if a record were lost; a wave
// that leaves through one raises the handle's status word.
// ---------------------------------------------------------------------------
#ifndef BB_ASYNC_SW
#define BB_ASYNC_SW 4  // search waves per workgroup (2 / 3 / 8: 7.65e9 / 8.04e9 / 9.36e9 vs 1.017e10, r03)
#endif
#ifndef BB_ASYNC_SPRIO
#define BB_ASYNC_SPRIO 3  // s_setprio of the search waves while they search (0: 5.6e9, 1: 9.58e9, 3: 9.60e9)
#endif
#ifndef BB_ASYNC_SLOTS
// in-lane quick-test slots per env: 1 (shipped, r04: 1.277e10) / 2 / 3: 1.246e10 / 1.155e10 (profiles/r04/ab/k1_*);
// 0: every drawn hand goes to the search waves
#define BB_ASYNC_SLOTS 1
#endif
#ifndef BB_ASYNC_DIAG_DUPSEARCH
#define BB_ASYNC_DIAG_DUPSEARCH 0  // diagnostics only: every search call run twice (tools/variants.py adup)
#endif
#ifndef BB_ASYNC_QPICK
// 1: the one in-lane slot starts from the hand's fewest-anchor piece (quick_rank_bf), 1.308e10 vs 1.280e10
// env-steps/s for slot 0 (0; profiles/r04/ab/q1_*)
#define BB_ASYNC_QPICK 1
#endif
#ifndef BB_ASYNC_DIAG
#define BB_ASYNC_DIAG 0  // per-wave counters into dbg_out (tools/diag_async.py, BB_DEBUG_MODE=16); 2: + env-wave
                         // phase cycles (each stamp costs ~10% of the iteration: a relative split only)
#endif
#if BB_ASYNC_DIAG >= 2
#define BB_ENV_STAMP(k)                                  \
  {                                                      \
    const uint64_t stamp_ = __builtin_amdgcn_s_memtime(); \
    dph[k] += stamp_ - dlast;                            \
    dlast = stamp_;                                      \
  }
#else
#define BB_ENV_STAMP(k)
#endif
#ifndef BB_ASYNC_SLEEP
#define BB_ASYNC_SLEEP 1  // s_sleep of an idle search wave between polls
#endif
#ifndef BB_ASYNC_LINEONLY
// search waves: slow_phase_wave's line-only second order above BB_SLOW_LINE_MIN tasks.  Round 3 measured it -1 to
// -4% (short exact phases); on the quota schedule the exact phase is ~29% of a call and it measured +0.4%
// (1.397e10 vs 1.392e10, three interleaved repeats; threshold 128: -2.8%; profiles/r05/ab/r05ab2_*)
#define BB_ASYNC_LINEONLY 1
#endif
#ifndef BB_SEARCH_QUOTA
// search waves: the quota pass schedule (gen_hands_quota, bb_solver.h); 0: gen_hands_multi's packed passes
#define BB_SEARCH_QUOTA 1
#endif
#ifndef BB_ASYNC_PHILOX_EARLY
#define BB_ASYNC_PHILOX_EARLY 0  // the policy uniform computed at the top of every iteration (every lane)
#endif
constexpr int kAEW = 4, kASW = BB_ASYNC_SW;
constexpr int kABlock = 64 * (kAEW + kASW);
constexpr int kAE = 64;                    // envs per env wave, one lane per env
constexpr int kAEnvs = kAE * kAEW;         // envs per workgroup
constexpr int kAPer = kAEnvs / 64;         // records a search-wave lane watches: k * 64 + lane

// The posted envs of a workgroup, one record per env, as structure of arrays (the lanes of a wave touch
// consecutive records: conflict-free LDS access).  In: board and stream state; back: stream state and the
// hand ids (has | ids << 1).
struct ARecs {
  uint64_t B[kAEnvs], hi[kAEnvs], lo[kAEnvs];
  uint64_t inc_hi[kAEnvs], inc_lo[kAEnvs];  // the stream increment (any search wave may take the env)
  uint32_t buf[kAEnvs], has_ids[kAEnvs];
};

__global__ void __launch_bounds__(kABlock, 1) rollout_async_kernel(EnvDev e, const PieceRow* g_rows,
                                                                  const uint8_t* g_d, StepArgs a, RollArgs r) {
  __shared__ Tables t;
  __shared__ uint32_t scratch[kABlock];  // 64 words per wave (the search waves' slow_phase_wave)
  __shared__ JumpRow jt[kJumpMax + 1];
  __shared__ ARecs arec;
  __shared__ uint32_t astat[kAEnvs];  // 0 idle, 1 posted, 3 claimed, 2 answered
  __shared__ uint32_t afin[kAEW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint32_t* lds = scratch + (threadIdx.x & ~63);
  if (threadIdx.x < kAEnvs) astat[threadIdx.x] = 0u;
  if (threadIdx.x < kAEW) afin[threadIdx.x] = 0u;
  stage_tables<true>(t, g_rows, g_d, jt, a.jump);  // ends with __syncthreads (also orders the inits above)

  if (wv >= kAEW) {
    // ---------------- search wave ----------------
    const int sw = wv - kAEW;
    Pcg rng;
    rng.hi = rng.lo = 0ull;
    rng.buf = 0u;
    rng.has = 0u;
    rng.inc_hi = rng.inc_lo = 0ull;
    int rid = lane;
    uint64_t B = 0ull;
#if BB_ASYNC_DIAG  // diagnostics (BB_DEBUG_MODE=16): calls, envs served, search cycles, polls, phase cycles
    uint64_t dcalls = 0, denvs = 0, dcyc = 0, dpolls = 0;
    uint64_t dprof[6] = {0, 0, 0, 0, 0, 0};
    uint64_t* const dprof_p = dprof;
#else
    uint64_t* const dprof_p = nullptr;
    (void)sw;
#endif
#pragma unroll 1
    for (;;) {
      // claim the first posted record among this lane's (posted -> 3 by compare-and-swap)
      uint32_t sv = 0u;
#pragma unroll
      for (int k = 0; k < kAPer; ++k) {
        if (sv != 1u &&
            __hip_atomic_load(&astat[k * 64 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 1u) {
          uint32_t expect = 1u;
          if (__hip_atomic_compare_exchange_strong(&astat[k * 64 + lane], &expect, 3u, __ATOMIC_RELAXED,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            sv = 1u;
            rid = k * 64 + lane;
          }
        }
      }
      const uint64_t req = __ballot(sv == 1u);
      if (req) {
        // acquire: the claimed records' fields were written before their poster's release of status 1
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        if (sv == 1u) {
          B = arec.B[rid];
          rng.hi = arec.hi[rid];
          rng.lo = arec.lo[rid];
          rng.buf = arec.buf[rid];
          rng.has = arec.has_ids[rid] & 1u;
          rng.inc_hi = arec.inc_hi[rid];
          rng.inc_lo = arec.inc_lo[rid];
        }
        __builtin_amdgcn_s_setprio(BB_ASYNC_SPRIO);
        uint32_t ids = 0;
#if BB_ASYNC_DIAG
        const uint64_t c0 = __builtin_amdgcn_s_memtime();
#endif
        // each env goes back to its env wave as soon as the round that decides it ends (1.105e10 vs
        // 1.076e10 with the hand-back at the call's end, r03)
        auto release = [&](bool d) {
          if (d && sv == 1u) {
            arec.hi[rid] = rng.hi;
            arec.lo[rid] = rng.lo;
            arec.buf[rid] = rng.buf;
            arec.has_ids[rid] = (rng.has ? 1u : 0u) | (ids << 1);
            lds_flag_store_release(&astat[rid], 2u);
          }
        };
#if BB_ASYNC_DIAG_DUPSEARCH
        const Pcg rng_dup = rng;
#endif
#if BB_SEARCH_QUOTA
        gen_hands_quota<64, (bool)BB_ASYNC_LINEONLY>(req, B, rng, ids, t.row, t.d, jt, lane, a.pack_first,
                                                     a.pack_next, lds, dprof_p, 0, release);
#else
        gen_hands_multi<64, (bool)BB_ASYNC_LINEONLY>(req, B, rng, ids, t.row, t.d, jt, lane, a.pack_first,
                                                     a.pack_next, lds, dprof_p, 0, release);
#endif
#if BB_ASYNC_DIAG_DUPSEARCH
        {  // diagnostics only: the same search once more, results dropped (its instructions are the search
           // waves' share of the kernel's SQ counts: counts of this build minus the shipped build's)
          Pcg r2 = rng_dup;
          uint32_t ids2 = 0;
          gen_hands_multi<64, (bool)BB_ASYNC_LINEONLY>(req, B, r2, ids2, t.row, t.d, jt, lane, a.pack_first,
                                                       a.pack_next, lds);
          if (ids2 == 0x7FFFFFFFu && r2.hi == 1ull) lds[lane] = ids2;  // keeps the call
        }
#endif
#if BB_ASYNC_DIAG
        dcyc += __builtin_amdgcn_s_memtime() - c0;
        dcalls += 1;
        denvs += (uint64_t)__popcll(req);
#endif
        __builtin_amdgcn_s_setprio(0);
      } else {
        uint32_t fin = 1u;
#pragma unroll
        for (int q = 0; q < kAEW; ++q) fin &= __hip_atomic_load(&afin[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (fin) break;  // wave-uniform (LDS word read by every lane)
#if BB_ASYNC_DIAG
        dpolls += 1;
#endif
        __builtin_amdgcn_s_sleep(BB_ASYNC_SLEEP);
      }
    }
#if BB_ASYNC_DIAG
    if (a.dbg_out && lane == 0) {
      uint64_t* o = a.dbg_out + 16 * ((size_t)(e.n + 63) / 64) + 16 * ((size_t)blockIdx.x * kASW + sw);
      o[0] = dcalls;
      o[1] = denvs;
      o[2] = dcyc;
      o[3] = dpolls;
      for (int q = 0; q < 6; ++q) o[4 + q] = dprof[q];
    }
#endif
    return;
  }

  // ---------------- env wave ----------------
  const int rid = wv * kAE + lane;  // this env's record
  const int i = blockIdx.x * kAEnvs + rid;
  const bool live = i < e.n;
  StepCtx s;
  s.seed_hi = s.seed_lo = 0ull;
  s.has_seed = false;
  int act = 0;
  uint64_t m[3] = {0ull, 0ull, 0ull};
  if (live) {
    s.i = i;
    act = r.first_action[i];
    s.B = e.board[i];
    s.hand = e.hand[i];
    s.score = e.score[i];
    s.combo = e.combo[i];
    s.max_combo = e.max_combo[i];
    s.moves = e.moves[i];
    s.lines_tot = e.lines[i];
    s.blocks = e.blocks[i];
    s.prev = e.prev[i];
    s.rng.hi = e.rng_hi[i];
    s.rng.lo = e.rng_lo[i];
    s.rng.buf = e.rng_buf[i];
    s.rng.inc_hi = e.inc_hi[i];
    s.rng.inc_lo = e.inc_lo[i];
    s.seed_hi = e.seed_hi[i];
    s.seed_lo = e.seed_lo[i];
    s.has_seed = e.has_seed[i] != 0;
    s.rng.has = hand_has32(s.hand);
  }
  // seeded envs re-seed on every reset (block_blast_env.py:212-215): post-reset hand, stream, mask once
  Pcg rs = s.rng;
  uint32_t r_hand = 0;
  uint64_t rm[3] = {0ull, 0ull, 0ull};
  if (live && s.has_seed) {
    uint64_t B0;
    reset_lane(t, true, s.seed_hi, s.seed_lo, rs, B0, r_hand, rm);
  }
  const size_t N = (size_t)e.n;
  const int T = r.steps;
  int st = 0;   // this env's completed steps
  int ph = 0;   // 0 ready to move, 1 posted (blocked), 2 hand known (finalize)
  // Bounds (never reached by a correct run): an iteration that moves or finalizes some env advances one of the
  // wave's 2 * kAE * T phases, so there are at most 2 * kAE * T of them; a run of iterations in which every
  // unfinished env waits on a search lasts as long as that search (at most 100 attempts), so 2^24 of them in a
  // row (seconds) means a lost record.  Either cap ends the wave instead of hanging the GPU, and the wave then
  // raises the handle's status word (kStatusAsyncCap): the host fails the next call with BB_ERR_DEVICE.
  const int64_t cap = r.work_cap > 0 ? r.work_cap : 2 * (int64_t)kAE * T + 4096;
  int64_t work_it = 0, idle_it = 0;  // idle_it: the current run of all-blocked iterations
#if BB_ASYNC_DIAG  // iterations, cycles, blocked env-iterations, iterations that moved no env | their cycles << 32
  uint64_t dit = 0, dblk = 0, didle = 0, didle_cyc = 0;
  const uint64_t dt0 = __builtin_amdgcn_s_memtime();
#endif
#if BB_ASYNC_DIAG >= 2  // env-wave phases: move+draw, quick test+post, poll, Philox, masks, reward, outputs+reset, policy
  uint64_t dph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t dlast = 0;
#endif
#pragma unroll 1
  while (work_it < cap && idle_it < (1 << 24)) {
    if (!__ballot(live && st < T)) break;
#if BB_ASYNC_DIAG
    const uint64_t dti = __builtin_amdgcn_s_memtime();
    dit += 1;
    dblk += (uint64_t)__popcll(__ballot(live && ph == 1));
    didle += __ballot(live && ph != 1 && st < T) ? 0u : 1u;
#endif
#if BB_ASYNC_DIAG >= 2
    dlast = __builtin_amdgcn_s_memtime();
#endif
    // 1. the move of every ready env and attempt 1's draws when it used the last slot
    //    (block_blast_env.py:237-245, engine.py:326-437)
    const bool mv = live && ph == 0 && st < T;
#if BB_ASYNC_PHILOX_EARLY
    // this step's policy uniform depends only on the env's step counter: its ten dependent Philox rounds
    // overlap the move's LDS round trips (one lane per env: no copy to share it with)
    const uint32_t u_next = policy_uniform(a.policy_seed, a.env_offset + (uint64_t)i, r.policy_step0 + st + 1);
#endif
    Pcg after = s.rng;
    bool drew = false;
    if (mv) {
      drew = apply_move_bf(t, s, act);
      if (drew) {
        const Pcg save = s.rng;
        uint32_t x0, x1, x2;
        draw3(s.rng, x0, x1, x2);
        after = s.rng;
        s.rng = save;
        s.hand = x0 | (x1 << 6) | (x2 << 12);
      }
    }
    BB_ENV_STAMP(0)
    // 2. in-lane quick test of attempt 1: fixed level-1 slots 0 .. BB_ASYNC_SLOTS - 1 (an accept is an exact
    //    success; anything else goes to a search wave, which redraws the attempt)
    if (drew) {
      const uint32_t q0 = s.hand & 63u, q1 = (s.hand >> 6) & 63u, q2 = (s.hand >> 12) & 63u;
      bool ok = false;
#if BB_ASYNC_QPICK
      ok = quick_rank_bf(s.B, q0, q1, q2, t.row, t.d, 0);
#else
#pragma unroll
      for (int k = 0; k < BB_ASYNC_SLOTS; ++k) ok = quick_slot_bf(s.B, q0, q1, q2, t.row, t.d, k) || ok;
#endif
      if (ok) s.rng = after;
      s.hand = (s.hand & 0x3FFFFu) | ((uint32_t)s.rng.has << 22);
      if (ok) {
        ph = 2;
      } else {  // post the env: post-move board, stream rolled back to attempt 1
        arec.B[rid] = s.B;
        arec.hi[rid] = s.rng.hi;
        arec.lo[rid] = s.rng.lo;
        arec.buf[rid] = s.rng.buf;
        arec.has_ids[rid] = s.rng.has ? 1u : 0u;
        arec.inc_hi[rid] = s.rng.inc_hi;
        arec.inc_lo[rid] = s.rng.inc_lo;
        lds_flag_store_release(&astat[rid], 1u);
        ph = 1;
      }
    } else if (mv) {
      ph = 2;  // no draw (or an invalid action): the hand is known
    }
    BB_ENV_STAMP(1)
    // 3. answered searches (polled after the moves, so that answers which arrived meanwhile finalize in this
    //    iteration: 1.017e10 vs 9.89e9 polled before them, r03): the stream after the accepted attempt, the hand
    if (live && ph == 1 && lds_flag_load_acquire(&astat[rid]) == 2u) {
      s.rng.hi = arec.hi[rid];
      s.rng.lo = arec.lo[rid];
      s.rng.buf = arec.buf[rid];
      const uint32_t hi = arec.has_ids[rid];
      s.rng.has = hi & 1u;
      s.hand = (hi >> 1) | ((hi & 1u) << 22);
      __hip_atomic_store(&astat[rid], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      ph = 2;
    }
    BB_ENV_STAMP(2)
    // 4. finalize every env whose hand is known: game over, reward, outputs, auto-reset, mask, policy
    const bool fin = live && ph == 2;
    if (fin) {
#if !BB_ASYNC_PHILOX_EARLY
      const uint32_t u_next = policy_uniform(a.policy_seed, a.env_offset + (uint64_t)i, r.policy_step0 + st + 1);
#endif
      BB_ENV_STAMP(3)
      masks_of(t, s.B, s.hand, m);
      BB_ENV_STAMP(4)
      double rew = -10.0;  // invalid action (block_blast_env.py:240-245)
      bool term = false;
      int holes = 0;
      if (s.valid) {
        const bool over = (m[0] | m[1] | m[2]) == 0ull;  // engine.py:440-441
        if (over) s.hand |= 1u << 21;
        int center;
        rew = move_reward(s, a, over, holes, center);
        s.prev = (uint32_t)(holes | (center << 8));
        term = over;
      }
      BB_ENV_STAMP(5)
      const size_t o = (size_t)st * N + (size_t)i;
      r.reward[o] = (float)rew;
      r.terminated[o] = term ? 1 : 0;
      if (r.lines) r.lines[o] = (uint8_t)s.lines;
      if (r.actions) r.actions[o] = act;
      if (term) {  // info['final_score'] / info['moves'] of the ending episode (wrappers.py:97-101)
        if (r.final_score) r.final_score[o] = s.score;
        if (r.final_moves) r.final_moves[o] = s.moves;
      }
      if (term && a.autoreset) {  // wrappers.py:97-102
        if (s.has_seed) {
          s.B = 0ull;
          s.hand = r_hand;
          s.rng.hi = rs.hi;
          s.rng.lo = rs.lo;
          s.rng.buf = rs.buf;
          s.rng.has = rs.has;
          m[0] = rm[0];
          m[1] = rm[1];
          m[2] = rm[2];
        } else {  // seed_value None: the stream continues across episodes
          reset_lane(t, false, s.seed_hi, s.seed_lo, s.rng, s.B, s.hand, m);
        }
        s.score = 0;
        s.combo = 0;
        s.max_combo = 0;
        s.moves = 0;
        s.lines_tot = 0;
        s.blocks = 0;
        s.prev = 0;
      }
      if (r.mask) {
        r.mask[3 * o + 0] = m[0];
        r.mask[3 * o + 1] = m[1];
        r.mask[3 * o + 2] = m[2];
      }
      BB_ENV_STAMP(6)
      act = random_policy_u(m[0], m[1], m[2], u_next);  // Philox (seed, env, policy_step0 + step + 1)
      st += 1;
      ph = 0;
      BB_ENV_STAMP(7)
    }
    if (!__ballot(mv || fin)) {  // every env blocked: leave the SIMD to the searches
      ++idle_it;
      __builtin_amdgcn_s_sleep(1);
#if BB_ASYNC_DIAG
      didle_cyc += __builtin_amdgcn_s_memtime() - dti;
#endif
    } else {
      ++work_it;
      idle_it = 0;
    }
  }
  // left through a cap with envs short of T steps: this launch's outputs and final state are incomplete
  if (__ballot(live && st < T) && lane == 0)
    __hip_atomic_store(e.status, kStatusAsyncCap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#if BB_ASYNC_DIAG
  if (a.dbg_out && lane == 0) {
    uint64_t* o = a.dbg_out + 16 * ((size_t)blockIdx.x * kAEW + wv);
    o[0] = dit;
    o[1] = __builtin_amdgcn_s_memtime() - dt0;
    o[2] = dblk;
    o[3] = didle | (didle_cyc << 32);
#if BB_ASYNC_DIAG >= 2
    for (int q = 0; q < 8; ++q) o[4 + q] = dph[q];
#endif
  }
#endif
  if (live) {
    e.board[i] = s.B;
    e.hand[i] = s.hand;
    e.rng_hi[i] = s.rng.hi;
    e.rng_lo[i] = s.rng.lo;
    e.rng_buf[i] = s.rng.buf;
    e.score[i] = s.score;
    e.combo[i] = s.combo;
    e.max_combo[i] = s.max_combo;
    e.moves[i] = s.moves;
    e.lines[i] = s.lines_tot;
    e.blocks[i] = s.blocks;
    e.prev[i] = (uint16_t)s.prev;
    if (T > 0) {
      e.mask[3 * i + 0] = m[0];
      e.mask[3 * i + 1] = m[1];
      e.mask[3 * i + 2] = m[2];
    }
    if (r.next_action) r.next_action[i] = act;
  }
  // every request this wave posted has been answered (an env is posted only while st < T), unless a cap
  // ended the wave: the search waves then finish what they claimed and leave
  if (lane == 0) lds_flag_store_release(&afin[wv], 1u);
}

// ---------------------------------------------------------------------------
// Observation expansion: engine.py:478-507 / block_blast_env.py:134-146.
// One thread per 16-byte output chunk -> fully coalesced dwordx4 stores.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float4 bits4(uint64_t v, int cell) {
  return make_float4((float)((v >> cell) & 1ull), (float)((v >> (cell + 1)) & 1ull),
                     (float)((v >> (cell + 2)) & 1ull), (float)((v >> (cell + 3)) & 1ull));
}

__device__ __forceinline__ uint64_t plane_of(const PieceRow* rows, uint64_t board, uint32_t hand, int plane) {
  if (plane == 0) return board;
  const int s = plane - 1;
  return ((hand_used(hand) >> s) & 1u) ? 0ull : rows[hand_id(hand, s)].shape;
}

// x[N][4][64] f32: 64 chunks per env.
__global__ void expand_x_kernel(const uint64_t* __restrict__ board, const uint32_t* __restrict__ hand,
                                const int64_t* __restrict__ index, const PieceRow* __restrict__ g_rows, int n,
                                float4* __restrict__ x) {
  __shared__ PieceRow rows[kPieces];
  if (threadIdx.x < kPieces) rows[threadIdx.x] = g_rows[threadIdx.x];
  __syncthreads();
  const int64_t total = (int64_t)n * 64;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < total;
       u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = u >> 6;
    const int chunk = (int)(u & 63);
    const int64_t src = index ? index[j] : j;
    const uint64_t v = plane_of(rows, board[src], hand[src], chunk >> 4);
    x[u] = bits4(v, (chunk & 15) * 4);
  }
}

// mask f32 [N][192]: 48 chunks per env; int8 [N][192]: 12 chunks of 16 B.
__global__ void expand_mask_kernel(const uint64_t* __restrict__ mbits, const int64_t* __restrict__ index, int n,
                                   float4* __restrict__ mf, int4* __restrict__ mi) {
  const int64_t totf = mf ? (int64_t)n * 48 : 0;
  const int64_t toti = mi ? (int64_t)n * 12 : 0;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < totf + toti;
       u += (int64_t)gridDim.x * blockDim.x) {
    if (u < totf) {
      const int64_t j = u / 48;
      const int chunk = (int)(u - j * 48);
      const int64_t src = index ? index[j] : j;
      const uint64_t w = mbits[3 * src + (chunk >> 4)];
      mf[u] = bits4(w, (chunk & 15) * 4);
    } else {
      const int64_t v = u - totf;
      const int64_t j = v / 12;
      const int chunk = (int)(v - j * 12);
      const int64_t src = index ? index[j] : j;
      const uint64_t w = mbits[3 * src + (chunk >> 2)];
      const uint32_t bits16 = (uint32_t)(w >> ((chunk & 3) * 16)) & 0xFFFFu;
      int4 o;
      uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t b4 = bits16 >> (4 * q);
        ow[q] = (b4 & 1u) | (((b4 >> 1) & 1u) << 8) | (((b4 >> 2) & 1u) << 16) | (((b4 >> 3) & 1u) << 24);
      }
      mi[v] = o;
    }
  }
}

// Recompute the mask column after a host-side state overwrite (bb_set_state).
__global__ void refresh_mask_kernel(EnvDev e, const PieceRow* __restrict__ g_rows) {
  __shared__ PieceRow rows[kPieces];
  if (threadIdx.x < kPieces) rows[threadIdx.x] = g_rows[threadIdx.x];
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= e.n) return;
  const uint64_t B = e.board[i];
  const uint32_t h = e.hand[i];
  const uint32_t used = hand_used(h);
  for (int s = 0; s < 3; ++s)
    e.mask[3 * i + s] = ((used >> s) & 1u) ? 0ull : anchors_of(rows[hand_id(h, s)], B);
}

__global__ void random_actions_kernel(const uint64_t* __restrict__ mbits, int n, uint64_t seed, uint64_t step,
                                      uint64_t offset, int32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = random_policy(mbits[3 * i], mbits[3 * i + 1], mbits[3 * i + 2], seed, offset + (uint64_t)i, step);
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
static inline int grid_for(int64_t units, int block) {
  int64_t g = (units + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

hipError_t launch_reset(const EnvDev& e, const PieceRow* rows, const uint8_t* d, const uint8_t* sel,
                        hipStream_t s) {
  hipLaunchKernelGGL(reset_kernel, dim3((e.n + kStepBlock - 1) / kStepBlock), dim3(kStepBlock), 0, s, e, rows, d,
                     sel);
  return hipGetLastError();
}

hipError_t launch_step(const EnvDev& e, const PieceRow* rows, const uint8_t* d, const int32_t* actions,
                       const StepArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(step_kernel, dim3((e.n + kStepBlock - 1) / kStepBlock), dim3(kStepBlock), 0, s, e, rows, d,
                     actions, a);
  hipError_t st = hipGetLastError();
  if (st != hipSuccess) return st;
  const int envs_per_block = kEscBlock / 64 * kEscGroup;
  hipLaunchKernelGGL(escalate_kernel, dim3((e.n + envs_per_block - 1) / envs_per_block), dim3(kEscBlock), 0, s, e,
                     rows, d, a);
  return hipGetLastError();
}

hipError_t launch_rollout(const EnvDev& e, const PieceRow* rows, const uint8_t* d, const StepArgs& a,
                          const RollArgs& r, hipStream_t s) {
  if (r.steps == 1) {  // bb_step in one launch
    const dim3 g((unsigned)(((int64_t)e.n + kStepEnvs - 1) / kStepEnvs * 64 / kStepRollBlock +
                            (((int64_t)e.n + kStepEnvs - 1) / kStepEnvs * 64 % kStepRollBlock ? 1 : 0)));
    if (r.info || r.reward_f64)
      hipLaunchKernelGGL(step_fused_kernel<true>, g, dim3(kStepRollBlock), 0, s, e, rows, d, a, r);
    else
      hipLaunchKernelGGL(step_fused_kernel<false>, g, dim3(kStepRollBlock), 0, s, e, rows, d, a, r);
  } else {  // bb_rollout (T >= 2; no info record, no fp64 reward)
    const dim3 g((unsigned)(((int64_t)e.n + kAEnvs - 1) / kAEnvs));
    hipLaunchKernelGGL(rollout_async_kernel, g, dim3(kABlock), 0, s, e, rows, d, a, r);
  }
  return hipGetLastError();
}

hipError_t launch_expand(const uint64_t* board, const uint32_t* hand, const uint64_t* mbits, const int64_t* index,
                         const PieceRow* rows, int n, float* x, float* mf, int8_t* mi, hipStream_t s) {
  if (x) {
    hipLaunchKernelGGL(expand_x_kernel, dim3(grid_for((int64_t)n * 64, 256)), dim3(256), 0, s, board, hand, index,
                       rows, n, reinterpret_cast<float4*>(x));
  }
  if (mf || mi) {
    const int64_t units = (mf ? (int64_t)n * 48 : 0) + (mi ? (int64_t)n * 12 : 0);
    hipLaunchKernelGGL(expand_mask_kernel, dim3(grid_for(units, 256)), dim3(256), 0, s, mbits, index, n,
                       reinterpret_cast<float4*>(mf), reinterpret_cast<int4*>(mi));
  }
  return hipGetLastError();
}

hipError_t launch_refresh_mask(const EnvDev& e, const PieceRow* rows, hipStream_t s) {
  hipLaunchKernelGGL(refresh_mask_kernel, dim3((e.n + 255) / 256), dim3(256), 0, s, e, rows);
  return hipGetLastError();
}

hipError_t launch_random_actions(const uint64_t* mbits, int n, uint64_t seed, uint64_t step, uint64_t offset,
                                 int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(random_actions_kernel, dim3((n + 255) / 256), dim3(256), 0, s, mbits, n, seed, step, offset,
                     out);
  return hipGetLastError();
}

}  // namespace bb

// bb_env.hip -- MI355X (gfx950) vectorised Block Blast environment.
//
// One env per lane, wave64.  Per-env state lives in HBM as structure-of-arrays
// (coalesced 2/4/8-byte columns); the 37-piece table and the pair-offset table
// are staged into LDS once per workgroup.
//
// A step is two launches on one stream:
//   step_kernel     -- every env: all state columns are loaded up front (one
//                      memory round trip), the action is applied on a uint64
//                      bitboard, lines cleared, scored; when all three slots are
//                      used a new hand is drawn (numpy-exact PCG64 stream) and
//                      tested for solvability under a per-lane work budget;
//                      then reward (fp64, reference order), game over, info,
//                      auto-reset, action mask and the fused random policy.
//                      Envs whose hand search ran out of budget are parked:
//                      post-move state + a pending flag.
//   escalate_kernel -- each wave owns 32 envs; its parked envs are searched
//                      together by the whole wave (gen_hands_multi: attempts of
//                      several envs packed into 64-lane passes) and then
//                      finalised exactly like step_kernel would have.
// Spreading the rare hard boards over 4x more waves than the step kernel
// keeps the slowest wave short.
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
#ifndef BB_ESC_MULTI
#define BB_ESC_MULTI 1  // escalate_kernel: parked envs searched together; 0: one env at a time
#endif
#ifndef BB_ESC_LDS_JUMP
#define BB_ESC_LDS_JUMP 0  // escalate_kernel (multi): PCG64 jump table staged in LDS
#endif

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

// Every lane gets the value of copy 0 of its env (lane l mod kE).
template <int kE>
__device__ __forceinline__ uint32_t copy0_bcast(uint32_t x) {
  if constexpr (kE == 64) return x;
  else if constexpr (kE == 32) return lower_half_bcast(x);
  else return (uint32_t)__shfl((int)x, (int)(threadIdx.x & 63) % kE);
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
#if BB_ESC_MULTI && BB_ESC_LDS_JUMP
  // 32-env waves nearly always hold a parked env: the jump table goes to LDS too
  __shared__ JumpRow jt[kJumpMax + 1];
  stage_tables<true>(t, g_rows, g_d, jt, a.jump);
  const JumpRow* J = jt;
#else
  stage_tables(t, g_rows, g_d);  // small groups mostly find nothing parked: no jump table in LDS
  const JumpRow* J = a.jump;
#endif
  if (!parked) return;
  uint32_t my_ids = 0;
#if BB_ESC_MULTI
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
#endif
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
// rollout: T steps of every env in one launch under the fused random policy
// (BASELINE config 2).  State stays in VGPRs for the whole rollout; a wave
// owns kRollEnvs envs (one per lane) and runs their hand searches itself,
// one parked env at a time with all 64 lanes (gen_hand_wave), so a hard
// search delays only its own wave and the per-step tail of the two-kernel
// bb_step averages out over the T steps.  Output for output identical to T
// bb_step calls chained through next_action (wrappers.py:128-137
// sample_valid_actions -> step, with the Philox policy in place of
// np.random.choice).
// ---------------------------------------------------------------------------
// Envs per wave: 32.  Lanes l and l + 32 both hold env l (identical state,
// identical per-env instructions, stores from the lower half only): the
// wave has two waves' worth of envs per SIMD at 65,536 envs, which hides the
// LDS / dependent-ALU latency, and the mirrored halves split the in-lane
// quick test of a new hand (each half tests its own fixed slots).  All 64
// lanes join the wave-cooperative searches.
#ifndef BB_ROLL_ENVS
#define BB_ROLL_ENVS 32
#endif
constexpr int kRollEnvs = BB_ROLL_ENVS;  // 32 (two copies per env), 16 (four) or 64 (one: 1 wave per SIMD)
static_assert(kRollEnvs == 16 || kRollEnvs == 32 || kRollEnvs == 64, "envs per wave");
#ifndef BB_STEP_ENVS
#define BB_STEP_ENVS 32  // bb_step's single-step instantiation: envs per wave (64 / copies)
#endif
constexpr int kStepEnvs = BB_STEP_ENVS;
#ifndef BB_STEP_ROLL_BLOCK
#define BB_STEP_ROLL_BLOCK 512  // bb_step's single-step instantiation: threads per workgroup
#endif
constexpr int kStepRollBlock = BB_STEP_ROLL_BLOCK;
#ifndef BB_ROLL_BLOCK
#define BB_ROLL_BLOCK 512  // 8 waves: at 65,536 envs one workgroup per CU, both waves of a SIMD in it
#endif
constexpr int kRollBlock = BB_ROLL_BLOCK;
#ifndef BB_ROLL_MINW
#define BB_ROLL_MINW 1
#endif
#ifndef BB_ROLL_FAIR
#define BB_ROLL_FAIR 2  // 1: alternate s_setprio between a SIMD's two waves every step; 2: behind one first
#endif
#ifndef BB_MULTI
#define BB_MULTI 1  // parked envs of a step searched together (gen_hands_multi); 0: one env at a time
#endif
#ifndef BB_ROLL_SLOTS
#define BB_ROLL_SLOTS 1  // in-lane quick-test slots per copy
#endif
#ifndef BB_ROLL_BFMOVE
#define BB_ROLL_BFMOVE 1  // rollout: branch-free apply_move (apply_move_bf)
#endif
#ifndef BB_ROLL_BFQUICK
#define BB_ROLL_BFQUICK 1  // rollout: branch-free in-lane quick slot (quick_slot_bf)
#endif
#ifndef BB_ROLL_PHILOX_TOP
#define BB_ROLL_PHILOX_TOP 0  // rollout: the policy uniform drawn at the top of every step (no branch)
#endif
#ifndef BB_STEP_LAZY_RESET
#define BB_STEP_LAZY_RESET 1  // bb_step: seeded-reset state read and expanded only by terminating envs
#endif
#ifndef BB_STEP_COND_STORE
// bb_step: 0 every state column written back; 1 only the columns that changed (measured: -2.5%, fewer bytes);
// 2 the PCG64 columns only where the stream moved (a draw or a reset), the rest unconditionally
#define BB_STEP_COND_STORE 2
#endif
#ifndef BB_ROLL_HALF_IDLE
// rollout: copy 1 exec-masked off through the move and the finalize (its duplicate work there is
// dropped; +0.8%, 8.87 vs 8.81e9 env-steps/s, 3 interleaved repeats, profiles/r03/ab/r03g_*)
#define BB_ROLL_HALF_IDLE 1
#endif
#ifndef BB_ROLL_DRAW_EARLY
#define BB_ROLL_DRAW_EARLY 0  // rollout: attempt 1 drawn before the move and quick-tested in every lane
#endif
#ifndef BB_ROLL_KSTEP
#define BB_ROLL_KSTEP BB_ROLL_SLOTS  // copy c tests slots c * KSTEP, c * KSTEP + 1, ...
#endif
#ifndef BB_WG_BALANCE
// hand searches balanced over the workgroup: after the in-lane quick tests every wave publishes its parked
// envs to LDS and each of the 8 waves searches an equal share of the workgroup's parked envs (two barriers
// per step).  1: bb_step's single step only; 2: also every step of bb_rollout; 0: off (each wave searches
// its own parked envs).  Measured slower and off: bb_step 2.71e9 vs 2.83e9 env-steps/s (the slowest wave is
// set by its hardest env, not by how many it holds), bb_rollout 5.65e9 vs 8.96e9 (profiles/r03/wgb/)
#define BB_WG_BALANCE 0
#endif

// One parked env handed to another wave of the workgroup (BB_WG_BALANCE): the board and stream state on
// the way in; the stream state and hand ids on the way back.
struct ParkRec {
  uint64_t B, hi, lo, inc_hi, inc_lo;
  uint32_t buf, has, ids, pad;
};

// kStepOut: the bb_step outputs (info record, fp64 reward) are written too --
// the instantiation bb_step uses at T = 1; the rollout path runs without them.
// kSingle: one step per launch (bb_step): the seeded-reset state is read and
// expanded only by the envs that terminate, and only the state columns the
// step changed are written back.
template <bool kStepOut, bool kSingle, int kE, int kBlock>
__global__ void __launch_bounds__(kBlock, BB_ROLL_MINW) rollout_kernel(EnvDev e, const PieceRow* g_rows, const uint8_t* g_d,
                                                             StepArgs a, RollArgs r) {
  static_assert(kE == 8 || kE == 16 || kE == 32 || kE == 64, "envs per wave");
  constexpr uint64_t kEnvMask = kE >= 64 ? ~0ull : ((1ull << (kE & 63)) - 1ull);
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
  // bb_step (kSingle, T = 1): the seeded-reset state (seed words, has_seed) is read only by the envs
  // that terminate, instead of being loaded and expanded into a post-reset hand by every env up front
  constexpr bool lazy_reset = kSingle && BB_STEP_LAZY_RESET;
  StepCtx s;
  s.seed_hi = s.seed_lo = 0ull;
  s.has_seed = false;
  int act = 0;
  // the action mask is recomputed by every step from board + hand: the stored column is never read
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
    if (!lazy_reset) {
      s.seed_hi = e.seed_hi[i];
      s.seed_lo = e.seed_lo[i];
      s.has_seed = e.has_seed[i] != 0;
    }
  }
  // loaded values: a single step's final stores skip the columns it left unchanged
  StepCtx s0;
  if constexpr (kSingle && BB_STEP_COND_STORE == 1) s0 = s;
  bool rng_moved = false;  // kSingle, BB_STEP_COND_STORE == 2: the stream advanced (a draw or a reset)
  // The two waves on a SIMD issue by priority, then age: the older one runs
  // nearly unimpeded and the younger one finishes up to 1.3x later, which
  // sets the launch time.  Partners (same workgroup, same SIMD) publish their
  // step counters in LDS; the one behind takes the higher priority.
  constexpr int kWaves = kBlock / 64;
  __shared__ uint32_t wave_simd[kWaves];
  __shared__ uint32_t prog[kWaves];
  const int wv = threadIdx.x >> 6;
  if (lane == 0) {
    wave_simd[wv] = ((uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3u;  // HW_ID.SIMD_ID
    prog[wv] = 0u;
  }
  stage_tables<true>(t, g_rows, g_d, jt, a.jump);  // ends with __syncthreads
  int pw = wv;  // partner wave: the other wave of this workgroup on this SIMD (itself if none)
#pragma unroll
  for (int k = 0; k < kWaves; ++k)
    if (k != wv && wave_simd[k] == wave_simd[wv]) pw = k;
  const uint32_t tie = wv < pw ? 1u : 0u;
  // the balanced search synchronises the workgroup every step: a wave without envs still joins the barriers
  constexpr bool kBalance = kSingle ? (BB_WG_BALANCE >= 1) : (BB_WG_BALANCE >= 2);
  __shared__ ParkRec prec[kBalance ? kWaves * kE : 1];
  __shared__ uint32_t pcnt[kWaves];
  if (!kBalance && __ballot(live) == 0ull) return;  // wave-uniform
  if (live) s.rng.has = hand_has32(s.hand);
  // A seeded env re-seeds with seed_value on every reset (block_blast_env.py:212-215), so its
  // post-reset hand, stream and mask are the same each episode: computed once, kept in registers.
  Pcg rs = s.rng;
  uint32_t r_hand = 0;
  uint64_t rm[3] = {0ull, 0ull, 0ull};
  if constexpr (!lazy_reset) {
    if (live && s.has_seed) {
      uint64_t B0;
      reset_lane(t, true, s.seed_hi, s.seed_lo, rs, B0, r_hand, rm);
    }
  }
  const size_t N = (size_t)e.n;
#if defined(BB_ROLL_DIAG) && BB_ROLL_DIAG == 3  // timing diagnostics: per-wave phase cycles (reference semantics)
  // move+quick, searches, finalize, #searches, attempts | 1-attempt searches << 32, passes | slow passes << 32,
  // quick cycles | slots << 32, disjoint | line cycles << 32
  // [9..14]: gen_hands_multi phases, [15]: HW_ID | XCC_ID << 32, [16]: wave start, [17]: wave end
  uint64_t dg[18] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  dg[15] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
           ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
  dg[16] = __builtin_amdgcn_s_memrealtime();  // 100 MHz, comparable across CUs
  uint32_t st[12];
#define BB_DIAG_T(x) const uint64_t x = __builtin_amdgcn_s_memtime()
#else
#define BB_DIAG_T(x)
#endif
  uint32_t partner = 0;
  // The policy uniforms are shared by an env's copies: on every kCopies-th
  // step copy c draws the uniform of step + 1 + c, and each step reads its
  // uniform from the copy that drew it (one Philox per lane per kCopies steps).
  constexpr int kCopies = 64 / kE;
  uint32_t u_drawn = 0;
#pragma unroll 1
  for (int step = 0; step < r.steps; ++step) {
#if BB_ROLL_FAIR == 1
    if (((uint32_t)step ^ tie) & 1u) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#elif BB_ROLL_FAIR == 2
    {  // the wave behind its SIMD partner (LDS step counters) takes the priority
      const int32_t lead = step - (int32_t)partner;
      if (lead < 0 || (lead == 0 && (((uint32_t)step ^ tie) & 1u))) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
      if (lane == 0) __hip_atomic_store(&prog[wv], (uint32_t)step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      partner = __hip_atomic_load(&prog[pw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // used next step
    }
#endif
#if BB_ROLL_PHILOX_TOP
    // this step's policy uniform, independent of the env state: computed first, with no branch, so
    // its Philox rounds interleave with the move; copy c draws step + 1 + c on even steps and the
    // same counter again on odd steps
    u_drawn = policy_uniform(a.policy_seed, a.env_offset + (uint64_t)i,
                             r.policy_step0 + (uint64_t)(step - step % kCopies) + 1 + half);
    const uint32_t u_next = __shfl(u_drawn, (lane % kE) + kE * (step % kCopies));
#endif
    BB_DIAG_T(c0);
    bool park = false;
    Pcg after = s.rng;  // stream state after attempt 1's draws
#if BB_ROLL_DRAW_EARLY && (!defined(BB_ROLL_DIAG) || BB_ROLL_DIAG == 3)
    // attempt 1's three draws do not depend on the move: drawn before it with no branch, so the
    // LCG multiplies overlap the move's table reads; the quick slot then runs in every lane (a wave
    // of 32 envs nearly always has one whose move empties its hand) and counts only where it did
    uint32_t ex0 = 0, ex1 = 0, ex2 = 0;
    if (live) draw3(after, ex0, ex1, ex2);
    if (live) {
#if BB_ROLL_BFMOVE
      const bool drew_now = apply_move_bf(t, s, act);
#else
      const bool drew_now = apply_move(t, s, act);
#endif
      const bool fits = quick_slot_bf(s.B, ex0, ex1, ex2, t.row, t.d, half * BB_ROLL_KSTEP);
      if (drew_now) {
        park = !fits;
        s.hand = ex0 | (ex1 << 6) | (ex2 << 12);
      }
    }
#elif BB_ROLL_HALF_IDLE && (!defined(BB_ROLL_DIAG) || BB_ROLL_DIAG == 3)
    // copy 1 idles through the move (and the finalize below): it takes the post-move board and the
    // drawn pieces from copy 0 (lane l -> l + 32, one v_permlane32_swap per dword) for its own
    // quick-test slot, and joins the wave search, which reads every env from copy 0's lane
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
    const uint32_t idq = copy0_bcast<kE>((uint32_t)ids0 | ((uint32_t)drew0 << 31));
    const uint64_t Bq = ((uint64_t)copy0_bcast<kE>((uint32_t)(s.B >> 32)) << 32) | copy0_bcast<kE>((uint32_t)s.B);
    if (live && (idq >> 31)) {
      park = !quick_slot_bf(Bq, idq & 63u, (idq >> 6) & 63u, (idq >> 12) & 63u, t.row, t.d, half * BB_ROLL_KSTEP);
    }
#else
    if (live) {
#if BB_ROLL_BFMOVE
      const bool drew_now = apply_move_bf(t, s, act);
#else
      const bool drew_now = apply_move(t, s, act);
#endif
      if (drew_now) {
        uint32_t ids = 0;
#if defined(BB_ROLL_DIAG) && BB_ROLL_DIAG == 2  // timing diagnostics only: first draw, no test (NOT reference)
        ids = draw_piece(s.rng);
        ids |= draw_piece(s.rng) << 6;
        ids |= draw_piece(s.rng) << 12;
#elif defined(BB_ROLL_DIAG) && BB_ROLL_DIAG == 1  // timing diagnostics only: no wave search (NOT reference)
        if (!quick_hand(s.B, s.rng, ids, t.row, t.d, a.lane_quick)) {
          ids = draw_piece(s.rng);
          ids |= draw_piece(s.rng) << 6;
          ids |= draw_piece(s.rng) << 12;
        }
#else
        // draw attempt 1 (both halves identically); each half quick-tests its own slots
        const Pcg save = s.rng;
        uint32_t x0, x1, x2;
        draw3(s.rng, x0, x1, x2);
        ids = x0 | (x1 << 6) | (x2 << 12);
#if BB_ROLL_BFQUICK && BB_ROLL_SLOTS == 1
        park = !quick_slot_bf(s.B, x0, x1, x2, t.row, t.d, half * BB_ROLL_KSTEP);
#else
        park = !quick_slots(s.B, x0, x1, x2, t.row, t.d, half * BB_ROLL_KSTEP, BB_ROLL_SLOTS);
#endif
        after = s.rng;
        s.rng = save;  // the wave search redraws the attempt unless a half accepts
#endif
        s.hand = ids;
      }
    }
#endif
    // accept if either copy accepted; else roll back for the wave search
#if BB_ROLL_HALF_IDLE
    uint64_t drew_bits = __ballot(live && half == 0 && s.drew);  // the other copies did not move: copy 0's flags
#pragma unroll
    for (int sft = kE; sft < 64; sft <<= 1) drew_bits |= drew_bits << sft;
    uint64_t acc = ~__ballot(park) & drew_bits;
#else
    uint64_t acc = ~__ballot(park) & __ballot(live && s.drew);
#endif
#pragma unroll
    for (int sft = kE; sft < 64; sft <<= 1) acc |= (acc >> sft) | (acc << (64 - sft));  // every copy sees the others
    const bool accepted = (acc >> lane) & 1ull;
    if (live && s.drew && (!BB_ROLL_HALF_IDLE || half == 0)) {
      rng_moved = true;
#if !defined(BB_ROLL_DIAG) || BB_ROLL_DIAG == 3
      if (accepted) s.rng = after;
      park = !accepted;
#endif
      s.hand = (s.hand & 0x3FFFFu) | ((uint32_t)s.rng.has << 22);
    }
    // hand searches the in-lane test left open: the whole wave, one env at a time
    uint64_t parked = __ballot(park) & kEnvMask;
    BB_DIAG_T(c1);
    if constexpr (kBalance) {
      // publish this wave's parked envs (record wv * kE + rank), then search slice wv of the
      // workgroup's list: envs gs .. ge-1 of the parked envs in wave order, held by lanes 0 .. ge-gs-1
      const int el = lane % kE;
      if (lane < kE && ((parked >> el) & 1ull)) {
        ParkRec& R = prec[wv * kE + __popcll(parked & ((1ull << el) - 1ull))];
        R.B = s.B;
        R.hi = s.rng.hi;
        R.lo = s.rng.lo;
        R.inc_hi = s.rng.inc_hi;
        R.inc_lo = s.rng.inc_lo;
        R.buf = s.rng.buf;
        R.has = s.rng.has;
      }
      if (lane == 0) pcnt[wv] = (uint32_t)__popcll(parked);
      __syncthreads();
      uint32_t cnt[kWaves];
      uint32_t P = 0;
#pragma unroll
      for (int q = 0; q < kWaves; ++q) {
        cnt[q] = pcnt[q];
        P += cnt[q];
      }
      if (P) {  // workgroup-uniform
        const int gs = (int)((wv * P) / kWaves), m = (int)(((wv + 1) * P) / kWaves) - gs;  // m <= kE
        int rec = 0;
        Pcg br = s.rng;
        uint64_t bB = 0ull;
        if (el < m) {
          int g = gs + el, q = 0;
#pragma unroll
          for (int w = 0; w < kWaves - 1; ++w)
            if (q == w && g >= (int)cnt[w]) {
              g -= (int)cnt[w];
              q = w + 1;
            }
          rec = q * kE + g;
          const ParkRec& R = prec[rec];
          bB = R.B;
          br.hi = R.hi;
          br.lo = R.lo;
          br.inc_hi = R.inc_hi;
          br.inc_lo = R.inc_lo;
          br.buf = R.buf;
          br.has = R.has;
        }
        if (m) {
          uint32_t ids = 0;
          gen_hands_multi<kE, kSingle>((1ull << m) - 1ull, bB, br, ids, t.row, t.d, jt, lane, a.pack_first,
                                              a.pack_next, lds);
          if (lane < kE && el < m) {
            ParkRec& R = prec[rec];
            R.hi = br.hi;
            R.lo = br.lo;
            R.buf = br.buf;
            R.has = br.has;
            R.ids = ids;
          }
        }
        __syncthreads();
        if ((parked >> el) & 1ull) {
          const ParkRec& R = prec[wv * kE + __popcll(parked & ((1ull << el) - 1ull))];
          s.rng.hi = R.hi;
          s.rng.lo = R.lo;
          s.rng.buf = R.buf;
          s.rng.has = R.has;
          s.hand = R.ids | (R.has << 22);
        }
      }
#if defined(BB_ROLL_DIAG) && BB_ROLL_DIAG == 3
      dg[3] += (uint64_t)__popcll(parked);
#endif
    } else
#if BB_MULTI
    if (parked) {
      uint32_t ids = 0;
#if defined(BB_ROLL_DIAG) && BB_ROLL_DIAG == 3
      dg[3] += (uint64_t)__popcll(parked);
      gen_hands_multi<kE, kSingle>(parked, s.B, s.rng, ids, t.row, t.d, jt, lane, a.pack_first, a.pack_next, lds,
                                 &dg[9]);
#else
      gen_hands_multi<kE, kSingle>(parked, s.B, s.rng, ids, t.row, t.d, jt, lane, a.pack_first, a.pack_next, lds);
#endif
      if ((parked >> (lane % kE)) & 1ull) s.hand = ids | ((uint32_t)s.rng.has << 22);
    }
#else
    while (parked) {
      const int k = __ffsll((unsigned long long)parked) - 1;
      parked &= parked - 1;
      Pcg w;
      w.hi = __shfl(s.rng.hi, k);
      w.lo = __shfl(s.rng.lo, k);
      w.inc_hi = __shfl(s.rng.inc_hi, k);
      w.inc_lo = __shfl(s.rng.inc_lo, k);
      w.buf = __shfl(s.rng.buf, k);
      w.has = __shfl((int)s.rng.has, k) != 0;
      const uint64_t wB = __shfl(s.B, k);
      uint32_t ids = 0;
#if defined(BB_ROLL_DIAG) && BB_ROLL_DIAG == 3
      for (int q = 0; q < 12; ++q) st[q] = 0;
      gen_hand_wave(wB, w, ids, 0, t.row, t.d, jt, lane, a.pack_first, a.pack_next, lds, st);
      dg[3] += 1 | ((uint64_t)st[9] << 32);
      dg[4] += st[0] | ((uint64_t)(st[0] == 1 ? 1u : 0u) << 32);
      dg[5] += st[1] | ((uint64_t)st[2] << 32);
      dg[6] += st[4] | ((uint64_t)st[8] << 32);
      dg[7] += st[5] | ((uint64_t)st[6] << 32);
      dg[8] += (st[0] == 1 && st[10] == 0) ? 1u : 0u;
#else
      gen_hand_wave(wB, w, ids, 0, t.row, t.d, jt, lane, a.pack_first, a.pack_next, lds);
#endif
      if ((lane % kE) == k) {
        s.rng = w;
        s.hand = ids | ((uint32_t)w.has << 22);
      }
    }
#endif
    BB_DIAG_T(c2);
#if !BB_ROLL_PHILOX_TOP
    if (step % kCopies == 0)
      u_drawn = policy_uniform(a.policy_seed, a.env_offset + (uint64_t)i, r.policy_step0 + step + 1 + half);
    const uint32_t u_next = __shfl(u_drawn, (lane % kE) + kE * (step % kCopies));
#endif
    if (live && (!BB_ROLL_HALF_IDLE || half == 0)) {
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
      const size_t o = (size_t)step * N + (size_t)i;
      if (primary) {
        r.reward[o] = (float)rew;
        r.terminated[o] = term ? 1 : 0;
        if (r.lines) r.lines[o] = (uint8_t)s.lines;
        if (r.actions) r.actions[o] = act;
        if (kStepOut && r.reward_f64) r.reward_f64[o] = rew;
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
          r.info[o] = inf;
        }
      }
      if (term && primary) {  // info['final_score'] / info['moves'] of the ending episode (wrappers.py:97-101)
        if (r.final_score) r.final_score[o] = s.score;
        if (r.final_moves) r.final_moves[o] = s.moves;
      }
      if (term && a.autoreset) {  // wrappers.py:97-102
        rng_moved = true;
        if constexpr (lazy_reset) {
          s.has_seed = e.has_seed[i] != 0;
          if (s.has_seed) {
            s.seed_hi = e.seed_hi[i];
            s.seed_lo = e.seed_lo[i];
          }
          reset_lane(t, s.has_seed, s.seed_hi, s.seed_lo, s.rng, s.B, s.hand, m);
        } else if (s.has_seed) {
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
      if (r.mask && primary) {
        r.mask[3 * o + 0] = m[0];
        r.mask[3 * o + 1] = m[1];
        r.mask[3 * o + 2] = m[2];
      }
      act = random_policy_u(m[0], m[1], m[2], u_next);  // Philox (seed, env, policy_step0 + step + 1)
    }
#if defined(BB_ROLL_DIAG) && BB_ROLL_DIAG == 3
    BB_DIAG_T(c3);
    dg[0] += c1 - c0;
    dg[1] += c2 - c1;
    dg[2] += c3 - c2;
#endif
  }
#if defined(BB_ROLL_DIAG) && BB_ROLL_DIAG == 3
  dg[17] = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && a.dbg_out)
    for (int q = 0; q < 18; ++q) a.dbg_out[18 * wave + q] = dg[q];
#endif
  if (primary && kSingle && BB_STEP_COND_STORE == 1) {  // only the columns that changed (a bb_step leaves most of rng / combo / lines alone)
    if (s.B != s0.B) e.board[i] = s.B;
    if (s.hand != s0.hand) e.hand[i] = s.hand;
    if (s.rng.hi != s0.rng.hi || s.rng.lo != s0.rng.lo) {
      e.rng_hi[i] = s.rng.hi;
      e.rng_lo[i] = s.rng.lo;
    }
    if (s.rng.buf != s0.rng.buf) e.rng_buf[i] = s.rng.buf;
    if (s.score != s0.score) e.score[i] = s.score;
    if (s.combo != s0.combo) e.combo[i] = s.combo;
    if (s.max_combo != s0.max_combo) e.max_combo[i] = s.max_combo;
    if (s.moves != s0.moves) e.moves[i] = s.moves;
    if (s.lines_tot != s0.lines_tot) e.lines[i] = s.lines_tot;
    if (s.blocks != s0.blocks) e.blocks[i] = s.blocks;
    if (s.prev != s0.prev) e.prev[i] = (uint16_t)s.prev;
  } else if (primary) {
    e.board[i] = s.B;
    e.hand[i] = s.hand;
    if (!(kSingle && BB_STEP_COND_STORE == 2) || rng_moved) {
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
  }
  if (primary) {
    e.mask[3 * i + 0] = m[0];
    e.mask[3 * i + 1] = m[1];
    e.mask[3 * i + 2] = m[2];
    if (r.next_action) r.next_action[i] = act;
  }
}

// ---------------------------------------------------------------------------
// bb_rollout with the hand searches taken off the step loop.
//
// rollout_kernel runs a wave's parked envs through the wave search inside the
// step: the whole wave (32 envs) waits for it, and with two waves per SIMD at
// 65,536 envs both are latency-bound (~41% VALU issue).  Here a workgroup holds
// kAEW env waves (32 envs each, the same two-copy layout and step code) and
// kASW search waves.  An env whose new hand the in-lane quick test leaves open
// posts its post-move board and rolled-back stream to an LDS record and is
// blocked; its wave goes on stepping its other envs (each env keeps its own
// step counter, outputs go to [its step][N]).  A search wave polls the records
// of its env waves, runs gen_hands_multi over every posted env at once and
// returns stream + hand; the env finalizes that step on its next iteration.
// Each env's trajectory is the one rollout_kernel computes (the same draws,
// the same tests, the same Philox keys), so the outputs are identical; only
// the order in which a wave's envs advance changes.  The SIMD gets a third
// wave of independent work, and a search no longer stalls 31 other envs.
//
// Termination: an env wave ends when each of its envs has done T steps (it
// never waits: blocked envs are polled once per iteration), and raises its
// flag; a search wave ends when the flags of all its env waves are up (a wave
// raises it only after every request it posted was answered).  An iteration
// cap on the env waves bounds the kernel even if a record were lost.
// ---------------------------------------------------------------------------
#ifndef BB_ASYNC
#define BB_ASYNC 1  // bb_rollout without bb_step outputs: env waves + search waves (0: rollout_kernel)
#endif
#ifndef BB_ASYNC_ENVS
#define BB_ASYNC_ENVS 64  // envs per env wave: 64 (one lane per env; 4 env + 4 search waves per CU: 1.074e10)
                          // or 32 (two copies per env, 8 env waves per CU: 1.006e10)
#endif
#ifndef BB_ASYNC_EW
#define BB_ASYNC_EW (256 / BB_ASYNC_ENVS)  // env waves per workgroup (256 envs: one workgroup per CU at 65,536)
#endif
#ifndef BB_ASYNC_SW
#define BB_ASYNC_SW 4  // search waves per workgroup; each serves BB_ASYNC_EW / BB_ASYNC_SW env waves (<= 64 envs)
#endif
#ifndef BB_ASYNC_SPRIO
#define BB_ASYNC_SPRIO 3  // s_setprio of the search waves while they search (0: 5.6e9, 1: 9.58e9, 3: 9.60e9)
#endif
#ifndef BB_ASYNC_POOL
#define BB_ASYNC_POOL 1  // every search wave takes posted envs of the whole workgroup (LDS compare-and-swap);
                         // 0: search wave s serves env waves 2s, 2s+1 (9.60e9 vs 9.89e9 pooled)
#endif
#ifndef BB_ASYNC_FAIR
// env waves: the one behind its SIMD partner takes s_setprio 1 (0: no priority).  With 64-env waves each SIMD
// holds one env wave, so there is no partner: off (1.093e10 vs 1.076e10 with the LDS counters kept)
#define BB_ASYNC_FAIR (BB_ASYNC_ENVS == 32)
#endif
#ifndef BB_ASYNC_SLOTS
#define BB_ASYNC_SLOTS 1  // in-lane quick-test slots per copy (copy c tests slots c * n .. c * n + n - 1)
#endif
#ifndef BB_ASYNC_SLOTS64
#define BB_ASYNC_SLOTS64 2  // 64-env waves: in-lane quick-test slots per env (0, 1: the two copies' slots)
#endif
#ifndef BB_ASYNC_PTOP
#define BB_ASYNC_PTOP 0  // 64-env waves: the policy uniform drawn at the top of every iteration
#endif
#ifndef BB_ASYNC_DEARLY
#define BB_ASYNC_DEARLY 0  // attempt 1's three draws made for every lane before the move
#endif
#ifndef BB_ASYNC_LINEONLY
#define BB_ASYNC_LINEONLY 0  // search waves: slow_phase_wave's line-only second order (bb_step's kLineOnly)
#endif
#ifndef BB_ASYNC_STEP
#define BB_ASYNC_STEP 0  // bb_step (T = 1, no info / fp64 reward) through rollout_async_kernel
#endif
#ifndef BB_ASYNC_EARLY
#define BB_ASYNC_EARLY 1  // search waves hand back each env when its round decides it, not at the call's end (1.105e10 vs 1.076e10)
#endif
#ifndef BB_ASYNC_LATEPOLL
#define BB_ASYNC_LATEPOLL 1  // env waves poll their posted envs after the moves (0: before them; 1.017e10 vs 9.89e9)
#endif
#ifndef BB_ASYNC_DIAG
#define BB_ASYNC_DIAG 0  // per-wave counters into dbg_out (tools/diag_async.py, BB_DEBUG_MODE=16)
#endif
#ifndef BB_ASYNC_SLEEP
#define BB_ASYNC_SLEEP 1  // s_sleep of an idle search wave between polls
#endif
constexpr int kAEW = BB_ASYNC_EW, kASW = BB_ASYNC_SW;
static_assert(kAEW % kASW == 0 || kASW % kAEW == 0 || BB_ASYNC_POOL, "search waves split the env waves");
constexpr int kABlock = 64 * (kAEW + kASW);
constexpr int kAE = BB_ASYNC_ENVS;
static_assert(kAE == 32 || kAE == 64, "async env waves: 32 or 64 envs");
constexpr int kAEnvs = kAE * kAEW;  // envs per workgroup

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
  constexpr int kE = kAE;
  constexpr int kCopies = 64 / kE;
  __shared__ Tables t;
  __shared__ uint32_t scratch[kABlock];  // 64 words per wave (the search waves' slow_phase_wave)
  __shared__ JumpRow jt[kJumpMax + 1];
  __shared__ ARecs arec;
  __shared__ uint32_t astat[kAEnvs];  // 0 idle, 1 posted, 2 answered
  __shared__ uint32_t afin[kAEW];
  __shared__ uint32_t wave_simd[kAEW + kASW];
  __shared__ uint32_t prog[kAEW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint32_t* lds = scratch + (threadIdx.x & ~63);
  if (threadIdx.x < kAEnvs) astat[threadIdx.x] = 0u;
  if (threadIdx.x < kAEW) afin[threadIdx.x] = 0u;
  if (lane == 0) {
    wave_simd[wv] = ((uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3u;  // HW_ID.SIMD_ID
    if (wv < kAEW) prog[wv] = 0u;
  }
  stage_tables<true>(t, g_rows, g_d, jt, a.jump);  // ends with __syncthreads (also orders the inits above)

  if (wv >= kAEW) {
    // ---------------- search wave ----------------
    const int sw = wv - kAEW;
    Pcg rng;
    rng.hi = rng.lo = 0ull;
    rng.buf = 0u;
    rng.has = 0u;
    rng.inc_hi = rng.inc_lo = 0ull;
    // pooled claims for rollouts; a single step (bb_step) keeps each search wave on its own env waves'
    // records, so that the step's parked envs are spread over the search waves instead of one taking all
    const bool pool = BB_ASYNC_POOL && r.steps > 1;
    constexpr int kPer = kAEnvs / 64;  // pool: records watched per lane, k * 64 + lane
    static_assert(kAEnvs % 64 == 0, "pool: whole records per lane");
    constexpr int kOwn = kAEnvs / kASW;  // own records per search wave (no pool)
    static_assert(kOwn <= 64, "a search wave serves <= 64 envs");
    int rid = pool ? lane : sw * kOwn + lane;
    const bool mine = lane < kOwn;
    uint64_t B = 0ull;
#if BB_ASYNC_DIAG  // diagnostics (BB_DEBUG_MODE=16): calls, envs served, search cycles, polls, phase cycles, rounds
    uint64_t dcalls = 0, denvs = 0, dcyc = 0, dpolls = 0;
    uint64_t dprof[6] = {0, 0, 0, 0, 0, 0};
    uint64_t* const dprof_p = dprof;
#else
    uint64_t* const dprof_p = nullptr;
#endif
#pragma unroll 1
    for (;;) {
      uint32_t sv = 0u;
      if (pool) {
        // claim the first posted record among this lane's (posted -> 3 by compare-and-swap)
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
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
      } else if (mine) {
        sv = __hip_atomic_load(&astat[rid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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
        bool released = false;
#if BB_ASYNC_EARLY
        // envs decided in an earlier round of the call go back to their env waves at once
        auto release = [&](bool d) {
          if (d && sv == 1u) {
            arec.hi[rid] = rng.hi;
            arec.lo[rid] = rng.lo;
            arec.buf[rid] = rng.buf;
            arec.has_ids[rid] = (rng.has ? 1u : 0u) | (ids << 1);
            lds_flag_store_release(&astat[rid], 2u);
            released = true;
          }
        };
        gen_hands_multi<64, (bool)BB_ASYNC_LINEONLY>(req, B, rng, ids, t.row, t.d, jt, lane, a.pack_first,
                                                     a.pack_next, lds, dprof_p, 0, release);
#else
        gen_hands_multi<64, (bool)BB_ASYNC_LINEONLY>(req, B, rng, ids, t.row, t.d, jt, lane, a.pack_first,
                                                     a.pack_next, lds);
#endif
#if BB_ASYNC_DIAG
        dcyc += __builtin_amdgcn_s_memtime() - c0;
        dcalls += 1;
        denvs += (uint64_t)__popcll(req);
#endif
        __builtin_amdgcn_s_setprio(0);
        if (sv == 1u && !released) {
          arec.hi[rid] = rng.hi;
          arec.lo[rid] = rng.lo;
          arec.buf[rid] = rng.buf;
          arec.has_ids[rid] = (rng.has ? 1u : 0u) | (ids << 1);
          lds_flag_store_release(&astat[rid], 2u);
        }
      } else {
        uint32_t fin = 1u;
#pragma unroll
        for (int q = 0; q < kAEW; ++q)  // every env wave (a cheap superset of the ones this wave serves)
          fin &= __hip_atomic_load(&afin[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (fin) break;  // wave-uniform (LDS word read by every lane)
#if BB_ASYNC_DIAG
        dpolls += 1;
#endif
        __builtin_amdgcn_s_sleep(BB_ASYNC_SLEEP);
      }
    }
#if BB_ASYNC_DIAG
    if (a.dbg_out && lane == 0) {
      uint64_t* o = a.dbg_out + 4 * ((size_t)(e.n + 31) / 32) + 12 * ((size_t)blockIdx.x * kASW + sw);
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
  const int half = lane / kE;  // copy index; 0 = primary copy of the env (stores)
  const int el = lane % kE;
  const int rid = wv * kE + el;  // this env's record
  const int i = blockIdx.x * kAEnvs + rid;
  const bool live = i < e.n;
  const bool primary = live && half == 0;
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
  int pw = wv;  // partner: the other env wave of this workgroup on this SIMD
#pragma unroll
  for (int k = 0; k < kAEW; ++k)
    if (k != wv && wave_simd[k] == wave_simd[wv]) pw = k;
  const uint32_t tie = wv < pw ? 1u : 0u;
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
  int ph = 0;   // copy 0: 0 ready to move, 1 posted (blocked), 2 hand known (finalize)
  uint32_t u_drawn = 0;
  uint32_t partner = 0;
  // Bounds (never reached by a correct run): an iteration that moves or finalizes some env advances one of the
  // wave's 2 * kE * T phases, so there are at most 2 * kE * T of them; a run of iterations in which every
  // unfinished env waits on a search lasts as long as that search (at most 100 attempts), so 2^24 of them in a
  // row (seconds) means a lost record.  Either cap ends the wave instead of hanging the GPU, and the wave then
  // raises the handle's status word (kStatusAsyncCap): the host fails the next call with BB_ERR_DEVICE.
  const int64_t cap = r.work_cap > 0 ? r.work_cap : 2 * (int64_t)kE * T + 4096;
  int64_t work_it = 0, idle_it = 0;  // idle_it: the current run of all-blocked iterations
#if BB_ASYNC_DIAG  // iterations, cycles, blocked env-iterations, iterations that moved no env | their cycles << 32
  uint64_t dit = 0, dblk = 0, didle = 0, didle_cyc = 0;
  const uint64_t dt0 = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll 1
  for (int it = 0; work_it < cap && idle_it < (1 << 24); ++it) {
    if (!__ballot(primary && st < T)) break;
#if BB_ASYNC_DIAG
    const uint64_t dti = __builtin_amdgcn_s_memtime();
    dit += 1;
    dblk += (uint64_t)__popcll(__ballot(primary && ph == 1));
    didle += __ballot(primary && ph != 1 && st < T) ? 0u : 1u;
#endif
    if (BB_ASYNC_FAIR) {  // the wave behind its SIMD partner (LDS iteration counters) takes the priority
      const int32_t lead = it - (int32_t)partner;
      if (lead < 0 || (lead == 0 && (((uint32_t)it ^ tie) & 1u))) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
      if (lane == 0) __hip_atomic_store(&prog[wv], (uint32_t)it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      partner = __hip_atomic_load(&prog[pw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // 1. answered searches: the stream after the accepted attempt and its hand
    auto poll = [&]() {
    if (primary && ph == 1) {
      if (lds_flag_load_acquire(&astat[rid]) == 2u) {
        s.rng.hi = arec.hi[rid];
        s.rng.lo = arec.lo[rid];
        s.rng.buf = arec.buf[rid];
        const uint32_t hi = arec.has_ids[rid];
        s.rng.has = hi & 1u;
        s.hand = (hi >> 1) | ((hi & 1u) << 22);
        __hip_atomic_store(&astat[rid], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ph = 2;
      }
    }
    };
    if (!BB_ASYNC_LATEPOLL) poll();
    // 2. the move of every ready env; a drawn hand is quick-tested by both copies (copy 1 takes the
    //    post-move board and the drawn pieces from copy 0, as in rollout_kernel)
    const bool mv = primary && ph == 0 && st < T;
    // one lane per env: this step's policy uniform depends only on the step counter, so it is drawn
    // here, without a branch, and its Philox rounds overlap the move's table reads
    const uint32_t u_top = (kCopies == 1 && BB_ASYNC_PTOP)
                               ? policy_uniform(a.policy_seed, a.env_offset + (uint64_t)i, r.policy_step0 + st + 1)
                               : 0u;
    Pcg after = s.rng;
    uint32_t ids0 = 0;
    bool drew0 = false;
#if BB_ASYNC_DEARLY
    // attempt 1's draws do not depend on the move: drawn for every lane before it (used where it drew)
    uint32_t ex0 = 0, ex1 = 0, ex2 = 0;
    draw3(after, ex0, ex1, ex2);
    if (mv) {
      drew0 = apply_move_bf(t, s, act);
      if (drew0) {
        ids0 = ex0 | (ex1 << 6) | (ex2 << 12);
        s.hand = ids0;
      }
    }
#else
    if (mv) {
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
#endif
    const uint32_t idq = copy0_bcast<kE>((uint32_t)ids0 | ((uint32_t)drew0 << 31));
    const uint64_t Bq = ((uint64_t)copy0_bcast<kE>((uint32_t)(s.B >> 32)) << 32) | copy0_bcast<kE>((uint32_t)s.B);
    bool park = false;
    if (live && (idq >> 31)) {
      const uint32_t q0 = idq & 63u, q1 = (idq >> 6) & 63u, q2 = (idq >> 12) & 63u;
      constexpr int kSl = kE == 64 ? BB_ASYNC_SLOTS64 : BB_ASYNC_SLOTS;  // slots tested by this lane
      bool ok = quick_slot_bf(Bq, q0, q1, q2, t.row, t.d, half * kSl);
#pragma unroll
      for (int k = 1; k < kSl; ++k) ok = quick_slot_bf(Bq, q0, q1, q2, t.row, t.d, half * kSl + k) || ok;
      park = !ok;
    }
    const uint64_t rej = __ballot(park);
    uint64_t okb = ~rej;  // either copy accepted
#pragma unroll
    for (int sft = kE; sft < 64; sft <<= 1) okb |= (okb >> sft) | (okb << (64 - sft));
    const bool accepted = (okb >> lane) & 1ull;
    if (mv) {
      if (drew0) {
        if (accepted) s.rng = after;
        s.hand = (s.hand & 0x3FFFFu) | ((uint32_t)s.rng.has << 22);
        if (accepted) {
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
      } else {
        ph = 2;  // no draw (or an invalid action): the hand is known
      }
    }
    if (BB_ASYNC_LATEPOLL) poll();  // after the moves: answers that arrived meanwhile finalize this iteration
    // 3. the policy uniforms: copy c draws the uniform of step st + 1 + c on the env's even steps
    const bool fin = primary && ph == 2;
    const uint32_t sb = copy0_bcast<kE>((uint32_t)st | ((uint32_t)fin << 31));
    const int stc = (int)(sb & 0x7FFFFFFFu);
    if (!(kCopies == 1 && BB_ASYNC_PTOP) && (sb >> 31) && (stc % kCopies) == 0)
      u_drawn = policy_uniform(a.policy_seed, a.env_offset + (uint64_t)i, r.policy_step0 + stc + 1 + half);
    const uint32_t u_next = (kCopies == 1 && BB_ASYNC_PTOP) ? u_top
                          : kCopies == 1 ? u_drawn : (uint32_t)__shfl((int)u_drawn, el + kE * (stc % kCopies));
    // 4. finalize every env whose hand is known (rollout_kernel's finalize)
    if (fin) {
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
      }
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
      act = random_policy_u(m[0], m[1], m[2], u_next);  // Philox (seed, env, policy_step0 + step + 1)
      st += 1;
      ph = 0;
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
  __builtin_amdgcn_s_setprio(0);
  // left through a cap with envs short of T steps: this launch's outputs and final state are incomplete
  if (__ballot(primary && st < T) && lane == 0)
    __hip_atomic_store(e.status, kStatusAsyncCap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#if BB_ASYNC_DIAG
  if (a.dbg_out && lane == 0) {
    uint64_t* o = a.dbg_out + 4 * ((size_t)blockIdx.x * kAEW + wv);
    o[0] = dit;
    o[1] = __builtin_amdgcn_s_memtime() - dt0;
    o[2] = dblk;
    o[3] = didle | (didle_cyc << 32);
  }
#endif
  if (primary) {
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
  auto grid = [&](int epw, int blk) { return dim3((unsigned)((((int64_t)e.n + epw - 1) / epw * 64 + blk - 1) / blk)); };
  if (r.steps == 1 && BB_ASYNC_STEP && !r.info && !r.reward_f64) {  // bb_step through the async kernel
    const dim3 g((unsigned)(((int64_t)e.n + kAEnvs - 1) / kAEnvs)), b(kABlock);
    hipLaunchKernelGGL(rollout_async_kernel, g, b, 0, s, e, rows, d, a, r);
  } else if (r.steps == 1) {  // bb_step
    const dim3 g = grid(kStepEnvs, kStepRollBlock), b(kStepRollBlock);
    if (r.info || r.reward_f64)
      hipLaunchKernelGGL((rollout_kernel<true, true, kStepEnvs, kStepRollBlock>), g, b, 0, s, e, rows, d, a, r);
    else
      hipLaunchKernelGGL((rollout_kernel<false, true, kStepEnvs, kStepRollBlock>), g, b, 0, s, e, rows, d, a, r);
  } else if (BB_ASYNC && kRollEnvs == 32 && !r.info && !r.reward_f64) {
    const dim3 g((unsigned)(((int64_t)e.n + kAEnvs - 1) / kAEnvs)), b(kABlock);
    hipLaunchKernelGGL(rollout_async_kernel, g, b, 0, s, e, rows, d, a, r);
  } else {
    const dim3 g = grid(kRollEnvs, kRollBlock), b(kRollBlock);
    if (r.info || r.reward_f64)
      hipLaunchKernelGGL((rollout_kernel<true, false, kRollEnvs, kRollBlock>), g, b, 0, s, e, rows, d, a, r);
    else
      hipLaunchKernelGGL((rollout_kernel<false, false, kRollEnvs, kRollBlock>), g, b, 0, s, e, rows, d, a, r);
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

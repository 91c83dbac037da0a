// bb_env.hip -- MI355X (gfx950) vectorised Block Blast environment.
//
// One env per lane, wave64, 64-thread workgroups.  Per-env state lives in HBM
// as structure-of-arrays (coalesced 4/8-byte columns); the 37-piece table and
// the pair-offset table are staged into LDS once per workgroup.  A step reads
// the state, applies the action on a uint64 bitboard, clears lines, scores,
// draws a new hand when all three slots are used (numpy-exact PCG64 stream +
// exact solvability test, hard boards escalated to the whole wave), computes
// the shaped fp64 reward, the 192-bit action mask and the game-over flag,
// auto-resets terminated envs, and writes state + outputs back.
//
// Reference semantics: src/environment/wrappers.py:75-116 (vec step, auto-reset)
// -> src/environment/block_blast_env.py:224-264 (step, invalid action, reward
// 148-193) -> src/game/engine.py:390-454 (make_move) and board.py.
#include <hip/hip_runtime.h>

#include "bb_device.h"
#include "bb_solver.h"
#include "bb_env_internal.h"

namespace bb {

constexpr int kBlock = 64;
// Per-lane search budget (anchors_of() evaluations) before a board is handed
// to the whole wave.
constexpr int kLaneBudget = 48;

struct Tables {
  PieceRow row[kPieces];
  uint8_t d[kPieces * kPieces];
};

__device__ __forceinline__ void stage_tables(Tables& t, const PieceRow* g_rows, const uint8_t* g_d) {
  const int tid = threadIdx.x;
  if (tid < kPieces) t.row[tid] = g_rows[tid];
  for (int i = tid; i < kPieces * kPieces; i += blockDim.x) t.d[i] = g_d[i];
  __syncthreads();
}

__device__ __forceinline__ void masks_of(const Tables& t, uint64_t B, uint32_t hand, uint64_t m[3]) {
  const uint32_t used = hand_used(hand);
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    m[s] = (used >> s) & 1u ? 0ull : anchors_of(t.row[hand_id(hand, s)], B);
  }
}

__device__ __forceinline__ Pcg load_pcg(const EnvDev& e, int i, uint32_t hand) {
  Pcg r;
  r.hi = e.rng_hi[i];
  r.lo = e.rng_lo[i];
  r.inc_hi = e.inc_hi[i];
  r.inc_lo = e.inc_lo[i];
  r.buf = e.rng_buf[i];
  r.has = hand_has32(hand);
  return r;
}

// ---------------------------------------------------------------------------
// reset: engine.py:127-153 + block_blast_env.py:210-217
// ---------------------------------------------------------------------------
__device__ __forceinline__ void reset_lane(const Tables& t, const EnvDev& e, int i, Pcg& rng, uint64_t& B,
                                           uint32_t& hand, uint64_t m[3]) {
  if (e.has_seed[i]) {  // re-seed with seed_value every episode
    rng.hi = e.seed_hi[i];
    rng.lo = e.seed_lo[i];
    rng.buf = 0;
    rng.has = false;
  }
  B = 0;
  uint32_t ids = 0;
  int attempt = 0;
  // On an empty board the first attempt always succeeds within a few anchor
  // evaluations; the budget is unlimited so this never escalates.
  gen_hand_lane(0ull, rng, ids, attempt, t.row, t.d, kUnlimited);
  hand = hand_pack(ids & 63u, (ids >> 6) & 63u, (ids >> 12) & 63u, 0u, false, rng.has);
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

__global__ void __launch_bounds__(kBlock) reset_kernel(EnvDev e, const PieceRow* g_rows, const uint8_t* g_d,
                                                       const uint8_t* sel) {
  __shared__ Tables t;
  stage_tables(t, g_rows, g_d);
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= e.n) return;
  if (sel && !sel[i]) return;
  Pcg rng = load_pcg(e, i, e.hand[i]);
  uint64_t B;
  uint32_t hand;
  uint64_t m[3];
  reset_lane(t, e, i, rng, B, hand, m);
  store_reset(e, i, rng, hand, m);
}

// ---------------------------------------------------------------------------
// step
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) step_kernel(EnvDev e, const PieceRow* g_rows, const uint8_t* g_d,
                                                      const int32_t* __restrict__ actions, StepArgs a) {
  __shared__ Tables t;
  stage_tables(t, g_rows, g_d);
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const bool live = i < e.n;

  uint64_t B = 0;
  uint32_t hand = 0;
  int act = -1;
  if (live) {
    B = e.board[i];
    hand = e.hand[i];
    act = actions[i];
  }

  // ---- validity: block_blast_env.py:237-245 -> engine.py:326-346 ----------
  const int p = act >> 6;           // a // 64 for a >= 0
  const int cell = act & 63;        // r*8 + c
  uint32_t used = hand_used(hand);
  bool valid = live && act >= 0 && act < 192 && !hand_over(hand) && !((used >> p) & 1u);
  PieceRow pr{};
  if (valid) {
    pr = t.row[hand_id(hand, p)];
    valid = ((pr.anchors >> cell) & 1ull) && ((pr.shape << cell) & B) == 0;
  }

  // Running per-env state (only loaded when the move is legal).
  Pcg rng{};
  int64_t score = 0;
  int combo = 0, max_combo = 0, moves = 0, lines_tot = 0, blocks = 0;
  int nblk = 0, lines = 0, cm = 1;
  int64_t gained = 0;
  bool pending = false;
  bool drew = false;
  int attempt = 0;
  uint32_t ids = hand & 0x3FFFFu;
  uint32_t has_bit = hand & (1u << 22);
  if (valid) {
    score = e.score[i];
    combo = e.combo[i];
    max_combo = e.max_combo[i];
    moves = e.moves[i];
    lines_tot = e.lines[i];
    blocks = e.blocks[i];
    // ---- make_move: engine.py:406-429 ----------------------------------
    nblk = (int)pr.ncells;
    B |= pr.shape << cell;
    used |= 1u << p;
    moves += 1;
    blocks += nblk;
    int rows, cols;
    B = clear_full(B, rows, cols);
    lines = rows + cols;
    if (lines > 0) {
      combo += 1;
      max_combo = combo > max_combo ? combo : max_combo;
      lines_tot += lines;
      cm = lines < 4 ? lines : 4;
    } else {
      combo = 0;
    }
    gained = nblk;
    if (lines > 0) {
      const int streak = combo + 1 < 8 ? combo + 1 : 8;  // post-increment combo (engine.py:261)
      gained += (int64_t)(lines * 8 * 10) * cm * streak;  // blocks_in_lines = lines*8 (engine.py:427)
    }
    score += gained;
    // ---- all three used -> new hand (engine.py:432-437) -----------------
    if (used == 7u) {
      rng = load_pcg(e, i, hand);
      used = 0;
      drew = true;
      pending = !gen_hand_lane(B, rng, ids, attempt, t.row, t.d, kLaneBudget);
    }
  }

  // ---- escalate budget-exhausted boards to the whole wave -----------------
  uint64_t pend = __ballot(pending);
  while (pend) {
    const int src = __ffsll((unsigned long long)pend) - 1;
    pend &= pend - 1;
    Pcg w;
    w.hi = __shfl(rng.hi, src);
    w.lo = __shfl(rng.lo, src);
    w.inc_hi = __shfl(rng.inc_hi, src);
    w.inc_lo = __shfl(rng.inc_lo, src);
    w.buf = __shfl(rng.buf, src);
    w.has = __shfl((int)rng.has, src) != 0;
    const uint64_t wB = __shfl(B, src);
    const int watt = __shfl(attempt, src);
    uint32_t wids = 0;
    gen_hand_wave(wB, w, wids, watt, t.row, t.d, lane);
    if (lane == src) {
      rng = w;
      ids = wids;
    }
  }

  // ---- finalise: game over, reward, info, auto-reset, mask ---------------
  if (!live) return;
  uint64_t m[3];
  if (valid) {
    // numpy's has_uint32 flag lives in the hand word.
    if (drew) has_bit = (uint32_t)rng.has << 22;
    hand = (ids & 0x3FFFFu) | (used << 18) | has_bit;
  }
  masks_of(t, B, hand, m);

  float rew32;
  double rew = -10.0;
  bool term = false;
  const uint32_t prev = valid ? (uint32_t)e.prev[i] : 0u;
  int holes = 0;
  int center = 0;
  if (valid) {
    const bool over = (m[0] | m[1] | m[2]) == 0ull;  // engine.py:440-441
    if (over) hand |= 1u << 21;
    // ---- _calculate_reward: block_blast_env.py:158-193, fp64 in order -----
    double R = 0.0;
    R = __dadd_rn(R, __dmul_rn((double)nblk, a.cfg.block_placed));
    R = __dadd_rn(R, a.cfg.survival_bonus);
    if (lines > 0) {
      double lr = __dmul_rn((double)lines, a.cfg.line_clear_base);
      lr = __dmul_rn(lr, (double)cm);
      R = __dadd_rn(R, lr);
      if (cm > 1) R = __dadd_rn(R, __dmul_rn((double)(cm - 1), a.cfg.combo_multiplier_bonus));
    }
    if (over) R = __dadd_rn(R, a.cfg.game_over_penalty);
    holes = count_holes(B);
    const int dh = holes - (int)(prev & 0xFFu);
    if (dh > 0) R = __dadd_rn(R, __dmul_rn((double)dh, a.cfg.hole_penalty));
    center = __popcll(B & kCenter);
    if (center <= (int)(prev >> 8)) R = __dadd_rn(R, a.center_tenth);  // openness >= previous
    rew = R;
    term = over;
  } else if (a.info) {
    holes = count_holes(B);
  }
  rew32 = (float)rew;

  if (a.info) {
    bb_info inf;
    inf.score = valid ? score : e.score[i];
    inf.score_gained = gained;
    inf.term_board = B;
    inf.moves = valid ? moves : e.moves[i];
    inf.lines = valid ? lines_tot : e.lines[i];
    inf.max_combo = valid ? max_combo : e.max_combo[i];
    inf.blocks = valid ? blocks : e.blocks[i];
    inf.term_hand = hand;
    inf.holes = (uint8_t)holes;
    inf.filled = (uint8_t)__popcll(B);
    inf.flags = (uint8_t)((valid ? 0u : 1u) | (term ? 2u : 0u) | (valid ? 4u : 0u));
    inf.last_blocks = (uint8_t)nblk;
    inf.last_lines = (uint8_t)lines;
    inf.last_cm = (uint8_t)cm;
    inf.pad[0] = inf.pad[1] = 0;
    a.info[i] = inf;
  }
  a.reward[i] = rew32;
  a.terminated[i] = term ? 1 : 0;
  if (a.reward_f64) a.reward_f64[i] = rew;
  if (a.lines) a.lines[i] = (uint8_t)lines;

  if (term && a.autoreset) {
    // wrappers.py:97-102: env.reset() with the stored seed_value.
    if (!drew) rng = load_pcg(e, i, hand);  // unseeded envs continue their stream
    reset_lane(t, e, i, rng, B, hand, m);
    store_reset(e, i, rng, hand, m);
  } else if (valid) {
    e.board[i] = B;
    e.hand[i] = hand;
    if (drew) {
      e.rng_hi[i] = rng.hi;
      e.rng_lo[i] = rng.lo;
      e.rng_buf[i] = rng.buf;
    }
    e.score[i] = score;
    e.combo[i] = combo;
    e.max_combo[i] = max_combo;
    e.moves[i] = moves;
    e.lines[i] = lines_tot;
    e.blocks[i] = blocks;
    e.prev[i] = (uint16_t)(holes | (center << 8));
    e.mask[3 * i + 0] = m[0];
    e.mask[3 * i + 1] = m[1];
    e.mask[3 * i + 2] = m[2];
  }
  if (a.mask_out) {
    a.mask_out[3 * i + 0] = m[0];
    a.mask_out[3 * i + 1] = m[1];
    a.mask_out[3 * i + 2] = m[2];
  }
  if (a.next_action) {
    a.next_action[i] = random_policy(m[0], m[1], m[2], a.policy_seed, a.env_offset + (uint64_t)i, a.policy_step);
  }
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
                                const int64_t* __restrict__ index, const PieceRow* __restrict__ g_rows,
                                int n, float4* __restrict__ x) {
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
__global__ void expand_mask_kernel(const uint64_t* __restrict__ mbits, const int64_t* __restrict__ index,
                                   int n, float4* __restrict__ mf, int4* __restrict__ mi) {
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
  hipLaunchKernelGGL(reset_kernel, dim3((e.n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, e, rows, d, sel);
  return hipGetLastError();
}

hipError_t launch_step(const EnvDev& e, const PieceRow* rows, const uint8_t* d, const int32_t* actions,
                       const StepArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(step_kernel, dim3((e.n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, e, rows, d, actions, a);
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

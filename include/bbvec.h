/*
 * bbvec.h -- C-ABI of the MI355X-native Block Blast vectorised environment and
 * masked-PPO rollout kernels (libbbvec.so, gfx950).
 *
 * This is the drop-in boundary under the reference's Python surface
 * (SURVEY.md section 8(b)).  The reference has no FFI of its own; each entry
 * point below names the reference interface it replaces, and INTEGRATION.md
 * shows the ctypes binding a maintainer would add.
 *
 * Conventions
 *   - Plain pointers and sizes only; no torch types.  "d_" pointers are device
 *     (HBM) pointers owned by the caller (e.g. tensor.data_ptr()); "h_" are host.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  All
 *     launches are asynchronous on that stream; nothing allocates or syncs
 *     inside bb_step / bb_obs / bb_masked_sample / bb_gae (graph-capturable).
 *   - Return value: 0 = BB_OK, negative = error; bb_last_error() explains.
 *     An invalid *action* is not an error: it is reproduced in-kernel as the
 *     reference does (reward -10, no state change; block_blast_env.py:240-245).
 *   - A handle is single-stream and not re-entrant (the reference is
 *     single-threaded).  Multi-GPU = one handle per process/device.
 *
 * Mask bit layout (shared by every entry point): uint64 mask[N][3], word p is
 * piece slot p, bit (r*8+c) set iff placing slot p at (r,c) is legal; flat
 * action a = p*64 + r*8 + c (block_blast_env.py:104-132).
 */
#ifndef BBVEC_H
#define BBVEC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BB_ABI_VERSION 8  /* 2: bb_step_out.final_score / final_moves; 3: bb_sync, BB_ERR_DEVICE;
                              4: bb_conv_in_* and bb_relu_bias_grad* removed;
                              5: bb_conv3x3_forward_stats / _stats_parts and bb_bn_forward_parts removed;
                              6: bb_build_id; bb_obs / bb_snapshot report BB_ERR_DEVICE;
                                 bb_conv3x3_f32_prep / _forward, bb_linear_f32;
                              7: bb_ppo_loss_forward_bf16 / _backward_bf16;
                              8: bb_dropout_forward, bb_linear_bgrad, bb_linear_wgrad, bb_linear_n1_*;
                                 bb_conv_in_forward / _wgrad; bb_bn_backward_res; bb_ppo_loss_fused and the
                                 loss forward's d_cnt (one launch, the statistics finalised in it);
                                 bb_conv3x3_wgrad_partial / _reduce / _chunks, bb_bn_backward_red,
                                 bb_conv_in_forward_prep, bb_linear_bgrad2, bb_conv3x3_forward_stats,
                                 bb_conv3x3_stats_blocks, bb_bn_forward_part, bb_conv3x3_forward_bstats,
                                 bb_bn_backward_part */

#define BB_OK 0
#define BB_ERR_ARG (-1)
#define BB_ERR_HIP (-2)
#define BB_ERR_STATE (-3)
#define BB_ERR_DEVICE (-4) /* a kernel reported a failure through the handle's status word */

#define BB_NUM_PIECES 37
#define BB_ACTIONS 192

typedef struct bb_env bb_env;

/* Reward weights: block_blast_env.py:63-73 (defaults), overridable from the
 * YAML `rewards:` section exactly like reward_config.update(). */
typedef struct bb_reward_cfg {
  double line_clear_base;        /* 1.0   */
  double block_placed;           /* 0.01  */
  double game_over_penalty;      /* -1.0  */
  double hole_penalty;           /* -0.05 */
  double center_bonus;           /* 0.02  */
  double combo_multiplier_bonus; /* 0.5   */
  double survival_bonus;         /* 0.001 */
} bb_reward_cfg;

/* Per-env info record written by bb_step (optional output).  Mirrors the
 * `info` dict of block_blast_env.py:266-288 (values AFTER the move, BEFORE any
 * auto-reset) plus the terminal-observation latch of wrappers.py:97-102. */
typedef struct bb_info {
  int64_t score;          /* info['score'] (== info['final_score'] on termination) */
  int64_t score_gained;   /* info['last_move']['score_gained'] */
  uint64_t term_board;    /* board bits before auto-reset (terminal_observation) */
  int32_t moves;          /* info['moves'] */
  int32_t lines;          /* info['lines_cleared'] (total) */
  int32_t max_combo;      /* info['max_combo'] */
  int32_t blocks;         /* info['blocks_placed'] (total) */
  uint32_t term_hand;     /* packed hand word before auto-reset (see bb_state) */
  uint8_t holes;          /* info['holes'] */
  uint8_t filled;         /* popcount(board): info['board_fill'] = filled / 64 */
  uint8_t flags;          /* bit0 invalid_action, bit1 terminated, bit2 has last_move */
  uint8_t last_blocks;    /* info['last_move']['blocks_placed'] */
  uint8_t last_lines;     /* info['last_move']['lines_cleared'] */
  uint8_t last_cm;        /* info['last_move']['combo_multiplier'] */
  uint8_t pad[2];
} bb_info;

/* Outputs of one bb_step.  reward and terminated are required, the rest may be
 * NULL.  `next_action`, when non-NULL, runs the fused synthetic random policy
 * (BASELINE config 2): for every env, u = Philox4x32-10(key=policy_seed,
 * ctr=(env_offset+i, policy_step)).x, k = (u * popcount(mask)) >> 32, and the
 * action is the k-th set bit of the post-step 192-bit mask (0 if empty). */
typedef struct bb_step_out {
  float* reward;          /* [N] f32 (wrappers.py:88,105)                       */
  uint8_t* terminated;    /* [N] 0/1; truncated is always false                  */
  double* reward_f64;     /* [N] optional: the fp64 reward BlockBlastEnv returns */
  uint64_t* mask;         /* [N][3] optional: post-step (post-reset) mask bits   */
  uint8_t* lines;         /* [N] optional: lines cleared by this move            */
  bb_info* info;          /* [N] optional                                        */
  int32_t* next_action;   /* [N] optional: fused random policy for the next step */
  uint64_t policy_seed;
  uint64_t policy_step;
  uint64_t env_offset;    /* global index of env 0 (multi-GPU shards)            */
  int64_t* final_score;   /* [N] optional: written ONLY for envs that terminated:
                             the episode's score before the auto-reset
                             (info['final_score'], wrappers.py:97-101)          */
  int32_t* final_moves;   /* [N] optional: likewise its moves (info['moves'];
                             scripts/train.py:196-201 reads both)               */
} bb_step_out;

/* Host view of the packed per-env state (bb_get_state / bb_set_state).
 * hand word: bits 0-5 slot0 piece id, 6-11 slot1, 12-17 slot2, 18-20 used,
 * 21 game_over, 22 pcg has_uint32.  Any pointer may be NULL (skipped). */
typedef struct bb_state_view {
  uint64_t* board;        /* [N] bit r*8+c = grid[r][c]                    */
  uint32_t* hand;         /* [N] packed hand word                           */
  int64_t* score;         /* [N]                                            */
  int32_t* combo;         /* [N] combo_count (engine.py:115)                */
  int32_t* max_combo;     /* [N]                                            */
  int32_t* moves;         /* [N]                                            */
  int32_t* lines;         /* [N] total_lines_cleared                        */
  int32_t* blocks;        /* [N] total_blocks_placed                        */
  uint8_t* prev_holes;    /* [N] BlockBlastEnv._prev_holes                  */
  uint8_t* prev_center;   /* [N] filled centre cells behind _prev_center_openness */
  uint64_t* rng;          /* [N][3] pcg state hi, state lo, uinteger        */
} bb_state_view;

/* ---- lifetime -------------------------------------------------------------
 * bb_create replaces VectorizedBlockBlastEnv.__init__ (wrappers.py:21-51) /
 * BlockBlastEnv.__init__ (block_blast_env.py:42-102).  autoreset=1 gives the
 * vec-env semantics (wrappers.py:97-102), 0 the single-env semantics.  The new
 * envs are unseeded until bb_seed + bb_reset. */
int bb_abi_version(void);
/* The id of the sources this library was built from: the first 16 hex digits of a SHA-256 over csrc/,
 * include/bbvec.h and the compiler flags (runtime/build.py source_id).  runtime/lib.load() refuses a
 * library whose id is not that of the sources beside it.  No reference counterpart. */
const char* bb_build_id(void);
int bb_create(int32_t num_envs, int32_t device, const bb_reward_cfg* cfg,
              int32_t autoreset, bb_env** out);
void bb_destroy(bb_env* env);
const char* bb_last_error(const bb_env* env); /* env may be NULL (last create error) */
int32_t bb_num_envs(const bb_env* env);

/* numpy-exact default_rng(seed) initialisation: SeedSequence(seed)
 * .generate_state(4, uint64) -> PCG64 set_seed.  out = {state_hi, state_lo,
 * inc_hi, inc_lo}.  Replaces np.random.default_rng (engine.py:109,138). */
int bb_pcg64_seed(uint64_t seed, uint64_t out[4]);

/* Per-env seeding (host arrays of length N).
 *   has_seed[i] == 1: seeded from seeds[i] (numpy default_rng(seeds[i])) now
 *     AND on every later reset -- the reference re-seeds each episode with
 *     seed_value (block_blast_env.py:212-215, engine.py:137-138);
 *   has_seed[i] == 2: same, but the post-seeding PCG64 words come from
 *     raw[i*4..i*4+3] = {state_hi, state_lo, inc_hi, inc_lo} (seeds that do
 *     not fit uint64, computed by the caller);
 *   has_seed[i] == 0: raw words (e.g. fresh OS entropy) and the stream
 *     continues across resets (seed_value None).
 * raw may be NULL when every has_seed is 1. */
int bb_seed(bb_env* env, const uint64_t* h_seeds, const uint8_t* h_has_seed,
            const uint64_t* h_raw);

/* Reset envs (all when d_env_mask is NULL, else those with mask[i] != 0):
 * engine.py:127-153 + block_blast_env.py:195-222. */
int bb_reset(bb_env* env, const uint8_t* d_env_mask, void* stream);

/* One step of every env with actions d_actions[N] (int32 flat actions):
 * VectorizedBlockBlastEnv.step (wrappers.py:75-116) -> BlockBlastEnv.step
 * (block_blast_env.py:224-264) -> GameEngine.make_move (engine.py:390-454).
 * If a launch fails, the handle refuses bb_step / bb_rollout / masked
 * bb_reset with BB_ERR_STATE until a full bb_reset (d_env_mask NULL): the
 * step kernel may already have parked envs whose search never ran. */
int bb_step(bb_env* env, const int32_t* d_actions, const bb_step_out* out,
            void* stream);

/* T steps of every env in ONE launch under the fused synthetic random policy
 * (BASELINE config 2; the reference's rollout loop of wrappers.py:128-137
 * sample_valid_actions -> wrappers.py:75-116 step, with the Philox policy of
 * bb_step_out.next_action in place of np.random.choice).  Output for output
 * and in the final state it equals T chained bb_step calls: call t takes
 * d_actions (t = 0) or call t-1's next_action, with policy_step =
 * policy_step0 + t + 1.  Per-step outputs are [T][N] (t-major); the env
 * state stays in registers between steps, so nothing but these outputs
 * touches HBM inside the rollout. */
typedef struct bb_rollout_out {
  float* reward;          /* [T][N] f32, required                             */
  uint8_t* terminated;    /* [T][N] 0/1, required                             */
  uint8_t* lines;         /* [T][N] optional: lines cleared by each move      */
  int32_t* actions;       /* [T][N] optional: the action applied at step t    */
  uint64_t* mask;         /* [T][N][3] optional: post-step (post-reset) masks */
  int32_t* next_action;   /* [N] optional: policy action after the last step  */
  uint64_t policy_seed;
  uint64_t policy_step0;
  uint64_t env_offset;    /* global index of env 0 (multi-GPU shards)         */
} bb_rollout_out;

int bb_rollout(bb_env* env, int32_t steps, const int32_t* d_actions,
               const bb_rollout_out* out, void* stream);

/* Device-side failures.  The rollout kernel bounds its own iterations so that
 * a logic error can never hang the GPU; if a bound is ever hit it writes the
 * handle's status word instead of failing silently.  Every later bb_step /
 * bb_rollout / bb_get_state / masked bb_reset then returns BB_ERR_DEVICE
 * (bb_last_error says which kernel and why) until a full bb_reset (d_env_mask
 * NULL).  Launches are asynchronous, so the check at the next call sees only
 * the launches that have finished by then; bb_sync waits for every launch on
 * `stream` and reports their status (BB_OK or BB_ERR_DEVICE / BB_ERR_HIP).
 * The reference has no device side; this replaces the exceptions its Python
 * step loop would raise (wrappers.py:75-116). */
int bb_sync(bb_env* env, void* stream);

/* Observation expansion (engine.py:478-507, block_blast_env.py:134-146,
 * wrappers.py:118-126).  Any output may be NULL:
 *   d_x      [N][4][8][8] f32: plane 0 board, planes 1-3 unused piece shapes
 *   d_mask_i8  [N][192] int8,  d_mask_f32 [N][192] f32,  d_mask_bits [N][3]. */
int bb_obs(bb_env* env, float* d_x, int8_t* d_mask_i8, float* d_mask_f32,
           uint64_t* d_mask_bits, void* stream);

/* Device pointers of the live state columns (board [N], hand [N], mask
 * [N][3]) for zero-copy snapshots into a device rollout buffer.  Valid until
 * bb_destroy; read them on the stream that runs bb_step. */
int bb_device_ptrs(bb_env* env, uint64_t** d_board, uint32_t** d_hand, uint64_t** d_mask);

/* Async device-to-device snapshot of the packed observation state into caller
 * buffers (the packed rollout-buffer record, ppo.py:100-102 without the f32
 * planes): board [N] u64, hand [N] u32, mask [N][3] u64.  Any may be NULL. */
int bb_snapshot(bb_env* env, uint64_t* d_board, uint32_t* d_hand, uint64_t* d_mask_bits, void* stream);

/* Synchronous state copies (tests / info / checkpoint).  bb_set_state also
 * overwrites the pcg state when v->rng is given. */
int bb_get_state(bb_env* env, const bb_state_view* h_view);
int bb_set_state(bb_env* env, const bb_state_view* h_view);

/* Diagnostics: per-env hand-search counters of the last bb_step, [N][4] =
 * {in-lane cycles, attempts | escalated << 32, wave cycles, board}.  Only
 * available when the env was created with BB_DEBUG_MODE having bit 1 set;
 * reading clears them.  NOTE: BB_DEBUG_MODE bit 1 (value 2) also switches the
 * escalate kernel from the shipped multi-env search (gen_hands_multi) to the
 * one-env-at-a-time wave search (gen_hand_wave) that these counters
 * instrument; both are exact (tests/test_gpu_solver_stress.py runs the
 * fallback), but the counters describe the fallback's work, not the shipped
 * path's. */
int bb_debug_counters(bb_env* env, uint64_t* h_out);

/* Synthetic random policy on its own (see bb_step_out.next_action). */
int bb_random_actions(const uint64_t* d_mask_bits, int32_t n, uint64_t seed,
                      uint64_t step, uint64_t env_offset, int32_t* d_actions,
                      void* stream);

/* Fused masked-categorical tail of BlockBlastNetwork.get_action_and_value
 * (network.py:173-180, 210-262; Categorical clamp semantics of torch 2.10):
 * logits f32 [n][192] (raw policy-head output, unmasked) + mask bits ->
 *   action (inverse-CDF sample with u from d_uniform[i] if non-NULL, else from
 *   Philox(seed, (env_offset+i, step)) word 1; argmax when deterministic),
 *   logp = log(clamp(p_a, 2^-23, 1-2^-23)), entropy = masked renormalised
 *   entropy with 1e-10 clamps.  Any of action/logp/entropy may be NULL.
 *   If d_action_in is non-NULL it is evaluated instead of sampling. */
int bb_masked_sample(const float* d_logits, const uint64_t* d_mask_bits,
                     int32_t n, const float* d_uniform, uint64_t seed,
                     uint64_t step, uint64_t env_offset, int32_t deterministic,
                     const int64_t* d_action_in, int64_t* d_action,
                     float* d_logp, float* d_entropy, void* stream);

/* bb_masked_sample with the Philox step read from device memory:
 * step = *d_step + step_add (no d_uniform, no d_action_in).  For a rollout
 * captured in a HIP graph (scripts/train.py:173-203 replayed per update):
 * the captured launches keep their step_add (0 .. T-1) and the caller
 * advances *d_step by T between replays, so every replay samples with fresh
 * uniforms, exactly as T eager calls with step = base + t would. */
int bb_masked_sample_dstep(const float* d_logits, const uint64_t* d_mask_bits,
                           int32_t n, uint64_t seed, const uint64_t* d_step,
                           uint64_t step_add, uint64_t env_offset,
                           int32_t deterministic, int64_t* d_action,
                           float* d_logp, float* d_entropy, void* stream);

/* GAE (RolloutBuffer.compute_returns_and_advantages, ppo.py:141-169) over
 * [T][N] f32 arrays, numpy-2 float32 operation order, no FMA contraction.
 * gamma and gamma_lambda are the f32 roundings of gamma and gamma*gae_lambda
 * (the latter multiplied in double first, as Python does). */
int bb_gae(const float* d_rewards, const float* d_values, const float* d_dones,
           const float* d_last_values, int32_t T, int32_t N, float gamma,
           float gamma_lambda, float* d_adv, float* d_ret, void* stream);

/* Packed rollout-buffer record -> network input for a minibatch
 * (RolloutBuffer.get_samples, ppo.py:171-213, with obs kept packed on device):
 * for j < n, src = d_index[j]: x[j] = expand(board[src], hand[src]),
 * mask_f32[j] = bits(mask[src]).  Either output may be NULL. */
int bb_gather_obs(const uint64_t* d_board, const uint32_t* d_hand,
                  const uint64_t* d_mask_bits, const int64_t* d_index,
                  int32_t n, float* d_x, float* d_mask_f32, void* stream);

/* Training-mode BatchNorm2d with an optional fused ReLU and an optional fused
 * bias of the preceding convolution, for the policy/value CNN's conv stack
 * (network.py:75-117 conv -> BatchNorm2d -> ReLU, ResidualBlock
 * network.py:14-30).  Input x is the convolution output WITHOUT its bias;
 * d_pre_bias (NULL = none) is that bias, added per channel before the
 * statistics, so the result equals nn.BatchNorm2d(conv(x) + bias).
 * dtype 0 = f32, 1 = bf16 activations; nhwc 0 = NCHW contiguous (HW * element
 * size a multiple of 16 bytes), 1 = NHWC / channels_last contiguous (C *
 * element size = 16 bytes times a power of two <= 256); weight / bias /
 * statistics are f32.  Forward = nn.BatchNorm2d training forward (batch mean,
 * biased variance for the normalisation; running_mean / running_var updated
 * with `momentum` and the unbiased variance when non-NULL, num_batches_tracked
 * incremented when non-NULL), then max(y, 0) if
 * relu.  d_ws is caller scratch of bb_bn_workspace_bytes(...) bytes (16-byte
 * aligned).  Backward takes the forward's input x and saved mean / inverse
 * std; with relu it recomputes the mask from x.  It writes dx and, where
 * non-NULL, dweight, dbias and d_dpre_bias = sum of dx per channel.  No
 * atomics: results are deterministic. */
int64_t bb_bn_workspace_bytes(int32_t dtype, int32_t nhwc, int32_t N, int32_t C, int32_t HW);
int bb_bn_forward(const void* d_x, int32_t dtype, int32_t nhwc, int32_t N, int32_t C, int32_t HW,
                  const float* d_pre_bias, const float* d_weight, const float* d_bias, float eps,
                  int32_t relu, double* d_ws, float* d_save_mean, float* d_save_invstd,
                  float* d_running_mean, float* d_running_var, float momentum,
                  int64_t* d_num_batches_tracked, void* d_y, void* stream);
/* bb_bn_forward with a residual input (ResidualBlock, network.py:14-30:
 * relu(bn2(conv2(.)) + x)): y = [relu](round(BatchNorm(x + pre_bias)) + res),
 * where round is the activation dtype's rounding (the BatchNorm output tensor
 * of the unfused module) and the sum is rounded once, as torch's add.  d_res
 * has x's shape, dtype and layout (16-byte aligned).  The backward is
 * bb_bn_backward_res (dy masked by y > 0, as threshold_backward; the masked dy
 * is also the residual's gradient). */
int bb_bn_forward_res(const void* d_x, const void* d_res, int32_t dtype, int32_t nhwc, int32_t N,
                      int32_t C, int32_t HW, const float* d_pre_bias, const float* d_weight,
                      const float* d_bias, float eps, int32_t relu, double* d_ws, float* d_save_mean,
                      float* d_save_invstd, float* d_running_mean, float* d_running_var, float momentum,
                      int64_t* d_num_batches_tracked, void* d_y, void* stream);
/* bb_bn_forward (d_res NULL) or bb_bn_forward_res from statistics partials a board convolution's forward
 * already produced (bb_conv3x3_forward_stats: d_part [nb_part][C][3] doubles, nb_part =
 * bb_conv3x3_stats_blocks(N, C)) instead of its own reduction pass over x: two launches (ABI 8). */
int bb_bn_forward_part(const void* d_x, const void* d_res, int32_t dtype, int32_t nhwc, int32_t N, int32_t C,
                       int32_t HW, const float* d_pre_bias, const float* d_weight, const float* d_bias, float eps,
                       int32_t relu, double* d_ws, float* d_save_mean, float* d_save_invstd, float* d_running_mean,
                       float* d_running_var, float momentum, int64_t* d_num_batches_tracked, void* d_y,
                       const double* d_part, int32_t nb_part, void* stream);
int bb_bn_backward(const void* d_x, const void* d_dy, int32_t dtype, int32_t nhwc, int32_t N,
                   int32_t C, int32_t HW, const float* d_pre_bias, const float* d_weight,
                   const float* d_bias, const float* d_save_mean, const float* d_save_invstd,
                   int32_t relu, double* d_ws, void* d_dx, float* d_dweight, float* d_dbias,
                   float* d_dpre_bias, void* stream);
/* bb_bn_backward with a board convolution's weight-gradient reduction (bb_conv3x3_wgrad_reduce's arguments)
 * run as extra workgroups of the BatchNorm finalisation's launch: two small launches in one (ABI 8). */
int bb_bn_backward_red(const void* d_x, const void* d_dy, int32_t dtype, int32_t nhwc, int32_t N, int32_t C, int32_t HW,
                       const float* d_pre_bias, const float* d_weight, const float* d_bias, const float* d_save_mean,
                       const float* d_save_invstd, int32_t relu, double* d_ws, void* d_dx, float* d_dweight,
                       float* d_dbias, float* d_dpre_bias, const float* d_conv_ws, int32_t conv_chunks,
                       int32_t conv_cin, int32_t conv_cout, int32_t conv_w_layout, float* d_conv_dw, void* stream);
/* bb_bn_backward / _red from reduction partials the board convolution that produced d_dy already made
 * (bb_conv3x3_forward_bstats: d_part [nb_part][C][3] doubles) instead of its own pass over x and dy; d_conv_ws
 * NULL: no carried weight-gradient reduction (ABI 8). */
int bb_bn_backward_part(const void* d_x, const void* d_dy, int32_t dtype, int32_t nhwc, int32_t N, int32_t C,
                        int32_t HW, const float* d_pre_bias, const float* d_weight, const float* d_bias,
                        const float* d_save_mean, const float* d_save_invstd, int32_t relu, double* d_ws, void* d_dx,
                        float* d_dweight, float* d_dbias, float* d_dpre_bias, const float* d_conv_ws,
                        int32_t conv_chunks, int32_t conv_cin, int32_t conv_cout, int32_t conv_w_layout,
                        float* d_conv_dw, const double* d_part, int32_t nb_part, void* stream);
/* The backward of bb_bn_forward_res with its ReLU: bb_bn_backward (relu = 0) over g = (y > 0 ? dy : 0), y the
 * forward's output (torch's threshold_backward): the reduction pass applies the mask and writes g to d_gres (x's
 * shape, dtype and layout; required), the elementwise pass reads it -- three launches, as bb_bn_backward, and no
 * pass of the mask's own.  g is also the residual's gradient.  d_conv_ws non-NULL: a preceding convolution's
 * weight-gradient reduction rides in the finalisation launch, as in bb_bn_backward_red. */
int bb_bn_backward_res(const void* d_x, const void* d_dy, const void* d_y, int32_t dtype, int32_t nhwc, int32_t N,
                       int32_t C, int32_t HW, const float* d_pre_bias, const float* d_weight, const float* d_bias,
                       const float* d_save_mean, const float* d_save_invstd, double* d_ws, void* d_dx,
                       float* d_dweight, float* d_dbias, float* d_dpre_bias, void* d_gres, const float* d_conv_ws,
                       int32_t conv_chunks, int32_t conv_cin, int32_t conv_cout, int32_t conv_w_layout,
                       float* d_conv_dw, void* stream);

/* The PPO minibatch loss (PPOAgent.update, ppo.py:362-401) with the masked
 * Categorical tail (network.py:173-180, 210-262), fused, forward and backward.
 * Per row i < B: logits f32 [B][192] (raw policy head), mask f32 [B][192]
 * (non-zero = legal), action, old log-prob, advantage, return and value.
 * Forward writes d_stats[6] = {policy_loss, value_loss, entropy, total_loss,
 * approx_kl, clip_fraction} (the reference's update metrics) and, if non-NULL,
 * d_loss[0] = total_loss, in one launch: d_ws is scratch of
 * bb_ppo_loss_workspace_bytes(B) bytes for the blocks' partial sums, which the
 * last block to finish adds in a fixed order (deterministic); d_cnt is one
 * uint32 counter, zero before the first launch and re-armed by each (ABI 8;
 * one counter per stream).  Backward takes d(total_loss) from d_grad_loss[0]
 * (device memory, so a HIP graph can replay it) and writes d/dlogits [B][192]
 * and d/dvalues [B], following torch autograd's rules for min / clamp / log.
 * bb_ppo_loss_fused is both in one launch (the caller knows the loss gradient
 * before the forward: the root of its backward), f32 (bf16 = 0) or bf16 (1)
 * logits / values and gradients. */
int64_t bb_ppo_loss_workspace_bytes(int32_t B);
int bb_ppo_loss_forward(const float* d_logits, const float* d_values, const float* d_mask,
                        const int64_t* d_actions, const float* d_old_logp, const float* d_adv,
                        const float* d_ret, int32_t B, float clip, float value_coef,
                        float entropy_coef, double* d_ws, uint32_t* d_cnt, float* d_stats, float* d_loss,
                        void* stream);
int bb_ppo_loss_backward(const float* d_logits, const float* d_values, const float* d_mask,
                         const int64_t* d_actions, const float* d_old_logp, const float* d_adv,
                         const float* d_ret, int32_t B, float clip, float value_coef,
                         float entropy_coef, const float* d_grad_loss, float* d_dlogits,
                         float* d_dvalues, void* stream);
/* The same loss on bf16 logits [B][192] and values [B] (the autocast network's outputs), widened exactly on
 * load; the backward writes d/dlogits and d/dvalues in bf16, rounded to nearest even: exactly the values of
 * autograd's casts around the f32 loss (bit-identical), without the four cast launches. */
int bb_ppo_loss_forward_bf16(const void* d_logits, const void* d_values, const float* d_mask,
                             const int64_t* d_actions, const float* d_old_logp, const float* d_adv,
                             const float* d_ret, int32_t B, float clip, float value_coef, float entropy_coef,
                             double* d_ws, uint32_t* d_cnt, float* d_stats, float* d_loss, void* stream);
int bb_ppo_loss_backward_bf16(const void* d_logits, const void* d_values, const float* d_mask,
                              const int64_t* d_actions, const float* d_old_logp, const float* d_adv,
                              const float* d_ret, int32_t B, float clip, float value_coef, float entropy_coef,
                              const float* d_grad_loss, void* d_dlogits, void* d_dvalues, void* stream);
int bb_ppo_loss_fused(const void* d_logits, const void* d_values, int32_t bf16, const float* d_mask,
                      const int64_t* d_actions, const float* d_old_logp, const float* d_adv, const float* d_ret,
                      int32_t B, float clip, float value_coef, float entropy_coef, const float* d_grad_loss,
                      void* d_dlogits, void* d_dvalues, double* d_ws, uint32_t* d_cnt, float* d_stats, float* d_loss,
                      void* stream);

/* The CNN's 3x3 / padding-1 convolutions over 8x8 boards (network.py:75-117,
 * ResidualBlock network.py:14-30; nn.Conv2d.forward and its autograd
 * backward) under bf16 autocast, for the layers with 64 or 128 channels in and
 * out.  Activations are bf16 NHWC (channels_last) [N][8][8][C], 16-byte
 * aligned; accumulation is f32.  bb_conv3x3_prep casts the nn.Conv2d weight
 * f32 [cout][cin][3][3] (w_layout 0) or [cout][3][3][cin] (w_layout 1, a
 * channels_last parameter) to bf16 (round to nearest even, as autocast) in two
 * images: d_wf [9][cout][cin] for the forward and d_wd [9][cin][cout], taps
 * reversed, for the data gradient.  bb_conv3x3_forward writes
 * y = conv(x, w) without bias (bf16 [N][8][8][cout]) from d_wf; the data
 * gradient is the same call on dy with d_wd and cin / cout swapped.
 * bb_conv3x3_wgrad writes the f32 weight gradient, in w_layout, of
 * y = conv(x, w) for the output gradient dy; d_ws is caller scratch of
 * bb_conv3x3_workspace_bytes(N, cin, cout) bytes.  No atomics: results are
 * deterministic. */
int64_t bb_conv3x3_workspace_bytes(int32_t N, int32_t cin, int32_t cout);
int bb_conv3x3_prep(const float* d_w, int32_t cin, int32_t cout, int32_t w_layout, void* d_wf, void* d_wd,
                    void* stream);
/* bb_conv3x3_prep for num_layers <= 16 layers in one launch (host arrays of
 * per-layer device pointers and sizes). */
int bb_conv3x3_prep_multi(int32_t num_layers, const float* const* h_w, const int32_t* h_cin,
                          const int32_t* h_cout, const int32_t* h_w_layout, void* const* h_wf,
                          void* const* h_wd, void* stream);
int bb_conv3x3_forward(const void* d_x, const void* d_w, int32_t N, int32_t cin, int32_t cout, void* d_y,
                       void* stream);
/* bb_conv3x3_forward plus a bf16 NHWC tensor d_add of y's shape, added to the
 * bf16-rounded convolution and rounded again (torch's bf16 add): the data
 * gradient of a ResidualBlock's first convolution with the identity path's
 * gradient folded in (network.py:14-30). */
int bb_conv3x3_forward_add(const void* d_x, const void* d_w, int32_t N, int32_t cin, int32_t cout,
                           const void* d_add, void* d_y, void* stream);
/* bb_conv3x3_forward that also writes, from its store pass, the following BatchNorm's batch-statistics
 * partials: per workgroup and output channel the f64 sum and sum of squares of the stored bf16 outputs
 * (d_part [bb_conv3x3_stats_blocks(N, cout)][cout][3], the third 0), for bb_bn_forward_part (ABI 8). */
int32_t bb_conv3x3_stats_blocks(int32_t N, int32_t cout);
int bb_conv3x3_forward_stats(const void* d_x, const void* d_w, int32_t N, int32_t cin, int32_t cout, void* d_y,
                             double* d_part, void* stream);
/* bb_conv3x3_forward run as a data gradient (y = dL/d(BatchNorm [+ ReLU] output)) that also writes that
 * BatchNorm's backward reduction partials: per workgroup and channel {sum g, sum g xhat, sum xhat}, g = y where
 * the forward's ReLU (relu != 0) passed, xhat = (bn_x - mean) invstd, bn_x the BatchNorm's bf16 NHWC input
 * (y's shape) and mean / invstd / weight / bias its forward's (bb_bn_backward_part; ABI 8). */
int bb_conv3x3_forward_bstats(const void* d_x, const void* d_w, int32_t N, int32_t cin, int32_t cout, void* d_y,
                              const void* d_bn_x, const float* d_mean, const float* d_invstd, const float* d_weight,
                              const float* d_bias, int32_t relu, double* d_part, void* stream);
int bb_conv3x3_wgrad(const void* d_x, const void* d_dy, int32_t N, int32_t cin, int32_t cout, float* d_ws,
                     int32_t w_layout, float* d_dw, void* stream);
/* bb_conv3x3_wgrad in two parts (ABI 8): the partial-sum kernel into d_ws, then the fixed-order sum of its
 * bb_conv3x3_wgrad_chunks(N, cin, cout) chunks into d_dw (alone, or inside bb_bn_backward_red); together
 * bit-identical to bb_conv3x3_wgrad. */
int32_t bb_conv3x3_wgrad_chunks(int32_t N, int32_t cin, int32_t cout);
int bb_conv3x3_wgrad_partial(const void* d_x, const void* d_dy, int32_t N, int32_t cin, int32_t cout, float* d_ws,
                             void* stream);
int bb_conv3x3_wgrad_reduce(const float* d_ws, int32_t chunks, int32_t cin, int32_t cout, int32_t w_layout,
                            float* d_dw, void* stream);

/* The same 3x3 convolutions in fp32 (no autocast: the reference's own precision), for (cin, cout) =
 * (128, 128), (64, 128) and (128, 64) (the last is the data gradient of the 64 -> 128 layer).  Every output
 * is the fp64 sum of 16-product fp32 MFMA chains, rounded to fp32 once (csrc/bb_conv32.hip): within
 * north_star's 1e-5 after the batch-statistics BatchNorms where MIOpen's 1,152-product order was not
 * (network.py:75-182 in train mode, scripts/train.py:122).  Activations f32 NHWC [N][8][8][C], 16-byte
 * aligned.  bb_conv3x3_f32_prep writes the f32 weight images d_wf [9][cout][cin] (forward) and
 * d_wd [9][cin][cout] (taps reversed, data gradient) from w_layout 0 / 1 as bb_conv3x3_prep; either output
 * may be NULL.  bb_conv3x3_f32_forward writes y = conv(x, w) without bias from d_wf; the data gradient is
 * the same call on dy with d_wd and cin / cout swapped.  Deterministic. */
int bb_conv3x3_f32_prep(const float* d_w, int32_t cin, int32_t cout, int32_t w_layout, float* d_wf, float* d_wd,
                        void* stream);
int bb_conv3x3_f32_forward(const float* d_x, const float* d_w, int32_t N, int32_t cin, int32_t cout, float* d_y,
                           void* stream);
/* nn.Linear's forward y = x w^T + bias in fp32 with the same accumulation (fp64 sum of 16-product fp32 MFMA
 * chains, the bias added in fp64, one rounding): the K = 8,192 first fc_encoder layer of the rollout's
 * forward (network.py:89-117, 135-182).  x [M][K], w [N][K] (nn.Linear.weight), y [M][N], all row-major and
 * 16-byte aligned; bias [N] or NULL; N % 128 == 0, K % 32 == 0.  Deterministic. */
int bb_linear_f32(const float* d_x, const float* d_w, const float* d_bias, int32_t M, int32_t N, int32_t K,
                  float* d_y, void* stream);

/* The end of the PPO minibatch step (PPOAgent.update, ppo.py:400-401):
 * nn.utils.clip_grad_norm_(params, max_norm) followed by
 * torch.optim.Adam(lr, betas, eps).step() (weight decay 0, no amsgrad), over
 * up to BB_OPT_MAX_TENSORS f32 parameter tensors given as host arrays of device
 * pointers: parameter, gradient, exp_avg, exp_avg_sq (same layout and numel
 * each) and Adam's per-tensor step count (f32 scalar on the device, incremented
 * first, as torch's fused / capturable Adam keeps it).  The gradient is scaled
 * by min(max_norm / (||g||_2 + 1e-6), 1) in place, as clip_grad_norm_ leaves
 * it; ||g|| over all tensors is written to d_total_norm when non-NULL.  d_ws is
 * caller scratch of bb_adam_clip_workspace_bytes(num_tensors, h_numel) bytes
 * (16-byte aligned).  Three kernel launches on `stream`; the tensor table is
 * passed by value, so the launches can be captured into a HIP graph.  The norm
 * is summed in a fixed order: deterministic.
 * Guard: zero d_ws once before the first call.  Then uint32 word
 * BB_ADAM_GUARD_WORD of d_ws holds 1 + the first chunk (BB_ADAM_CHUNK gradient
 * elements, chunks numbered across the tensors in table order) whose sum of
 * squares was non-finite or above 1e16.  The next word counts such chunks.
 * Both are sticky until the caller clears them.  The update itself is not
 * altered (runtime/kernels.py adam_guard_check reads and clears them). */
#define BB_OPT_MAX_TENSORS 48
#define BB_ADAM_GUARD_WORD 2
#define BB_ADAM_CHUNK 2048
int64_t bb_adam_clip_workspace_bytes(int32_t num_tensors, const int64_t* h_numel);
int bb_adam_clip_step(int32_t num_tensors, float* const* h_param, float* const* h_grad,
                      float* const* h_exp_avg, float* const* h_exp_avg_sq, float* const* h_step,
                      const int64_t* h_numel, double lr, double beta1, double beta2, double eps,
                      float max_norm, double* d_ws, float* d_total_norm, void* stream);

/* bf16 autocast's parameter casts for the CNN's nn.Linear layers
 * (network.py:89-117 under torch.autocast), all tensors in one launch: dir 0
 * casts f32 -> bf16 (round to nearest even), dir 1 bf16 -> f32 (their
 * gradients).  h_perm_c (NULL = none) > 0 marks a tensor of O rows whose f32
 * side is [O][perm_c][perm_hw] and whose bf16 side is [O][perm_hw][perm_c] (the
 * first FC weight against a channels_last flatten); perm_c * perm_hw <= 8192. */
int bb_cast_multi(int32_t num_tensors, int32_t dir, const void* const* h_src, void* const* h_dst,
                  const int64_t* h_numel, const int32_t* h_perm_c, const int32_t* h_perm_hw, void* stream);

/* The CNN's bf16 Linear tails (network.py:89-117: nn.Linear -> nn.ReLU -> nn.Dropout under autocast), not
 * part of the env boundary.
 * bb_dropout_forward: nn.Dropout(p)'s training forward, in place over n bf16 values (n % 8 == 0, 16-byte
 * aligned): y * (1 / (1 - p)) where the element is kept, else 0.  Element i is dropped when draw i % 4 of
 * Philox4x32-10(counter = (i / 4, offset), key = seed) is below p * 2^32.  d_rng is a device int64[4]
 * {seed, offset, 0, 0}: the launch reads (seed, offset), and the last of its workgroups advances offset by
 * one (words 2-3 are its scratch and stay 0 between launches), so every launch -- and every replay of a
 * captured graph -- draws a new mask.  One launch.
 * bb_linear_bgrad: the backward of y = dropout(relu(x w^T + b)) up to its GEMMs.  d_yd = the saved output
 * (bf16 [rows][cols]): g = dy * scale where yd > 0, else 0 (scale = the dropout's 1 / (1 - p), or 1), written
 * to d_g; d_yd = NULL: g = dy (plain Linear, nothing written).  d_db[c] = sum over rows of g[., c], f32 sums
 * in a fixed order rounded to bf16 (deterministic).  One launch: row chunks of 64 columns each publish
 * partial sums to d_ws (bb_linear_bgrad_workspace_bytes(rows, cols) bytes) and the last chunk to finish adds
 * them; d_cnt holds bb_linear_bgrad_counters(cols) uint32 counters that must be zero before the first launch
 * and are zero again after each (the launch re-arms them) -- one counter block per stream: launches that run
 * concurrently must not share one. */
int bb_dropout_forward(void* d_y, int64_t n, float p, int64_t* d_rng, void* stream);

/* The CNN's input layer, conv 4 -> 64 3x3 pad 1 over 8x8 boards (network.py:75-87, the first nn.Conv2d, without
 * its bias: the BatchNorm after it adds that) under bf16 autocast, not part of the env boundary.  x: N boards
 * of f32 [4][8][8] (x_nhwc 0) or [8][8][4] (x_nhwc 1, channels_last), 16-byte aligned; w: f32 [64][4][3][3]
 * (wl 0) or [64][3][3][4] (wl 1).  x and w are rounded to bf16 as autocast casts them, products summed in f32.
 * bb_conv_in_forward: y = bf16 [N][8][8][64] (NHWC).  One launch.
 * bb_conv_in_wgrad: dw (f32, w's layout) = sum over boards and pixels of dy (bf16 NHWC [N][8][8][64]) times
 * the bf16 input, f32 sums: per-workgroup partials in d_ws (bb_conv_in_wgrad_workspace_bytes(N) bytes) added
 * in a fixed order (deterministic).  Two launches. */
int64_t bb_conv_in_wgrad_workspace_bytes(int32_t N);
int bb_conv_in_forward(const float* d_x, int32_t x_nhwc, const float* d_w, int32_t wl, int32_t N, void* d_y,
                       void* stream);
int bb_conv_in_wgrad(const float* d_x, int32_t x_nhwc, const void* d_dy, int32_t N, float* d_ws, int32_t wl,
                     float* d_dw, void* stream);
/* bb_conv_in_forward plus bb_conv3x3_prep_multi's weight images of the other layers (same table arguments) in one
 * launch: both run at the start of the CNN's forward and are independent. */
int bb_conv_in_forward_prep(const float* d_x, int32_t x_nhwc, const float* d_w, int32_t wl, int32_t N, void* d_y,
                            int32_t count, const float* const* h_w, const int32_t* h_cin, const int32_t* h_cout,
                            const int32_t* h_w_layout, void* const* h_wf, void* const* h_wd, void* stream);
/* bb_linear_wgrad: a Linear's weight gradient dW = g^T x (g bf16 [rows][N], x bf16 [rows][K] with row stride
 * ldx >= K a multiple of 8, dW bf16 [N][K], all row-major; N and K multiples of 32, 16-byte aligned rows, rows <= 16384), f32 sums in a fixed order
 * rounded once (deterministic).  One launch: splits of 256 rows publish 32 x 32 partials to d_ws
 * (bb_linear_wgrad_workspace_bytes(rows, N, K) bytes) and the last split of a tile adds them; d_cnt: the
 * bb_linear_wgrad_counters(N, K) uint32 counters, zero before and after each launch (as bb_linear_bgrad's,
 * and the same counter block may serve both on one stream). */
/* bb_linear_n1_forward / _backward: a bf16 Linear with one output (the value head's Linear(128, 1)), x bf16
 * [rows][K] with row stride ldx (>= K, a multiple of 8), w bf16 [K], b bf16 [1] (NULL: none), K a multiple of
 * 8, 16-byte aligned.  Forward: y[r] = bf16(sum_k x[r][k] w[k] + b), f32 sums.  Backward: dx[r][k] = bf16(gy[r] w[k]), dW[k] = sum_r gy[r] x[r][k],
 * db = sum_r gy[r] (d_db NULL: skipped), f32 sums in a fixed order rounded to bf16; row chunks publish
 * partials to d_ws (bb_linear_n1_workspace_bytes(rows, K) bytes) with bb_linear_n1_counters(K) zeroed
 * counters in d_cnt (as bb_linear_bgrad).  One launch each. */
int64_t bb_linear_n1_workspace_bytes(int32_t rows, int32_t K);
int32_t bb_linear_n1_counters(int32_t K);
int bb_linear_n1_forward(const void* d_x, const void* d_w, const void* d_b, int32_t rows, int32_t K, int32_t ldx,
                         void* d_y, void* stream);
int bb_linear_n1_backward(const void* d_gy, const void* d_x, const void* d_w, int32_t rows, int32_t K, int32_t ldx,
                          void* d_dx, void* d_dw, void* d_db, float* d_ws, uint32_t* d_cnt, void* stream);
int64_t bb_linear_wgrad_workspace_bytes(int32_t rows, int32_t N, int32_t K);
int32_t bb_linear_wgrad_counters(int32_t N, int32_t K);
int bb_linear_wgrad(const void* d_g, const void* d_x, int32_t rows, int32_t N, int32_t K, int32_t ldx, void* d_dw,
                    float* d_ws, uint32_t* d_cnt, void* stream);
int64_t bb_linear_bgrad_workspace_bytes(int32_t rows, int32_t cols);
int32_t bb_linear_bgrad_counters(int32_t cols);
int bb_linear_bgrad(const void* d_dy, const void* d_yd, int32_t rows, int32_t cols, float scale, void* d_g,
                    void* d_db, float* d_ws, uint32_t* d_cnt, void* stream);
/* bb_linear_bgrad over two layers' output gradients side by side (ABI 8): columns [0, split) of dy come from d_dy
 * ([rows][split]), columns [split, cols) from d_dy2 ([rows][cols - split]); d_yd, d_g are [rows][cols] (the
 * policy and value heads' first layers as one GEMM). */
int bb_linear_bgrad2(const void* d_dy, const void* d_dy2, int32_t split, const void* d_yd, int32_t rows, int32_t cols,
                     float scale, void* d_g, void* d_db, float* d_ws, uint32_t* d_cnt, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BBVEC_H */

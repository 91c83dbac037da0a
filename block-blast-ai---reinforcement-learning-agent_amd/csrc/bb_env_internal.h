// bb_env_internal.h -- device state layout shared by the kernels and the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bbvec.h"
#include "bb_device.h"

namespace bb {

// Structure-of-arrays per-env state in HBM.
// Hot columns (read+written every step): board, hand, score, combo,
// max_combo, moves, lines, blocks, prev, mask.  PCG columns are touched only
// on the steps that draw a hand (every third legal move) and on resets.
struct EnvDev {
  int n;
  uint64_t* board;      // bitboard
  uint32_t* hand;       // 3 x 6-bit ids | used<<18 | over<<21 | has_uint32<<22
  int64_t* score;
  int32_t* combo;
  int32_t* max_combo;
  int32_t* moves;
  int32_t* lines;
  int32_t* blocks;
  uint16_t* prev;       // _prev_holes | filled-centre-cells << 8
  uint64_t* mask;       // [n][3] current action-mask bits
  uint64_t* rng_hi;     // PCG64 state
  uint64_t* rng_lo;
  uint32_t* rng_buf;    // buffered 32-bit half
  uint64_t* inc_hi;     // PCG64 increment (constant per seed)
  uint64_t* inc_lo;
  uint64_t* seed_hi;    // state right after default_rng(seed_value)
  uint64_t* seed_lo;
  uint8_t* has_seed;    // seed_value is not None -> re-seed on reset
  uint8_t* pend;        // parked by step_kernel, finished by escalate_kernel
  uint64_t* pscratch;   // parked env's unfinished attempt + move summary
  uint32_t* status;     // device-side failure word (host-pinned, device-mapped); 0 = ok, see kStatus*
};

// Device-side failure codes written to EnvDev::status (the host turns them into BB_ERR_DEVICE).
constexpr uint32_t kStatusAsyncCap = 1u;  // rollout_async_kernel: an env wave left through an iteration cap

struct StepArgs {
  bb_reward_cfg cfg;
  double center_tenth;  // reward_config['center_bonus'] * 0.1 (block_blast_env.py:190)
  int autoreset;
  int lane_budget;      // per-lane solver budget before wave escalation
  int lane_quick;       // > 0: in-lane test of this many fixed slots instead of the budget search
  int pack_first;       // attempts drawn in the first wave pass (>= 1)
  int pack_next;        // attempts per later pass (0: double each pass)
  const JumpRow* jump;  // PCG64 jump-ahead table [kJumpMax + 1]
  int dbg;              // diagnostics only (BB_DEBUG_MODE): bit0 = skip solvability test,
                        // bit1 = write per-env solver counters to dbg_out
  uint64_t* dbg_out;    // [n][4]: lane cycles, attempts | escalated << 32, wave cycles, board
  float* reward;
  uint8_t* terminated;
  double* reward_f64;
  uint64_t* mask_out;
  uint8_t* lines;
  bb_info* info;
  int32_t* next_action;
  uint64_t policy_seed;
  uint64_t policy_step;
  uint64_t env_offset;
  int64_t* final_score;  // [N] optional: score of the envs that terminated (before the auto-reset)
  int32_t* final_moves;  // [N] optional: their moves
};

// bb_rollout: T fused steps (see rollout_kernel).  Per-step outputs are [T][N].
struct RollArgs {
  int steps;
  const int32_t* first_action;  // [N] action of step 0
  float* reward;                // [T][N]
  uint8_t* terminated;          // [T][N]
  uint8_t* lines;               // [T][N] optional
  int32_t* actions;             // [T][N] optional: action applied at step t
  uint64_t* mask;               // [T][N][3] optional: post-step mask bits
  int32_t* next_action;         // [N] optional: policy action after the last step
  uint64_t policy_step0;        // step t's next action uses policy_step0 + t + 1
  bb_info* info;                // [T][N] optional: bb_step's info record (bb_step through this kernel, T = 1)
  double* reward_f64;           // [T][N] optional: the fp64 reward
  int64_t* final_score;         // [T][N] optional: written where the env terminated at step t (pre-reset score)
  int32_t* final_moves;         // [T][N] optional: likewise its moves
  int64_t work_cap;             // rollout_async_kernel: working iterations per env wave (0: 2 * 64 * T + 4096;
                                // smaller only to test the cap's error path, BB_DEBUG_ASYNC_CAP)
};

hipError_t launch_reset(const EnvDev& e, const PieceRow* rows, const uint8_t* d, const uint8_t* sel, hipStream_t s);
hipError_t launch_step(const EnvDev& e, const PieceRow* rows, const uint8_t* d, const int32_t* actions,
                       const StepArgs& a, hipStream_t s);
hipError_t launch_rollout(const EnvDev& e, const PieceRow* rows, const uint8_t* d, const StepArgs& a,
                          const RollArgs& r, hipStream_t s);
hipError_t launch_expand(const uint64_t* board, const uint32_t* hand, const uint64_t* mbits, const int64_t* index,
                         const PieceRow* rows, int n, float* x, float* mf, int8_t* mi, hipStream_t s);
hipError_t launch_refresh_mask(const EnvDev& e, const PieceRow* rows, hipStream_t s);
hipError_t launch_random_actions(const uint64_t* mbits, int n, uint64_t seed, uint64_t step, uint64_t offset,
                                 int32_t* out, hipStream_t s);
hipError_t launch_masked_sample(const float* logits, const uint64_t* mbits, int n, const float* uniform,
                                uint64_t seed, uint64_t step, const uint64_t* d_step, uint64_t offset,
                                int deterministic, const int64_t* action_in, int64_t* action, float* logp,
                                float* ent, hipStream_t s);
hipError_t launch_gae(const float* r, const float* v, const float* d, const float* last, int T, int N, float gamma,
                      float gl, float* adv, float* ret, hipStream_t s);

int64_t bn_workspace_bytes(int dtype, int nhwc, int N, int C, int HW);
hipError_t launch_bn_forward(const void* x, const void* res, int dtype, int nhwc, int N, int C, int HW,
                             const float* pb, const float* w, const float* b, float eps, int relu, double* ws,
                             float* save_mean, float* save_invstd, float* rmean, float* rvar, float momentum,
                             int64_t* nbt, void* y, hipStream_t s, const double* ext_part = nullptr, int ext_nb = 0);
// a board convolution's weight-gradient partial-sum reduction (csrc/bb_conv.hip conv_wgrad_reduce's arguments),
// run inside a BatchNorm backward finalisation's launch by bb_bn_backward_red
struct WgradReduceJob {  // conv_wgrad_reduce's arguments
  const float* part;
  int nchunk, cout, cin, wl;
  float* dw;
};
hipError_t launch_bn_backward(const void* x, const void* dy, int dtype, int nhwc, int N, int C, int HW,
                              const float* pb, const float* w, const float* b, const float* mean, const float* invstd,
                              int relu, double* ws, void* dx, float* dw, float* db, float* dpb, hipStream_t s,
                              const void* mask = nullptr, void* gout = nullptr, const WgradReduceJob* job = nullptr,
                              const double* ext_part = nullptr, int ext_nb = 0);

bool conv3x3_supported(int cin, int cout);
int64_t conv3x3_wgrad_workspace_bytes(int nb, int cin, int cout);
hipError_t launch_conv3x3_prep(const float* w, int cin, int cout, int wl, void* wf, void* wd, hipStream_t s);
hipError_t launch_conv3x3_prep_multi(int count, const float* const* w, const int32_t* cin, const int32_t* cout,
                                     const int32_t* wl, void* const* wf, void* const* wd, hipStream_t s);
// BatchNorm reduction sums from a board convolution's store pass (conv_fwd_kernel): part [blocks][cout][3];
// bx NULL: forward statistics of the output, else the output is a BatchNorm's output gradient and bx, mean,
// invstd, w, b, relu that BatchNorm's input and forward coefficients
struct ConvStatsArgs {
  double* part;
  const uint16_t* bx;
  const float* mean;
  const float* invstd;
  const float* w;
  const float* b;
  int relu;
};
hipError_t launch_conv3x3_forward(const void* x, const void* w, int nb, int cin, int cout, void* y, hipStream_t s,
                                  const void* radd = nullptr, const ConvStatsArgs* stats = nullptr);
int conv3x3_stats_blocks(int nb, int cout);
hipError_t launch_conv3x3_wgrad(const void* x, const void* dy, int nb, int cin, int cout, float* ws, int wl,
                                float* dw, hipStream_t s);
// the weight gradient in two parts: the partial-sum kernel, and the fixed-order sum of its `used` chunks (which
// bb_bn_backward_red can run inside the next BatchNorm finalisation's launch)
int conv3x3_wgrad_chunks_used(int nb, int cin, int cout);
hipError_t launch_conv3x3_wgrad_partial(const void* x, const void* dy, int nb, int cin, int cout, float* ws,
                                        hipStream_t s);
hipError_t launch_conv3x3_wgrad_reduce(const float* ws, int used, int cin, int cout, int wl, float* dw, hipStream_t s);

// the input layer, conv 4 -> 64 (x f32 NCHW or NHWC, w f32 [64][4][3][3] wl 0 or [64][3][3][4] wl 1)
int64_t conv_in_wgrad_workspace_bytes(int nb);
hipError_t launch_conv_in_forward(const float* x, int x_nhwc, const float* w, int wl, int nb, void* y, hipStream_t s);
hipError_t launch_conv_in_forward_prep(const float* x, int x_nhwc, const float* w, int wl, int nb, void* y, int count,
                                       const float* const* pw, const int32_t* cin, const int32_t* cout,
                                       const int32_t* pwl, void* const* wf, void* const* wd, hipStream_t s);
hipError_t launch_conv_in_wgrad(const float* x, int x_nhwc, const void* dy, int nb, float* ws, int wl, float* dw,
                                hipStream_t s);

bool conv3x3_f32_supported(int cin, int cout);
hipError_t launch_conv3x3_f32_prep(const float* w, int cin, int cout, int wl, float* wf, float* wd, hipStream_t s);
hipError_t launch_conv3x3_f32_forward(const float* x, const float* w, int nb, int cin, int cout, float* y,
                                      hipStream_t s);
hipError_t launch_linear_f32(const float* x, const float* w, const float* bias, int M, int N, int K, float* y,
                             hipStream_t s);

int64_t ppo_loss_workspace_bytes(int B);
// logits / values (and backward's dlogits / dvalues): f32, or bf16 when bf16 != 0
hipError_t launch_ppo_loss_forward(const void* logits, const void* values, int bf16, const float* mask,
                                   const int64_t* actions, const float* old_logp, const float* adv, const float* ret,
                                   int B, float clip, float vcoef, float ecoef, double* ws, uint32_t* cnt, float* stats,
                                   float* loss, hipStream_t s);
hipError_t launch_ppo_loss_backward(const void* logits, const void* values, int bf16, const float* mask,
                                    const int64_t* actions, const float* old_logp, const float* adv, const float* ret,
                                    int B, float clip, float vcoef, float ecoef, const float* gloss, void* dlogits,
                                    void* dvalues, hipStream_t s);
hipError_t launch_ppo_loss_fused(const void* logits, const void* values, int bf16, const float* mask,
                                 const int64_t* actions, const float* old_logp, const float* adv, const float* ret,
                                 int B, float clip, float vcoef, float ecoef, const float* gloss, void* dlogits,
                                 void* dvalues, double* ws, uint32_t* cnt, float* stats, float* loss, hipStream_t s);

constexpr int kOptMaxTensors = 48;  // == BB_OPT_MAX_TENSORS
int64_t adam_clip_workspace_bytes(int count, const int64_t* n);
hipError_t launch_adam_clip(int count, float* const* p, float* const* g, float* const* m, float* const* v,
                            float* const* step, const int64_t* n, double lr, double beta1, double beta2, double eps,
                            float max_norm, double* ws, float* norm_out, hipStream_t s);
hipError_t launch_cast_multi(int count, int dir, const void* const* src, void* const* dst, const int64_t* n,
                             const int32_t* perm_c, const int32_t* perm_hw, hipStream_t s);
// bf16 Linear tails (bb_optim.hip): in-place dropout with a self-advancing device generator word, and the
// masked-scale + ReLU-mask + bias-gradient pass of the backward
hipError_t launch_dropout_fwd(void* y, int64_t n, float p, int64_t* rng, hipStream_t s);
int64_t linear_bgrad_workspace_bytes(int rows, int cols);
int linear_bgrad_counters(int cols);
hipError_t launch_linear_bgrad(const void* dy, const void* yd, int rows, int cols, float scale, void* g, void* db,
                               float* part, uint32_t* cnt, hipStream_t s, const void* dy2 = nullptr, int split = 0);
int64_t linear_n1_workspace_bytes(int rows, int K);
int linear_n1_counters(int K);
hipError_t launch_linear_n1_forward(const void* x, const void* w, const void* b, int rows, int K, int ldx, void* y,
                                    hipStream_t s);
hipError_t launch_linear_n1_backward(const void* gy, const void* x, const void* w, int rows, int K, int ldx, void* dx,
                                     void* dw, void* db, float* part, uint32_t* cnt, hipStream_t s);
int64_t linear_wgrad_workspace_bytes(int rows, int N, int K);
int linear_wgrad_counters(int N, int K);
hipError_t launch_linear_wgrad(const void* g, const void* x, int rows, int N, int K, int ldx, void* dw, float* part,
                               uint32_t* cnt, hipStream_t s);

// Host helpers (bb_tables.cpp).
void build_piece_tables(PieceRow rows[kPieces], uint8_t dtab[kPieces * kPieces]);
void build_jump_table(JumpRow rows[kJumpMax + 1]);
void pcg64_seed_numpy(uint64_t seed, uint64_t out[4]);

}  // namespace bb

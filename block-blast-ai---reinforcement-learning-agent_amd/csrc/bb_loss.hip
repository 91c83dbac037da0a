// bb_loss.hip -- the PPO minibatch loss of PPOAgent.update (ppo.py:362-401)
// with the masked-categorical tail of BlockBlastNetwork (network.py:173-180,
// 210-262), forward and backward, fused (gfx950).
//
// Issued as torch ops the loss is ~45 elementwise / reduction kernels forward
// and as many backward, each a few microseconds on 2,048 x 192 logits; here it
// is one wave per minibatch row, one launch each way (the last block to finish
// finalises the statistics), or one launch for both when the caller supplies
// the loss gradient up front (the graph root's seed: bb_ppo_loss_fused).
//
// Per row (torch fp32 semantics, same operation order as the torch path):
//   p      = softmax(logits + where(mask, 0, -inf))
//   P      = p / sum(p)                         Categorical(probs) normalisation
//   logp   = log(clamp(P[a], eps, 1 - eps))     Categorical.log_prob (clamp_probs)
//   ent    = masked entropy of p (network.py:232-262, clamps 1e-10)
//   ratio  = exp(logp - old_logp)
//   pol    = -min(ratio * A, clamp(ratio, 1 - c, 1 + c) * A)
//   vloss  = (value - ret)^2
// Loss = mean(pol) + vcoef * mean(vloss) - ecoef * mean(ent); the statistics
// (policy / value / entropy / total loss, approx_kl = mean((r - 1) - log r),
// clip_fraction = mean(|r - 1| > c)) come from fp64 block partials summed in a
// fixed order.  Backward follows torch's autograd rules: torch.min splits ties
// half/half, clamp passes the gradient on its closed interval, log divides by
// the clamped value.  Logits and values may be bf16 (the autocast network's
// outputs): widened exactly on load, and their gradients rounded to bf16 (to
// nearest even) on store -- the values of autograd's casts around an fp32 loss,
// without the four cast kernels.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <math.h>

#include "bb_env_internal.h"

namespace bb {

namespace {

constexpr int kLossThreads = 256;
constexpr int kRowsPerBlock = kLossThreads / 64;
constexpr int kStats = 5;  // partial sums: pol, vloss, ent, kl, clipped
constexpr float kEps32 = 1.1920928955078125e-07f;  // torch.finfo(float32).eps

__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = __fadd_rn(v, __shfl_xor(v, o));
  return v;
}

// The forward quantities of one row, 3 entries per lane (action j * 64 + lane).
struct RowFwd {
  bool valid[3];
  float p[3];     // softmax of the masked logits
  float s;        // sum of p
  float pa;       // P[a] = p[a] / s (all lanes)
  float ms_raw;   // sum of the masked p
  float ms;       // clamp(ms_raw, 1e-10)
  float q[3];     // masked p / ms
  float logp, ent;
};

// logits / values / their gradients: f32, or bf16 (BF)
template <bool BF>
__device__ __forceinline__ float ldv(const void* __restrict__ p, int64_t i) {
  if constexpr (BF) return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(p)[i] << 16);
  return reinterpret_cast<const float*>(p)[i];
}
template <bool BF>
__device__ __forceinline__ void stv(void* __restrict__ p, int64_t i, float v) {
  if constexpr (BF) {
    const __hip_bfloat16 b = __float2bfloat16(v);  // round to nearest even, as torch's cast
    reinterpret_cast<uint16_t*>(p)[i] = *reinterpret_cast<const uint16_t*>(&b);
  } else {
    reinterpret_cast<float*>(p)[i] = v;
  }
}

template <bool BF>
__device__ __forceinline__ void row_forward(const void* __restrict__ logits, const float* __restrict__ mask,
                                            int64_t row, int64_t a, int lane, RowFwd& r) {
  float x[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    x[j] = ldv<BF>(logits, row * 192 + j * 64 + lane);
    r.valid[j] = mask[row * 192 + j * 64 + lane] != 0.f;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 3; ++j)
    if (r.valid[j]) mx = fmaxf(mx, x[j]);
  mx = wmax(mx);
  float e[3], se = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    e[j] = r.valid[j] ? expf(__fsub_rn(x[j], mx)) : 0.f;
    se = __fadd_rn(se, e[j]);
  }
  se = wsum(se);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    r.p[j] = __fdiv_rn(e[j], se);
    s = __fadd_rn(s, r.p[j]);
  }
  r.s = wsum(s);
  const int aj = (int)(a >> 6), al = (int)(a & 63);
  r.pa = __fdiv_rn(__shfl(aj == 0 ? r.p[0] : (aj == 1 ? r.p[1] : r.p[2]), al), r.s);
  r.logp = logf(fminf(fmaxf(r.pa, kEps32), 1.f - kEps32));
  float ms = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) ms = __fadd_rn(ms, r.valid[j] ? r.p[j] : 0.f);
  r.ms_raw = wsum(ms);
  r.ms = fmaxf(r.ms_raw, 1e-10f);
  float h = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    r.q[j] = __fdiv_rn(r.valid[j] ? r.p[j] : 0.f, r.ms);
    h = __fadd_rn(h, r.valid[j] ? __fmul_rn(r.q[j], logf(fmaxf(r.q[j], 1e-10f))) : 0.f);
  }
  r.ent = -wsum(h);
}

// Last-arriver hand-off of the blocks' partial sums, ordered by the HIP memory model (as bb_optim.hip's): stored by
// agent-scope atomic stores (written through, sc1) and drained, a workgroup barrier, then one lane counts the block
// with an agent-scope release add (buffer_wbl2 sc1 + s_waitcnt before it); the lane whose add returns the last count
// issues an agent-scope acquire fence (buffer_inv sc1) and its block, after a barrier, reads all partials with
// agent-scope loads, finalises and re-arms the counter atomically.
#ifndef BB_HANDOFF_ORDER
#define BB_HANDOFF_ORDER __ATOMIC_RELEASE  // A/B only: __ATOMIC_RELAXED is the round-5 form (tools/variants.py hrx)
#endif
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) uint32_t guint32;
__device__ __forceinline__ void wt_store(double* p, double v) {
  __hip_atomic_store((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double wt_load(const double* p) {
  return __hip_atomic_load((const gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool wt_arrive_last(uint32_t* c, uint32_t n) {
  const bool last = __hip_atomic_fetch_add((guint32*)c, 1u, BB_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT) == n - 1u;
  if (last && BB_HANDOFF_ORDER != __ATOMIC_RELAXED) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return last;
}
__device__ __forceinline__ void wt_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// stats = [policy_loss, value_loss, entropy, total_loss, approx_kl, clip_fraction]; loss = stats[3]
__device__ __forceinline__ void loss_stats_out(const double t[kStats], int B, float vcoef, float ecoef,
                                               float* __restrict__ stats, float* __restrict__ loss) {
  float m[kStats];
  for (int k = 0; k < kStats; ++k) m[k] = (float)(t[k] / (double)B);
  const float total = __fadd_rn(__fadd_rn(m[0], __fmul_rn(vcoef, m[1])), __fmul_rn(ecoef, -m[2]));
  stats[0] = m[0];
  stats[1] = m[1];
  stats[2] = m[2];
  stats[3] = total;
  stats[4] = m[3];
  stats[5] = m[4];
  if (loss) loss[0] = total;
}

// One wave per row.  STATS: the loss terms' fp64 block partials -> part; with cnt, the last block to arrive
// adds every block's partials (lane b of a wave per block b, b + 64, ...; the lanes and then the waves in a
// fixed order) and writes stats / loss, re-arming cnt.  GRAD: d loss / d logits, d values for the loss gradient
// gloss[0] (the backward's formulas; with STATS too, the forward and backward of one minibatch in one launch).
template <bool BF, bool STATS, bool GRAD>
__global__ void __launch_bounds__(kLossThreads) ppo_loss_kernel(
    const void* __restrict__ logits, const void* __restrict__ values, const float* __restrict__ mask,
    const int64_t* __restrict__ actions, const float* __restrict__ old_logp, const float* __restrict__ adv,
    const float* __restrict__ ret, int B, float clip, float vcoef, float ecoef, const float* __restrict__ gloss,
    void* __restrict__ dlogits, void* __restrict__ dvalues, double* __restrict__ part, uint32_t* cnt,
    float* __restrict__ stats, float* __restrict__ loss) {
  __shared__ double red[kStats][kRowsPerBlock];
  __shared__ int last_block;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double acc[kStats] = {0.0, 0.0, 0.0, 0.0, 0.0};
  const float g = GRAD ? gloss[0] : 0.f;
  const float invB = 1.f / (float)B;
  for (int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + w; row < B; row += (int64_t)gridDim.x * kRowsPerBlock) {
    const int64_t a = actions[row];
    RowFwd r;
    row_forward<BF>(logits, mask, row, a, lane, r);
    const float A = adv[row];
    const float ratio = expf(__fsub_rn(r.logp, old_logp[row]));
    const float s1 = __fmul_rn(ratio, A), s2 = __fmul_rn(fminf(fmaxf(ratio, 1.f - clip), 1.f + clip), A);
    if (STATS) {
      const float dv = __fsub_rn(ldv<BF>(values, row), ret[row]);
      const float rm1 = __fsub_rn(ratio, 1.f);
      acc[0] += (double)(-fminf(s1, s2));
      acc[1] += (double)__fmul_rn(dv, dv);
      acc[2] += (double)r.ent;
      acc[3] += (double)__fsub_rn(rm1, logf(ratio));
      acc[4] += fabsf(rm1) > clip ? 1.0 : 0.0;
    }
    if (GRAD) {
      // d loss / d min(s1, s2) = -g / B; torch.min splits ties half/half
      const float gmin = -g * invB;
      const float g1 = s1 < s2 ? gmin : (s1 > s2 ? 0.f : 0.5f * gmin);
      const float g2 = s2 < s1 ? gmin : (s2 > s1 ? 0.f : 0.5f * gmin);
      const bool in_clip = ratio >= 1.f - clip && ratio <= 1.f + clip;
      const float glogp = (g1 * A + (in_clip ? g2 * A : 0.f)) * ratio;  // d exp(x)/dx = exp(x)
      if (lane == 0) stv<BF>(dvalues, row, vcoef * g * invB * 2.f * __fsub_rn(ldv<BF>(values, row), ret[row]));  // mse
      const float gent = -ecoef * g * invB;  // ecoef * (-mean(ent))
      // log(clamp(P_a, eps, 1 - eps)): passes where eps <= P_a <= 1 - eps, divided by the clamped value
      const float gPa = (r.pa >= kEps32 && r.pa <= 1.f - kEps32) ? glogp / r.pa : 0.f;
      // P = p / s: gp_k = [k == a] gPa / s - gPa p_a / s^2
      const int aj = (int)(a >> 6), al = (int)(a & 63);
      const float p_a = __shfl(aj == 0 ? r.p[0] : (aj == 1 ? r.p[1] : r.p[2]), al);
      const float corr = gPa * p_a / (r.s * r.s);
      // entropy = -sum m q log(clamp(q, 1e-10)), q = m p / clamp(ms, 1e-10):
      //   d/dq_j = -m_j (log(clamp(q_j)) + [q_j >= 1e-10])
      float gq[3], sgqm = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        gq[j] = 0.f;
        if (r.valid[j]) gq[j] = -gent * (logf(fmaxf(r.q[j], 1e-10f)) + (r.q[j] >= 1e-10f ? 1.f : 0.f));
        sgqm += r.valid[j] ? gq[j] * r.p[j] : 0.f;
      }
      sgqm = wsum(sgqm);
      const float gms = r.ms_raw >= 1e-10f ? -sgqm / (r.ms * r.ms) : 0.f;
      float gp[3], dot = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        gp[j] = ((j == aj && lane == al) ? gPa / r.s : 0.f) - corr;
        if (r.valid[j]) gp[j] += gq[j] / r.ms + gms;
        dot += gp[j] * r.p[j];
      }
      dot = wsum(dot);
      // softmax backward: dz_k = p_k (gp_k - sum_j gp_j p_j); masked entries have p = 0
#pragma unroll
      for (int j = 0; j < 3; ++j) stv<BF>(dlogits, row * 192 + j * 64 + lane, r.p[j] * (gp[j] - dot));
    }
  }
  if (!STATS) return;
  if (lane == 0)
    for (int k = 0; k < kStats; ++k) red[k][w] = acc[k];
  __syncthreads();
  if (threadIdx.x < kStats) {
    double t = 0.0;
    for (int k = 0; k < kRowsPerBlock; ++k) t += red[threadIdx.x][k];
    wt_store(part + (int64_t)blockIdx.x * kStats + threadIdx.x, t);
    wt_drain();
  }
  __syncthreads();  // wave 0's partial stores have drained
  if (threadIdx.x == 0) last_block = wt_arrive_last(cnt, (uint32_t)gridDim.x);
  __syncthreads();
  if (!last_block) return;
  // every block's partials: lane l of wave k adds blocks (l + 64 j) for stat k (waves 0-3 take stats 0-3, wave 0
  // then stat 4), the lanes' sums in lane order through LDS
  __shared__ double lsum[kStats][64];
  const int nb = gridDim.x;
  for (int k = w; k < kStats; k += kLossThreads / 64) {
    double t = 0.0;
    for (int b0 = lane; b0 < nb; b0 += 8 * 64) {
      double v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = b0 + 64 * j < nb ? wt_load(part + (int64_t)(b0 + 64 * j) * kStats + k) : 0.0;
#pragma unroll
      for (int j = 0; j < 8; ++j) t += v[j];
    }
    lsum[k][lane] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[kStats];
    for (int k = 0; k < kStats; ++k) {
      t[k] = 0.0;
      for (int l = 0; l < 64; ++l) t[k] += lsum[k][l];
    }
    loss_stats_out(t, B, vcoef, ecoef, stats, loss);
    __hip_atomic_store((guint32*)cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next launch
  }
}

int loss_blocks(int B) {
  int b = (B + kRowsPerBlock - 1) / kRowsPerBlock;
  return b < 1 ? 1 : (b > 4096 ? 4096 : b);
}

}  // namespace

int64_t ppo_loss_workspace_bytes(int B) { return (int64_t)sizeof(double) * kStats * loss_blocks(B); }

// stats / loss from one launch: block partials summed by the last block to arrive (cnt: a zeroed counter)
hipError_t launch_ppo_loss_forward(const void* logits, const void* values, int bf16, const float* mask,
                                   const int64_t* actions, const float* old_logp, const float* adv, const float* ret,
                                   int B, float clip, float vcoef, float ecoef, double* ws, uint32_t* cnt, float* stats,
                                   float* loss, hipStream_t s) {
  if (B <= 0 || !cnt) return hipErrorInvalidValue;
  const int nb = loss_blocks(B);
  if (bf16)
    hipLaunchKernelGGL((ppo_loss_kernel<true, true, false>), dim3(nb), dim3(kLossThreads), 0, s, logits, values, mask,
                       actions, old_logp, adv, ret, B, clip, vcoef, ecoef, nullptr, nullptr, nullptr, ws, cnt, stats,
                       loss);
  else
    hipLaunchKernelGGL((ppo_loss_kernel<false, true, false>), dim3(nb), dim3(kLossThreads), 0, s, logits, values, mask,
                       actions, old_logp, adv, ret, B, clip, vcoef, ecoef, nullptr, nullptr, nullptr, ws, cnt, stats,
                       loss);
  return hipGetLastError();
}

hipError_t launch_ppo_loss_backward(const void* logits, const void* values, int bf16, const float* mask,
                                    const int64_t* actions, const float* old_logp, const float* adv, const float* ret,
                                    int B, float clip, float vcoef, float ecoef, const float* gloss, void* dlogits,
                                    void* dvalues, hipStream_t s) {
  if (B <= 0) return hipErrorInvalidValue;
  if (bf16)
    hipLaunchKernelGGL((ppo_loss_kernel<true, false, true>), dim3(loss_blocks(B)), dim3(kLossThreads), 0, s, logits,
                       values, mask, actions, old_logp, adv, ret, B, clip, vcoef, ecoef, gloss, dlogits, dvalues,
                       nullptr, nullptr, nullptr, nullptr);
  else
    hipLaunchKernelGGL((ppo_loss_kernel<false, false, true>), dim3(loss_blocks(B)), dim3(kLossThreads), 0, s, logits,
                       values, mask, actions, old_logp, adv, ret, B, clip, vcoef, ecoef, gloss, dlogits, dvalues,
                       nullptr, nullptr, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_ppo_loss_fused(const void* logits, const void* values, int bf16, const float* mask,
                                 const int64_t* actions, const float* old_logp, const float* adv, const float* ret,
                                 int B, float clip, float vcoef, float ecoef, const float* gloss, void* dlogits,
                                 void* dvalues, double* ws, uint32_t* cnt, float* stats, float* loss, hipStream_t s) {
  if (B <= 0 || !cnt) return hipErrorInvalidValue;
  const int nb = loss_blocks(B);
  if (bf16)
    hipLaunchKernelGGL((ppo_loss_kernel<true, true, true>), dim3(nb), dim3(kLossThreads), 0, s, logits, values, mask,
                       actions, old_logp, adv, ret, B, clip, vcoef, ecoef, gloss, dlogits, dvalues, ws, cnt, stats,
                       loss);
  else
    hipLaunchKernelGGL((ppo_loss_kernel<false, true, true>), dim3(nb), dim3(kLossThreads), 0, s, logits, values, mask,
                       actions, old_logp, adv, ret, B, clip, vcoef, ecoef, gloss, dlogits, dvalues, ws, cnt, stats,
                       loss);
  return hipGetLastError();
}

}  // namespace bb

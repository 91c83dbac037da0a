// bb_ppo.hip -- fused rollout-side PPO kernels (gfx950).
//
//  * masked_sample_kernel: the masking / softmax / Categorical / sample /
//    log-prob / masked-entropy tail of BlockBlastNetwork.get_action_and_value
//    (network.py:173-180, 210-262) in one pass, one wave64 per env row: the 192
//    logits are 3 per lane, reductions are butterfly shuffles, the sample is an
//    inverse-CDF over a double-precision wave prefix scan.
//  * gae_kernel: RolloutBuffer.compute_returns_and_advantages (ppo.py:141-169),
//    one thread per env walking t = T-1..0; coalesced [T][N] rows; numpy-2
//    float32 operation order with explicit round-to-nearest ops (no FMA).
#include <hip/hip_runtime.h>
#include <math.h>

#include "bb_device.h"
#include "bb_env_internal.h"

namespace bb {

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = __fadd_rn(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = __dadd_rn(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double wave_incl_scan_d(double v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    double u = __shfl_up(v, o);
    if (lane >= o) v = __dadd_rn(v, u);
  }
  return v;
}

constexpr float kEps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps (clamp_probs)

__global__ void __launch_bounds__(256) masked_sample_kernel(const float* __restrict__ logits,
                                                            const uint64_t* __restrict__ mbits, int n,
                                                            const float* __restrict__ uniform, uint64_t seed,
                                                            uint64_t step, const uint64_t* __restrict__ d_step,
                                                            uint64_t offset, int deterministic,
                                                            const int64_t* __restrict__ action_in,
                                                            int64_t* __restrict__ action_out,
                                                            float* __restrict__ logp_out, float* __restrict__ ent_out) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  if (d_step) step += d_step[0];  // graph replays: the base step lives in device memory
  for (int row = wave; row < n; row += nwaves) {
    float x[3];
    bool v[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      x[j] = logits[(int64_t)row * 192 + j * 64 + lane];
      v[j] = (mbits[(int64_t)row * 3 + j] >> lane) & 1ull;
    }
    // logits + where(mask, 0, -inf) then F.softmax (network.py:173-180, 213)
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (v[j]) mx = fmaxf(mx, x[j]);
    mx = wave_max(mx);
    float e[3];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      e[j] = v[j] ? expf(__fsub_rn(x[j], mx)) : 0.f;
      s = __fadd_rn(s, e[j]);
    }
    s = wave_sum(s);
    float pr[3];
    float s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      pr[j] = __fdiv_rn(e[j], s);
      s2 = __fadd_rn(s2, pr[j]);
    }
    s2 = wave_sum(s2);
    // Categorical(probs): P = probs / probs.sum(-1)
    float P[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) P[j] = __fdiv_rn(pr[j], s2);

    int64_t a;
    if (action_in) {
      a = action_in[row];
    } else if (deterministic) {
      // torch.argmax(probs): first index of the maximum
      float best = -1.f;
      int bidx = 0;
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (pr[j] > best) {
          best = pr[j];
          bidx = j * 64 + lane;
        }
      float wbest = wave_max(best);
      int cand = best == wbest ? bidx : 1 << 30;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o));
      a = cand;
    } else {
      double u;
      if (uniform) {
        u = (double)uniform[row];
      } else {
        uint32_t w[4];
        philox_words(seed, offset + (uint64_t)row, step, w);
        u = (double)w[1] * 2.3283064365386963e-10;  // 2^-32
      }
      double tot[3];
      double inc[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        inc[j] = wave_incl_scan_d((double)P[j], lane);
        tot[j] = __shfl(inc[j], 63);
      }
      const double total = __dadd_rn(__dadd_rn(tot[0], tot[1]), tot[2]);
      const double target = __dmul_rn(u, total);
      double base = 0.0;
      a = -1;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        uint64_t hit = __ballot(v[j] && __dadd_rn(base, inc[j]) > target);
        if (a < 0 && hit) a = j * 64 + (__ffsll((unsigned long long)hit) - 1);
        base = __dadd_rn(base, tot[j]);
      }
      if (a < 0) {  // rounding fell past the last mass: take the last legal action
        int last = -1;
#pragma unroll
        for (int j = 0; j < 3; ++j)
          if (v[j]) last = j * 64 + lane;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o));
        a = last < 0 ? 0 : last;
      }
    }
    // dist.log_prob(a) = log(clamp(P_a, eps, 1 - eps))
    const int aj = (int)(a >> 6), al = (int)(a & 63);
    float pa = __shfl(aj == 0 ? P[0] : (aj == 1 ? P[1] : P[2]), al);
    float lp = logf(fminf(fmaxf(pa, kEps), 1.f - kEps));
    // _masked_entropy (network.py:232-262)
    float ms = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) ms = __fadd_rn(ms, v[j] ? pr[j] : 0.f);
    ms = fmaxf(wave_sum(ms), 1e-10f);
    float h = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float q = __fdiv_rn(v[j] ? pr[j] : 0.f, ms);
      const float lq = logf(fmaxf(q, 1e-10f));
      h = __fadd_rn(h, v[j] ? __fmul_rn(q, lq) : 0.f);
    }
    h = -wave_sum(h);
    if (lane == 0) {
      if (action_out) action_out[row] = a;
      if (logp_out) logp_out[row] = lp;
      if (ent_out) ent_out[row] = h;
    }
  }
}

__global__ void gae_kernel(const float* __restrict__ r, const float* __restrict__ v, const float* __restrict__ d,
                           const float* __restrict__ last, int T, int N, float gamma, float gl,
                           float* __restrict__ adv, float* __restrict__ ret) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  float gae = 0.f;
  float nv = last[i];
  for (int t = T - 1; t >= 0; --t) {
    const int64_t k = (int64_t)t * N + i;
    const float vt = v[k];
    const float nnt = __fsub_rn(1.0f, d[k]);
    // delta = r + gamma*nv*nnt - v        (ppo.py:165)
    const float delta = __fsub_rn(__fadd_rn(r[k], __fmul_rn(__fmul_rn(gamma, nv), nnt)), vt);
    // gae = delta + gamma*lambda*nnt*gae  (ppo.py:166)
    gae = __fadd_rn(delta, __fmul_rn(__fmul_rn(gl, nnt), gae));
    adv[k] = gae;
    ret[k] = __fadd_rn(gae, vt);  // ppo.py:169
    nv = vt;
  }
}

hipError_t launch_masked_sample(const float* logits, const uint64_t* mbits, int n, const float* uniform,
                                uint64_t seed, uint64_t step, const uint64_t* d_step, uint64_t offset,
                                int deterministic, const int64_t* action_in, int64_t* action, float* logp,
                                float* ent, hipStream_t s) {
  int64_t waves = n;
  int64_t blocks = (waves * 64 + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(masked_sample_kernel, dim3((unsigned)blocks), dim3(256), 0, s, logits, mbits, n, uniform, seed,
                     step, d_step, offset, deterministic, action_in, action, logp, ent);
  return hipGetLastError();
}

hipError_t launch_gae(const float* r, const float* v, const float* d, const float* last, int T, int N, float gamma,
                      float gl, float* adv, float* ret, hipStream_t s) {
  hipLaunchKernelGGL(gae_kernel, dim3((N + 255) / 256), dim3(256), 0, s, r, v, d, last, T, N, gamma, gl, adv, ret);
  return hipGetLastError();
}

}  // namespace bb

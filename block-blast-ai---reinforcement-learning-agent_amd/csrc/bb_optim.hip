// bb_optim.hip -- the tail of the PPO minibatch step (gfx950): gradient-norm
// clipping + Adam in three launches, and the CNN's autocast weight casts of the
// Linear layers in one launch each way.
//
// PPOAgent.update (ppo.py:400-401) runs nn.utils.clip_grad_norm_(params, 0.5)
// and torch.optim.Adam(lr, eps=1e-5).step() after every minibatch backward.
// torch issues them as a per-tensor norm kernel, a few scalar kernels, a
// multi-tensor scale and two multi-tensor Adam launches (~115 us per step at
// 5.29 M parameters, ~2 TB/s); here they are
//   adam_norm_kernel     : sum of g^2 per chunk of 2,048 elements -> fp64 partials
//   adam_finalize_kernel : one workgroup adds the partials in a fixed order
//                          (deterministic), clip coefficient
//                          min(max_norm / (||g|| + 1e-6), 1), step += 1 per
//                          tensor, Adam's bias corrections;
//   adam_update_kernel   : g *= coef (written back, as clip_grad_norm_ leaves
//                          it), then torch's fused Adam arithmetic
//                          (fused_adam_utils.cuh adam_math, ADAM_MODE::ORIGINAL:
//                          the moment updates in double, step size lr / bc1,
//                          denom sqrt(v) / sqrt(bc2) + eps).
// Every kernel is one HBM pass over its operands; the tensor table travels in
// the kernel arguments, so a HIP graph can capture the launches.
//
// Casts: under bf16 autocast every nn.Linear of the CNN casts its f32 weight
// and bias to bf16 in a kernel of its own, and autograd casts the bf16 weight
// gradients back (24 launches per step, plus a strided permute-copy of the
// first FC weight for the channels_last flatten, network.py trunk).
// cast_multi_kernel does all tensors of one direction in one launch; a tensor
// with perm_c > 0 is [O][perm_c][perm_hw] on the f32 side and [O][perm_hw][perm_c]
// on the bf16 side (transposed per row through LDS, both sides coalesced).
//
// Linear tails under bf16 autocast (network.py:89-117, nn.Linear -> nn.ReLU -> nn.Dropout(0.1)):
//   dropout_fwd_kernel  : nn.Dropout's training forward over the ReLU GEMM's bf16 output, in place
//                         (y * scale where a Philox4x32-10 draw keeps the element, else 0); the generator's
//                         (seed, offset) live in a device word the launch advances itself, so a captured
//                         HIP graph draws fresh masks on every replay without a host-side refill;
//   linear_bgrad_kernel : the backward up to the GEMMs -- g = dy * scale where the saved output
//                         (after ReLU and dropout) is > 0, else 0 (dropout's masked scale, then
//                         threshold_backward, as autograd rounds them), and the bias gradient
//                         db = sum over rows of g (f32 sums in a fixed order, bf16 out) -- one pass
//                         instead of torch's masked-scale, threshold, semaphore memset and reduction.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <math.h>

#include <algorithm>

#include "bb_env_internal.h"

namespace bb {

namespace {

constexpr int kOptThreads = 256;
constexpr int kOptChunk = 2048;  // elements per workgroup (8 per thread)
constexpr int kCastChunk = 8192; // elements per workgroup in the casts (one permuted row at most)

struct AdamTable {
  float* p[kOptMaxTensors];
  float* g[kOptMaxTensors];
  float* m[kOptMaxTensors];
  float* v[kOptMaxTensors];
  float* step[kOptMaxTensors];
  int64_t n[kOptMaxTensors];
  int32_t chunk0[kOptMaxTensors + 1];  // first chunk of tensor t; chunk0[count] = total
  int32_t count;
};

struct CastTable {
  const void* src[kOptMaxTensors];
  void* dst[kOptMaxTensors];
  int64_t n[kOptMaxTensors];
  int32_t perm_c[kOptMaxTensors];
  int32_t perm_hw[kOptMaxTensors];
  int32_t chunk0[kOptMaxTensors + 1];
  int32_t count;
};

// workspace: [0, kHdr) doubles of header (coef, norm, per-tensor bc1 / sqrt(bc2) as floats), then partials
constexpr int kHdr = 8 + kOptMaxTensors;

template <typename Tab>
__device__ __forceinline__ int find_tensor(const Tab& tab, int chunk) {
  int t = 0;
  while (t + 1 < tab.count && tab.chunk0[t + 1] <= chunk) ++t;  // uniform scan over <= 48 kernel arguments
  return t;
}

__device__ double block_sum(double x, double* red) {
  // fixed-order tree over the workgroup (deterministic)
  for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = x;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < kOptThreads / 64; ++i) s += red[i];
  return s;
}

// BB_ADAM_NORM_CPB chunks per workgroup, their loads all in flight before the adds; every chunk's sum is its
// own partial, added in the same order for any setting (bit-identical partials).  4: 15.2 us vs 11.0 us for
// one chunk per workgroup (fewer workgroups in flight; tools/variants.py an4).
#ifndef BB_ADAM_NORM_CPB
#define BB_ADAM_NORM_CPB 1
#endif
constexpr int kNormCpb = BB_ADAM_NORM_CPB;

__global__ void __launch_bounds__(kOptThreads) adam_norm_kernel(const AdamTable tab, double* __restrict__ ws) {
  __shared__ double red[kNormCpb][kOptThreads / 64];
  constexpr int L = kOptChunk / (kOptThreads * 4);  // float4 loads per thread per chunk
  const int nchunks = tab.chunk0[tab.count];
  float acc[kNormCpb];
  float4 q[kNormCpb][L];
  bool fast[kNormCpb];
#pragma unroll
  for (int j = 0; j < kNormCpb; ++j) {
    acc[j] = 0.f;
    const int chunk = blockIdx.x * kNormCpb + j;
    fast[j] = false;
    if (chunk >= nchunks) continue;
    const int t = find_tensor(tab, chunk);
    const int64_t base = int64_t(chunk - tab.chunk0[t]) * kOptChunk;
    const float* g = tab.g[t];
    fast[j] = ((reinterpret_cast<uintptr_t>(g) & 15) == 0) && base + kOptChunk <= tab.n[t];
    if (fast[j]) {
#pragma unroll
      for (int k = 0; k < L; ++k)
        q[j][k] = *reinterpret_cast<const float4*>(g + base + threadIdx.x * 4 + k * kOptThreads * 4);
    } else {
      for (int64_t i = base + threadIdx.x; i < tab.n[t] && i < base + kOptChunk; i += kOptThreads)
        acc[j] += g[i] * g[i];
    }
  }
#pragma unroll
  for (int j = 0; j < kNormCpb; ++j)
    if (fast[j])
#pragma unroll
      for (int k = 0; k < L; ++k) acc[j] += q[j][k].x * q[j][k].x + q[j][k].y * q[j][k].y + q[j][k].z * q[j][k].z +
                                           q[j][k].w * q[j][k].w;
  // block_sum's fixed-order tree, per chunk
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < kNormCpb; ++j) {
    double x = double(acc[j]);
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
    if (lane == 0) red[j][w] = x;
  }
  __syncthreads();
  if (threadIdx.x < kNormCpb) {
    const int chunk = blockIdx.x * kNormCpb + threadIdx.x;
    double s = 0.0;
    for (int i = 0; i < kOptThreads / 64; ++i) s += red[threadIdx.x][i];
    if (chunk < nchunks) ws[kHdr + chunk] = s;
  }
}

// Guard on the norm's inputs: a chunk partial (the sum of g^2 over 2,048 elements) that is not finite or above
// kGuardChunkSq (a chunk L2 norm above 1e8, ~1e5x the largest this network's gradients reach) is an operand that
// no gradient kernel should have produced -- e.g. a read of an unwritten workspace.  The finaliser records the
// first such chunk in header word kGuardWord as chunk + 1 (sticky: only the first offence is kept until the host
// clears it) and counts offences in kGuardWord + 1; the update itself is not altered (clip_grad_norm_'s
// arithmetic on whatever the gradients hold).  PPOAgent.update reads the word once per update and raises.
constexpr double kGuardChunkSq = 1e16;
constexpr int kGuardWord = 2;  // uint32 words 2, 3 of the header (floats 2..15 are unused)

__global__ void __launch_bounds__(kOptThreads) adam_finalize_kernel(const AdamTable tab, double* __restrict__ ws,
                                                                    float max_norm, double beta1, double beta2,
                                                                    float* __restrict__ norm_out) {
  __shared__ double red[kOptThreads / 64];
  __shared__ uint32_t bad_first, bad_count;
  if (threadIdx.x == 0) {
    bad_first = 0xffffffffu;
    bad_count = 0u;
  }
  __syncthreads();
  const int nchunks = tab.chunk0[tab.count];
  double s = 0.0;
  uint32_t my_first = 0xffffffffu, my_count = 0u;
  auto guard = [&](double v, int c) {
    if (!(v <= kGuardChunkSq)) {  // NaN fails the comparison too
      my_first = min(my_first, (uint32_t)c);
      ++my_count;
    }
  };
  int i = threadIdx.x;
  for (; i + 7 * kOptThreads < nchunks; i += 8 * kOptThreads) {  // 8 loads in flight, added in order
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ws[kHdr + i + j * kOptThreads];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s += v[j];
      guard(v[j], i + j * kOptThreads);
    }
  }
  for (; i < nchunks; i += kOptThreads) {
    const double v = ws[kHdr + i];
    s += v;
    guard(v, i);
  }
  if (my_count) {
    atomicMin(&bad_first, my_first);
    atomicAdd(&bad_count, my_count);
  }
  s = block_sum(s, red);  // (its barrier orders the LDS atomics above before thread 0's reads below)
  float* hdr = reinterpret_cast<float*>(ws);
  if (threadIdx.x == 0) {
    uint32_t* gw = reinterpret_cast<uint32_t*>(ws) + kGuardWord;
    if (bad_count) {
      if (gw[0] == 0u) gw[0] = bad_first + 1u;
      gw[1] += bad_count;
    }
    // clip_grad_norm_: total_norm (f32), clip_coef = max_norm / (total_norm + 1e-6), clamped to <= 1
    const float norm = float(sqrt(s));
    const float coef = fminf(max_norm / (norm + 1e-6f), 1.0f);
    hdr[0] = coef;
    hdr[1] = norm;
    if (norm_out) *norm_out = norm;
  }
  if (threadIdx.x < tab.count) {
    // torch's fused Adam: state_steps += 1, then the bias corrections from the new step
    const int t = threadIdx.x;
    const float st = *tab.step[t] + 1.0f;
    *tab.step[t] = st;
    const double bc1 = 1.0 - pow(beta1, double(st));
    const double bc2 = 1.0 - pow(beta2, double(st));
    hdr[16 + 2 * t] = float(bc1);
    hdr[16 + 2 * t + 1] = float(sqrt(bc2));
  }
}

__device__ __forceinline__ void adam_elem(float& p, float& g, float& m, float& v, float coef, double lr, double beta1,
                                          double beta2, double eps, float bc1, float bc2s) {
  g = g * coef;
  m = float(beta1 * double(m) + (1.0 - beta1) * double(g));
  v = float(beta2 * double(v) + (1.0 - beta2) * double(g) * double(g));
  const float step_size = float(lr / double(bc1));
  const float denom = float(double(sqrtf(v) / bc2s) + eps);
  p -= step_size * m / denom;
}

__global__ void __launch_bounds__(kOptThreads) adam_update_kernel(const AdamTable tab, const double* __restrict__ ws,
                                                                  double lr, double beta1, double beta2, double eps) {
  const int chunk = blockIdx.x;
  const int t = find_tensor(tab, chunk);
  const int64_t base = int64_t(chunk - tab.chunk0[t]) * kOptChunk;
  const int64_t n = tab.n[t];
  const float* hdr = reinterpret_cast<const float*>(ws);
  const float coef = hdr[0], bc1 = hdr[16 + 2 * t], bc2s = hdr[16 + 2 * t + 1];
  float *P = tab.p[t], *G = tab.g[t], *M = tab.m[t], *V = tab.v[t];
  const bool vec = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(G) | reinterpret_cast<uintptr_t>(M) |
                     reinterpret_cast<uintptr_t>(V)) & 15) == 0;
  if (vec && base + kOptChunk <= n) {
#pragma unroll
    for (int k = 0; k < kOptChunk; k += kOptThreads * 4) {
      const int64_t i = base + k + threadIdx.x * 4;
      float4 p = *reinterpret_cast<float4*>(P + i), g = *reinterpret_cast<float4*>(G + i);
      float4 m = *reinterpret_cast<float4*>(M + i), v = *reinterpret_cast<float4*>(V + i);
      adam_elem(p.x, g.x, m.x, v.x, coef, lr, beta1, beta2, eps, bc1, bc2s);
      adam_elem(p.y, g.y, m.y, v.y, coef, lr, beta1, beta2, eps, bc1, bc2s);
      adam_elem(p.z, g.z, m.z, v.z, coef, lr, beta1, beta2, eps, bc1, bc2s);
      adam_elem(p.w, g.w, m.w, v.w, coef, lr, beta1, beta2, eps, bc1, bc2s);
      *reinterpret_cast<float4*>(P + i) = p;
      *reinterpret_cast<float4*>(G + i) = g;
      *reinterpret_cast<float4*>(M + i) = m;
      *reinterpret_cast<float4*>(V + i) = v;
    }
  } else {
    for (int64_t i = base + threadIdx.x; i < n && i < base + kOptChunk; i += kOptThreads) {
      float p = P[i], g = G[i], m = M[i], v = V[i];
      adam_elem(p, g, m, v, coef, lr, beta1, beta2, eps, bc1, bc2s);
      P[i] = p;
      G[i] = g;
      M[i] = m;
      V[i] = v;
    }
  }
}

__device__ __forceinline__ uint16_t f2bf_rne(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);  // round to nearest even, as autocast's cast
  return *reinterpret_cast<uint16_t*>(&b);
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

// DIR 0: f32 -> bf16, DIR 1: bf16 -> f32
template <int DIR>
__global__ void __launch_bounds__(kOptThreads) cast_multi_kernel(const CastTable tab) {
  __shared__ float tile[kCastChunk + kCastChunk / 64];  // one permuted row, padded every 64 floats
  const int chunk = blockIdx.x;
  const int t = find_tensor(tab, chunk);
  const int pc = tab.perm_c[t];
  const int64_t n = tab.n[t];
  if (pc > 0) {  // one row [perm_c][perm_hw] (f32 side) <-> [perm_hw][perm_c] (bf16 side) per workgroup
    const int hw = tab.perm_hw[t], row = pc * hw;
    const int64_t base = int64_t(chunk - tab.chunk0[t]) * row;
    auto pad = [](int i) { return i + (i >> 6); };
    if (DIR == 0) {
      const float* s = static_cast<const float*>(tab.src[t]) + base;
      uint16_t* d = static_cast<uint16_t*>(tab.dst[t]) + base;
      for (int i = threadIdx.x; i < row; i += kOptThreads) tile[pad(i)] = s[i];  // i = c * hw + q
      __syncthreads();
      for (int j = threadIdx.x; j < row; j += kOptThreads) {  // j = q * pc + c
        const int q = j / pc, c = j - q * pc;
        d[j] = f2bf_rne(tile[pad(c * hw + q)]);
      }
    } else {
      const uint16_t* s = static_cast<const uint16_t*>(tab.src[t]) + base;
      float* d = static_cast<float*>(tab.dst[t]) + base;
      for (int j = threadIdx.x; j < row; j += kOptThreads) tile[pad(j)] = bf2f(s[j]);  // j = q * pc + c
      __syncthreads();
      for (int i = threadIdx.x; i < row; i += kOptThreads) {  // i = c * hw + q
        const int c = i / hw, q = i - c * hw;
        d[i] = tile[pad(q * pc + c)];
      }
    }
    return;
  }
  const int64_t base = int64_t(chunk - tab.chunk0[t]) * kCastChunk;
  const int64_t end = base + kCastChunk < n ? base + kCastChunk : n;
  if (DIR == 0) {
    const float* s = static_cast<const float*>(tab.src[t]);
    uint16_t* d = static_cast<uint16_t*>(tab.dst[t]);
    const bool vec = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0;
    int64_t i = base + threadIdx.x * 8;
    if (vec)
      for (; i + 8 <= end; i += kOptThreads * 8) {
        const float4 a = *reinterpret_cast<const float4*>(s + i), b = *reinterpret_cast<const float4*>(s + i + 4);
        uint4 o;
        o.x = uint32_t(f2bf_rne(a.x)) | (uint32_t(f2bf_rne(a.y)) << 16);
        o.y = uint32_t(f2bf_rne(a.z)) | (uint32_t(f2bf_rne(a.w)) << 16);
        o.z = uint32_t(f2bf_rne(b.x)) | (uint32_t(f2bf_rne(b.y)) << 16);
        o.w = uint32_t(f2bf_rne(b.z)) | (uint32_t(f2bf_rne(b.w)) << 16);
        *reinterpret_cast<uint4*>(d + i) = o;
      }
    // scalar tail (or the whole chunk when unaligned)
    const int64_t tail0 = vec ? base + ((end - base) / 8) * 8 : base;
    for (int64_t k = tail0 + threadIdx.x; k < end; k += kOptThreads) d[k] = f2bf_rne(s[k]);
  } else {
    const uint16_t* s = static_cast<const uint16_t*>(tab.src[t]);
    float* d = static_cast<float*>(tab.dst[t]);
    const bool vec = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0;
    if (vec)
      for (int64_t i = base + threadIdx.x * 8; i + 8 <= end; i += kOptThreads * 8) {
        const uint4 h = *reinterpret_cast<const uint4*>(s + i);
        *reinterpret_cast<float4*>(d + i) = make_float4(__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xffff0000u),
                                                        __uint_as_float(h.y << 16), __uint_as_float(h.y & 0xffff0000u));
        *reinterpret_cast<float4*>(d + i + 4) = make_float4(__uint_as_float(h.z << 16),
                                                            __uint_as_float(h.z & 0xffff0000u),
                                                            __uint_as_float(h.w << 16),
                                                            __uint_as_float(h.w & 0xffff0000u));
      }
    const int64_t tail0 = vec ? base + ((end - base) / 8) * 8 : base;
    for (int64_t k = tail0 + threadIdx.x; k < end; k += kOptThreads) d[k] = bf2f(s[k]);
  }
}

// ---------------------------------------------------------------- Linear tails (dropout, bias gradient)
constexpr int kDropThreads = 256;  // 8 bf16 per thread per pass
#ifndef BB_DROP_BLOCKS
#define BB_DROP_BLOCKS 128
#endif
constexpr int kDropMaxBlocks = BB_DROP_BLOCKS;
#ifndef BB_DROP_UNROLL
#define BB_DROP_UNROLL 4
#endif
constexpr int kDropUnroll = BB_DROP_UNROLL;
// linear_bgrad_kernel shape: BB_BGRAD_CFG 0 = 64 columns x 32 row lanes (256 threads), row chunks of ~128 rows
// (BB_BGRAD_CHUNK)
// with the write-through hand-off; 1 = 8 columns x 1024 row lanes, all rows in one workgroup; 2 = 16 columns x
// 512 row lanes, all rows; 3 = 8 columns x 256 row lanes, row chunks of ~512 rows with the hand-off
#ifndef BB_BGRAD_CFG
#define BB_BGRAD_CFG 0
#endif
constexpr int kBgradCL = BB_BGRAD_CFG == 0 ? 8 : BB_BGRAD_CFG == 2 ? 2 : 1;  // column lanes of 8 columns
constexpr int kBgradThreads = BB_BGRAD_CFG == 0 || BB_BGRAD_CFG == 3 ? 256 : 1024;
constexpr int kBgradCols = 8 * kBgradCL;
#ifndef BB_BGRAD_CHUNK
#define BB_BGRAD_CHUNK 128
#endif
constexpr int kBgradChunk = BB_BGRAD_CFG == 0 ? BB_BGRAD_CHUNK : BB_BGRAD_CFG == 3 ? 512 : 0;  // rows per chunk
constexpr int kBgradMaxSplit = 64;

// Last-arriver hand-off between workgroups, ordered by the HIP memory model rather than by hardware behaviour:
// partial sums stored with agent-scope atomic stores (written through, sc1), a workgroup barrier (every wave's
// stores issued before the count), then one lane counts the workgroup with an agent-scope release add
// (buffer_wbl2 sc1 + s_waitcnt vmcnt(0) before it: the partials of every wave that passed the barrier are
// published); the lane whose add returns the last count issues an agent-scope acquire fence (buffer_inv sc1)
// before its workgroup -- after a barrier, or in the same wave -- loads the partials.  The other workgroups skip
// the acquire (acq_rel on every add: 1.510 against 1.478 ms per bf16 step, profiles/r06/handoff/).  The re-arm
// of the counter is an agent-scope atomic store.
#ifndef BB_HANDOFF_ORDER
#define BB_HANDOFF_ORDER __ATOMIC_RELEASE  // A/B only: __ATOMIC_RELAXED is the round-5 form (tools/variants.py hrx)
#endif
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) uint32_t guint32;
__device__ __forceinline__ void wt_store(float* p, float v) {
  __hip_atomic_store((gfloat*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float wt_load(const float* p) {
  return __hip_atomic_load((const gfloat*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// true in the lane whose add completes the count n (it has then acquired every other workgroup's release)
__device__ __forceinline__ bool wt_arrive_last(uint32_t* c, uint32_t n) {
  const bool last = __hip_atomic_fetch_add((guint32*)c, 1u, BB_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT) == n - 1u;
  if (last && BB_HANDOFF_ORDER != __ATOMIC_RELAXED) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return last;
}
__device__ __forceinline__ void wt_rearm(uint32_t* c) {
  __hip_atomic_store((guint32*)c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the waves' own stores complete before the barrier that precedes the arrive (the release covers them too;
// kept so a wave never reaches the barrier with its partial stores still in flight)
__device__ __forceinline__ void wt_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct Philox4 {
  uint32_t v[4];
};

// Philox4x32-10 (Salmon et al., SC'11): counter c, key k.
__device__ __forceinline__ Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                 uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return Philox4{{c0, c1, c2, c3}};
}

// rng: {seed, offset, arrivals, 0} (int64).  Element i keeps its value when draw (i / 4, lane i % 4) of
// counter (i / 4, offset) >= thresh (P(drop) = thresh / 2^32).  The last workgroup to arrive advances the
// offset by one and clears the arrival count, so the next launch (or graph replay) draws a new mask.
__global__ void __launch_bounds__(kDropThreads) dropout_fwd_kernel(uint16_t* y, int64_t n, uint32_t thresh,
                                                                   float scale, int64_t* rng) {
  const uint64_t seed = (uint64_t)rng[0], off = (uint64_t)rng[1];
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32), o0 = (uint32_t)off, o1 = (uint32_t)(off >> 32);
  // kDropUnroll vectors of 8 per thread in flight: loads first (y is read and written in place, so the
  // compiler would not hoist the next vector's load above this one's store)
  const int64_t stride = (int64_t)gridDim.x * kDropThreads * 8;
  for (int64_t i0 = ((int64_t)blockIdx.x * kDropThreads + threadIdx.x) * 8; i0 < n; i0 += stride * kDropUnroll) {
    uint4 h[kDropUnroll];
#pragma unroll
    for (int u = 0; u < kDropUnroll; ++u)
      if (i0 + u * stride < n) h[u] = *reinterpret_cast<const uint4*>(y + i0 + u * stride);
#pragma unroll
    for (int u = 0; u < kDropUnroll; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n) break;
      const uint64_t q = (uint64_t)i >> 2;
      const Philox4 a = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), o0, o1, k0, k1);
      const Philox4 b = philox4x32_10((uint32_t)(q + 1), (uint32_t)((q + 1) >> 32), o0, o1, k0, k1);
      const uint32_t r[8] = {a.v[0], a.v[1], a.v[2], a.v[3], b.v[0], b.v[1], b.v[2], b.v[3]};
      uint32_t w[4] = {h[u].x, h[u].y, h[u].z, h[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint16_t lo = r[2 * k] >= thresh ? f2bf_rne(bf2f((uint16_t)w[k]) * scale) : 0;
        const uint16_t hi = r[2 * k + 1] >= thresh ? f2bf_rne(bf2f((uint16_t)(w[k] >> 16)) * scale) : 0;
        w[k] = (uint32_t)lo | ((uint32_t)hi << 16);
      }
      *reinterpret_cast<uint4*>(y + i) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
  __syncthreads();  // every thread's (seed, offset) load has returned before the block counts itself
  if (threadIdx.x == 0) {
    const uint64_t prev = __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(rng + 2), 1ull,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (uint64_t)gridDim.x - 1) {  // the last block: every block has read the offset
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(rng + 1), (unsigned long long)(off + 1),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(rng + 2), 0ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Grid (column blocks of kBgradCols, row chunks): kBgradCL column lanes x 8 columns, the rest row lanes; each
// thread's 8 column sums over its chunk's rows in row order, a wave's row lanes added by a fixed xor tree, the
// waves in wave order (LDS).  One chunk: those are db.  Several: each chunk publishes its partial sums
// (write-through) and the last chunk of a column block to arrive adds them in chunk order (deterministic
// whatever the arrival order), writes db and re-arms the block's counter (cnt: zero between launches).
// yd == nullptr: g is dy itself (not written).  VEC: cols % 8 == 0 and 16-byte aligned rows.
template <bool VEC>
__global__ void __launch_bounds__(kBgradThreads) linear_bgrad_kernel(const uint16_t* __restrict__ dy,
                                                                      const uint16_t* __restrict__ yd, int rows,
                                                                      int cols, int chunk_rows, float scale,
                                                                      uint16_t* __restrict__ g,
                                                                      uint16_t* __restrict__ db, float* part,
                                                                      uint32_t* cnt, const uint16_t* __restrict__ dy2,
                                                                      int split) {
  constexpr int RL = kBgradThreads / kBgradCL;
  __shared__ float wsum[kBgradThreads / 64][kBgradCols];
  const int cl = threadIdx.x % kBgradCL, rl = threadIdx.x / kBgradCL;
  const int c0 = blockIdx.x * kBgradCols + cl * 8;
  const int r0 = blockIdx.y * chunk_rows, r1 = min(rows, r0 + chunk_rows);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (VEC) {
    if (c0 < cols) {
      // dy2: columns split.. come from a second row-major source (two layers' gradients side by side)
      const bool second = dy2 && c0 >= split;
      const uint16_t* src = second ? dy2 + (c0 - split) : dy + c0;
      const int lds = second ? cols - split : (dy2 ? split : cols);
#pragma unroll 4
      for (int r = r0 + rl; r < r1; r += RL) {
        const int64_t o = (int64_t)r * cols + c0;
        const uint4 h = *reinterpret_cast<const uint4*>(src + (int64_t)r * lds);
        uint32_t w[4] = {h.x, h.y, h.z, h.w};
        if (yd) {
          const uint4 m = *reinterpret_cast<const uint4*>(yd + o);
          const uint32_t mm[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            // bf16 > 0: sign clear and not +0
            const uint16_t lo = ((int16_t)(mm[k] & 0xffffu) > 0) ? f2bf_rne(bf2f((uint16_t)w[k]) * scale) : 0;
            const uint16_t hi = ((int16_t)(mm[k] >> 16) > 0) ? f2bf_rne(bf2f((uint16_t)(w[k] >> 16)) * scale) : 0;
            w[k] = (uint32_t)lo | ((uint32_t)hi << 16);
          }
          *reinterpret_cast<uint4*>(g + o) = make_uint4(w[0], w[1], w[2], w[3]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[2 * k] += bf2f((uint16_t)w[k]);
          acc[2 * k + 1] += bf2f((uint16_t)(w[k] >> 16));
        }
      }
    }
  } else {
    for (int r = r0 + rl; r < r1; r += RL) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        if (c < cols) {
          const int64_t o = (int64_t)r * cols + c;
          uint16_t v = dy[o];
          if (yd) {
            v = ((int16_t)yd[o] > 0) ? f2bf_rne(bf2f(v) * scale) : 0;
            g[o] = v;
          }
          acc[j] += bf2f(v);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int m = kBgradCL; m < 64; m <<= 1) acc[j] += __shfl_xor(acc[j], m, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane < kBgradCL)
#pragma unroll
    for (int j = 0; j < 8; ++j) wsum[wave][lane * 8 + j] = acc[j];
  __syncthreads();
  const int nsplit = gridDim.y;
  if (threadIdx.x >= kBgradCols) return;
  const int c = blockIdx.x * kBgradCols + threadIdx.x;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kBgradThreads / 64; ++k) s += wsum[k][threadIdx.x];
  if (nsplit == 1) {
    if (c < cols) db[c] = f2bf_rne(s);
    return;
  }
  // (the threads left are one wave: kBgradCols <= 64)
  float* col = part + (size_t)blockIdx.x * nsplit * kBgradCols + threadIdx.x;
  wt_store(col + (size_t)blockIdx.y * kBgradCols, s);
  wt_drain();
  int arrived = 0;
  if (threadIdx.x == 0) arrived = wt_arrive_last(cnt + blockIdx.x, (uint32_t)nsplit);
  if (!__shfl(arrived, 0, 64)) return;  // lane 0's add has returned
  float v[kBgradMaxSplit];
#pragma unroll
  for (int k = 0; k < kBgradMaxSplit; ++k) v[k] = k < nsplit ? wt_load(col + (size_t)k * kBgradCols) : 0.f;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < kBgradMaxSplit; ++k) t += v[k];  // chunk order; absent chunks add +0
  if (c < cols) db[c] = f2bf_rne(t);
  if (threadIdx.x == 0) wt_rearm(cnt + blockIdx.x);  // every chunk has counted itself: re-armed for the next launch
}

// Weight gradient of a bf16 Linear, dW[n][k] = sum_r g[r][n] x[r][k] (autograd's g^T x for the CNN's small
// FC / head layers, where hipBLASLt's tiles leave all but a few CUs idle over the 2,048-row reduction).
// Grid (K / 32, N / 32, row splits of 256): a workgroup loads its 256 rows of both 32-column strips at once
// (8 x 16 B per thread in flight), wave w takes rows 64 w .. 64 w + 63 (mfma_f32_16x16x16_bf16, 2 x 2 tiles);
// both operands are row-major in HBM and reach the MFMA k-major through ds_read_b64_tr_b16 (lane 4q + p of a
// 16-lane group addresses row q, columns 4p .. 4p + 3 of its 4 x 16 block).  The 4 waves' sums are added in
// wave order (LDS, one output per thread per pass); with several splits each publishes its 32 x 32 partial
// write-through and the last split
// to arrive adds them in split order (deterministic) and re-arms the tile's counter; the sum is rounded to
// bf16 once.
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr int kWgT = 32;        // dW tile
constexpr int kWgSplit = 256;   // rows per workgroup
constexpr int kWgMaxSplit = 64;

__device__ __forceinline__ s16x4 tr_read(const uint16_t* lds) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)lds);
}

__global__ void __launch_bounds__(256) linear_wgrad_kernel(const uint16_t* __restrict__ g,
                                                           const uint16_t* __restrict__ x, int rows, int N, int K,
                                                           int ldx, uint16_t* __restrict__ dw, float* part,
                                                           uint32_t* cnt) {
  __shared__ __attribute__((aligned(16))) uint16_t gs[kWgSplit][kWgT];
  __shared__ __attribute__((aligned(16))) uint16_t xs[kWgSplit][kWgT];
  __shared__ float red[4][kWgT * kWgT];
  __shared__ int last_split;
  const int n0 = blockIdx.y * kWgT, k0 = blockIdx.x * kWgT, r0 = blockIdx.z * kWgSplit;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  {  // rows r0 + (t >> 2) + 64 u, 16-byte piece t & 3 of each 64-byte strip row
    const int lr = t >> 2, lp = (t & 3) * 8;
    uint4 rg[4], rx[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = r0 + lr + 64 * u;
      if (r < rows) {
        rg[u] = *reinterpret_cast<const uint4*>(g + (int64_t)r * N + n0 + lp);
        rx[u] = *reinterpret_cast<const uint4*>(x + (int64_t)r * ldx + k0 + lp);
      } else {
        rg[u] = make_uint4(0u, 0u, 0u, 0u);
        rx[u] = rg[u];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      *reinterpret_cast<uint4*>(&gs[lr + 64 * u][lp]) = rg[u];
      *reinterpret_cast<uint4*>(&xs[lr + 64 * u][lp]) = rx[u];
    }
  }
  __syncthreads();
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int rrow = 64 * wave + 16 * ks + 4 * grp + q;  // this lane's block row
    s16x4 af[2], bf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = tr_read(&gs[rrow][16 * i + 4 * p]);  // A[m = n][k = row]
#pragma unroll
    for (int j = 0; j < 2; ++j) bf[j] = tr_read(&xs[rrow][16 * j + 4 * p]);  // B[k = row][n = k]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af[i], bf[j], acc[i][j], 0, 0, 0);
  }
  // C[m = 4 grp + e][n = li] of tile (i, j) -> LDS; thread t then owns outputs t + 256 u, summed in wave order
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave][(16 * i + 4 * grp + e) * kWgT + 16 * j + li] = acc[i][j][e];
  __syncthreads();
  constexpr int kOut = kWgT * kWgT / 256;
  float v[kOut];
#pragma unroll
  for (int u = 0; u < kOut; ++u) {
    const int o = t + 256 * u;
    v[u] = ((red[0][o] + red[1][o]) + red[2][o]) + red[3][o];
  }
  const int nsplit = gridDim.z;
  const int tile = blockIdx.y * gridDim.x + blockIdx.x;
  if (nsplit > 1) {  // publish, count; the last split adds every split's partial in split order
    float* tp = part + (size_t)tile * nsplit * (kWgT * kWgT);
#pragma unroll
    for (int u = 0; u < kOut; ++u) wt_store(tp + (size_t)blockIdx.z * (kWgT * kWgT) + t + 256 * u, v[u]);
    wt_drain();
    __syncthreads();  // every wave's partial stores have drained
    if (t == 0) last_split = wt_arrive_last(cnt + tile, (uint32_t)nsplit);
    __syncthreads();
    if (!last_split) return;
#pragma unroll
    for (int u = 0; u < kOut; ++u) {
      const float* src = tp + t + 256 * u;
      float sum = 0.f;
      for (int z0 = 0; z0 < nsplit; z0 += 8) {
        float ps[8];
#pragma unroll
        for (int z = 0; z < 8; ++z) ps[z] = z0 + z < nsplit ? wt_load(src + (size_t)(z0 + z) * (kWgT * kWgT)) : 0.f;
#pragma unroll
        for (int z = 0; z < 8; ++z) sum += ps[z];  // split order; absent splits add +0
      }
      v[u] = sum;
    }
    if (t == 0) wt_rearm(cnt + tile);  // every split has counted itself: re-armed for the next launch
  }
#pragma unroll
  for (int u = 0; u < kOut; ++u) {
    const int o = t + 256 * u, m = o / kWgT, n = o % kWgT;
    dw[(int64_t)(n0 + m) * K + k0 + n] = f2bf_rne(v[u]);
  }
}

// A bf16 Linear with ONE output (network.py's value head, Linear(128, 1), under autocast): torch runs it as a
// bias copy + a GEMM forward and a GEMM for dx, a GEMM for dW and a reduction for db backward.
// linear_n1_fwd_kernel: y[r] = bf16(sum_k x[r][k] w[k] + b), 16 lanes per row (8 columns per load), the lanes'
// sums added by a fixed xor tree.
// linear_n1_bwd_kernel: dx[r][k] = bf16(gy[r] w[k]) (the K = 1 GEMM's exact product, rounded once), dW[k] =
// sum_r gy[r] x[r][k] and db = sum_r gy[r] in f32, laid out as bb_linear_bgrad (64 columns x row chunks,
// write-through partials, the last chunk adds them in chunk order; db is column block 0's 65th sum).
constexpr int kN1Rows = 16;
constexpr int kN1Slots = kBgradCols + 1;

__global__ void __launch_bounds__(256) linear_n1_fwd_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ w,
                                                            const uint16_t* __restrict__ b, int rows, int K, int ldx,
                                                            uint16_t* __restrict__ y) {
  const int r = blockIdx.x * kN1Rows + (threadIdx.x >> 4), l = threadIdx.x & 15;
  float s = 0.f;
  if (r < rows)
    for (int k = 8 * l; k < K; k += 128) {
      const uint4 xv = *reinterpret_cast<const uint4*>(x + (int64_t)r * ldx + k);
      const uint4 wv = *reinterpret_cast<const uint4*>(w + k);
      const uint32_t xa[4] = {xv.x, xv.y, xv.z, xv.w}, wa[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s += bf2f((uint16_t)xa[e]) * bf2f((uint16_t)wa[e]);
        s += bf2f((uint16_t)(xa[e] >> 16)) * bf2f((uint16_t)(wa[e] >> 16));
      }
    }
#pragma unroll
  for (int m = 8; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
  if (l == 0 && r < rows) y[r] = f2bf_rne(s + (b ? bf2f(b[0]) : 0.f));
}

__global__ void __launch_bounds__(256) linear_n1_bwd_kernel(const uint16_t* __restrict__ gy,
                                                            const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ w, int rows, int K,
                                                            int ldx, int chunk_rows, uint16_t* __restrict__ dx,
                                                            uint16_t* __restrict__ dw, uint16_t* __restrict__ db,
                                                            float* part, uint32_t* cnt) {
  __shared__ float wsum[4][kN1Slots];
  __shared__ int last_chunk;
  const int t = threadIdx.x, cl = t & 7, rl = t >> 3, lane = t & 63, wave = t >> 6;
  const int c0 = blockIdx.x * kBgradCols + cl * 8;
  const int r0 = blockIdx.y * chunk_rows, r1 = min(rows, r0 + chunk_rows);
  const bool live = c0 < K;
  float wv[8], acc[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) acc[j] = 0.f;
  if (live) {
    const uint4 h = *reinterpret_cast<const uint4*>(w + c0);
    const uint32_t ha[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      wv[2 * e] = bf2f((uint16_t)ha[e]);
      wv[2 * e + 1] = bf2f((uint16_t)(ha[e] >> 16));
    }
  }
#pragma unroll 2
  for (int r = r0 + rl; r < r1; r += 32) {
    const float gv = bf2f(gy[r]);
    acc[8] += gv;
    if (live) {
      const int64_t o = (int64_t)r * K + c0;
      const uint4 h = *reinterpret_cast<const uint4*>(x + (int64_t)r * ldx + c0);
      const uint32_t xa[4] = {h.x, h.y, h.z, h.w};
      uint32_t d[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = bf2f((uint16_t)xa[e]), hi = bf2f((uint16_t)(xa[e] >> 16));
        acc[2 * e] += gv * lo;
        acc[2 * e + 1] += gv * hi;
        d[e] = (uint32_t)f2bf_rne(gv * wv[2 * e]) | ((uint32_t)f2bf_rne(gv * wv[2 * e + 1]) << 16);
      }
      *reinterpret_cast<uint4*>(dx + o) = make_uint4(d[0], d[1], d[2], d[3]);
    }
  }
#pragma unroll
  for (int j = 0; j < 9; ++j)
#pragma unroll
    for (int m = 8; m < 64; m <<= 1) acc[j] += __shfl_xor(acc[j], m, 64);
  if (lane < 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) wsum[wave][lane * 8 + j] = acc[j];
    if (lane == 0) wsum[wave][kBgradCols] = acc[8];
  }
  __syncthreads();
  float v = 0.f;
  if (t < kN1Slots) v = ((wsum[0][t] + wsum[1][t]) + wsum[2][t]) + wsum[3][t];  // wave order
  const int nsplit = gridDim.y;
  if (nsplit > 1) {
    float* col = part + (size_t)blockIdx.x * nsplit * kN1Slots + t;
    if (t < kN1Slots) wt_store(col + (size_t)blockIdx.y * kN1Slots, v);
    wt_drain();
    __syncthreads();  // the storing waves have drained
    if (t == 0) last_chunk = wt_arrive_last(cnt + blockIdx.x, (uint32_t)nsplit);
    __syncthreads();
    if (!last_chunk) return;
    if (t < kN1Slots) {
      float sum = 0.f;
      for (int z0 = 0; z0 < nsplit; z0 += 8) {
        float ps[8];
#pragma unroll
        for (int z = 0; z < 8; ++z) ps[z] = z0 + z < nsplit ? wt_load(col + (size_t)(z0 + z) * kN1Slots) : 0.f;
#pragma unroll
        for (int z = 0; z < 8; ++z) sum += ps[z];  // chunk order
      }
      v = sum;
    }
    if (t == 0) wt_rearm(cnt + blockIdx.x);
  }
  if (t < kBgradCols) {
    const int c = blockIdx.x * kBgradCols + t;
    if (c < K) dw[c] = f2bf_rne(v);
  } else if (t == kBgradCols && blockIdx.x == 0 && db) {
    db[0] = f2bf_rne(v);
  }
}

int build_adam_table(AdamTable& tab, int count, float* const* p, float* const* g, float* const* m, float* const* v,
                     float* const* step, const int64_t* n) {
  if (count <= 0 || count > kOptMaxTensors) return -1;
  tab.count = count;
  int64_t c = 0;
  for (int t = 0; t < count; ++t) {
    if (n[t] <= 0 || !p[t] || !g[t] || !m[t] || !v[t] || !step[t]) return -1;
    tab.p[t] = p[t];
    tab.g[t] = g[t];
    tab.m[t] = m[t];
    tab.v[t] = v[t];
    tab.step[t] = step[t];
    tab.n[t] = n[t];
    tab.chunk0[t] = int32_t(c);
    c += (n[t] + kOptChunk - 1) / kOptChunk;
    if (c > (1 << 30)) return -1;
  }
  tab.chunk0[count] = int32_t(c);
  return int(c);
}

}  // namespace

int64_t adam_clip_workspace_bytes(int count, const int64_t* n) {
  if (count <= 0 || count > kOptMaxTensors) return -1;
  int64_t c = 0;
  for (int t = 0; t < count; ++t) {
    if (n[t] <= 0) return -1;
    c += (n[t] + kOptChunk - 1) / kOptChunk;
  }
  return (kHdr + c) * int64_t(sizeof(double));
}

hipError_t launch_adam_clip(int count, float* const* p, float* const* g, float* const* m, float* const* v,
                            float* const* step, const int64_t* n, double lr, double beta1, double beta2, double eps,
                            float max_norm, double* ws, float* norm_out, hipStream_t s) {
  AdamTable tab;
  const int chunks = build_adam_table(tab, count, p, g, m, v, step, n);
  if (chunks <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(adam_norm_kernel, dim3((chunks + kNormCpb - 1) / kNormCpb), dim3(kOptThreads), 0, s, tab, ws);
  hipLaunchKernelGGL(adam_finalize_kernel, dim3(1), dim3(kOptThreads), 0, s, tab, ws, max_norm, beta1, beta2,
                     norm_out);
  hipLaunchKernelGGL(adam_update_kernel, dim3(chunks), dim3(kOptThreads), 0, s, tab, ws, lr, beta1, beta2, eps);
  return hipGetLastError();
}

hipError_t launch_cast_multi(int count, int dir, const void* const* src, void* const* dst, const int64_t* n,
                             const int32_t* perm_c, const int32_t* perm_hw, hipStream_t s) {
  if (count <= 0 || count > kOptMaxTensors || (dir != 0 && dir != 1)) return hipErrorInvalidValue;
  CastTable tab;
  tab.count = count;
  int64_t c = 0;
  for (int t = 0; t < count; ++t) {
    const int pc = perm_c ? perm_c[t] : 0, ph = perm_hw ? perm_hw[t] : 0;
    if (n[t] <= 0 || !src[t] || !dst[t] || pc < 0) return hipErrorInvalidValue;
    if (pc > 0 && (ph <= 0 || int64_t(pc) * ph > kCastChunk || n[t] % (int64_t(pc) * ph) != 0))
      return hipErrorInvalidValue;
    tab.src[t] = src[t];
    tab.dst[t] = dst[t];
    tab.n[t] = n[t];
    tab.perm_c[t] = pc;
    tab.perm_hw[t] = pc > 0 ? ph : 0;
    tab.chunk0[t] = int32_t(c);
    c += pc > 0 ? n[t] / (int64_t(pc) * ph) : (n[t] + kCastChunk - 1) / kCastChunk;
    if (c > (1 << 30)) return hipErrorInvalidValue;
  }
  tab.chunk0[count] = int32_t(c);
  if (dir == 0)
    hipLaunchKernelGGL(cast_multi_kernel<0>, dim3(c), dim3(kOptThreads), 0, s, tab);
  else
    hipLaunchKernelGGL(cast_multi_kernel<1>, dim3(c), dim3(kOptThreads), 0, s, tab);
  return hipGetLastError();
}

hipError_t launch_dropout_fwd(void* y, int64_t n, float p, int64_t* rng, hipStream_t s) {
  if (n <= 0 || n % 8 || !y || !rng || !(p > 0.f && p < 1.f) || (reinterpret_cast<uintptr_t>(y) & 15))
    return hipErrorInvalidValue;
  // torch's fused dropout: scale = 1 / (1 - p) with 1 - p held as a float
  const float keep = (float)(1.0 - (double)p);
  const float scale = (float)(1.0 / (double)keep);
  const double t = (double)p * 4294967296.0;
  const uint32_t thresh = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  int64_t blocks = (n / 8 + kDropThreads - 1) / kDropThreads;
  if (blocks > kDropMaxBlocks) blocks = kDropMaxBlocks;  // grid-stride: few arrivals on the generator word
  hipLaunchKernelGGL(dropout_fwd_kernel, dim3((unsigned)blocks), dim3(kDropThreads), 0, s, (uint16_t*)y, n,
                     thresh, scale, rng);
  return hipGetLastError();
}

static int bgrad_split(int rows) {
  return kBgradChunk ? std::min(kBgradMaxSplit, (rows + kBgradChunk - 1) / kBgradChunk) : 1;
}

int64_t linear_bgrad_workspace_bytes(int rows, int cols) {
  if (rows <= 0 || cols <= 0) return -1;
  return ((cols + kBgradCols - 1) / kBgradCols) * (int64_t)bgrad_split(rows) * kBgradCols * (int64_t)sizeof(float);
}

int linear_bgrad_counters(int cols) { return cols > 0 ? (cols + kBgradCols - 1) / kBgradCols : -1; }

hipError_t launch_linear_bgrad(const void* dy, const void* yd, int rows, int cols, float scale, void* g, void* db,
                               float* part, uint32_t* cnt, hipStream_t s, const void* dy2, int split) {
  if (rows <= 0 || cols <= 0 || !dy || !db || (yd && !g) || !part || !cnt) return hipErrorInvalidValue;
  const bool vec = cols % 8 == 0 &&
                   ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(yd) | reinterpret_cast<uintptr_t>(g) |
                     reinterpret_cast<uintptr_t>(dy2)) & 15) == 0;
  if (dy2 && (!vec || split <= 0 || split >= cols || split % 8 || (cols - split) % 8)) return hipErrorInvalidValue;
  const int nsplit = bgrad_split(rows);
  const int chunk = (rows + nsplit - 1) / nsplit;
  const dim3 grid((cols + kBgradCols - 1) / kBgradCols, nsplit);
  if (vec)
    hipLaunchKernelGGL(linear_bgrad_kernel<true>, grid, dim3(kBgradThreads), 0, s, (const uint16_t*)dy,
                       (const uint16_t*)yd, rows, cols, chunk, scale, (uint16_t*)g, (uint16_t*)db, part, cnt,
                       (const uint16_t*)dy2, split);
  else
    hipLaunchKernelGGL(linear_bgrad_kernel<false>, grid, dim3(kBgradThreads), 0, s, (const uint16_t*)dy,
                       (const uint16_t*)yd, rows, cols, chunk, scale, (uint16_t*)g, (uint16_t*)db, part, cnt,
                       (const uint16_t*)nullptr, 0);
  return hipGetLastError();
}

int64_t linear_wgrad_workspace_bytes(int rows, int N, int K) {
  if (rows <= 0 || N <= 0 || K <= 0 || N % kWgT || K % kWgT) return -1;
  const int64_t nsplit = (rows + kWgSplit - 1) / kWgSplit;
  return nsplit > kWgMaxSplit ? -1 : (int64_t)(N / kWgT) * (K / kWgT) * nsplit * kWgT * kWgT * (int64_t)sizeof(float);
}

int linear_wgrad_counters(int N, int K) { return (N % kWgT || K % kWgT) ? -1 : (N / kWgT) * (K / kWgT); }

hipError_t launch_linear_wgrad(const void* g, const void* x, int rows, int N, int K, int ldx, void* dw, float* part,
                               uint32_t* cnt, hipStream_t s) {
  if (linear_wgrad_workspace_bytes(rows, N, K) < 0 || !g || !x || !dw || !part || !cnt || ldx < K || ldx % 8 ||
      ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(x)) & 15))
    return hipErrorInvalidValue;
  const int nsplit = (rows + kWgSplit - 1) / kWgSplit;
  hipLaunchKernelGGL(linear_wgrad_kernel, dim3(K / kWgT, N / kWgT, nsplit), dim3(256), 0, s, (const uint16_t*)g,
                     (const uint16_t*)x, rows, N, K, ldx, (uint16_t*)dw, part, cnt);
  return hipGetLastError();
}

int64_t linear_n1_workspace_bytes(int rows, int K) {
  if (rows <= 0 || K <= 0 || K % 8) return -1;
  return (int64_t)((K + kBgradCols - 1) / kBgradCols) * bgrad_split(rows) * kN1Slots * (int64_t)sizeof(float);
}

int linear_n1_counters(int K) { return K > 0 ? (K + kBgradCols - 1) / kBgradCols : -1; }

hipError_t launch_linear_n1_forward(const void* x, const void* w, const void* b, int rows, int K, int ldx, void* y,
                                    hipStream_t s) {
  if (rows <= 0 || K <= 0 || K % 8 || ldx < K || ldx % 8 || !x || !w || !y ||
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w)) & 15))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(linear_n1_fwd_kernel, dim3((rows + kN1Rows - 1) / kN1Rows), dim3(256), 0, s, (const uint16_t*)x,
                     (const uint16_t*)w, (const uint16_t*)b, rows, K, ldx, (uint16_t*)y);
  return hipGetLastError();
}

hipError_t launch_linear_n1_backward(const void* gy, const void* x, const void* w, int rows, int K, int ldx, void* dx,
                                     void* dw, void* db, float* part, uint32_t* cnt, hipStream_t s) {
  if (linear_n1_workspace_bytes(rows, K) < 0 || ldx < K || ldx % 8 || !gy || !x || !w || !dx || !dw || !part || !cnt ||
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(dx)) & 15))
    return hipErrorInvalidValue;
  const int nsplit = bgrad_split(rows);
  const int chunk = (rows + nsplit - 1) / nsplit;
  hipLaunchKernelGGL(linear_n1_bwd_kernel, dim3((K + kBgradCols - 1) / kBgradCols, nsplit), dim3(256), 0, s,
                     (const uint16_t*)gy, (const uint16_t*)x, (const uint16_t*)w, rows, K, ldx, chunk, (uint16_t*)dx,
                     (uint16_t*)dw, (uint16_t*)db, part, cnt);
  return hipGetLastError();
}

}  // namespace bb

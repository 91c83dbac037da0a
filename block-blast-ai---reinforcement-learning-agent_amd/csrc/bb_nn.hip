// bb_nn.hip -- training-mode BatchNorm2d (+ fused ReLU, + the preceding
// convolution's bias) for the policy/value CNN (gfx950).
//
// BlockBlastNetwork's conv stack is conv -> BatchNorm2d -> ReLU on 8x8 boards
// (network.py:75-117, ResidualBlock network.py:14-30).  With batch statistics
// over N x 64 positions per channel, MIOpen's spatial BatchNorm took 80 us
// forward and 200 us backward per layer at N = 2048 (bf16), about a third of a
// PPO minibatch step, and the convolution bias cost a separate add forward and
// a reduction backward; these kernels are HBM passes:
//   forward : per-channel sum / sum of squares of x, accumulated in fp64 from
//             the first add -> normalise, scale, shift, optional ReLU, saved mean
//             / inverse std, running-stat update (momentum, unbiased variance),
//             exactly nn.BatchNorm2d's training forward of u = conv(x) + bias.
//             The bias only shifts the batch mean, so it cancels in the output:
//             the output is (x - mean_x) * invstd * w + b with mean_x the mean of
//             x itself (one rounding, no u = x + bias rounding amplified by the
//             normalisation) and mean_u = mean_x + bias (fp64) feeds the running
//             mean; the saved mean is mean_x.  A one-pass fp32 sum of squares
//             loses the variance to cancellation when |mean| >> std (the fp32
//             train-mode logits ended 1.2e-5 from the fp64 network with it,
//             tests/test_gpu_network_oracle.py);
//   backward: per-channel sum(g), sum(g * xhat), sum(xhat) with g = dy masked
//             by the ReLU (recomputed from x) -> dx, dweight, dbias and the
//             convolution bias gradient sum(dx).
// Reductions are two-level without atomics: every block writes fp64 partials
// (its rows, all its channels), one wave per channel adds them up in a fixed
// order, so results are deterministic run to run.
// Layout NCHW or NHWC (channels_last) contiguous, f32 or bf16 activations, f32
// parameters and stats.  Loads and stores are 16-byte vectors along the
// contiguous dimension (HW resp. C times the element size % 16 == 0).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <math.h>

#include <type_traits>

#include "bb_env_internal.h"

namespace bb {

namespace {

constexpr int kBnThreads = 256;
// rows in flight per thread in the NHWC reductions (forward: one tensor; backward: x and dy)
#ifndef BB_BN_UNROLL_BWD
#define BB_BN_UNROLL_BWD 2  // 2: -0.5% on the update step against 4 (8: +0.5%), profiles/r02/optim/bnab_*
#endif
#ifndef BB_BN_UNROLL_FWD
#define BB_BN_UNROLL_FWD 8
#endif
template <bool BWD>
constexpr int kUnroll = BWD ? BB_BN_UNROLL_BWD : BB_BN_UNROLL_FWD;
constexpr int kQ = 3;       // partial quantities per channel

template <typename T>
struct Vec;  // 16 bytes of T as floats
template <>
struct Vec<float> {
  static constexpr int N = 4;
  __device__ static void load(const void* p, int64_t i, float* f) {
    const float4 v = reinterpret_cast<const float4*>(p)[i];
    f[0] = v.x;
    f[1] = v.y;
    f[2] = v.z;
    f[3] = v.w;
  }
  __device__ static void store(void* p, int64_t i, const float* f) {
    reinterpret_cast<float4*>(p)[i] = make_float4(f[0], f[1], f[2], f[3]);
  }
  __device__ static float round(float x) { return x; }
};
template <>
struct Vec<__hip_bfloat16> {
  static constexpr int N = 8;
  __device__ static void load(const void* p, int64_t i, float* f) {
    const uint4 v = reinterpret_cast<const uint4*>(p)[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = __uint_as_float(w[k] << 16);
      f[2 * k + 1] = __uint_as_float(w[k] & 0xFFFF0000u);
    }
  }
  __device__ static uint32_t rne(float x) {  // f32 -> bf16 bits, round to nearest even (NaN kept quiet)
    const uint32_t u = __float_as_uint(x);
    const uint32_t r = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
    return (u & 0x7FFFFFFFu) > 0x7F800000u ? ((u >> 16) | 0x40u) : r;  // a select, not a branch
  }
  __device__ static float round(float x) { return __uint_as_float(rne(x) << 16); }  // the bf16 tensor value
  __device__ static void store(void* p, int64_t i, const float* f) {
    uint4 v;
    v.x = rne(f[0]) | (rne(f[1]) << 16);
    v.y = rne(f[2]) | (rne(f[3]) << 16);
    v.z = rne(f[4]) | (rne(f[5]) << 16);
    v.w = rne(f[6]) | (rne(f[7]) << 16);
    reinterpret_cast<uint4*>(p)[i] = v;
  }
};

// The ReLU of a block's output applied to its gradient from the saved output (torch's threshold_backward,
// F.relu's rule): g = y > 0 ? dy : 0 -- the ResidualBlock tail, whose ReLU follows the residual add, so the
// mask cannot be recomputed from the BatchNorm input alone.
template <typename T>
__device__ __forceinline__ void mask_grad(const void* mask, int64_t i, float* fg) {
  float fm[Vec<T>::N];
  Vec<T>::load(mask, i, fm);
#pragma unroll
  for (int j = 0; j < Vec<T>::N; ++j) fg[j] = fm[j] > 0.f ? fg[j] : 0.f;
}

// Per-channel coefficients of the reduction passes (forward reads only pb).
struct ChanCoef {
  float pb, mu, is, sc, sh;
};

__device__ __forceinline__ ChanCoef coef_of(int c, const float* pre_bias, const float* mean, const float* invstd,
                                            const float* w, const float* b, bool bwd) {
  ChanCoef k;
  (void)pre_bias;  // the statistics are those of x: the bias cancels (see the top of the file)
  k.pb = 0.f;
  k.mu = bwd ? mean[c] : 0.f;
  k.is = bwd ? invstd[c] : 0.f;
  k.sc = bwd ? k.is * w[c] : 0.f;
  k.sh = bwd ? b[c] : 0.f;
  return k;
}

// One element's contribution: forward (x, x^2, 0), for f32 activations in fp64 from the first add (the fp32
// rollout forward's precision, tests/test_gpu_network_oracle.py), for bf16 ones in f32 per thread as in
// round 4 (the bf16 training step's activations carry 8 bits); backward (g, g*xhat, xhat) in f32.
template <typename T, bool BWD>
using Acc = typename std::conditional<BWD || !std::is_same<T, float>::value, float, double>::type;

template <typename T, bool BWD>
__device__ __forceinline__ void accumulate(float xv, float gv, const ChanCoef& k, int relu, Acc<T, BWD>& s,
                                           Acc<T, BWD>& q, Acc<T, BWD>& t) {
  if constexpr (BWD) {
    const float u = xv + k.pb;
    const float g = (relu && (u - k.mu) * k.sc + k.sh <= 0.f) ? 0.f : gv;  // the forward's exact ops
    const float xh = (u - k.mu) * k.is;
    s += g;
    q += g * xh;
    t += xh;
  } else {
    const Acc<T, BWD> u = (Acc<T, BWD>)xv;
    s += u;
    q += u * u;
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// NCHW reduction, block (c, s): channel c, images s, s + S, ... -> part[s][c][kQ].
template <typename T, bool BWD, bool MASK = false>
__global__ void __launch_bounds__(kBnThreads) bn_reduce_nchw(const void* __restrict__ x, const void* __restrict__ dy,
                                                             int N, int C, int HW, const float* __restrict__ pre_bias,
                                                             const float* __restrict__ w, const float* __restrict__ b,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd, int relu,
                                                             const void* __restrict__ mask, void* __restrict__ gout,
                                                             double* __restrict__ part) {
  __shared__ double red[kQ][kBnThreads / 64];
  constexpr int V = Vec<T>::N;
  const int c = blockIdx.x;
  const int cpr = HW / V;  // 16-byte chunks per (n, c) row
  const int rows_per_iter = kBnThreads / cpr;
  const int r = threadIdx.x / cpr, kk = threadIdx.x % cpr;
  const ChanCoef k = coef_of(c, pre_bias, mean, invstd, w, b, BWD);
  Acc<T, BWD> s = 0, q = 0, t = 0;
  if (r < rows_per_iter) {
    for (int n = blockIdx.y * rows_per_iter + r; n < N; n += gridDim.y * rows_per_iter) {
      const int64_t i = ((int64_t)n * C + c) * cpr + kk;
      float fx[V], fg[V];
      Vec<T>::load(x, i, fx);
      if (BWD) Vec<T>::load(dy, i, fg);
      if (BWD && MASK) {
        mask_grad<T>(mask, i, fg);
        Vec<T>::store(gout, i, fg);  // the masked gradient, for the apply pass and the residual (exact in T)
      }
#pragma unroll
      for (int j = 0; j < V; ++j) accumulate<T, BWD>(fx[j], BWD ? fg[j] : 0.f, k, relu, s, q, t);
    }
  }
  const double v[kQ] = {wave_sum((double)s), wave_sum((double)q), wave_sum((double)t)};
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int m = 0; m < kQ; ++m) red[m][wv] = v[m];
  __syncthreads();
  if (threadIdx.x < kQ) {
    double a = 0.0;
    for (int k2 = 0; k2 < kBnThreads / 64; ++k2) a += red[threadIdx.x][k2];
    part[((int64_t)blockIdx.y * C + c) * kQ + threadIdx.x] = a;
  }
}

// NHWC reduction: thread t owns the V channels of chunk t % cpr of rows
// t / cpr, t / cpr + rows_per_iter, ... (cpr = C / V divides kBnThreads, so
// its channels never change); block b writes part[b][c][kQ] for every c.
template <typename T, bool BWD, bool MASK = false>
__global__ void __launch_bounds__(kBnThreads) bn_reduce_nhwc(const void* __restrict__ x, const void* __restrict__ dy,
                                                             int R, int C, const float* __restrict__ pre_bias,
                                                             const float* __restrict__ w, const float* __restrict__ b,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd, int relu,
                                                             const void* __restrict__ mask, void* __restrict__ gout,
                                                             double* __restrict__ part) {
  constexpr int V = Vec<T>::N;
  constexpr int NQ = BWD ? kQ : 2;  // the forward has no third quantity
  __shared__ Acc<T, BWD> red[NQ][kBnThreads * V];
  const int cpr = C / V;
  const int rows_per_iter = kBnThreads / cpr;
  const int r = threadIdx.x / cpr, kc = threadIdx.x % cpr;
  ChanCoef k[V];
  Acc<T, BWD> s[V], q[V], t[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    k[j] = coef_of(kc * V + j, pre_bias, mean, invstd, w, b, BWD);
    s[j] = q[j] = t[j] = 0.f;
  }
  const int stride = gridDim.x * rows_per_iter;
  for (int n0 = blockIdx.x * rows_per_iter + r; n0 < R; n0 += kUnroll<BWD> * stride) {
    float fx[kUnroll<BWD>][V], fg[kUnroll<BWD>][BWD ? V : 1];
#pragma unroll
    for (int u = 0; u < kUnroll<BWD>; ++u) {  // all loads in flight before the arithmetic
      const int n = n0 + u * stride;
      if (n < R) {
        Vec<T>::load(x, (int64_t)n * cpr + kc, fx[u]);
        if (BWD) Vec<T>::load(dy, (int64_t)n * cpr + kc, fg[u]);
        if (BWD && MASK) {
          mask_grad<T>(mask, (int64_t)n * cpr + kc, fg[u]);
          Vec<T>::store(gout, (int64_t)n * cpr + kc, fg[u]);  // the masked gradient (exact in T)
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll<BWD>; ++u) {
      if (n0 + u * stride >= R) break;
#pragma unroll
      for (int j = 0; j < V; ++j) accumulate<T, BWD>(fx[u][j], BWD ? fg[u][j] : 0.f, k[j], relu, s[j], q[j], t[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    red[0][threadIdx.x * V + j] = s[j];
    red[1][threadIdx.x * V + j] = q[j];
    if (BWD) red[NQ - 1][threadIdx.x * V + j] = t[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kBnThreads) {
    const int cc = c / V, jc = c % V;
    double a[kQ] = {0.0, 0.0, 0.0};
    for (int rr = 0; rr < rows_per_iter; ++rr)
      for (int m = 0; m < NQ; ++m) a[m] += (double)red[m][(rr * cpr + cc) * V + jc];
    for (int m = 0; m < kQ; ++m) part[((int64_t)blockIdx.x * C + c) * kQ + m] = a[m];
  }
}

// A board convolution's weight-gradient partial sums, added in chunk order (csrc/bb_conv.hip
// conv_wgrad_reduce's arithmetic, bit for bit): dw[co][ci][t] (wl 0) or dw[co][t][ci] (wl 1).
__device__ __forceinline__ void wgrad_reduce_at(const WgradReduceJob& j, int i) {
  const int n = 9 * j.cout * j.cin;
  if (i >= n) return;
  float s = 0.f;
  int c = 0;
  for (; c + 16 <= j.nchunk; c += 16) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = j.part[(size_t)(c + k) * n + i];
#pragma unroll
    for (int k = 0; k < 16; ++k) s += v[k];
  }
  for (; c < j.nchunk; ++c) s += j.part[(size_t)c * n + i];
  const int ci = i % j.cin, co = (i / j.cin) % j.cout, t = i / (j.cin * j.cout);
  j.dw[j.wl ? (co * 9 + t) * j.cin + ci : (co * j.cin + ci) * 9 + t] = s;
}

// Per-channel coefficients of the elementwise passes, packed 8 floats per
// channel so an apply thread loads them as two 16-byte vectors:
//   forward  {pre_bias, mean, invstd * weight, bias, -, -, -, -}
//   backward {pre_bias, mean, invstd * weight, bias, invstd, mean(g), mean(g * xhat), -}
constexpr int kCoef = 8;

// The per-channel sums over the nb block partials part[blk][c][kQ], one wave
// per channel (fixed order), valid in lane 0.
__device__ __forceinline__ bool channel_sums(const double* __restrict__ part, int nb, int C, int& c, double a[kQ]) {
  c = blockIdx.x * (kBnThreads / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= C) return false;
  a[0] = a[1] = a[2] = 0.0;
  int blk = lane;
  // 8 partial rows' loads in flight per lane before their (in-order) adds: the loop is a chain of
  // dependent HBM latencies otherwise (one wave per channel, rows C * kQ doubles apart)
  for (; blk + 7 * 64 < nb; blk += 8 * 64) {
    double v[8][kQ];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int m = 0; m < kQ; ++m) v[j][m] = part[((int64_t)(blk + 64 * j) * C + c) * kQ + m];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int m = 0; m < kQ; ++m) a[m] += v[j][m];
  }
  for (; blk < nb; blk += 64)
    for (int m = 0; m < kQ; ++m) a[m] += part[((int64_t)blk * C + c) * kQ + m];
  for (int m = 0; m < kQ; ++m) a[m] = wave_sum(a[m]);
  return lane == 0;
}

// BB_BN_FIN_CPB: channels per finalisation block -- 4: one wave per channel (round 4), 1: the whole block
// sums one channel (4x the workgroups on the partials' strided rows; each lane a fixed sequence of rows, the
// lanes' sums by the xor tree, the waves' in order: deterministic).
#ifndef BB_BN_FIN_CPB
#define BB_BN_FIN_CPB 1
#endif
constexpr int kFinCpb = BB_BN_FIN_CPB;
static_assert(kFinCpb == 1 || kFinCpb == 4, "BB_BN_FIN_CPB: 1 or 4");

// NQR: the quantities read (the forward's third is 0 and skipped)
template <int NQR>
__device__ __forceinline__ bool channel_sums_block(const double* __restrict__ part, int nb, int C, int& c,
                                                   double a[kQ]) {
  __shared__ double red[kQ][kBnThreads / 64];
  // blocks b, b + 8, ... share an XCD (round-robin dealing, MI355X_MICROARCH.md): give them consecutive
  // channels, so the partial rows' cache lines (5 channels per 128 B) are fetched into one L2, not eight
  c = (C % 8 == 0 && (int)gridDim.x >= C) ? ((int)blockIdx.x % 8) * (C / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
  a[0] = a[1] = a[2] = 0.0;
  int blk = threadIdx.x;
  for (; blk + kBnThreads < nb; blk += 2 * kBnThreads) {  // two rows' loads in flight
    double v[2][NQR];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < NQR; ++m) v[j][m] = part[((int64_t)(blk + kBnThreads * j) * C + c) * kQ + m];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < NQR; ++m) a[m] += v[j][m];
  }
  if (blk < nb)
#pragma unroll
    for (int m = 0; m < NQR; ++m) a[m] += part[((int64_t)blk * C + c) * kQ + m];
  for (int m = 0; m < kQ; ++m) a[m] = wave_sum(a[m]);
  if ((threadIdx.x & 63) == 0)
    for (int m = 0; m < kQ; ++m) red[m][threadIdx.x >> 6] = a[m];
  __syncthreads();
  if (threadIdx.x != 0) return false;
  for (int m = 0; m < kQ; ++m) a[m] = ((red[m][0] + red[m][1]) + red[m][2]) + red[m][3];
  return true;
}

template <int NQR = kQ>
__device__ __forceinline__ bool fin_sums(const double* __restrict__ part, int nb, int C, int& c, double a[kQ]) {
  if (kFinCpb == 1) return channel_sums_block<NQR>(part, nb, C, c, a);
  return channel_sums(part, nb, C, c, a);
}

// Forward finalisation: mean, inverse std of the biased variance (the
// normalisation), running statistics with the unbiased variance
// (nn.BatchNorm2d, momentum = exponential_average_factor), num_batches_tracked
// += 1, coefficients.
__global__ void __launch_bounds__(kBnThreads) bn_finalize_fwd(const double* __restrict__ part, int nb, int C, double M,
                                                              float eps, const float* __restrict__ pre_bias,
                                                              const float* __restrict__ w, const float* __restrict__ b,
                                                              float* __restrict__ save_mean,
                                                              float* __restrict__ save_invstd,
                                                              float* __restrict__ rmean, float* __restrict__ rvar,
                                                              float momentum, int64_t* __restrict__ nbt,
                                                              float* __restrict__ coef) {
  int c;
  double a[kQ];
  if (!fin_sums<2>(part, nb, C, c, a)) return;
  const double m = a[0] / M;  // mean of x (the bias-free input)
  double var = a[1] / M - m * m;
  if (var < 0.0) var = 0.0;
  const float mu = (float)m, is = (float)(1.0 / sqrt(var + (double)eps));
  save_mean[c] = mu;
  save_invstd[c] = is;
  const float mu_u = (float)(m + (pre_bias ? (double)pre_bias[c] : 0.0));  // the mean of u = x + bias
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu_u;
  if (rvar) rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(M > 1.0 ? var * M / (M - 1.0) : var);
  if (nbt && c == 0) nbt[0] += 1;
  float4* o = reinterpret_cast<float4*>(coef + kCoef * c);
  o[0] = make_float4(0.f, mu, is * w[c], b[c]);
}

// Backward finalisation: dweight = sum(g * xhat), dbias = sum(g), the
// convolution bias gradient sum(dx) (dx = sc * (g - mg - xhat * mgx) summed in
// fp64), coefficients.
// With a WgradReduceJob (bb_bn_backward_red): blocks from the finalisation's on add a preceding board convolution's
// weight-gradient partials instead -- two independent small passes in one launch.
__global__ void __launch_bounds__(kBnThreads) bn_finalize_bwd(const double* __restrict__ part, int nb, int C, double M,
                                                              const float* __restrict__ pre_bias,
                                                              const float* __restrict__ w, const float* __restrict__ b,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd, float* __restrict__ dw,
                                                              float* __restrict__ db, float* __restrict__ dpb,
                                                              float* __restrict__ coef, WgradReduceJob job) {
  const int fin_blocks = (C + kFinCpb - 1) / kFinCpb;
  if ((int)blockIdx.x >= fin_blocks) {
    wgrad_reduce_at(job, ((int)blockIdx.x - fin_blocks) * kBnThreads + threadIdx.x);
    return;
  }
  int c;
  double a[kQ];
  if (!fin_sums(part, nb, C, c, a)) return;
  const float invM = (float)(1.0 / M);
  const double sg = a[0], sgx = a[1], sx = a[2];
  const float is = invstd[c], sc = is * w[c];
  const float mg = (float)sg * invM, mgx = (float)sgx * invM;
  if (dw) dw[c] = (float)sgx;
  if (db) db[c] = (float)sg;
  if (dpb) dpb[c] = (float)((double)sc * (sg - M * (double)mg) - (double)sc * (double)mgx * sx);
  float4* o = reinterpret_cast<float4*>(coef + kCoef * c);
  o[0] = make_float4(0.f, mean[c], sc, b[c]);  // mean[c]: the forward's saved mean of x (bias-free)
  o[1] = make_float4(is, mg, mgx, 0.f);
}

// BB_BN_APPLY_UNROLL chunks of a thread's grid-stride sequence loaded before any is computed (1: one at a time).
// Measured on the bf16 update step (round 6, tools/gpu_update_ab2.sh, three interleaved repeats per box): 2 within
// -0.3..0%, 4 +1.7%, 8 +2.5%; BB_BN_APPLY_PT 1 / 2 / 4 / 16 / 32 chunks per thread +23% / +8% / +1% / +1% / +7%.
// The passes' 4.4 TB/s is not a loads-in-flight limit.
#ifndef BB_BN_APPLY_UNROLL
#define BB_BN_APPLY_UNROLL 1
#endif
constexpr int kApplyU = BB_BN_APPLY_UNROLL;

// Channel of element j of 16-byte chunk i: NCHW rows are (n, c) with HW / V
// chunks each (one channel per chunk); NHWC rows are (n, h, w) with C / V
// chunks of V channels each.  The NHWC grid stride is a multiple of C / V, so
// a thread's channels are fixed and their coefficients stay in registers.
// With res (ResidualBlock, network.py:14-30: relu(bn2(conv2(.)) + x)): the BatchNorm
// output is rounded to T as its tensor would be, the residual added in f32 and
// the sum stored (one rounding, as torch's add), then the ReLU.
template <typename T, bool NHWC>
__global__ void __launch_bounds__(kBnThreads) bn_apply_fwd(const void* __restrict__ x, const void* __restrict__ res,
                                                           void* __restrict__ y, int64_t total, int C, int cpr,
                                                           int relu, const float* __restrict__ coef) {
  constexpr int V = Vec<T>::N;
  constexpr int NC = NHWC ? V : 1;
  const float4* cf = reinterpret_cast<const float4*>(coef);
  const int64_t g0 = (int64_t)blockIdx.x * kBnThreads + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBnThreads;
  float4 k[NC];
  if (NHWC) {
    const int c0 = (int)(g0 % cpr) * V;
#pragma unroll
    for (int j = 0; j < NC; ++j) k[j] = cf[(c0 + j) * (kCoef / 4)];
  }
  for (int64_t i0 = g0; i0 < total; i0 += kApplyU * stride) {
    float f[kApplyU][V], fr[kApplyU][V];
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {  // every load in flight before the arithmetic
      const int64_t i = i0 + u * stride;
      if (i < total) {
        Vec<T>::load(x, i, f[u]);
        if (res) Vec<T>::load(res, i, fr[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= total) break;
      if (!NHWC) k[0] = cf[(int)((i / cpr) % C) * (kCoef / 4)];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float4& q = k[NHWC ? j : 0];  // {pb, mu, sc, sh}
        float v = (f[u][j] + q.x - q.y) * q.z + q.w;
        if (res) v = Vec<T>::round(v) + fr[u][j];
        f[u][j] = relu ? fmaxf(v, 0.f) : v;
      }
      Vec<T>::store(y, i, f[u]);
    }
  }
}

template <typename T, bool NHWC>
__global__ void __launch_bounds__(kBnThreads) bn_apply_bwd(const void* __restrict__ x, const void* __restrict__ dy,
                                                           void* __restrict__ dx, int64_t total, int C, int cpr,
                                                           int relu, const float* __restrict__ coef) {
  constexpr int V = Vec<T>::N;
  constexpr int NC = NHWC ? V : 1;
  const float4* cf = reinterpret_cast<const float4*>(coef);
  const int64_t g0 = (int64_t)blockIdx.x * kBnThreads + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBnThreads;
  float4 k0[NC], k1[NC];
  if (NHWC) {
    const int c0 = (int)(g0 % cpr) * V;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      k0[j] = cf[(c0 + j) * (kCoef / 4)];
      k1[j] = cf[(c0 + j) * (kCoef / 4) + 1];
    }
  }
  for (int64_t i0 = g0; i0 < total; i0 += kApplyU * stride) {
    float fx[kApplyU][V], fg[kApplyU][V];
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {  // every load in flight before the arithmetic
      const int64_t i = i0 + u * stride;
      if (i < total) {
        Vec<T>::load(x, i, fx[u]);
        Vec<T>::load(dy, i, fg[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= total) break;
      if (!NHWC) {
        const int c = (int)((i / cpr) % C);
        k0[0] = cf[c * (kCoef / 4)];
        k1[0] = cf[c * (kCoef / 4) + 1];
      }
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float4& a = k0[NHWC ? j : 0];  // {pb, mu, sc, sh}
        const float4& q = k1[NHWC ? j : 0];  // {is, mg, mgx, -}
        const float u_ = fx[u][j] + a.x;
        const float g = (relu && (u_ - a.y) * a.z + a.w <= 0.f) ? 0.f : fg[u][j];  // the forward's exact ops
        const float xh = (u_ - a.y) * q.x;
        fx[u][j] = a.z * (g - q.y - xh * q.z);
      }
      Vec<T>::store(dx, i, fx[u]);
    }
  }
}

// ---------------------------------------------------------------- launch plan
#ifndef BB_BN_RBLOCKS
#define BB_BN_RBLOCKS 512  // NHWC reduction blocks at most
#endif
struct Plan {
  int V, cpr, nb;  // vector width, 16-byte chunks per contiguous row, reduction blocks
  dim3 rgrid;      // reduction grid
  int64_t chunks;
};

Plan plan_for(int esz, int nhwc, int N, int C, int HW) {
  Plan p;
  p.V = 16 / esz;
  p.chunks = (int64_t)N * C * HW / p.V;
  if (nhwc) {
    p.cpr = C / p.V;
    const int rows_per_iter = kBnThreads / p.cpr;
    const int64_t R = (int64_t)N * HW;
    int64_t g = (R + (int64_t)rows_per_iter * 8 - 1) / ((int64_t)rows_per_iter * 8);
    p.nb = (int)(g < 1 ? 1 : (g > BB_BN_RBLOCKS ? BB_BN_RBLOCKS : g));  // >= 8 rows per thread
    p.rgrid = dim3(p.nb);
  } else {
    p.cpr = HW / p.V;
    const int rows_per_iter = kBnThreads / p.cpr;
    int s = (1024 + C - 1) / C;  // enough blocks to fill the chip, >= 4 rows per thread-row
    const int max_s = (N + rows_per_iter * 4 - 1) / (rows_per_iter * 4);
    if (s > max_s) s = max_s;
    if (s < 1) s = 1;
    if (s > 65535) s = 65535;
    p.nb = s;
    p.rgrid = dim3(C, s);
  }
  return p;
}

// Elementwise grids: NHWC threads keep V channels' coefficients in registers,
// so they stride over >= 8 chunks each to amortise loading them.
#ifndef BB_BN_APPLY_PT
#define BB_BN_APPLY_PT 8
#endif
int grid_for_elems(int64_t chunks, int nhwc) {
  const int64_t per_thread = nhwc ? BB_BN_APPLY_PT : 1;
  int64_t g = (chunks + kBnThreads * per_thread - 1) / (kBnThreads * per_thread);
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

template <typename T, bool BWD>
void launch_reduce(const Plan& p, int nhwc, const void* x, const void* dy, int N, int C, int HW, const float* pb,
                   const float* w, const float* b, const float* mean, const float* invstd, int relu, double* part,
                   hipStream_t s, const void* mask = nullptr, void* gout = nullptr) {
  if (nhwc) {
    if (BWD && mask)
      hipLaunchKernelGGL((bn_reduce_nhwc<T, BWD, true>), p.rgrid, dim3(kBnThreads), 0, s, x, dy, N * HW, C, pb, w, b,
                         mean, invstd, relu, mask, gout, part);
    else
      hipLaunchKernelGGL((bn_reduce_nhwc<T, BWD>), p.rgrid, dim3(kBnThreads), 0, s, x, dy, N * HW, C, pb, w, b, mean,
                         invstd, relu, nullptr, nullptr, part);
  } else {
    if (BWD && mask)
      hipLaunchKernelGGL((bn_reduce_nchw<T, BWD, true>), p.rgrid, dim3(kBnThreads), 0, s, x, dy, N, C, HW, pb, w, b,
                         mean, invstd, relu, mask, gout, part);
    else
      hipLaunchKernelGGL((bn_reduce_nchw<T, BWD>), p.rgrid, dim3(kBnThreads), 0, s, x, dy, N, C, HW, pb, w, b, mean,
                         invstd, relu, nullptr, nullptr, part);
  }
}

// Workspace (16-byte aligned): coefficients [C][kCoef] floats (float4 loads),
// then the block partials [nb][C][kQ] doubles.
struct Ws {
  float* coef;
  double* part;
};
Ws split_ws(double* ws, int C) {
  Ws w;
  w.coef = reinterpret_cast<float*>(ws);
  w.part = ws + kCoef / 2 * C;
  return w;
}

template <typename T>
hipError_t bn_forward_t(const void* x, const void* res, int nhwc, int N, int C, int HW, const float* pb, const float* w,
                        const float* b, float eps, int relu, double* ws, float* save_mean, float* save_invstd,
                        float* rmean, float* rvar, float momentum, int64_t* nbt, void* y, hipStream_t s,
                        const double* ext_part, int ext_nb) {
  const Plan p = plan_for(sizeof(T), nhwc, N, C, HW);
  const Ws k = split_ws(ws, C);
  // ext_part: the block partials a preceding board convolution's store pass produced (conv_fwd_kernel stats)
  const double* part = ext_part ? ext_part : k.part;
  const int nbp = ext_part ? ext_nb : p.nb;
  if (!ext_part) launch_reduce<T, false>(p, nhwc, x, nullptr, N, C, HW, pb, w, b, nullptr, nullptr, 0, k.part, s);
  hipLaunchKernelGGL(bn_finalize_fwd, dim3((C + kFinCpb - 1) / kFinCpb), dim3(kBnThreads), 0, s, part, nbp, C, (double)N * HW, eps,
                     pb, w, b, save_mean, save_invstd, rmean, rvar, momentum, nbt, k.coef);
  const dim3 ge(grid_for_elems(p.chunks, nhwc));
  if (nhwc)
    hipLaunchKernelGGL((bn_apply_fwd<T, true>), ge, dim3(kBnThreads), 0, s, x, res, y, p.chunks, C, p.cpr, relu,
                       k.coef);
  else
    hipLaunchKernelGGL((bn_apply_fwd<T, false>), ge, dim3(kBnThreads), 0, s, x, res, y, p.chunks, C, p.cpr, relu,
                       k.coef);
  return hipGetLastError();
}

template <typename T>
hipError_t bn_backward_t(const void* x, const void* dy, int nhwc, int N, int C, int HW, const float* pb,
                         const float* w, const float* b, const float* mean, const float* invstd, int relu, double* ws,
                         void* dx, float* dw, float* db, float* dpb, hipStream_t s, const void* mask, void* gout,
                         const WgradReduceJob* job, const double* ext_part, int ext_nb) {
  const Plan p = plan_for(sizeof(T), nhwc, N, C, HW);
  const Ws k = split_ws(ws, C);
  // with a mask (the ResidualBlock tail): the reduction writes the masked gradient g to gout, and the
  // elementwise pass reads g as its dy (no mask there).  ext_part (no mask): the reduction's partials came
  // from the board convolution that produced dy (conv_fwd_kernel's backward statistics)
  if (ext_part && mask) return hipErrorInvalidValue;
  const double* part = ext_part ? ext_part : k.part;
  const int nbp = ext_part ? ext_nb : p.nb;
  if (!ext_part) launch_reduce<T, true>(p, nhwc, x, dy, N, C, HW, pb, w, b, mean, invstd, relu, k.part, s, mask, gout);
  if (mask) dy = gout;
  WgradReduceJob jb{};
  int red_blocks = 0;
  if (job) {
    jb = *job;
    red_blocks = (9 * jb.cout * jb.cin + kBnThreads - 1) / kBnThreads;
  }
  hipLaunchKernelGGL(bn_finalize_bwd, dim3((C + kFinCpb - 1) / kFinCpb + red_blocks), dim3(kBnThreads), 0, s, part, nbp, C,
                     (double)N * HW, pb, w, b, mean, invstd, dw, db, dpb, k.coef, jb);
  const dim3 ge(grid_for_elems(p.chunks, nhwc));
  if (nhwc)
    hipLaunchKernelGGL((bn_apply_bwd<T, true>), ge, dim3(kBnThreads), 0, s, x, dy, dx, p.chunks, C, p.cpr, relu,
                       k.coef);
  else
    hipLaunchKernelGGL((bn_apply_bwd<T, false>), ge, dim3(kBnThreads), 0, s, x, dy, dx, p.chunks, C, p.cpr, relu,
                       k.coef);
  return hipGetLastError();
}

}  // namespace

int64_t bn_workspace_bytes(int dtype, int nhwc, int N, int C, int HW) {
  const Plan p = plan_for(dtype == 1 ? 2 : 4, nhwc, N, C, HW);
  return (int64_t)sizeof(double) * C * (kCoef / 2 + kQ * (int64_t)p.nb);
}

hipError_t launch_bn_forward(const void* x, const void* res, int dtype, int nhwc, int N, int C, int HW,
                             const float* pb, const float* w, const float* b, float eps, int relu, double* ws,
                             float* save_mean, float* save_invstd, float* rmean, float* rvar, float momentum,
                             int64_t* nbt, void* y, hipStream_t s, const double* ext_part, int ext_nb) {
  if (dtype == 1)
    return bn_forward_t<__hip_bfloat16>(x, res, nhwc, N, C, HW, pb, w, b, eps, relu, ws, save_mean, save_invstd, rmean,
                                        rvar, momentum, nbt, y, s, ext_part, ext_nb);
  return bn_forward_t<float>(x, res, nhwc, N, C, HW, pb, w, b, eps, relu, ws, save_mean, save_invstd, rmean, rvar, momentum,
                             nbt, y, s, ext_part, ext_nb);
}

hipError_t launch_bn_backward(const void* x, const void* dy, int dtype, int nhwc, int N, int C, int HW,
                              const float* pb, const float* w, const float* b, const float* mean, const float* invstd,
                              int relu, double* ws, void* dx, float* dw, float* db, float* dpb, hipStream_t s,
                              const void* mask, void* gout, const WgradReduceJob* job, const double* ext_part,
                              int ext_nb) {
  if (dtype == 1)
    return bn_backward_t<__hip_bfloat16>(x, dy, nhwc, N, C, HW, pb, w, b, mean, invstd, relu, ws, dx, dw, db, dpb, s,
                                         mask, gout, job, ext_part, ext_nb);
  return bn_backward_t<float>(x, dy, nhwc, N, C, HW, pb, w, b, mean, invstd, relu, ws, dx, dw, db, dpb, s, mask, gout,
                              job, ext_part, ext_nb);
}

}  // namespace bb

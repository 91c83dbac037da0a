// bb_nn.hip -- training-mode BatchNorm2d (+ fused ReLU) for the policy/value
// CNN (gfx950).
//
// BlockBlastNetwork's conv stack is conv -> BatchNorm2d -> ReLU on 8x8 boards
// (network.py:75-117, ResidualBlock network.py:14-30).  With batch statistics
// over N x 64 positions per channel, MIOpen's spatial BatchNorm took 80 us
// forward and 200 us backward per layer at N = 2048 (bf16), about a third of a
// PPO minibatch step; these kernels are HBM passes:
//   forward : per-channel sum / sum of squares (fp32 lanes, fp64 block and
//             global accumulation) -> normalise, scale, shift, optional ReLU,
//             saved mean / inverse std, running-stat update (momentum,
//             unbiased variance), exactly nn.BatchNorm2d's training forward;
//   backward: per-channel sum(g) and sum(g * xhat) with g = dy masked by the
//             ReLU (recomputed from x) -> dx, dweight, dbias.
// Layout NCHW contiguous, f32 or bf16 activations, f32 parameters and stats.
// Loads and stores are 16-byte vectors along HW (HW * element size % 16 == 0).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <math.h>

#include "bb_env_internal.h"

namespace bb {

namespace {

constexpr int kBnThreads = 256;

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
    if ((u & 0x7FFFFFFFu) > 0x7F800000u) return (u >> 16) | 0x40u;
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
  }
  __device__ static void store(void* p, int64_t i, const float* f) {
    uint4 v;
    v.x = rne(f[0]) | (rne(f[1]) << 16);
    v.y = rne(f[2]) | (rne(f[3]) << 16);
    v.z = rne(f[4]) | (rne(f[5]) << 16);
    v.w = rne(f[6]) | (rne(f[7]) << 16);
    reinterpret_cast<uint4*>(p)[i] = v;
  }
};

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int k = 0; k < kBnThreads / 64; ++k) s += red[k];
  return s;  // valid in thread 0
}

// Per-channel finalisation (one thread per channel): mean, inverse std of the
// biased variance (the normalisation), running statistics with the unbiased
// variance (nn.BatchNorm2d, momentum = exponential_average_factor).
__global__ void bn_finalize_fwd(int C, double M, const double* __restrict__ ws, float eps,
                                float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                float* __restrict__ rmean, float* __restrict__ rvar, float momentum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double m = ws[2 * c] / M;
  double var = ws[2 * c + 1] / M - m * m;
  if (var < 0.0) var = 0.0;
  save_mean[c] = (float)m;
  save_invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)m;
  if (rvar) rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(M > 1.0 ? var * M / (M - 1.0) : var);
}

// Block (c, s): channel c, images s, s + S, ...  ws[2c] += sum x, ws[2c+1] += sum x^2.
template <typename T>
__global__ void __launch_bounds__(kBnThreads) bn_reduce_fwd(const void* __restrict__ x, int N, int C, int HW,
                                                            double* __restrict__ ws) {
  __shared__ double red[2][kBnThreads / 64];
  constexpr int V = Vec<T>::N;
  const int c = blockIdx.x;
  const int cpr = HW / V;  // 16-byte chunks per (n, c) row
  const int rows_per_iter = kBnThreads / cpr;
  const int r = threadIdx.x / cpr, k = threadIdx.x % cpr;
  float s = 0.f, q = 0.f;
  if (r < rows_per_iter) {
    for (int n = blockIdx.y * rows_per_iter + r; n < N; n += gridDim.y * rows_per_iter) {
      float f[V];
      Vec<T>::load(x, ((int64_t)n * C + c) * cpr + k, f);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        s += f[j];
        q += f[j] * f[j];
      }
    }
  }
  const double bs = block_sum((double)s, red[0]);
  const double bq = block_sum((double)q, red[1]);
  if (threadIdx.x == 0) {
    atomicAdd(&ws[2 * c], bs);
    atomicAdd(&ws[2 * c + 1], bq);
  }
}

template <typename T>
__global__ void __launch_bounds__(kBnThreads) bn_apply_fwd(const void* __restrict__ x, void* __restrict__ y, int N,
                                                           int C, int HW, const float* __restrict__ w,
                                                           const float* __restrict__ b, int relu,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd) {
  constexpr int V = Vec<T>::N;
  const int cpr = HW / V;
  const int64_t total = (int64_t)N * C * cpr;
  for (int64_t i = (int64_t)blockIdx.x * kBnThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kBnThreads) {
    const int c = (int)((i / cpr) % C);
    const float mu = mean[c], sc = invstd[c] * w[c], sh = b[c];
    float f[V];
    Vec<T>::load(x, i, f);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float v = (f[j] - mu) * sc + sh;
      f[j] = relu ? fmaxf(v, 0.f) : v;
    }
    Vec<T>::store(y, i, f);
  }
}

// ws[2c] += sum g, ws[2c+1] += sum g * xhat, g = dy (masked where the fused ReLU clipped).
template <typename T>
__global__ void __launch_bounds__(kBnThreads) bn_reduce_bwd(const void* __restrict__ x, const void* __restrict__ dy,
                                                            int N, int C, int HW, const float* __restrict__ w,
                                                            const float* __restrict__ b,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, int relu,
                                                            double* __restrict__ ws) {
  __shared__ double red[2][kBnThreads / 64];
  constexpr int V = Vec<T>::N;
  const int c = blockIdx.x;
  const int cpr = HW / V;
  const int rows_per_iter = kBnThreads / cpr;
  const int r = threadIdx.x / cpr, k = threadIdx.x % cpr;
  const float mu = mean[c], is = invstd[c], sc = is * w[c], sh = b[c];
  float s = 0.f, q = 0.f;
  if (r < rows_per_iter) {
    for (int n = blockIdx.y * rows_per_iter + r; n < N; n += gridDim.y * rows_per_iter) {
      const int64_t i = ((int64_t)n * C + c) * cpr + k;
      float fx[V], fg[V];
      Vec<T>::load(x, i, fx);
      Vec<T>::load(dy, i, fg);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float g = (relu && (fx[j] - mu) * sc + sh <= 0.f) ? 0.f : fg[j];  // forward's exact ops
        s += g;
        q += g * (fx[j] - mu) * is;
      }
    }
  }
  const double bs = block_sum((double)s, red[0]);
  const double bq = block_sum((double)q, red[1]);
  if (threadIdx.x == 0) {
    atomicAdd(&ws[2 * c], bs);
    atomicAdd(&ws[2 * c + 1], bq);
  }
}

template <typename T>
__global__ void __launch_bounds__(kBnThreads) bn_apply_bwd(const void* __restrict__ x, const void* __restrict__ dy,
                                                           void* __restrict__ dx, int N, int C, int HW,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd, int relu,
                                                           const double* __restrict__ ws, float* __restrict__ dw,
                                                           float* __restrict__ db) {
  constexpr int V = Vec<T>::N;
  const int cpr = HW / V;
  const int64_t total = (int64_t)N * C * cpr;
  const float invM = (float)(1.0 / ((double)N * HW));
  const int64_t g0 = (int64_t)blockIdx.x * kBnThreads + threadIdx.x;
  if (g0 < C) {
    if (dw) dw[g0] = (float)ws[2 * g0 + 1];
    if (db) db[g0] = (float)ws[2 * g0];
  }
  for (int64_t i = g0; i < total; i += (int64_t)gridDim.x * kBnThreads) {
    const int c = (int)((i / cpr) % C);
    const float mu = mean[c], is = invstd[c], sc = is * w[c], sh = b[c];
    const float mg = (float)ws[2 * c] * invM, mgx = (float)ws[2 * c + 1] * invM;
    float fx[V], fg[V];
    Vec<T>::load(x, i, fx);
    Vec<T>::load(dy, i, fg);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float g = (relu && (fx[j] - mu) * sc + sh <= 0.f) ? 0.f : fg[j];
      const float xh = (fx[j] - mu) * is;
      fx[j] = sc * (g - mg - xh * mgx);
    }
    Vec<T>::store(dx, i, fx);
  }
}

int split_for(int N, int C, int HW, int V) {
  // enough blocks per channel to fill the chip (>= 4 per CU overall), >= 4 rows per thread-row
  const int rows_per_iter = kBnThreads / (HW / V);
  int s = (1024 + C - 1) / C;
  const int max_s = (N + rows_per_iter * 4 - 1) / (rows_per_iter * 4);
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  if (s > 65535) s = 65535;
  return s;
}

int grid_for_elems(int64_t chunks) {
  int64_t g = (chunks + kBnThreads - 1) / kBnThreads;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

template <typename T>
hipError_t bn_forward_t(const void* x, int N, int C, int HW, const float* w, const float* b, float eps, int relu,
                        double* ws, float* save_mean, float* save_invstd, float* rmean, float* rvar,
                        float momentum, void* y, hipStream_t s) {
  constexpr int V = Vec<T>::N;
  hipError_t st = hipMemsetAsync(ws, 0, sizeof(double) * 2 * C, s);
  if (st != hipSuccess) return st;
  hipLaunchKernelGGL(bn_reduce_fwd<T>, dim3(C, split_for(N, C, HW, V)), dim3(kBnThreads), 0, s, x, N, C, HW, ws);
  hipLaunchKernelGGL(bn_finalize_fwd, dim3((C + 255) / 256), dim3(256), 0, s, C, (double)N * HW, ws, eps, save_mean,
                     save_invstd, rmean, rvar, momentum);
  hipLaunchKernelGGL(bn_apply_fwd<T>, dim3(grid_for_elems((int64_t)N * C * (HW / V))), dim3(kBnThreads), 0, s, x, y,
                     N, C, HW, w, b, relu, save_mean, save_invstd);
  return hipGetLastError();
}

template <typename T>
hipError_t bn_backward_t(const void* x, const void* dy, int N, int C, int HW, const float* w, const float* b,
                         const float* mean, const float* invstd, int relu, double* ws, void* dx, float* dw, float* db,
                         hipStream_t s) {
  constexpr int V = Vec<T>::N;
  hipError_t st = hipMemsetAsync(ws, 0, sizeof(double) * 2 * C, s);
  if (st != hipSuccess) return st;
  hipLaunchKernelGGL(bn_reduce_bwd<T>, dim3(C, split_for(N, C, HW, V)), dim3(kBnThreads), 0, s, x, dy, N, C, HW, w,
                     b, mean, invstd, relu, ws);
  const int64_t chunks = (int64_t)N * C * (HW / V);
  hipLaunchKernelGGL(bn_apply_bwd<T>, dim3(grid_for_elems(chunks > C ? chunks : C)), dim3(kBnThreads), 0, s, x, dy,
                     dx, N, C, HW, w, b, mean, invstd, relu, ws, dw, db);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_bn_forward(const void* x, int dtype, int N, int C, int HW, const float* w, const float* b, float eps,
                             int relu, double* ws, float* save_mean, float* save_invstd, float* rmean, float* rvar,
                             float momentum, void* y, hipStream_t s) {
  if (dtype == 1)
    return bn_forward_t<__hip_bfloat16>(x, N, C, HW, w, b, eps, relu, ws, save_mean, save_invstd, rmean, rvar,
                                        momentum, y, s);
  return bn_forward_t<float>(x, N, C, HW, w, b, eps, relu, ws, save_mean, save_invstd, rmean, rvar, momentum, y, s);
}

hipError_t launch_bn_backward(const void* x, const void* dy, int dtype, int N, int C, int HW, const float* w,
                              const float* b, const float* mean, const float* invstd, int relu, double* ws, void* dx,
                              float* dw, float* db, hipStream_t s) {
  if (dtype == 1)
    return bn_backward_t<__hip_bfloat16>(x, dy, N, C, HW, w, b, mean, invstd, relu, ws, dx, dw, db, s);
  return bn_backward_t<float>(x, dy, N, C, HW, w, b, mean, invstd, relu, ws, dx, dw, db, s);
}

}  // namespace bb

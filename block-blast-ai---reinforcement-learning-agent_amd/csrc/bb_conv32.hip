// bb_conv32.hip -- the CNN's 3x3 / pad-1 convolutions on 8x8 boards and its long-K Linear layer in fp32
// (gfx950), accumulated so that the result is as close to the exact sum as one fp32 rounding allows.
//
// The policy's fp32 forward (network.py:75-117, ResidualBlock network.py:14-30) runs in training mode in the
// rollout (scripts/train.py:122 keeps agent.train(): batch-statistics BatchNorm after every convolution).
// MIOpen's fp32 128-channel convolutions (K = 9 x 128 = 1,152 products per output) accumulate in one long
// order, and the batch-statistics BatchNorms amplify that rounding: the logits ended 1.28e-5 from the fp64
// truth, over north_star's 1e-5.  Here every output is a sum of short fp32 chains: each
// 16-channel block of one tap is one v_mfma_f32_16x16x4_f32 chain of 16 products (exact fp32, bit-for-bit an
// fmaf chain, MI355X_MICROARCH.md), and the blocks are added in fp64 (72 blocks at 128 channels), rounded to
// fp32 once at the end.  The error is then ~0.5 ulp of the result plus a 16-term chain's, against a
// 1,152-term chain's.
//
//   y[b,p,co] = sum_{t,ci} x[b,p+d_t,ci] * w[co,ci,t],   d_t = (t/3 - 1, t%3 - 1), zero outside the board
//   dx[b,q,ci] = the same kernel over dy with w'[t'][ci][co] = w[co][ci][8 - t']
//
// Layouts: x, y, dy, dx f32 NHWC (channels_last), [nb][64][C]; weight images f32 [9][COUT][CIN] (forward) and
// [9][CIN][COUT] tap-reversed (data gradient), written by conv32_prep_kernel from nn.Conv2d's [COUT][CIN][3][3]
// (w_layout 0) or a channels_last parameter [COUT][3][3][CIN] (w_layout 1).
//
// Workgroup: 8 waves, 2 boards (128 pixel rows) x all COUT.  Waves: COUT 128 -> 2 (co) x 4 (px) waves of 64 co x
// 32 px; COUT 64 -> 1 x 8 waves of 64 co x 16 px.  The input tile (2 boards, plus 16 zero rows for the taps
// that leave the board) is copied to LDS once (global -> LDS direct); the weights stream through a 2-slot LDS
// ring in stages of one tap x 32 input channels.  MFMA operands: lane l of a 16x16x4 step holds
// A[co0 + (l & 15)][k] and B[k][px0 + (l & 15)] for k = 4 (l >> 4) + s of a 16-channel block, s = 0..3 the
// step: one ds_read_b128 per operand and block (the k order inside a block is a permutation of the channels,
// the same for A and B).  LDS rows are XOR-swizzled by 16-byte chunk (input: chunk ^ (row & 15); weights:
// chunk ^ ((co >> 1) & 7)) so the 16 lanes of each ds_read_b128 group hit 16 different bank quads; a zero row
// keeps the key of the row it replaces.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bb_env_internal.h"

namespace bb {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kC32Threads = 512;
constexpr int kC32Boards = 2;
constexpr int kC32Rows = kC32Boards * 64;
constexpr int kC32Zero = 16;
#ifndef BB_CONV32_SCI
// input channels per weight stage of the 128-input-channel layers (32 or 64): 64 measured 103.9 vs 99.0 TFLOP/s on
// conv 128 -> 128 at 65,536 boards (tools/bench_conv32.py, profiles/r05/conv32/)
#define BB_CONV32_SCI 64
#endif
#ifndef BB_CONV32_RING
#define BB_CONV32_RING 2  // weight-stage LDS ring slots (stages copied RING - 1 ahead); 3: 103.3 TFLOP/s at SCI 32
#endif
#ifndef BB_CONV32_BLOCK
#define BB_CONV32_BLOCK 16  // channels per fp32 MFMA chain before the fp64 add (16 or 32)
#endif

__device__ __forceinline__ void c32_glds16(const void* g, uint8_t* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// The same copy from inline asm: the compiler does not track it, so it inserts no vmcnt(0) before the LDS reads of
// the current stage while later stages' copies are in flight; counted waits (C32_WAIT_VM) cover it.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved; nothing else in these kernels keeps it live
__device__ __forceinline__ void c32_glds16_async(const void* g, uint8_t* lds_base) {
  const uint32_t l = (uint32_t)(size_t)((__attribute__((address_space(3))) uint8_t*)lds_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
}
#pragma clang diagnostic pop
// s_waitcnt with vmcnt = n and lgkmcnt = 0 (expcnt not waited)
#define C32_WAIT_VM_LGKM0(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (7 << 4) | (((n) >> 4) << 14))

__global__ void __launch_bounds__(256) conv32_prep_kernel(const float* __restrict__ w, int cout, int cin, int wl,
                                                          float* __restrict__ wf, float* __restrict__ wd) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= cout * cin * 9) return;
  const int co = i / (9 * cin);
  const int t = wl ? (i / cin) % 9 : i % 9;
  const int ci = wl ? i % cin : (i / 9) % cin;
  const float v = w[i];
  if (wf) wf[(t * cout + co) * cin + ci] = v;
  if (wd) wd[((8 - t) * cin + ci) * cout + co] = v;
}

template <int CIN>
constexpr int c32_sci() { return CIN == 128 ? BB_CONV32_SCI : 32; }
template <int SCI>
__device__ __forceinline__ int c32_wkey(int co) {  // weight rows of 8 chunks (two per bank line) or 16 (one)
  return SCI == 64 ? (co & 15) : ((co >> 1) & 7);
}

template <int CIN, int COUT>
__global__ void __launch_bounds__(kC32Threads) conv32_fwd_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ w, float* __restrict__ y,
                                                                 int nb) {
  constexpr int RB = CIN * 4;                       // bytes per pixel row
  constexpr int NCH = CIN / 4;                      // 16-byte chunks per pixel row (16 or 32)
  constexpr int XBYTES = (kC32Rows + kC32Zero) * RB;
  constexpr int kC32Sci = c32_sci<CIN>();           // input channels per weight stage
  constexpr int kC32Ring = BB_CONV32_RING;
  constexpr int NCB = CIN / kC32Sci;                // weight stages per tap
  constexpr int NS = 9 * NCB;                       // stages
  constexpr int WROW = kC32Sci * 4;                 // 128- or 256-byte weight rows
  constexpr int WCH = kC32Sci / 4;                  // 16-byte chunks per weight row
  constexpr int WBYTES = COUT * WROW;
  constexpr int NW = kC32Threads / 64;
  constexpr int GPW = WBYTES / 1024 / NW;           // 1-KB weight copies per wave per stage
  constexpr int WN = COUT / 64;                     // waves along co
  constexpr int WM = NW / WN;                       // waves along px
  constexpr int TN = 4;                             // 16-co tiles per wave
  constexpr int TM = kC32Rows / WM / 16;            // 16-px tiles per wave
  constexpr int KB = kC32Sci / 16;                  // 16-channel blocks per stage
  constexpr int FL = BB_CONV32_BLOCK / 16;          // blocks per fp64 add
  static_assert(NCH >= 16 && GPW >= 1 && TM >= 1, "shape");
  __shared__ __attribute__((aligned(16))) uint8_t sm[XBYTES + kC32Ring * WBYTES];
  uint8_t* const xs = sm;

  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int b0 = blockIdx.x * kC32Boards;
  const int r16 = lane & 15, g = lane >> 4;

  // input tile: physical chunk e = 64 k + lane holds row e / NCH, logical chunk (e % NCH) ^ (row & 15)
  for (int k = wid; k < kC32Rows * NCH / 64; k += NW) {
    const int e = k * 64 + lane, r = e / NCH, lc = (e % NCH) ^ (r & 15);
    const int b = min(b0 + (r >> 6), nb - 1);  // boards past the batch read the last one (never stored)
    c32_glds16_async(x + (size_t(b) * 64 + (r & 63)) * CIN + lc * 4, xs + k * 1024);
  }
  auto stage_w = [&](int st) {  // stage st: tap st / NCB, channels SCI (st % NCB) ... -> slot st % RING
    uint8_t* wb = sm + XBYTES + (st % kC32Ring) * WBYTES;
    const float* ws = w + (size_t)(st / NCB) * COUT * CIN + (st % NCB) * kC32Sci;
#pragma unroll
    for (int kq = 0; kq < GPW; ++kq) {
      const int k = wid + kq * NW;
      const int e = k * 64 + lane, r = e / WCH, lc = (e % WCH) ^ c32_wkey<kC32Sci>(r);
      c32_glds16_async(ws + r * CIN + lc * 4, wb + k * 1024);
    }
  };
#pragma unroll
  for (int st = 0; st < kC32Ring - 1; ++st) stage_w(st);
  for (int i = tid; i < kC32Zero * NCH; i += kC32Threads)
    *reinterpret_cast<uint4*>(xs + kC32Rows * RB + i * 16) = make_uint4(0, 0, 0, 0);
  C32_WAIT_VM_LGKM0((kC32Ring - 2) * GPW);  // the input tile and stage 0 (this wave's copies)
  __syncthreads();

  const int co0 = (wid % WN) * 64;
  const int px0 = (wid / WN) * (kC32Rows / WM);
  int abase[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int co = co0 + 16 * j + r16;
    abase[j] = co * WROW;
  }
  double dacc[TN][TM][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) dacc[j][i][e] = 0.0;
  int brow[TM];

  for (int st = 0; st < NS; ++st) {
    // its slot was last read in stage st - 1, before that stage's barrier
    if (st + kC32Ring - 1 < NS) stage_w(st + kC32Ring - 1);
    const int cb = st % NCB;
    if (cb == 0) {
      const int t = st / NCB, dy = t / 3 - 1, dx = t % 3 - 1;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int px = px0 + 16 * i + r16;
        const int p = px & 63, yy = (p >> 3) + dy, xc = (p & 7) + dx;
        brow[i] = ((unsigned)yy < 8u && (unsigned)xc < 8u) ? (px & ~63) + yy * 8 + xc
                                                           : kC32Rows + ((px + 8 * dy + dx) & 15);
      }
    }
    const uint8_t* wb = sm + XBYTES + (st % kC32Ring) * WBYTES;
    f32x4 af[KB][TN], bf[KB][TM];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int co = co0 + 16 * j + r16;
        af[kb][j] = *reinterpret_cast<const f32x4*>(wb + abase[j] + (((4 * kb + g) ^ c32_wkey<kC32Sci>(co)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = brow[i];
        bf[kb][i] = *reinterpret_cast<const f32x4*>(xs + row * RB + (((cb * WCH + 4 * kb + g) ^ (row & 15)) << 4));
      }
    }
#pragma unroll
    for (int kb0 = 0; kb0 < KB; kb0 += FL) {
      f32x4 acc[TN][TM];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = kb0; kb < kb0 + FL; ++kb)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[kb][j][s], bf[kb][i][s], acc[j][i], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) dacc[j][i][e] += (double)acc[j][i][e];
    }
    // the next stage's weights (this wave's copies; the barrier covers the rest): every copy but the stages issued
    // after it
    {
      const int after = min(NS, st + kC32Ring) - (st + 2);
      if (after >= 1 && kC32Ring >= 3) C32_WAIT_VM_LGKM0(GPW);
      else C32_WAIT_VM_LGKM0(0);
    }
    __syncthreads();
  }
  // D[co0 + 16 j + 4 g + e][px0 + 16 i + r16]: 4 consecutive channels of one pixel = one 16-byte store
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int px = px0 + 16 * i + r16;
    if (b0 + (px >> 6) >= nb) continue;
    float* yo = y + (size_t(b0) * 64 + px) * COUT + co0 + 4 * g;
#pragma unroll
    for (int j = 0; j < TN; ++j)
      *reinterpret_cast<f32x4*>(yo + 16 * j) = f32x4{(float)dacc[j][i][0], (float)dacc[j][i][1],
                                                     (float)dacc[j][i][2], (float)dacc[j][i][3]};
  }
}

// ---------------------------------------------------------------------------
// y[m][n] = sum_k x[m][k] w[n][k] + bias[n] in fp32 with the same accumulation (nn.Linear's forward,
// network.py:89-117: the first fc_encoder layer has K = 8,192, where hipBLASLt's fp32 order cost more than
// north_star's 1e-5 at the logits after the batch-statistics BatchNorms, tools/diag_net_fp32.py).  Every
// output is the fp64 sum of 16-product fp32 MFMA chains plus the bias, rounded once.  x [M][K], w [N][K]
// row-major (K contiguous), y [M][N]; N % 128 == 0, K % 32 == 0.  Workgroup: BM (64 or 128) rows x 128 columns,
// waves BM / 32 (m) x 2 (n) of 32 x 64; stages of 32 k through a 2-slot LDS ring (direct global -> LDS copies),
// rows of 128 bytes XOR-swizzled by chunk ^ ((row >> 1) & 7).
// ---------------------------------------------------------------------------
// Two tile heights: 128 rows (8 waves; each W stage serves twice the rows, registers capped for two
// workgroups per CU, 12 VGPRs spilled) when the grid still has >= BB_LINEAR32_BIG workgroups, else 64 rows (4 waves) so that
// small batches spread over more CUs.  Microbench (tools/bench_conv32.py, 8192 -> 512): 65,536 rows
// 7.97 -> 5.42 ms with the taller tile; 2,048 rows 0.42 ms (64) vs 0.75 ms (128).
#ifndef BB_LINEAR32_BIG
#define BB_LINEAR32_BIG 1024
#endif
constexpr int kL32BN = 128, kL32BK = 32;
template <int BM>
constexpr int l32_threads() { return 64 * (BM / 32) * 2; }  // waves: BM / 32 (m) x 2 (n), each 32 m x 64 n

template <int BM>
__global__ void __launch_bounds__(l32_threads<BM>()) __attribute__((amdgpu_waves_per_eu(BM == 128 ? 4 : 1)))
linear32_kernel(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
                float* __restrict__ y, int M, int N, int K) {
  constexpr int kL32BM = BM, kL32Threads = l32_threads<BM>();
  constexpr int ABYTES = kL32BM * kL32BK * 4, BBYTES = kL32BN * kL32BK * 4;
  constexpr int SBYTES = ABYTES + BBYTES;
  constexpr int NW = kL32Threads / 64;
  constexpr int TM = 2, TN = 4;  // 16 x 16 tiles per wave: 32 m x 64 n
  constexpr int GA = ABYTES / 1024 / NW, GB = BBYTES / 1024 / NW;  // 1-KB copies per wave per stage
  static_assert(GA >= 1 && GB >= 1, "stage smaller than one copy per wave");
  __shared__ __attribute__((aligned(16))) uint8_t sm[2 * SBYTES];
  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r16 = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * kL32BM, n0 = blockIdx.y * kL32BN;
  const int NS = K / kL32BK;
  auto stage = [&](int st) {
    uint8_t* a = sm + (st & 1) * SBYTES;
    uint8_t* b = a + ABYTES;
    const int k0 = st * kL32BK;
#pragma unroll
    for (int kq = 0; kq < GA; ++kq) {
      const int kk = wid + kq * NW, e = kk * 64 + lane, r = e / 8, lc = (e % 8) ^ ((r >> 1) & 7);
      const int row = min(m0 + r, M - 1);  // rows past M read the last one (never stored)
      c32_glds16_async(x + (size_t)row * K + k0 + lc * 4, a + kk * 1024);
    }
#pragma unroll
    for (int kq = 0; kq < GB; ++kq) {
      const int kk = wid + kq * NW, e = kk * 64 + lane, r = e / 8, lc = (e % 8) ^ ((r >> 1) & 7);
      c32_glds16_async(w + (size_t)(n0 + r) * K + k0 + lc * 4, b + kk * 1024);
    }
  };
  stage(0);
  C32_WAIT_VM_LGKM0(0);
  __syncthreads();
  const int wm = (wid % (kL32BM / 32)) * 32, wn = (wid / (kL32BM / 32)) * 64;
  double dacc[TN][TM][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) dacc[j][i][e] = 0.0;
  for (int st = 0; st < NS; ++st) {
    if (st + 1 < NS) stage(st + 1);  // its slot was last read in stage st - 1, before that stage's barrier
    const uint8_t* a = sm + (st & 1) * SBYTES;
    const uint8_t* b = a + ABYTES;
#pragma unroll
    for (int kb = 0; kb < kL32BK / 16; ++kb) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm + 16 * i + r16;
        af[i] = *reinterpret_cast<const f32x4*>(a + r * 128 + (((4 * kb + g) ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn + 16 * j + r16;
        bf[j] = *reinterpret_cast<const f32x4*>(b + r * 128 + (((4 * kb + g) ^ ((r >> 1) & 7)) << 4));
      }
      f32x4 acc[TN][TM];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(bf[j][s4], af[i][s4], acc[j][i], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) dacc[j][i][e] += (double)acc[j][i][e];
    }
    C32_WAIT_VM_LGKM0(0);  // the next stage (this wave's copies; the barrier covers the rest)
    __syncthreads();
  }
  // D[n = wn + 16 j + 4 g + e][m = wm + 16 i + r16]: 4 consecutive outputs of one row = one 16-byte store
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm + 16 * i + r16;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn + 16 * j + 4 * g;
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (float)(dacc[j][i][e] + (bias ? (double)bias[n + e] : 0.0));
      *reinterpret_cast<f32x4*>(y + (size_t)m * N + n) = f32x4{o[0], o[1], o[2], o[3]};
    }
  }
}

template <int CIN, int COUT>
hipError_t c32_fwd_t(const float* x, const float* w, int nb, float* y, hipStream_t s) {
  hipLaunchKernelGGL((conv32_fwd_kernel<CIN, COUT>), dim3((nb + kC32Boards - 1) / kC32Boards), dim3(kC32Threads), 0,
                     s, x, w, y, nb);
  return hipGetLastError();
}

}  // namespace

bool conv3x3_f32_supported(int cin, int cout) {
  return (cin == 128 && cout == 128) || (cin == 64 && cout == 128) || (cin == 128 && cout == 64);
}

hipError_t launch_conv3x3_f32_prep(const float* w, int cin, int cout, int wl, float* wf, float* wd, hipStream_t s) {
  const int n = cout * cin * 9;
  hipLaunchKernelGGL(conv32_prep_kernel, dim3((n + 255) / 256), dim3(256), 0, s, w, cout, cin, wl, wf, wd);
  return hipGetLastError();
}

hipError_t launch_conv3x3_f32_forward(const float* x, const float* w, int nb, int cin, int cout, float* y,
                                      hipStream_t s) {
  if (nb <= 0 || !conv3x3_f32_supported(cin, cout)) return hipErrorInvalidValue;
  if (cin == 64) return c32_fwd_t<64, 128>(x, w, nb, y, s);
  if (cout == 64) return c32_fwd_t<128, 64>(x, w, nb, y, s);
  return c32_fwd_t<128, 128>(x, w, nb, y, s);
}

hipError_t launch_linear_f32(const float* x, const float* w, const float* bias, int M, int N, int K, float* y,
                             hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || N % kL32BN || K % kL32BK) return hipErrorInvalidValue;
  if ((long)((M + 127) / 128) * (N / kL32BN) >= BB_LINEAR32_BIG)
    hipLaunchKernelGGL(linear32_kernel<128>, dim3((M + 127) / 128, N / kL32BN), dim3(l32_threads<128>()), 0, s, x,
                       w, bias, y, M, N, K);
  else
    hipLaunchKernelGGL(linear32_kernel<64>, dim3((M + 63) / 64, N / kL32BN), dim3(l32_threads<64>()), 0, s, x, w,
                       bias, y, M, N, K);
  return hipGetLastError();
}

}  // namespace bb

// bb_conv.hip -- the CNN's 3x3 / pad-1 convolutions on 8x8 board planes, bf16
// MFMA with f32 accumulation (gfx950).
//
// BlockBlastNetwork's conv stack (network.py:75-117, ResidualBlock
// network.py:14-30) is conv 4->64, conv 64->128 and five conv 128->128, all
// 3x3 with padding 1 over 8x8 boards.  Under bf16 autocast MIOpen ran the
// 128-channel layers at 0.4-0.7 PFLOP/s and its split-K weight gradient needed
// zero fills and casts around it (the PPO optimizer step).  These
// kernels are written for the 8x8 board: a board is 64 pixel rows of C channels
// in NHWC, the nine taps are row shifts inside a board, and a tap that leaves
// the board reads a zero row of LDS instead of branching.
//
//   forward  y[b,p,co]  = sum_{t,ci} x[b,p+d_t,ci] * w[co,ci,t]
//   data grad dx[b,q,ci] = sum_{t,co} dy[b,q-d_t,co] * w[co,ci,t]
//            = the forward kernel over dy with w'[t'][ci][co] = w[co][ci][8-t']
//   weight grad dw[co,ci,t] = sum_{b,p} dy[b,p,co] * x[b,p+d_t,ci]
// with d_t = (t/3 - 1, t%3 - 1) and zero outside the board.  Activations are
// bf16 NHWC (channels_last), weights f32 [Cout][Cin][3][3] (nn.Conv2d) cast to
// bf16 with round-to-nearest-even as autocast does, accumulation f32, y and dx
// rounded to bf16, dw f32.  The weight gradient is split over board chunks
// into f32 partials that one pass adds in a fixed order: no atomics, results
// are deterministic run to run.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include <algorithm>

#include "bb_env_internal.h"

namespace bb {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int kThreads = 256;
#ifndef BB_CONV_FWD_BOARDS
#define BB_CONV_FWD_BOARDS 2
#endif
// forward: boards (64 pixel rows each) per workgroup; 1 only with 128 output channels
template <int COUT>
constexpr int fwd_boards() { return (BB_CONV_FWD_BOARDS == 1 && COUT == 128) ? 1 : 2; }
constexpr int kWgBoards = 2;     // weight grad: boards per LDS stage
constexpr int kWgTile = 64;      // weight grad: 64 x 64 (co, ci) tile, all nine taps

__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);  // round to nearest even
  return *reinterpret_cast<uint16_t*>(&b);
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return uint32_t(f2bf(lo)) | (uint32_t(f2bf(hi)) << 16);
}

// ---------------------------------------------------------------------------
// weight prep: w f32 [COUT][CIN][9] (wl 0) or [COUT][9][CIN] (wl 1, a
// channels_last parameter) -> wf bf16 [9][COUT][CIN] (forward) and wd bf16
// [9][CIN][COUT] with tap 8 - t (data gradient)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) conv_prep_kernel(const float* __restrict__ w, int cout, int cin, int wl,
                                                             uint16_t* __restrict__ wf, uint16_t* __restrict__ wd) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= cout * cin * 9) return;
  const int co = i / (9 * cin);
  const int t = wl ? (i / cin) % 9 : i % 9;
  const int ci = wl ? i % cin : (i / 9) % cin;
  const uint16_t b = f2bf(w[i]);
  wf[(t * cout + co) * cin + ci] = b;
  wd[((8 - t) * cin + ci) * cout + co] = b;
}

// All layers' weight prep in one launch (one kernel per layer otherwise): the
// table of up to kPrepMax layers travels in the kernel arguments.
constexpr int kPrepMax = 16;
struct PrepTable {
  const float* w[kPrepMax];
  uint16_t* wf[kPrepMax];
  uint16_t* wd[kPrepMax];
  int cin[kPrepMax], cout[kPrepMax], wl[kPrepMax];
  int block0[kPrepMax + 1];  // first workgroup of layer l
  int count;
};

__device__ __forceinline__ void prep_block(const PrepTable& tab, int blk) {  // workgroup blk of the table's launch
  int l = 0;
  while (l + 1 < tab.count && tab.block0[l + 1] <= blk) ++l;
  const int cout = tab.cout[l], cin = tab.cin[l], wl = tab.wl[l];
  const int i = (blk - tab.block0[l]) * kThreads + threadIdx.x;
  if (i >= cout * cin * 9) return;
  const int co = i / (9 * cin);
  const int t = wl ? (i / cin) % 9 : i % 9;
  const int ci = wl ? i % cin : (i / 9) % cin;
  const uint16_t b = f2bf(tab.w[l][i]);
  tab.wf[l][(t * cout + co) * cin + ci] = b;
  tab.wd[l][((8 - t) * cin + ci) * cout + co] = b;
}

__global__ void __launch_bounds__(kThreads) conv_prep_multi_kernel(const PrepTable tab) { prep_block(tab, blockIdx.x); }

// A prep table's launch geometry (PrepTable.block0); -1: a layer the HIP convolutions do not take
int build_prep_table(PrepTable& tab, int count, const float* const* w, const int32_t* cin, const int32_t* cout,
                     const int32_t* wl, void* const* wf, void* const* wd);

// LDS image of pixel rows of C bf16 channels: 16-byte chunk c of row r sits at
// chunk c ^ key(r).  The B fragment of mfma_f32_16x16x32_bf16 puts pixel n of a
// 16-pixel tile in lanes n + 16 hq, chunk 4 cb + hq; ds_read_b128 serves lanes in
// groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} (and +32): each group reads
// chunk parity hq & 1 = 0 for pixels n in {0-3, 12-15} and 1 for n in {4-11},
// or the reverse.  The key leaves bit 0 of the chunk alone and XORs the row's
// residue mod 8 into bits 1-3 (256-B rows) or (row & 1, row >> 1 & 3) into the
// bank line half and bits 1-2 (128-B rows, two per bank line): both pixel sets
// are 8 consecutive rows mod 8 under every tap shift, so the 16 lanes of a group
// hit 16 different 16-byte bank quads (r03's key r & 15 conflicted on the odd
// column shifts: 40% extra LDS cycles).  Zero rows sit at ROWS + (row mod 16),
// which keeps the key of the row they replace.
template <int C>
__device__ __forceinline__ int fwd_key(int r) {
  return C == 128 ? ((r & 7) << 1) : (((r >> 1) & 3) << 1);
}

// Direct global -> LDS copy of one 16-byte chunk per lane: lane L of the wave
// lands at lds_base + 16 L (lds_base wave-uniform); the global address is per
// lane, so swizzled LDS images are written by permuting the sources.
__device__ __forceinline__ void glds16(const void* g, uint8_t* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// The same copy issued from inline asm: the compiler then does not track it,
// so it inserts no vmcnt(0) before LDS reads of OTHER buffers while it is in
// flight; the caller waits for it with a counted BB_WAIT_VM before the barrier
// that precedes reading its buffer.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved; nothing else in these kernels keeps it live
__device__ __forceinline__ void glds16_async(const void* g, uint8_t* lds_base) {
  const uint32_t l = (uint32_t)(size_t)((__attribute__((address_space(3))) uint8_t*)lds_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
}
#pragma clang diagnostic pop

// s_waitcnt with vmcnt = n (expcnt, lgkmcnt not waited)
#define BB_WAIT_VM(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (7 << 4) | (15 << 8) | (((n) >> 4) << 14))
// s_waitcnt with vmcnt = n and lgkmcnt = 0
#define BB_WAIT_VM_LGKM0(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (7 << 4) | (((n) >> 4) << 14))

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------------------
// forward / data gradient.  Workgroup (4 waves): 2 boards = 128 pixel rows x
// all COUT; two workgroups share a CU, so one's copies and barriers overlap
// the other's MFMAs.  D[co][px] = sum_k W[co][k] X[k][px] on
// mfma_f32_32x32x16_bf16 with A = the weights, B = the (shifted) input rows,
// both from LDS (ds_read_b128), the fragments of k-step k+1 read while k
// computes; each lane ends with 4 consecutive output channels of one pixel per
// register group (8-byte stores).  The input tile is copied once (direct
// global -> LDS).  The weights stream from L2 in stages of one tap x 32 input
// channels (COUT rows of 64 B) through a ring of kFwdRing LDS buffers, copied
// kFwdRing - 1 stages ahead; each wave waits (counted vmcnt) only for its own
// copies of the next stage before the barrier.
// Waves: COUT = 128 -> 2 (co) x 2 (px) waves of 64 co x 64 px;
//        COUT =  64 -> 1 x 4 waves of 64 co x 32 px.
// A tap that leaves the board reads one of 16 zero rows, the one whose
// swizzle matches the row it replaces (no extra bank conflict).  Boards past
// the batch read board nb-1 (their outputs are not stored; taps never cross
// boards).  Weight rows of 64 B hold 16-byte chunk c at c ^ ((co >> 2) & 3).
// ---------------------------------------------------------------------------
constexpr int kFwdThreads = 256;
constexpr int kZeroRows = 16;
#ifndef BB_CONV_FWD_RING
#define BB_CONV_FWD_RING 2  // 3: -29%, 5 with 32-channel stages: -14% (tools/variants.py cf*)
#endif
#ifndef BB_CONV_FWD_SCI
#define BB_CONV_FWD_SCI 64
#endif
#ifndef BB_CONV_FWD_UNROLL
#define BB_CONV_FWD_UNROLL 1  // conv_fwd_kernel's stage loop unrolled with precomputed operand bases (0: rolled)
#endif
#ifndef BB_CONV_MFMA16
#define BB_CONV_MFMA16 1  // forward tiles on mfma_f32_16x16x32_bf16 (0: 32x32x16)
#endif
#ifndef BB_CONV_STORE_LDS
#define BB_CONV_STORE_LDS 1  // forward output staged through LDS for 16-byte coalesced stores
#endif
#ifndef BB_CONV_WG16
#define BB_CONV_WG16 0  // 1: weight-gradient tiles on mfma_f32_16x16x32_bf16 (parity-green, 14% slower)
#endif
#ifndef BB_CONV_DIAG
#define BB_CONV_DIAG 0  // diagnostics only: 1 = no output stores, 2 = one tap of the nine
#endif
constexpr int kFwdRing = BB_CONV_FWD_RING;

template <int SCI>
__device__ __forceinline__ int wkey(int co) {
  return SCI == 32 ? (co >> 2) & 3 : (co >> 1) & 7;
}

__device__ __forceinline__ uint32_t add2_bf16(uint32_t a, uint32_t b) {  // two bf16 sums, rounded once (torch's add)
  return pack2(__uint_as_float(a << 16) + __uint_as_float(b << 16),
               __uint_as_float(a & 0xFFFF0000u) + __uint_as_float(b & 0xFFFF0000u));
}

// radd (NULL = none, shipped LDS-staged store path only): y = bf16(conv) + radd, rounded again -- the
// data gradient of a ResidualBlock's first convolution plus the identity path's gradient, as autograd's
// separate add kernel computed it
// st.part (NULL = none, same path, radd NULL): BatchNorm reduction sums from the store pass, per channel over
// the workgroup's pixels (f32 per thread over its rows, the lanes of a channel by a fixed xor tree, the waves
// added in order in f64) -> st.part[(blockIdx.x * COUT + c) * 3 + q], bn_reduce_nhwc's partial layout:
//   st.bx NULL: the following BatchNorm's forward statistics, q = {sum y, sum y^2, 0} of the stored bf16
//               outputs (bb_bn_forward_part finalises from them without its own pass over y);
//   st.bx set : this is a data gradient dy of a BatchNorm [+ ReLU] output whose input was st.bx (bf16, y's
//               shape): q = {sum g, sum g xhat, sum xhat}, g = dy masked where the forward's ReLU was off,
//               xhat = (x - mean) invstd -- bn_reduce_nhwc's backward arithmetic (bb_bn_backward_part).
// BSTATS: the backward-statistics instantiation (st.bx set); the others carry none of its code.
template <int CIN, int COUT, bool BSTATS = false>
__global__ void __launch_bounds__(kFwdThreads) conv_fwd_kernel(const uint16_t* __restrict__ x,
                                                               const uint16_t* __restrict__ w,
                                                               uint16_t* __restrict__ y, int nb,
                                                               const uint16_t* __restrict__ radd,
                                                               const ConvStatsArgs st) {
  constexpr int RB = CIN * 2;                 // bytes per pixel row
  constexpr int NCH = CIN / 8;                // 16-byte chunks per pixel row
  constexpr int FB = fwd_boards<COUT>();
  constexpr int ROWS = FB * 64;               // pixel rows
  constexpr int XBYTES = (ROWS + kZeroRows) * RB;
  constexpr int SCI = BB_CONV_FWD_SCI;        // input channels per weight stage (32 or 64)
  constexpr int NCB = CIN / SCI;              // stages per tap
  constexpr int NS = (BB_CONV_DIAG == 2 ? 1 : 9) * NCB;  // stages
  constexpr int WBYTES = COUT * SCI * 2;      // one stage: COUT rows of SCI * 2 bytes
  constexpr int NW = kFwdThreads / 64;        // 4 waves
  constexpr int GPW = WBYTES / 1024 / NW;     // weight copies per wave per stage
  constexpr int DIST = kFwdRing - 1;          // stages in flight ahead
  constexpr int WN = COUT / 64;               // waves along co
  constexpr int WM = NW / WN;                 // waves along px
  constexpr int TM = (ROWS / WM) / 32;        // 32-px MFMA tiles per wave
  constexpr int TN = 2;                       // 32-co MFMA tiles per wave
  constexpr int KK = SCI / 16;                // k-steps per stage
  static_assert(GPW >= 1, "weight stage smaller than one copy per wave");
  __shared__ __attribute__((aligned(16))) uint8_t sm[XBYTES + kFwdRing * WBYTES];
  uint8_t* const xs = sm;

  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int b0 = blockIdx.x * FB;

  // input tile: LDS chunk e = 64 k + lane holds row e / NCH, logical chunk (e % NCH) ^ key(row)
#pragma unroll
  for (int k = wid; k < ROWS * NCH / 64; k += NW) {
    const int e = k * 64 + lane, r = e / NCH, lc = (e % NCH) ^ fwd_key<CIN>(r);
    const int b = min(b0 + (r >> 6), nb - 1);
    glds16_async(x + (size_t(b) * 64 + (r & 63)) * CIN + lc * 8, xs + k * 1024);
  }
  // weight stage st (tap st / NCB, channels 32 (st % NCB) ...) -> ring slot st % kFwdRing
  auto stage_w = [&](int st) {
    uint8_t* wb = sm + XBYTES + (st % kFwdRing) * WBYTES;
    const uint16_t* ws = w + (size_t)(st / NCB) * COUT * CIN + (st % NCB) * SCI;
#pragma unroll
    for (int kq = 0; kq < GPW; ++kq) {
      const int k = wid + kq * NW;
      const int e = k * 64 + lane, r = e / (SCI / 8), lc = (e % (SCI / 8)) ^ wkey<SCI>(r);
      glds16_async(ws + r * CIN + lc * 8, wb + k * 1024);
    }
  };
#pragma unroll
  for (int st = 0; st < DIST; ++st) stage_w(st);
  for (int i = tid; i < kZeroRows * NCH; i += kFwdThreads)
    *reinterpret_cast<uint4*>(xs + ROWS * RB + i * 16) = make_uint4(0, 0, 0, 0);
  BB_WAIT_VM_LGKM0((DIST - 1) * GPW);  // the input tile and stage 0 have landed
  raw_barrier();

#if BB_CONV_MFMA16
  // mfma_f32_16x16x32_bf16 tiles (holds a higher clock than 32x32x16 under load, MI355X_MICROARCH.md):
  // lane l holds A[co0 + 16jn + (l & 15)][k 8(l >> 4) + j], B[k 8(l >> 4) + j][px0 + 16im + (l & 15)],
  // D[co0 + 16jn + 4(l >> 4) + reg][px0 + 16im + (l & 15)]
  constexpr int TN16 = 4;                     // 16-co tiles per wave (64 co)
  constexpr int TM16 = (ROWS / WM) / 16;      // 16-px tiles per wave
  constexpr int KK16 = SCI / 32;              // k-steps of 32 per stage
  const int r16 = lane & 15, hq = lane >> 4;
  const int co0 = (wid % WN) * 64;
  const int px0 = (wid / WN) * (ROWS / WM);
  int abase[TN16], akey[TN16];
#pragma unroll
  for (int j = 0; j < TN16; ++j) {
    const int co = co0 + 16 * j + r16;
    abase[j] = co * SCI * 2;
    akey[j] = wkey<SCI>(co);
  }
  f32x4 acc[TN16][TM16];
#pragma unroll
  for (int j = 0; j < TN16; ++j)
#pragma unroll
    for (int i = 0; i < TM16; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[j][i][e] = 0.f;

#if BB_CONV_FWD_UNROLL
  // every stage unrolled: tap, channel block and ring slot are compile-time, so an operand address is one
  // precomputed per-lane base XOR a constant (the swizzle keys only flip chunk bits that the k offset does not
  // carry, see fwd_key) and the ring slot rides in the ds_read offset
  int aq[TN16], bq[TM16];
#pragma unroll
  for (int j = 0; j < TN16; ++j) aq[j] = abase[j] + ((hq ^ akey[j]) << 4);
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    if (st + DIST < NS) stage_w(st + DIST);  // its slot was last read in stage st-1, before the barrier
    const int cb = st % NCB;
    if (cb == 0) {
      const int t = st / NCB, dy = t / 3 - 1, dx = t % 3 - 1;
#pragma unroll
      for (int i = 0; i < TM16; ++i) {
        const int px = px0 + 16 * i + r16;
        const int p = px & 63, yy = (p >> 3) + dy, xc = (p & 7) + dx;
        const int row = ((unsigned)yy < 8u && (unsigned)xc < 8u) ? (px & ~63) + yy * 8 + xc
                                                                  : ROWS + ((px + 8 * dy + dx) & 15);
        bq[i] = row * RB + ((hq ^ fwd_key<CIN>(row)) << 4);
      }
    }
    const int woff = XBYTES + (st % kFwdRing) * WBYTES;
    bf16x8 afr[2][TN16], bfr[2][TM16];
    auto load = [&](int kk, int set) {
#pragma unroll
      for (int j = 0; j < TN16; ++j)
        afr[set][j] = *reinterpret_cast<const bf16x8*>(sm + woff + (aq[j] ^ (kk << 6)));
#pragma unroll
      for (int i = 0; i < TM16; ++i)
        bfr[set][i] = *reinterpret_cast<const bf16x8*>(xs + (bq[i] ^ ((cb * (SCI / 8) + 4 * kk) << 4)));
    };
    load(0, 0);
#pragma unroll
    for (int kk = 0; kk < KK16; ++kk) {
      if (kk + 1 < KK16) load(kk + 1, (kk + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < TN16; ++j)
#pragma unroll
        for (int i = 0; i < TM16; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[kk & 1][j], bfr[kk & 1][i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int after = min(NS, st + DIST + 1) - (st + 2);
    if (after >= 4) BB_WAIT_VM(4 * GPW);
    else if (after == 3) BB_WAIT_VM(3 * GPW);
    else if (after == 2) BB_WAIT_VM(2 * GPW);
    else if (after == 1) BB_WAIT_VM(GPW);
    else BB_WAIT_VM(0);
    raw_barrier();
  }
#else
  int rb[TM16], key[TM16];
  for (int st = 0; st < NS; ++st) {
    if (st + DIST < NS) stage_w(st + DIST);  // its slot was last read in stage st-1, before the barrier
    const int cb = st % NCB;
    if (cb == 0) {
      const int t = st / NCB, dy = t / 3 - 1, dx = t % 3 - 1;
#pragma unroll
      for (int i = 0; i < TM16; ++i) {
        const int px = px0 + 16 * i + r16;
        const int p = px & 63, yy = (p >> 3) + dy, xc = (p & 7) + dx;
        const int row = ((unsigned)yy < 8u && (unsigned)xc < 8u) ? (px & ~63) + yy * 8 + xc
                                                                  : ROWS + ((px + 8 * dy + dx) & 15);
        rb[i] = row * RB;
        key[i] = fwd_key<CIN>(row);
      }
    }
    const uint8_t* wb = sm + XBYTES + (st % kFwdRing) * WBYTES;
    bf16x8 afr[2][TN16], bfr[2][TM16];
    auto load = [&](int kk, int set) {
#pragma unroll
      for (int j = 0; j < TN16; ++j)
        afr[set][j] = *reinterpret_cast<const bf16x8*>(wb + abase[j] + (((4 * kk + hq) ^ akey[j]) << 4));
#pragma unroll
      for (int i = 0; i < TM16; ++i)
        bfr[set][i] = *reinterpret_cast<const bf16x8*>(xs + rb[i] + (((cb * (SCI / 8) + 4 * kk + hq) ^ key[i]) << 4));
    };
    load(0, 0);
#pragma unroll
    for (int kk = 0; kk < KK16; ++kk) {
      if (kk + 1 < KK16) load(kk + 1, (kk + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < TN16; ++j)
#pragma unroll
        for (int i = 0; i < TM16; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[kk & 1][j], bfr[kk & 1][i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int after = min(NS, st + DIST + 1) - (st + 2);
    if (after >= 4) BB_WAIT_VM(4 * GPW);
    else if (after == 3) BB_WAIT_VM(3 * GPW);
    else if (after == 2) BB_WAIT_VM(2 * GPW);
    else if (after == 1) BB_WAIT_VM(GPW);
    else BB_WAIT_VM(0);
    raw_barrier();
  }
#endif
#if BB_CONV_STORE_LDS
  // the output tile goes through LDS (free after the last stage's barrier) so that every global
  // store is a whole 16-byte chunk of a pixel row: row px of COUT bf16, 16-byte chunk c at c ^ (px & 15)
  constexpr int OCH = COUT / 8;  // 16-byte chunks per output row
  constexpr int NIT = ROWS * OCH / kFwdThreads;  // store-pass chunks per thread
  static_assert(ROWS * OCH % kFwdThreads == 0, "whole store-pass iterations");
  uint8_t* const os = sm;
  // backward statistics: the BatchNorm input's chunks of this thread's store-pass positions, loaded now so
  // their latency hides behind the tile's LDS staging
  uint4 bxv[BSTATS ? NIT : 1];
  if constexpr (BSTATS) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = tid + it * kFwdThreads, px = e / OCH, c = e % OCH;
      bxv[it] = b0 + (px >> 6) < nb
                    ? *reinterpret_cast<const uint4*>(st.bx + (size_t(b0) * 64 + px) * COUT + c * 8)
                    : make_uint4(0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < TM16; ++i) {
    const int px = px0 + 16 * i + r16;
#pragma unroll
    for (int j = 0; j < TN16; ++j) {
      const int co = co0 + 16 * j + 4 * hq;  // 4 channels = half of chunk co / 8
      uint2 v;
      v.x = pack2(acc[j][i][0], acc[j][i][1]);
      v.y = pack2(acc[j][i][2], acc[j][i][3]);
      *reinterpret_cast<uint2*>(os + px * (COUT * 2) + (((co >> 3) ^ (px & 15 & (OCH - 1))) << 4) + ((co & 4) << 1)) = v;
    }
  }
  __syncthreads();
  static_assert(kFwdThreads % OCH == 0, "a thread's output chunk column must stay fixed");
  double* const stats = st.part;
  constexpr bool bwd = BSTATS;
  float ss[8], sq[8], sx[8];  // stats: the 8 channels of chunk column tid % OCH
  float kmu[8], kis[8], ksc[8], ksh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ss[j] = sq[j] = sx[j] = 0.f;
    kmu[j] = kis[j] = ksc[j] = ksh[j] = 0.f;
  }
  if (stats && bwd) {
    const int c0 = (tid % OCH) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      kmu[j] = st.mean[c0 + j];
      kis[j] = st.invstd[c0 + j];
      ksc[j] = kis[j] * st.w[c0 + j];
      ksh[j] = st.b[c0 + j];
    }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + it * kFwdThreads;
    const int px = e / OCH, c = e % OCH;
    if (b0 + (px >> 6) >= nb) continue;
    if (BB_CONV_DIAG == 1 && acc[0][0][0] != 1.2345e-30f) continue;
    const size_t o = (size_t(b0) * 64 + px) * COUT + c * 8;
    uint4 v = *reinterpret_cast<const uint4*>(os + px * (COUT * 2) + ((c ^ (px & 15 & (OCH - 1))) << 4));
    if (radd) {
      const uint4 a = *reinterpret_cast<const uint4*>(radd + o);
      v = make_uint4(add2_bf16(v.x, a.x), add2_bf16(v.y, a.y), add2_bf16(v.z, a.z), add2_bf16(v.w, a.w));
    }
    if (stats) {
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
      float f[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f[2 * k] = __uint_as_float(vv[k] << 16);
        f[2 * k + 1] = __uint_as_float(vv[k] & 0xFFFF0000u);
      }
      if constexpr (bwd) {
        const uint4 xa = bxv[it];
        const uint32_t xw[4] = {xa.x, xa.y, xa.z, xa.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xv = __uint_as_float((j & 1) ? (xw[j >> 1] & 0xFFFF0000u) : (xw[j >> 1] << 16));
          const float u = xv + 0.f;  // bn_reduce's u = x + pb, pb = 0
          const float g = (st.relu && (u - kmu[j]) * ksc[j] + ksh[j] <= 0.f) ? 0.f : f[j];  // the forward's ops
          const float xh = (u - kmu[j]) * kis[j];
          ss[j] += g;
          sq[j] += g * xh;
          sx[j] += xh;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ss[j] += f[j];
          sq[j] += f[j] * f[j];
        }
      }
    }
    *reinterpret_cast<uint4*>(y + o) = v;
  }
  if (stats) {  // uniform: every thread reaches the barrier
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int m = OCH; m < 64; m <<= 1) {
        ss[j] += __shfl_xor(ss[j], m, 64);
        sq[j] += __shfl_xor(sq[j], m, 64);
        sx[j] += __shfl_xor(sx[j], m, 64);
      }
    float* red = reinterpret_cast<float*>(sm + ROWS * COUT * 2);  // past the output tile: [wave][3][COUT]
    static_assert(ROWS * COUT * 2 + NW * 3 * COUT * 4 <= XBYTES + kFwdRing * WBYTES, "stats scratch");
    if (lane < OCH)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(wid * 3 + 0) * COUT + lane * 8 + j] = ss[j];
        red[(wid * 3 + 1) * COUT + lane * 8 + j] = sq[j];
        red[(wid * 3 + 2) * COUT + lane * 8 + j] = sx[j];
      }
    __syncthreads();
    for (int t = tid; t < COUT * 3; t += kFwdThreads) {
      const int c = t / 3, m = t % 3;
      double a = 0.0;
#pragma unroll
      for (int wv = 0; wv < NW; ++wv) a += (double)red[(wv * 3 + m) * COUT + c];
      stats[(size_t)blockIdx.x * COUT * 3 + t] = a;
    }
  }
#else
#pragma unroll
  for (int i = 0; i < TM16; ++i) {
    const int px = px0 + 16 * i + r16;
    if (b0 + (px >> 6) >= nb) continue;
    if (BB_CONV_DIAG == 1 && acc[0][i][0] != 1.2345e-30f) continue;
    uint16_t* yo = y + (size_t(b0) * 64 + px) * COUT + co0 + 4 * hq;
#pragma unroll
    for (int j = 0; j < TN16; ++j) {
      uint2 v;
      v.x = pack2(acc[j][i][0], acc[j][i][1]);
      v.y = pack2(acc[j][i][2], acc[j][i][3]);
      *reinterpret_cast<uint2*>(yo + 16 * j) = v;
    }
  }
#endif
#else
  const int r = lane & 31, h = lane >> 5;
  const int co0 = (wid % WN) * 64;
  const int px0 = (wid / WN) * (ROWS / WM);
  int abase[TN], akey[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int co = co0 + 32 * j + r;
    abase[j] = co * SCI * 2;
    akey[j] = wkey<SCI>(co);
  }

  f32x16 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][i][e] = 0.f;

  int rb[TM], key[TM];
  for (int st = 0; st < NS; ++st) {
    if (st + DIST < NS) stage_w(st + DIST);  // its slot was last read in stage st-1, before the barrier
    const int cb = st % NCB;
    if (cb == 0) {
      const int t = st / NCB, dy = t / 3 - 1, dx = t % 3 - 1;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int px = px0 + 32 * i + r;
        const int p = px & 63, yy = (p >> 3) + dy, xc = (p & 7) + dx;
        const int row = ((unsigned)yy < 8u && (unsigned)xc < 8u) ? (px & ~63) + yy * 8 + xc
                                                                  : ROWS + ((px + 8 * dy + dx) & 15);
        rb[i] = row * RB;
        key[i] = fwd_key<CIN>(row);
      }
    }
    const uint8_t* wb = sm + XBYTES + (st % kFwdRing) * WBYTES;
    bf16x8 afr[2][TN], bfr[2][TM];
    auto load = [&](int kk, int set) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        afr[set][j] = *reinterpret_cast<const bf16x8*>(wb + abase[j] + (((2 * kk + h) ^ akey[j]) << 4));
#pragma unroll
      for (int i = 0; i < TM; ++i)
        bfr[set][i] = *reinterpret_cast<const bf16x8*>(xs + rb[i] + (((cb * (SCI / 8) + 2 * kk + h) ^ key[i]) << 4));
    };
    load(0, 0);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      // the reads of k-step kk+1 are issued before the MFMAs of kk (the scheduler
      // would otherwise reuse the registers and wait on every k-step's reads)
      if (kk + 1 < KK) load(kk + 1, (kk + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr[kk & 1][j], bfr[kk & 1][i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // the next stage must have landed: this wave's copies (counted), the others' (barrier)
    const int after = min(NS, st + DIST + 1) - (st + 2);
    if (after >= 4) BB_WAIT_VM(4 * GPW);
    else if (after == 3) BB_WAIT_VM(3 * GPW);
    else if (after == 2) BB_WAIT_VM(2 * GPW);
    else if (after == 1) BB_WAIT_VM(GPW);
    else BB_WAIT_VM(0);
    raw_barrier();
  }

  // epilogue: lane holds D[co0 + 32j + 8g + 4h + (0..3)][px0 + 32i + r]
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int px = px0 + 32 * i + r;
    if (b0 + (px >> 6) >= nb) continue;
    if (BB_CONV_DIAG == 1 && acc[0][i][0] != 1.2345e-30f) continue;
    uint16_t* yo = y + (size_t(b0) * 64 + px) * COUT + co0 + 4 * h;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 v;
        v.x = pack2(acc[j][i][4 * g + 0], acc[j][i][4 * g + 1]);
        v.y = pack2(acc[j][i][4 * g + 2], acc[j][i][4 * g + 3]);
        *reinterpret_cast<uint2*>(yo + 32 * j + 8 * g) = v;
      }
  }
#endif
}

// ---------------------------------------------------------------------------
// weight gradient.  Workgroup (8 waves): one 64 (co) x 64 (ci) tile, all nine
// taps, over a chunk of boards, 2 boards per LDS stage.  Stages go through a
// ring of 4 LDS buffers by direct global -> LDS copies issued 3 stages ahead;
// each wave waits (counted vmcnt) only for its copies of the next stage before
// the barrier, so the HBM latency of a stage is covered by three stages of
// MFMAs.  Both operands have the pixel as their k index, so they are read with
// ds_read_b64_tr_b16 from plain NHWC rows (the hardware transposes 4 rows x 16
// channels per 16-lane group); the shifted input rows of a tap point at a zero
// row when they leave the board.  Waves 4k + (wc, wi) take board k of each
// stage and accumulate D_t[32 co][32 ci] for the nine taps (144 f32 per lane);
// at the end the second half hands its sums to the first through LDS, which
// writes the chunk's partial [chunk][t][co][ci]; conv_wgrad_reduce adds the
// chunks in order.  The grid runs the 4 tiles of a chunk next to each other,
// so the second read of each slice of dy and x comes from cache.
// LDS rows are 128 B (64 channels); 8-byte unit u of row r sits at
// u ^ (((r >> 1) & 1) << 3), which makes a 32-lane half's 4 consecutive rows x
// 32 channels conflict-free; the 4 zero rows follow the same pattern, and an
// off-board row v reads zero row v & 3 (the bank segment v would have used).
// ---------------------------------------------------------------------------
constexpr int kWgThreads = 512;
constexpr int kWgRing = 4;

__device__ __forceinline__ int wg_off(int r, int u) { return r * 128 + ((u ^ (((r >> 1) & 1) << 3)) << 3); }

template <int CIN, int COUT>
__global__ void __launch_bounds__(kWgThreads) conv_wgrad_kernel(const uint16_t* __restrict__ x,
                                                                const uint16_t* __restrict__ dy,
                                                                float* __restrict__ part, int nb, int bpc) {
  constexpr int SROWS = kWgBoards * 64;                // pixel rows per stage and operand
  constexpr int SBYTES = 2 * SROWS * 128;              // dy rows then x rows
  constexpr int ZOFF = kWgRing * SBYTES;               // 4 zero rows after the ring
  constexpr int NWAVE = kWgThreads / 64;
  constexpr int GPS = SBYTES / 1024 / NWAVE;           // copies per wave per stage (4)
  __shared__ __attribute__((aligned(16))) uint8_t sm[kWgRing * SBYTES + 4 * 128];

  constexpr int TCI = CIN / kWgTile;
  constexpr int NT = TCI * (COUT / kWgTile);
  // XCD-aware order: workgroup ids go round-robin over the 8 XCDs, so the NT tiles of
  // one chunk (which read the same dy and x slices) get ids 8 apart = the same XCD's L2
  const int id = blockIdx.x, xcd = id & 7, k8 = id >> 3;
  const int tile = k8 % NT;
  const int chunk = (k8 / NT) * 8 + xcd;
  if (chunk * bpc >= nb) return;  // the whole workgroup: no barrier reached
  const int co_t = (tile / TCI) * kWgTile, ci_t = (tile % TCI) * kWgTile;
  const int bb = chunk * bpc;
  const int be = min(nb, bb + bpc);
  const int nst = (be - bb + kWgBoards - 1) / kWgBoards;
  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if (tid < 32) *reinterpret_cast<uint4*>(sm + ZOFF + tid * 16) = make_uint4(0, 0, 0, 0);

  // stage copy: wave-instruction k (1 KB = 8 rows of 128 B) of [operand][row];
  // lane L -> row 8k' + L/8, physical 16-byte chunk L%8 = logical chunk ^ 4*((row>>1)&1)
  auto stage = [&](int si) {
    const int s0 = bb + si * kWgBoards;
    uint8_t* base = sm + (si & (kWgRing - 1)) * SBYTES;
#pragma unroll
    for (int kq = 0; kq < GPS; ++kq) {
      const int k = wid + kq * NWAVE;
      const int op = k / (SROWS / 8), r = (k % (SROWS / 8)) * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ ((((r >> 1) & 1)) << 2);
      const int b = min(s0 + (r >> 6), nb - 1);  // past the chunk: any valid board, skipped below
      const size_t pix = size_t(b) * 64 + (r & 63);
      const uint16_t* src = op == 0 ? dy + pix * COUT + co_t + lc * 8 : x + pix * CIN + ci_t + lc * 8;
      glds16_async(src, base + k * 1024);
    }
  };

  const int half = wid >> 2, wc = wid & 1, wi = (wid >> 1) & 1;
  const int gi = lane & 15, g = lane >> 4, hh = g >> 1, q = gi >> 2, p = gi & 3;
  const int ucol = (g & 1) * 4 + p;   // 8-byte unit within the wave's 32 channels
  const int ua = wc * 8 + ucol;       // dy unit (co)
  const int ub = wi * 8 + ucol;       // x unit (ci)

#if BB_CONV_WG16
  // mfma_f32_16x16x32_bf16: k = 32 pixels; lane group g (= lane >> 4) holds k 8g..8g+7, column lane & 15;
  // tile (jc, ji) of the wave's 32 x 32 is acc[t][2 jc + ji]
  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int z = 0; z < 4; ++z)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t][z][e] = 0.f;
#else
  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
#endif

  const int pre = min(nst, kWgRing - 1);
  for (int si = 0; si < pre; ++si) stage(si);
  // stage 0 landed (the later ones may still be in flight), zero rows written
  if (pre == 3) BB_WAIT_VM_LGKM0(2 * GPS);
  else if (pre == 2) BB_WAIT_VM_LGKM0(GPS);
  else BB_WAIT_VM_LGKM0(0);
  raw_barrier();
  for (int si = 0; si < nst; ++si) {
    if (si + kWgRing - 1 < nst) stage(si + kWgRing - 1);  // its buffer was last read in stage si-1
    const int s0 = bb + si * kWgBoards;
    if (s0 + half < be) {
      const int sdy = (si & (kWgRing - 1)) * SBYTES + half * 64 * 128;
      const int sx = sdy + SROWS * 128;
#if BB_CONV_WG16
      // A (dy^T) fragments: k-step ks (32 pixels) x co tile jc: pixels 32ks + 8g + q (+4), channels 16jc + 4p..
      bf16x8 afr[2][2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int jc = 0; jc < 2; ++jc) {
          const int o0 = 32 * ks + 8 * g + q;
          const int u = wc * 8 + 4 * jc + p;
          const bf16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(sm + sdy + wg_off(o0, u)));
          const bf16x4 ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(sm + sdy + wg_off(o0 + 4, u)));
          afr[ks][jc] = __builtin_shufflevector(alo, ahi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      // B (shifted x) fragments of tap t, k-step ks, ci tile ji: input board row 4ks + g + dy, columns q + dx, q + 4 + dx
      auto bload = [&](int t, int ks, int ji) {
        const int dy = t / 3 - 1, dx = t % 3 - 1;
        const int iy = 4 * ks + g + dy, ix0 = q + dx, ix1 = q + 4 + dx;
        const int u = wi * 8 + 4 * ji + p;
        const bool vy = (unsigned)iy < 8u;
        const int v0 = iy * 8 + ix0, v1 = iy * 8 + ix1;
        const int off0 = (vy && (unsigned)ix0 < 8u) ? sx + wg_off(v0, u) : ZOFF + wg_off(v0 & 3, u);
        const int off1 = (vy && (unsigned)ix1 < 8u) ? sx + wg_off(v1, u) : ZOFF + wg_off(v1 & 3, u);
        const bf16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(sm + off0));
        const bf16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(sm + off1));
        return __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7);
      };
#pragma unroll
      for (int n = 0; n < 18; ++n) {  // (tap, k-step) pairs
        const int t = n >> 1, ks = n & 1;
        const bf16x8 b0 = bload(t, ks, 0), b1 = bload(t, ks, 1);
#pragma unroll
        for (int jc = 0; jc < 2; ++jc) {
          acc[t][2 * jc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[ks][jc], b0, acc[t][2 * jc], 0, 0, 0);
          acc[t][2 * jc + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[ks][jc], b1, acc[t][2 * jc + 1], 0, 0, 0);
        }
      }
#else
      // A (dy^T) fragments of the 4 k-steps: board-local pixels 16ks + 8hh + q (+4)
      bf16x8 afr[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int o0 = 16 * ks + 8 * hh + q;
        const bf16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(sm + sdy + wg_off(o0, ua)));
        const bf16x4 ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(sm + sdy + wg_off(o0 + 4, ua)));
        afr[ks] = __builtin_shufflevector(alo, ahi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      // B (shifted x) fragment of input board row u + hh, columns q + dx and q + 4 + dx: tap (dy, dx) of
      // k-step ks reads u = 2ks + dy, so (ks, +1) and (ks + 1, -1) share one read: 27 reads for 36 MFMAs
      auto bload = [&](int u, int dx) {
        const int iy = u + hh, ix0 = q + dx, ix1 = q + 4 + dx;
        const bool vy = (unsigned)iy < 8u;
        const int v0 = iy * 8 + ix0, v1 = iy * 8 + ix1;
        const int off0 = (vy && (unsigned)ix0 < 8u) ? sx + wg_off(v0, ub) : ZOFF + wg_off(v0 & 3, ub);
        const int off1 = (vy && (unsigned)ix1 < 8u) ? sx + wg_off(v1, ub) : ZOFF + wg_off(v1 & 3, ub);
        const bf16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(sm + off0));
        const bf16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(sm + off1));
        return __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7);
      };
      bf16x8 bfr[2];
      bfr[0] = bload(-1, -1);
#pragma unroll
      for (int n = 0; n < 27; ++n) {
        const int dxi = n / 9, u = n % 9 - 1;
        if (n + 1 < 27) bfr[(n + 1) & 1] = bload((n + 1) % 9 - 1, (n + 1) / 9 - 1);
        __builtin_amdgcn_sched_barrier(0);
        if (u & 1) {  // odd u: (ks, dy) = ((u - 1) / 2, +1) and ((u + 1) / 2, -1)
          if (u >= 1) acc[6 + dxi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr[(u - 1) / 2], bfr[n & 1], acc[6 + dxi], 0, 0, 0);
          if (u <= 5) acc[dxi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr[(u + 1) / 2], bfr[n & 1], acc[dxi], 0, 0, 0);
        } else {      // even u: (u / 2, 0)
          acc[3 + dxi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr[u / 2], bfr[n & 1], acc[3 + dxi], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    #endif
    }
    // the next stage must have landed (this wave's copies; the barrier covers the others')
    const int after = min(nst, si + kWgRing) - (si + 2);  // stages issued after stage si+1
    if (after >= 2) BB_WAIT_VM(2 * GPS);
    else if (after == 1) BB_WAIT_VM(GPS);
    else BB_WAIT_VM(0);
    raw_barrier();
  }

  // the second half's sums -> LDS (3 taps = 48 KB at a time) -> added by the first half
  const int r = lane & 31, h = lane >> 5;
  float* pp = part + (size_t)chunk * 9 * COUT * CIN;
  float* red = reinterpret_cast<float*>(sm);
  const int slot = (wid & 3) * 64 + lane;  // the partner waves (wid, wid + 4) share a slot
#pragma unroll
  for (int t0 = 0; t0 < 9; t0 += 3) {
    if (half == 1) {
#pragma unroll
      for (int t = t0; t < t0 + 3; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e)
#if BB_CONV_WG16
          red[((t - t0) * 16 + e) * 256 + slot] = acc[t][e >> 2][e & 3];
#else
          red[((t - t0) * 16 + e) * 256 + slot] = acc[t][e];
#endif
    }
    __syncthreads();
    if (half == 0) {
#pragma unroll
      for (int t = t0; t < t0 + 3; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
#if BB_CONV_WG16
          // tile z = e >> 2 = 2 jc + ji, register e & 3: co 16 jc + 4g + reg, ci 16 ji + (lane & 15)
          const int co = co_t + 32 * wc + 16 * (e >> 3) + 4 * g + (e & 3);
          const int ci = ci_t + 32 * wi + 16 * ((e >> 2) & 1) + (lane & 15);
          pp[((size_t)t * COUT + co) * CIN + ci] = acc[t][e >> 2][e & 3] + red[((t - t0) * 16 + e) * 256 + slot];
#else
          const int co = co_t + 32 * wc + (e & 3) + 8 * (e >> 2) + 4 * h;
          pp[((size_t)t * COUT + co) * CIN + ci_t + 32 * wi + r] = acc[t][e] + red[((t - t0) * 16 + e) * 256 + slot];
#endif
        }
    }
    __syncthreads();
  }
}

// dw[co][ci][t] (wl 0) or dw[co][t][ci] (wl 1) = sum over chunks, in chunk order
__global__ void __launch_bounds__(kThreads) conv_wgrad_reduce(const float* __restrict__ part, int nchunk, int cout,
                                                              int cin, int wl, float* __restrict__ dw) {
  const int i = blockIdx.x * kThreads + threadIdx.x;  // over [t][co][ci]
  const int n = 9 * cout * cin;
  if (i >= n) return;
  float s = 0.f;
  int c = 0;
  for (; c + 16 <= nchunk; c += 16) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = part[(size_t)(c + k) * n + i];
#pragma unroll
    for (int k = 0; k < 16; ++k) s += v[k];
  }
  for (; c < nchunk; ++c) s += part[(size_t)c * n + i];
  const int ci = i % cin, co = (i / cin) % cout, t = i / (cin * cout);
  dw[wl ? (co * 9 + t) * cin + ci : (co * cin + ci) * 9 + t] = s;
}

int wgrad_chunks(int nb, int cin, int cout) {
  const int tiles = (cin / kWgTile) * (cout / kWgTile);
  int nchunk = 256 / tiles;  // one 8-wave workgroup per CU
  const int maxc = (nb + kWgBoards - 1) / kWgBoards;
  if (nchunk > maxc) nchunk = maxc;
  if (nchunk < 1) nchunk = 1;
  return nchunk;
}

int wgrad_bpc(int nb, int nchunk) {
  int bpc = (nb + nchunk - 1) / nchunk;
  return (bpc + kWgBoards - 1) / kWgBoards * kWgBoards;
}

template <int CIN, int COUT>
hipError_t fwd_t(const void* x, const void* w, int nb, void* y, hipStream_t s, const void* radd,
                 const ConvStatsArgs& st) {
  if (nb <= 0 || (radd && st.part)) return hipErrorInvalidValue;
  // variant builds: no fused add / statistics
  if ((radd || st.part) && !(BB_CONV_MFMA16 && BB_CONV_STORE_LDS)) return hipErrorInvalidValue;
  const dim3 grid((nb + fwd_boards<COUT>() - 1) / fwd_boards<COUT>());
  if (st.part && st.bx)
    hipLaunchKernelGGL((conv_fwd_kernel<CIN, COUT, true>), grid, dim3(kFwdThreads), 0, s, (const uint16_t*)x,
                       (const uint16_t*)w, (uint16_t*)y, nb, (const uint16_t*)radd, st);
  else
    hipLaunchKernelGGL((conv_fwd_kernel<CIN, COUT>), grid, dim3(kFwdThreads), 0, s, (const uint16_t*)x,
                       (const uint16_t*)w, (uint16_t*)y, nb, (const uint16_t*)radd, st);
  return hipGetLastError();
}

int wgrad_used(int nb, int cin, int cout) {  // chunks that hold boards
  const int bpc = wgrad_bpc(nb, wgrad_chunks(nb, cin, cout));
  return (nb + bpc - 1) / bpc;
}

template <int CIN, int COUT>
hipError_t wgrad_partial_t(const void* x, const void* dy, int nb, float* ws, hipStream_t s) {
  const int bpc = wgrad_bpc(nb, wgrad_chunks(nb, CIN, COUT));
  const int used8 = (wgrad_used(nb, CIN, COUT) + 7) / 8 * 8;
  hipLaunchKernelGGL((conv_wgrad_kernel<CIN, COUT>), dim3((CIN / kWgTile) * (COUT / kWgTile) * used8), dim3(kWgThreads),
                     0, s, (const uint16_t*)x, (const uint16_t*)dy, ws, nb, bpc);
  return hipGetLastError();
}

hipError_t wgrad_reduce(const float* ws, int used, int cin, int cout, int wl, float* dw, hipStream_t s) {
  const int n = 9 * cout * cin;
  hipLaunchKernelGGL(conv_wgrad_reduce, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, ws, used, cout, cin,
                     wl, dw);
  return hipGetLastError();
}

template <int CIN, int COUT>
hipError_t wgrad_t(const void* x, const void* dy, int nb, float* ws, int wl, float* dw, hipStream_t s) {
  hipError_t st = wgrad_partial_t<CIN, COUT>(x, dy, nb, ws, s);
  if (st != hipSuccess) return st;
  return wgrad_reduce(ws, wgrad_used(nb, CIN, COUT), CIN, COUT, wl, dw, s);
}

// ---------------------------------------------------------------------------
// The input layer, conv 4 -> 64 (network.py:75-87's first Conv2d) under bf16 autocast: x f32 (the stacked
// board + piece planes, NCHW or channels_last) and w f32 rounded to bf16 as autocast casts them, products
// exact, f32 sums, y bf16 NHWC.  K = 36 (k = 4 t + ci) is padded to 64 for mfma_f32_16x16x32_bf16 with
// A = the weights (M = co), B = the board's im2col (N = pixel): a lane's C values are 4 consecutive output
// channels of one pixel, staged through LDS so a wave stores its board's 8 KB as whole 16-byte chunks.
// Weight gradient dw[co][k] = sum_{b,p} dy[b,p,co] x[b,p+d_t,ci]: M = co, N = k (36 -> 48), K = pixels, dy
// transposed through LDS; a workgroup's partial [t][co][ci] goes to conv_wgrad_reduce (fixed chunk order).
// ---------------------------------------------------------------------------
constexpr int kInCout = 64, kInK = 36, kInWaves = 4;
#ifndef BB_IN_WG_CHUNKS
#define BB_IN_WG_CHUNKS 128
#endif
#ifndef BB_IN_FWD_BLOCKS
#define BB_IN_FWD_BLOCKS 256
#endif
constexpr int kInWgChunks = BB_IN_WG_CHUNKS;  // weight-gradient workgroups (partials) at most
constexpr int kInFwdBlocks = BB_IN_FWD_BLOCKS;  // forward workgroups at most (4 boards each per pass)

__device__ __forceinline__ bf16x8 pack8(float4 a, float4 b) {
  bf16x8 r;
  r[0] = (short)f2bf(a.x); r[1] = (short)f2bf(a.y); r[2] = (short)f2bf(a.z); r[3] = (short)f2bf(a.w);
  r[4] = (short)f2bf(b.x); r[5] = (short)f2bf(b.y); r[6] = (short)f2bf(b.z); r[7] = (short)f2bf(b.w);
  return r;
}

__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// one lane's A fragments of the input-layer weights: A[co = 16 mt + l16][k = 32 s + 8 g + j], k = 4 t + ci,
// straight from the f32 weight (L2-resident; 16-byte loads for a channels_last weight), rounded to bf16
__device__ __forceinline__ float4 in_weight_taps(const float* __restrict__ w, int wl, int co, int t) {
  if (t >= 9) return make_float4(0.f, 0.f, 0.f, 0.f);
  if (wl) return *reinterpret_cast<const float4*>(w + (co * 9 + t) * 4);
  return make_float4(w[(co * 4) * 9 + t], w[(co * 4 + 1) * 9 + t], w[(co * 4 + 2) * 9 + t], w[(co * 4 + 3) * 9 + t]);
}

__device__ __forceinline__ void in_weight_frags(const float* __restrict__ w, int wl, int g, int l16, bf16x8 afr[4][2]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int co = 16 * mt + l16, t = 8 * s2 + 2 * g;
      afr[mt][s2] = pack8(in_weight_taps(w, wl, co, t), in_weight_taps(w, wl, co, t + 1));
    }
}

// With prep_blocks > 0 the launch's last prep_blocks workgroups build the other layers' bf16 weight images
// (conv_prep_multi's work, independent of this layer: both run at the start of the forward, in one launch).
__global__ void __launch_bounds__(256) conv_in_fwd_kernel(const float* __restrict__ x, int x_nhwc,
                                                          const float* __restrict__ w, int wl, int nb,
                                                          uint16_t* __restrict__ y, const PrepTable pt,
                                                          int prep_blocks) {
  __shared__ float4 xpad[kInWaves][100];      // per wave: [(r + 1) * 10 + c + 1] -> 4 channels
  __shared__ uint4 ost[kInWaves][64 * 8];     // per wave: [pixel][16-B chunk ^ (pixel & 7)] of 8 channels
  const int fwd_blocks = (int)gridDim.x - prep_blocks;
  if ((int)blockIdx.x >= fwd_blocks) {
    prep_block(pt, (int)blockIdx.x - fwd_blocks);
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
  const int stride = fwd_blocks * kInWaves;
  int b = blockIdx.x * kInWaves + wave;
  // the first board's load in flight with the weight fragments' (every wave works alone: no barrier)
  float4 xv = b < nb ? reinterpret_cast<const float4*>(x + (size_t)b * 256)[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = lane; i < 100; i += 64) xpad[wave][i] = make_float4(0.f, 0.f, 0.f, 0.f);
  bf16x8 afr[4][2];
  in_weight_frags(w, wl, g, l16, afr);
  for (; b < nb; b += stride) {
    if (x_nhwc) {  // lane = pixel
      xpad[wave][((lane >> 3) + 1) * 10 + (lane & 7) + 1] = xv;
    } else {  // lane: channel lane >> 4, pixels 4 (lane & 15) .. + 3
      const int ci = lane >> 4, p0 = (lane & 15) * 4, r = p0 >> 3, c0 = p0 & 7;
      float* f = reinterpret_cast<float*>(xpad[wave]) + ((r + 1) * 10 + c0 + 1) * 4 + ci;
      f[0] = xv.x;
      f[4] = xv.y;
      f[8] = xv.z;
      f[12] = xv.w;
    }
    if (b + stride < nb) xv = reinterpret_cast<const float4*>(x + (size_t)(b + stride) * 256)[lane];  // next board
    lds_wait();
    f32x4 acc[4][4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int p = 16 * nt + l16, r = p >> 3, c = p & 7;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int t0 = 8 * s2 + 2 * g;  // taps t0, t0 + 1 (k = 4 t + ci)
        // loads at clamped taps, then a value select (a select of addresses becomes a flat load from LDS or stack)
        const int ta = min(t0, 8), tb = min(t0 + 1, 8);
        float4 v0 = xpad[wave][(r + ta / 3) * 10 + c + ta % 3];
        float4 v1 = xpad[wave][(r + tb / 3) * 10 + c + tb % 3];
        if (t0 >= 9) v0 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t0 + 1 >= 9) v1 = make_float4(0.f, 0.f, 0.f, 0.f);
        const bf16x8 bfr = pack8(v0, v1);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[mt][s2], bfr, acc[mt][nt], 0, 0, 0);
      }
    }
    // C[co = 16 mt + 4 g + i][pixel = 16 nt + l16] -> ost (8 bytes: 4 channels)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int p = 16 * nt + l16, chunk = 2 * mt + (g >> 1);
        uint2 v;
        v.x = pack2(acc[mt][nt][0], acc[mt][nt][1]);
        v.y = pack2(acc[mt][nt][2], acc[mt][nt][3]);
        reinterpret_cast<uint2*>(&ost[wave][p * 8 + (chunk ^ (p & 7))])[g & 1] = v;
      }
    lds_wait();
    uint4* yb = reinterpret_cast<uint4*>(y + (size_t)b * 64 * kInCout);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = lane + 64 * q, p = idx >> 3, ch = idx & 7;
      yb[idx] = ost[wave][p * 8 + (ch ^ (p & 7))];
    }
  }
}

__device__ __forceinline__ s16x4 in_tr_read(const uint16_t* lds) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)lds);
}

__global__ void __launch_bounds__(256) conv_in_wgrad_kernel(const float* __restrict__ x, int x_nhwc,
                                                            const uint16_t* __restrict__ dy, int nb,
                                                            float* __restrict__ part) {
  // per wave: dy [64 pixels][64 co] bf16 as stored (read k-major by ds_read_b64_tr_b16), then the padded
  // board; after the board loop the same bytes hold waves 1-3's sums for wave 0 to add
  constexpr int kDy = 64 * 64 * 2, kXp = 100 * 16, kPerWave = kDy + kXp;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kInWaves * kPerWave];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
  const int q4 = l16 >> 2, p4 = l16 & 3;  // this lane's row / column group in a transposed read
  uint16_t* dys = reinterpret_cast<uint16_t*>(smem + wave * kPerWave);
  float4* xpad = reinterpret_cast<float4*>(smem + wave * kPerWave + kDy);
  for (int i = lane; i < 100; i += 64) xpad[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  f32x4 acc[4][3];  // C[co = 16 mt + 4 g + i][k = 16 nt + l16]
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int stride = gridDim.x * kInWaves;
  int b = blockIdx.x * kInWaves + wave;
  // board bb's dy (8 x 16 B per lane) and x (16 B) into registers
#define BB_IN_FETCH(bb)                                                              \
  {                                                                                  \
    const uint4* db_ = reinterpret_cast<const uint4*>(dy + (size_t)(bb) * 64 * kInCout); \
    dv0 = db_[lane];                                                                 \
    dv1 = db_[lane + 64];                                                            \
    dv2 = db_[lane + 128];                                                           \
    dv3 = db_[lane + 192];                                                           \
    dv4 = db_[lane + 256];                                                           \
    dv5 = db_[lane + 320];                                                           \
    dv6 = db_[lane + 384];                                                           \
    dv7 = db_[lane + 448];                                                           \
    xv = reinterpret_cast<const float4*>(x + (size_t)(bb) * 256)[lane];              \
  }
  uint4 dv0, dv1, dv2, dv3, dv4, dv5, dv6, dv7;
  float4 xv;
  if (b < nb) BB_IN_FETCH(b)
  for (; b < nb; b += stride) {
    {  // [pixel][co], as in HBM
      uint4* d_ = reinterpret_cast<uint4*>(dys) + lane;
      d_[0] = dv0, d_[64] = dv1, d_[128] = dv2, d_[192] = dv3, d_[256] = dv4, d_[320] = dv5, d_[384] = dv6, d_[448] = dv7;
    }
    if (x_nhwc) {
      xpad[((lane >> 3) + 1) * 10 + (lane & 7) + 1] = xv;
    } else {
      const int ci = lane >> 4, p0 = (lane & 15) * 4, r = p0 >> 3, c0 = p0 & 7;
      float* f = reinterpret_cast<float*>(xpad) + ((r + 1) * 10 + c0 + 1) * 4 + ci;
      f[0] = xv.x;
      f[4] = xv.y;
      f[8] = xv.z;
      f[12] = xv.w;
    }
    if (b + stride < nb) BB_IN_FETCH(b + stride)  // the next board's loads in flight during this one
    lds_wait();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 afr[4];  // A[co = 16 mt + l16][pixel = 32 s + 8 g + j]: two 4-pixel transposed reads
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const s16x4 lo = in_tr_read(dys + (32 * s2 + 8 * g + q4) * 64 + 16 * mt + 4 * p4);
        const s16x4 hi = in_tr_read(dys + (32 * s2 + 8 * g + 4 + q4) * 64 + 16 * mt + 4 * p4);
        afr[mt] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) {
        const int k = 16 * nt + l16, t = k >> 2, ci = k & 3, r = 4 * s2 + g;  // pixels (r, 0 .. 7)
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = k < kInK ? reinterpret_cast<const float*>(xpad)[((r + t / 3) * 10 + j + t % 3) * 4 + ci] : 0.f;
        const bf16x8 bfr = pack8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[mt], bfr, acc[mt][nt], 0, 0, 0);
      }
    }
  }
#undef BB_IN_FETCH
  __syncthreads();  // every wave is done with its LDS images
  float* red = reinterpret_cast<float*>(smem);  // [3][9][64][4]: waves 1-3
  constexpr int kW = 9 * kInCout * 4;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) {
      const int k = 16 * nt + l16, t = k >> 2, ci = k & 3;
      if (wave > 0 && k < kInK)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[(wave - 1) * kW + (t * kInCout + 16 * mt + 4 * g + i) * 4 + ci] = acc[mt][nt][i];
    }
  __syncthreads();
  if (wave > 0) return;
  float* out = part + (size_t)blockIdx.x * kW;  // [t][co][ci], conv_wgrad_reduce's chunk layout
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) {
      const int k = 16 * nt + l16, t = k >> 2, ci = k & 3;
      if (k < kInK)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int o = (t * kInCout + 16 * mt + 4 * g + i) * 4 + ci;
          out[o] = ((acc[mt][nt][i] + red[o]) + red[kW + o]) + red[2 * kW + o];  // wave order
        }
    }
}

int in_wgrad_chunks(int nb) { return nb <= 0 ? 0 : std::min(kInWgChunks, (nb + kInWaves - 1) / kInWaves); }

}  // namespace

bool conv3x3_supported(int cin, int cout) {
  return (cin == 64 || cin == 128) && (cout == 64 || cout == 128);
}

int64_t conv3x3_wgrad_workspace_bytes(int nb, int cin, int cout) {
  const int nchunk = wgrad_chunks(nb, cin, cout);
  return (int64_t)nchunk * 9 * cin * cout * (int64_t)sizeof(float);
}

hipError_t launch_conv3x3_prep(const float* w, int cin, int cout, int wl, void* wf, void* wd, hipStream_t s) {
  const int n = cout * cin * 9;
  hipLaunchKernelGGL(conv_prep_kernel, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, w, cout, cin, wl,
                     (uint16_t*)wf, (uint16_t*)wd);
  return hipGetLastError();
}

namespace {
int build_prep_table(PrepTable& tab, int count, const float* const* w, const int32_t* cin, const int32_t* cout,
                     const int32_t* wl, void* const* wf, void* const* wd) {
  if (count <= 0 || count > kPrepMax) return -1;
  tab.count = count;
  int blocks = 0;
  for (int l = 0; l < count; ++l) {
    if (!w[l] || !wf[l] || !wd[l] || !conv3x3_supported(cin[l], cout[l]) || (wl[l] != 0 && wl[l] != 1)) return -1;
    tab.w[l] = w[l];
    tab.wf[l] = static_cast<uint16_t*>(wf[l]);
    tab.wd[l] = static_cast<uint16_t*>(wd[l]);
    tab.cin[l] = cin[l];
    tab.cout[l] = cout[l];
    tab.wl[l] = wl[l];
    tab.block0[l] = blocks;
    blocks += (cout[l] * cin[l] * 9 + kThreads - 1) / kThreads;
  }
  tab.block0[count] = blocks;
  return blocks;
}
}  // namespace

hipError_t launch_conv3x3_prep_multi(int count, const float* const* w, const int32_t* cin, const int32_t* cout,
                                     const int32_t* wl, void* const* wf, void* const* wd, hipStream_t s) {
  PrepTable tab;
  const int blocks = build_prep_table(tab, count, w, cin, cout, wl, wf, wd);
  if (blocks <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv_prep_multi_kernel, dim3(blocks), dim3(kThreads), 0, s, tab);
  return hipGetLastError();
}

hipError_t launch_conv3x3_forward(const void* x, const void* w, int nb, int cin, int cout, void* y, hipStream_t s,
                                  const void* radd, const ConvStatsArgs* stats) {
  ConvStatsArgs st{};
  if (stats) st = *stats;
  if (cin == 64 && cout == 64) return fwd_t<64, 64>(x, w, nb, y, s, radd, st);
  if (cin == 64 && cout == 128) return fwd_t<64, 128>(x, w, nb, y, s, radd, st);
  if (cin == 128 && cout == 64) return fwd_t<128, 64>(x, w, nb, y, s, radd, st);
  return fwd_t<128, 128>(x, w, nb, y, s, radd, st);
}

int conv3x3_stats_blocks(int nb, int cout) {
  if (nb <= 0) return -1;
  const int fb = cout == 128 ? fwd_boards<128>() : fwd_boards<64>();
  return (nb + fb - 1) / fb;
}

int conv3x3_wgrad_chunks_used(int nb, int cin, int cout) { return wgrad_used(nb, cin, cout); }

hipError_t launch_conv3x3_wgrad_partial(const void* x, const void* dy, int nb, int cin, int cout, float* ws,
                                        hipStream_t s) {
  if (cin == 64 && cout == 64) return wgrad_partial_t<64, 64>(x, dy, nb, ws, s);
  if (cin == 64 && cout == 128) return wgrad_partial_t<64, 128>(x, dy, nb, ws, s);
  if (cin == 128 && cout == 64) return wgrad_partial_t<128, 64>(x, dy, nb, ws, s);
  return wgrad_partial_t<128, 128>(x, dy, nb, ws, s);
}

hipError_t launch_conv3x3_wgrad_reduce(const float* ws, int used, int cin, int cout, int wl, float* dw, hipStream_t s) {
  return wgrad_reduce(ws, used, cin, cout, wl, dw, s);
}

hipError_t launch_conv3x3_wgrad(const void* x, const void* dy, int nb, int cin, int cout, float* ws, int wl,
                                float* dw, hipStream_t s) {
  if (cin == 64 && cout == 64) return wgrad_t<64, 64>(x, dy, nb, ws, wl, dw, s);
  if (cin == 64 && cout == 128) return wgrad_t<64, 128>(x, dy, nb, ws, wl, dw, s);
  if (cin == 128 && cout == 64) return wgrad_t<128, 64>(x, dy, nb, ws, wl, dw, s);
  return wgrad_t<128, 128>(x, dy, nb, ws, wl, dw, s);
}

int64_t conv_in_wgrad_workspace_bytes(int nb) {
  return nb > 0 ? (int64_t)in_wgrad_chunks(nb) * 9 * kInCout * 4 * (int64_t)sizeof(float) : -1;
}

hipError_t launch_conv_in_forward(const float* x, int x_nhwc, const float* w, int wl, int nb, void* y, hipStream_t s) {
  if (nb <= 0 || !x || !w || !y || (wl != 0 && wl != 1) || (reinterpret_cast<uintptr_t>(x) & 15) ||
      (reinterpret_cast<uintptr_t>(y) & 15))
    return hipErrorInvalidValue;
  const int blocks = std::min((nb + kInWaves - 1) / kInWaves, kInFwdBlocks);
  PrepTable pt{};
  hipLaunchKernelGGL(conv_in_fwd_kernel, dim3(blocks), dim3(256), 0, s, x, x_nhwc ? 1 : 0, w, wl, nb, (uint16_t*)y, pt,
                     0);
  return hipGetLastError();
}

hipError_t launch_conv_in_forward_prep(const float* x, int x_nhwc, const float* w, int wl, int nb, void* y, int count,
                                       const float* const* pw, const int32_t* cin, const int32_t* cout,
                                       const int32_t* pwl, void* const* wf, void* const* wd, hipStream_t s) {
  if (nb <= 0 || !x || !w || !y || (wl != 0 && wl != 1) || (reinterpret_cast<uintptr_t>(x) & 15) ||
      (reinterpret_cast<uintptr_t>(y) & 15) || count <= 0 || count > kPrepMax)
    return hipErrorInvalidValue;
  PrepTable pt;
  const int pblocks = build_prep_table(pt, count, pw, cin, cout, pwl, wf, wd);
  if (pblocks <= 0) return hipErrorInvalidValue;
  const int blocks = std::min((nb + kInWaves - 1) / kInWaves, kInFwdBlocks);
  hipLaunchKernelGGL(conv_in_fwd_kernel, dim3(blocks + pblocks), dim3(256), 0, s, x, x_nhwc ? 1 : 0, w, wl, nb,
                     (uint16_t*)y, pt, pblocks);
  return hipGetLastError();
}

hipError_t launch_conv_in_wgrad(const float* x, int x_nhwc, const void* dy, int nb, float* ws, int wl, float* dw,
                                hipStream_t s) {
  if (nb <= 0 || !x || !dy || !ws || !dw || (wl != 0 && wl != 1) || (reinterpret_cast<uintptr_t>(x) & 15) ||
      (reinterpret_cast<uintptr_t>(dy) & 15))
    return hipErrorInvalidValue;
  const int chunks = in_wgrad_chunks(nb);
  hipLaunchKernelGGL(conv_in_wgrad_kernel, dim3(chunks), dim3(256), 0, s, x, x_nhwc ? 1 : 0, (const uint16_t*)dy, nb,
                     ws);
  hipError_t st = hipGetLastError();
  if (st != hipSuccess) return st;
  const int n = 9 * kInCout * 4;
  hipLaunchKernelGGL(conv_wgrad_reduce, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, ws, chunks,
                     kInCout, 4, wl, dw);
  return hipGetLastError();
}

}  // namespace bb

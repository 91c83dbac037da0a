// Diagnostics (not product): issue cost of the VALU instructions the env
// kernels lean on (64-bit shifts, 64-bit multiply-adds, 32-bit multiplies,
// popcounts, cross-lane moves), one and two waves per SIMD.  Each lane runs 8
// independent chains; cycles per wave-instruction from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_rates tools/ubench/valu_rates.hip && /tmp/valu_rates
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CH 8
#define ITERS 256

template <int OP>
__global__ void kern(uint64_t* out, uint64_t seed) {
  uint64_t x[CH];
  uint32_t s = (threadIdx.x * 7 + 3) & 63;
  for (int k = 0; k < CH; ++k) x[k] = seed * (k + 1) + threadIdx.x;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      if (OP == 0) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(x[k]) : "v"(s));
      if (OP == 1) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(x[k]) : "v"(s));
      if (OP == 2) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(x[k]) : "v"(s));
      if (OP == 3) { uint32_t lo = (uint32_t)x[k]; asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(lo) : "v"(s)); x[k] = (x[k] & ~0xffffffffull) | lo; }
      if (OP == 4) { uint32_t lo = (uint32_t)x[k]; asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(lo) : "v"(s)); x[k] = (x[k] & ~0xffffffffull) | lo; }
      if (OP == 5) { uint32_t lo = (uint32_t)x[k]; asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(lo) : "v"(s)); x[k] = (x[k] & ~0xffffffffull) | lo; }
      if (OP == 6) { uint32_t lo = (uint32_t)x[k]; asm volatile("v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(s)); x[k] = (x[k] & ~0xffffffffull) | lo; }
      if (OP == 7) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(x[k]));
      if (OP == 8) { uint32_t lo = (uint32_t)x[k]; asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(lo) : "v"(s)); x[k] = (x[k] & ~0xffffffffull) | lo; }
      if (OP == 9) asm volatile("v_mov_b64 %0, %0" : "+v"(x[k]));
      if (OP == 10) { uint32_t lo = (uint32_t)x[k]; asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(lo) : "v"(s)); x[k] = (x[k] & ~0xffffffffull) | lo; }
      if (OP == 11) { uint32_t lo = (uint32_t)x[k], hi = (uint32_t)(x[k] >> 32); asm volatile("v_nop\n\tv_permlane32_swap_b32 %0, %1" : "+v"(lo), "+v"(hi)); x[k] = ((uint64_t)hi << 32) | lo; }
      if (OP == 12) { uint32_t lo = (uint32_t)x[k]; asm volatile("v_ffbl_b32 %0, %0" : "+v"(lo)); x[k] = (x[k] & ~0xffffffffull) | lo; }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t acc = 0;
  for (int k = 0; k < CH; ++k) acc ^= x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) out[gridDim.x * blockDim.x + (blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

static const char* names[] = {"v_lshrrev_b64", "v_lshlrev_b64", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32",
                              "v_bcnt_u32_b32", "v_add_u32", "v_lshl_add_u64", "v_mul_u32_u24", "v_mov_b64",
                              "v_alignbit_b32", "v_permlane32_swap", "v_ffbl_b32"};

template <int OP>
void run(int threads) {
  const int blocks = 256;
  const size_t n = (size_t)blocks * threads;
  uint64_t* d;
  hipMalloc(&d, (n + n / 64) * 8);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, d, 12345);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, d, 12345);
  hipDeviceSynchronize();
  uint64_t* h = (uint64_t*)malloc(n / 64 * 8);
  hipMemcpy(h, d + n, n / 64 * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (size_t i = 0; i < n / 64; ++i) s += (double)h[i];
  s /= (double)(n / 64);
  // extra ops per chain step for the 32-bit cases (the 64-bit repack) are included: compare against v_add_u32
  printf("%-20s waves/SIMD %d  cycles per wave-instruction %.2f\n", names[OP], threads / 256, s / (ITERS * CH));
  free(h);
  hipFree(d);
}

template <int OP>
void run2() { run<OP>(256); run<OP>(512); }

int main() {
  run2<0>(); run2<1>(); run2<2>(); run2<3>(); run2<4>(); run2<5>(); run2<6>(); run2<7>(); run2<8>(); run2<9>();
  run2<10>(); run2<11>(); run2<12>();
  return 0;
}

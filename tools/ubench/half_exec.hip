// Diagnostics (not product): does a wave64 VALU instruction with only lanes
// 0-31 active (exec upper half zero) issue faster than a full one on gfx950?
// 8 independent chains of v_add_u32 / v_lshrrev_b64 under a lane condition.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/half_exec tools/ubench/half_exec.hip && /tmp/half_exec
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CH 8
#define ITERS 512

template <int OP>
__global__ void kern(uint64_t* out, int active) {
  uint32_t x[CH];
  uint64_t y[CH];
  for (int k = 0; k < CH; ++k) x[k] = threadIdx.x * (k + 3), y[k] = ((uint64_t)x[k] << 20) | k;
  const uint32_t s = (threadIdx.x * 7 + 3) & 31;
  const int lane = threadIdx.x & 63;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (lane < active) {
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(s));
        if (OP == 1) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(y[k]) : "v"(s));
        if (OP == 2) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(y[k]) : "v"(s));
      }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t acc = 0;
  for (int k = 0; k < CH; ++k) acc ^= x[k] ^ y[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) out[gridDim.x * blockDim.x + (blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int OP>
void run(const char* name, int threads, int active) {
  const int blocks = 256;
  const size_t n = (size_t)blocks * threads;
  uint64_t* d;
  (void)hipMalloc(&d, (n + n / 64) * 8);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, d, active);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, d, active);
  (void)hipDeviceSynchronize();
  uint64_t* h = (uint64_t*)malloc(n / 64 * 8);
  (void)hipMemcpy(h, d + n, n / 64 * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (size_t i = 0; i < n / 64; ++i) s += (double)h[i];
  s /= (double)(n / 64);
  printf("%-16s waves/SIMD %d active lanes %2d: cycles per wave-instruction %.2f\n", name, threads / 256, active,
         s / (ITERS * CH));
  free(h);
  (void)hipFree(d);
}

int main() {
  for (int w = 256; w <= 512; w += 256) {
    for (int a : {64, 32, 16}) {
      run<0>("v_add_u32", w, a);
      run<1>("v_lshrrev_b64", w, a);
      run<2>("v_mad_u64_u32", w, a);
    }
  }
  return 0;
}

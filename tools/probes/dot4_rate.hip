// Probe: issue cost of v_dot4_u32_u8 against v_mad_u32_u24 on gfx950, 8
// independent accumulator chains per lane, 1 or 4 waves per SIMD (grid of
// 256 CUs x 4 or 16 waves). Prints ns per instruction per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
template <int OP>
__global__ void __launch_bounds__(1024) k(uint32_t *out, uint32_t a, uint32_t b, int n) {
  uint32_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x + i;
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) acc[i] = __builtin_amdgcn_udot4(acc[i], a, acc[i], false);
      else acc[i] = __umul24(acc[i], a) + b;  // v_mad_u32_u24
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  uint32_t *d;
  hipMalloc(&d, 256 * 1024 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int n = 4096;
  for (int op = 0; op < 2; ++op)
    for (int waves = 4; waves <= 16; waves *= 4) {
      float best = 1e9f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        if (op == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(64 * waves), 0, 0, d, 0x01020304u, 7u, n);
        else hipLaunchKernelGGL(k<1>, dim3(256), dim3(64 * waves), 0, 0, d, 0x01020304u, 7u, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      // per SIMD: waves/4 waves, each n*8 instructions
      const double per = best * 1e6 / ((double)n * 8 * (waves / 4));
      printf("%s waves/SIMD %d: %.3f ns per wave-instruction per SIMD (%.2f cycles at 2.4 GHz)\n",
             op == 0 ? "v_dot4_u32_u8 " : "v_mad_u32_u24", waves / 4, per, per * 2.4);
    }
  return 0;
}

// Microbenchmark (diagnostic, standalone): does a CU's scalar unit limit many
// waves running wave-uniform (SGPR) dependent chains at once? Each wave of a
// W-wave workgroup (one workgroup per CU, 256 workgroups) runs the same
// 64-bit shift/xor chain either on SGPRs (wave-uniform values) or on VGPRs
// (the same values, marked divergent). Reports cycles per chain step per wave.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/salu_tput.hip -o /tmp/salu_tput
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <bool VEC>
__global__ void k_chain(uint64_t *out, const uint32_t *seedv, int n) {
  uint64_t a;
  if (VEC) a = ((uint64_t)seedv[threadIdx.x & 63] << 32) | seedv[(threadIdx.x + 1) & 63];
  else a = ((uint64_t)__builtin_amdgcn_readfirstlane(seedv[0]) << 32) | __builtin_amdgcn_readfirstlane(seedv[1]);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    a = (a << 3) ^ (a >> 7);
    a ^= (uint64_t)i;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 64 + (threadIdx.x >> 6)] = t1 - t0;
  if (a == 0x12345) out[0] = a;
}

int main() {
  uint64_t *d;
  uint32_t *s;
  (void)hipMalloc(&d, 256 * 64 * sizeof(uint64_t));
  (void)hipMalloc(&s, 64 * sizeof(uint32_t));
  uint32_t hs[64];
  for (int i = 0; i < 64; ++i) hs[i] = 0x9E3779B9u * (i + 1);
  (void)hipMemcpy(s, hs, sizeof(hs), hipMemcpyHostToDevice);
  const int n = 8192;
  static uint64_t h[256 * 64];
  for (int vec = 0; vec < 2; ++vec)
    for (int w : {1, 2, 4, 8, 16}) {
      for (int rep = 0; rep < 2; ++rep) {
        if (vec) hipLaunchKernelGGL(k_chain<true>, dim3(256), dim3(64 * w), 0, 0, d, s, n);
        else hipLaunchKernelGGL(k_chain<false>, dim3(256), dim3(64 * w), 0, 0, d, s, n);
      }
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      double sum = 0;
      for (int b = 0; b < 256; ++b)
        for (int k = 0; k < w; ++k) sum += (double)h[b * 64 + k];
      printf("%s waves/CU %2d: %.1f cycles/step per wave\n", vec ? "VGPR" : "SGPR", w, sum / (256.0 * w) / n);
    }
  return 0;
}

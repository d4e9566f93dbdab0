// Microbenchmark (diagnostic, standalone): cycles per instruction of a lone
// wave's dependent chains of the kinds k_prog's serial decoder runs:
//   salu64   s_lshl_b64 / s_xor_b64 chain on wave-uniform values
//   vcmp_ff1 v_cmp (SGPR vs VGPR) -> s_ff1_i32_b64 -> SGPR (ballot + ffs)
//   readlane v_readlane_b32 with an SGPR lane index feeding the next index
//   ldsuni   ds_read_b32 at a uniform address -> v_readfirstlane -> address
//   branchy  a data-dependent scalar branch per step
// One workgroup of one wave; s_memtime (core clock) around each loop.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/salu_lat.hip -o tools/probes/salu_lat
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__global__ void k_lat(uint64_t *out, uint64_t seed, int n) {
  __shared__ uint32_t tab[256];
  const int lane = threadIdx.x;
  for (int i = lane; i < 256; i += 64) tab[i] = (uint32_t)(i * 2654435761u) >> 24;
  __syncthreads();
  const uint32_t vl = (uint32_t)(lane * 977u) & 0xFFFF;
  const int vv = (int)((lane * 13) & 63);
  uint64_t t0, t1;
  // 1: 64-bit scalar chain (2 ops per step)
  uint64_t a = uni((uint32_t)seed) | ((uint64_t)uni((uint32_t)(seed >> 32)) << 32);
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    a = (a << 3) ^ (a >> 7);
    a ^= (uint64_t)i;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[0] = t1 - t0; out[8] = a; }
  // 1b: four independent 64-bit scalar chains in the same loop (ILP)
  uint64_t b1 = a ^ 1, b2 = a ^ 2, b3 = a ^ 3, b4 = a ^ 4;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    b1 = (b1 << 3) ^ (b1 >> 7);
    b2 = (b2 << 5) ^ (b2 >> 9);
    b3 = (b3 << 7) ^ (b3 >> 11);
    b4 = (b4 << 9) ^ (b4 >> 13);
    b1 ^= (uint64_t)i;
    b2 ^= (uint64_t)i;
    b3 ^= (uint64_t)i;
    b4 ^= (uint64_t)i;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[6] = t1 - t0; out[14] = b1 ^ b2 ^ b3 ^ b4; }
  // 1c: s_memrealtime over the same chain as 1 (100 MHz reference clock)
  uint64_t c = a;
  t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) {
    c = (c << 3) ^ (c >> 7);
    c ^= (uint64_t)i;
  }
  t1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) { out[7] = t1 - t0; out[15] = c; }
  // 2: ballot + ffs chain
  uint32_t w = uni((uint32_t)seed) & 0xFFFF;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(w < vl);
    const int l = m ? __ffsll((unsigned long long)m) : 0;
    w = (w * 5 + (uint32_t)l) & 0xFFFF;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[1] = t1 - t0; out[9] = w; }
  // 3: readlane chain
  int idx = (int)(seed & 63);
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) idx = __builtin_amdgcn_readlane(vv, idx) ^ (i & 1);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[2] = t1 - t0; out[10] = idx; }
  // 4: uniform LDS read chain
  uint32_t p = (uint32_t)seed & 255;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) p = uni(tab[p]) ^ (uint32_t)(i & 1);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[3] = t1 - t0; out[11] = p; }
  // 5: data-dependent scalar branches
  uint32_t q = uni((uint32_t)seed);
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (q & 1) q = q * 3 + 1;
    else q >>= 1;
    q += (uint32_t)i;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[4] = t1 - t0; out[12] = q; }
  // 6: mbcnt + cmp + ballot chain (nth_set)
  uint64_t z = a | 1;
  int r = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(z >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)z, 0u));
    const uint64_t m = __builtin_amdgcn_ballot_w64(below == (uint32_t)(r & 7)) & z;
    r = m ? __ffsll((unsigned long long)m) : 1;
    z = (z << 1) | (z >> 63);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[5] = t1 - t0; out[13] = r; }
}

int main() {
  uint64_t *d;
  hipMalloc(&d, 16 * sizeof(uint64_t));
  const int n = 4096;
  hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, d, 0x123456789abcdefull, n);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, d, 0x123456789abcdefull, n);
  uint64_t h[16];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char *names[7] = {"salu64 (2 ops/step)", "vcmp_ff1", "readlane", "ldsuni", "branchy", "nth_set",
                          "salu64 x4 independent"};
  for (int i = 0; i < 7; ++i) printf("%-22s %.1f cycles/step\n", names[i], (double)h[i] / n);
  printf("salu64 chain: %.2f ns/step by s_memrealtime (100 MHz)\n", (double)h[7] * 10.0 / n);
  return 0;
}

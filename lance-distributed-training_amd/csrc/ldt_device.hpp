// ldt_device.hpp — device helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace ldt {

// ---------------------------------------------------------------------------
// Block-wide exclusive scan (256 threads = 4 waves of 64).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// Returns the exclusive prefix of v over the block; *total = block sum.
// `scratch` must hold >= 5 ints; contains a __syncthreads.
__device__ __forceinline__ int block_excl_scan256(int v, int *scratch, int *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int inc = wave_incl_scan(v);
  if (lane == 63) scratch[wave] = inc;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    int s = scratch[w];
    if (w < wave) base += s;
    tot += s;
  }
  *total = tot;
  __syncthreads();
  return base + inc - v;
}

} // namespace ldt

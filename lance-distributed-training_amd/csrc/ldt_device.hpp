// ldt_device.hpp — device helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldt_types.hpp"

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

// 64-bit variant (row and batch totals of large datasets pass 2^31).
// `scratch` must hold >= 4 int64; contains a __syncthreads.
__device__ __forceinline__ int64_t block_excl_scan256_i64(int64_t v, long long *scratch,
                                                          int64_t *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t t = __shfl_up(inc, d, 64);
    if (lane >= d) inc += t;
  }
  if (lane == 63) scratch[wave] = inc;
  __syncthreads();
  int64_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int64_t s = scratch[w];
    if (w < wave) base += s;
    tot += s;
  }
  *total = tot;
  __syncthreads();
  return base + inc - v;
}

// ---------------------------------------------------------------------------
// Pillow Resample.c precompute_coeffs + normalize_coeffs_8bpc for one output
// index, BILINEAR (support 1.0), box (0, in). IEEE double, no contraction, so
// the result equals the x86-64 build of Pillow bit for bit.
// ---------------------------------------------------------------------------
static __device__ int resample_coeffs_one(int inSize, int outSize, int xx, int ksize, int32_t *k,
                                   int *xmin_out) {
#pragma clang fp contract(off)
  const double scale = (double)inSize / (double)outSize;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const double center = (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > inSize) xmax = inSize;
  xmax -= xmin;
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) {
    double t = ((double)(x + xmin) - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    double wv = t < 1.0 ? 1.0 - t : 0.0;
    ww += wv;
  }
  for (int x = 0; x < ksize; ++x) {
    double wv = 0.0;
    if (x < xmax) {
      double t = ((double)(x + xmin) - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      wv = t < 1.0 ? 1.0 - t : 0.0;
      if (ww != 0.0) wv = wv / ww;
    }
    const double v = wv * (double)(1 << kPrecisionBits);
    k[x] = (int32_t)(wv < 0 ? (-0.5 + v) : (0.5 + v));
  }
  *xmin_out = xmin;
  return xmax;
}

__device__ __forceinline__ uint32_t clip8(int32_t in) {
  if (in >= (1 << kPrecisionBits << 8)) return 255;
  if (in <= 0) return 0;
  return (uint32_t)(in >> kPrecisionBits);
}

// ---------------------------------------------------------------------------
// Source-row staging for the resize kernel.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// jdsample.c fancy upsampling value of chroma component c at full-res (x, y).
__device__ __forceinline__ int chroma_at(const ImgDesc &d, const uint8_t *pl, int c, int x, int y) {
  const int stride = d.plane_stride[c];
  const int hf = d.hf[c], vf = d.vf[c];
  if (hf == 1 && vf == 1) return pl[(int64_t)y * stride + x];
  const int dw = d.cdw[c], dh = d.cdh[c];
  if (hf == 2 && vf == 2) {
    const int cx = x >> 1, cy = y >> 1;
    if (dw <= 2) return pl[(int64_t)cy * stride + cx];
    const int ny = (y & 1) ? min(cy + 1, dh - 1) : max(cy - 1, 0);
    const int nx = (x & 1) ? min(cx + 1, dw - 1) : max(cx - 1, 0);
    const uint8_t *r0 = pl + (int64_t)cy * stride, *r1 = pl + (int64_t)ny * stride;
    const int thiscol = r0[cx] * 3 + r1[cx];
    const int nextcol = r0[nx] * 3 + r1[nx];
    return (thiscol * 3 + nextcol + 8 - (x & 1)) >> 4;
  }
  if (hf == 2 && vf == 1) {
    const int cx = x >> 1;
    const uint8_t *r0 = pl + (int64_t)y * stride;
    if (dw <= 2) return r0[cx];
    const int nx = (x & 1) ? min(cx + 1, dw - 1) : max(cx - 1, 0);
    return (r0[cx] * 3 + r0[nx] + 1 + (x & 1)) >> 2;
  }
  return pl[(int64_t)(y / vf) * stride + (x / hf)];
}

// jdcolor.c ycc_rgb_convert with the 16-bit fixed-point tables evaluated inline.
__device__ __forceinline__ void ycc_to_rgb(int Y, int cb, int cr, uint8_t *o) {
  const int xcr = cr - 128, xcb = cb - 128;
  const int cr_r = (91881 * xcr + 32768) >> 16;         // FIX(1.40200)
  const int cb_b = (116130 * xcb + 32768) >> 16;        // FIX(1.77200)
  const int g = (-22554 * xcb + 32768 + (-46802) * xcr) >> 16; // FIX(0.34414), FIX(0.71414)
  o[0] = (uint8_t)clampi(Y + cr_r, 0, 255);
  o[1] = (uint8_t)clampi(Y + g, 0, 255);
  o[2] = (uint8_t)clampi(Y + cb_b, 0, 255);
}

} // namespace ldt

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


// Destuff classification of 16 bytes (jdhuff.c jpeg_fill_bit_buffer /
// jdmarker.c semantics): wv[1..4] hold them, wv[0] and wv[5] the words on
// either side; p0 is the position of the first one relative to the scan start
// and L the scan's length. keep: bytes kept (FF00 -> FF, fill bytes and marker
// bytes dropped); rst: RSTn codes (segment boundaries); local_end: index of an
// end-of-scan marker's FF (16: none).
__host__ __device__ __forceinline__ void ds_classify16(const uint32_t wv[6], int64_t p0, int64_t L,
                                              uint32_t &keep, uint32_t &rst, int &local_end) {
  keep = rst = 0;
  local_end = 16;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int64_t p = p0 + j;
    const uint32_t prev = (wv[(j + 3) >> 2] >> (8 * ((j + 3) & 3))) & 255;
    const uint32_t cur = (wv[(j + 4) >> 2] >> (8 * ((j + 4) & 3))) & 255;
    const uint32_t next = (wv[(j + 5) >> 2] >> (8 * ((j + 5) & 3))) & 255;
    const bool in = p >= 0 && p < L;
    const bool next_in = p + 1 < L;
    bool drop = false;
    if (cur == 0xFF) {
      const uint32_t nx = next_in ? next : 0u;
      if (nx == 0x00) {
        drop = false;                        // stuffed data byte 0xFF
      } else if (nx == 0xFF || (nx >= 0xD0 && nx <= 0xD7)) {
        drop = true;                         // fill byte or RSTn prefix
      } else if (in && next_in) {
        if (local_end == 16) local_end = j;  // end-of-scan marker
        drop = true;
      } else {
        drop = true;                         // trailing 0xFF at end of cell
      }
    } else if (prev == 0xFF && p > 0) {
      if (cur == 0x00) drop = true;          // stuffing zero
      else if (cur >= 0xD0 && cur <= 0xD7) {
        drop = true;
        if (in) rst |= 1u << j;              // RSTn code: segment boundary
      }
    }
    if (in && !drop) keep |= 1u << j;
  }
}


// The same classification driven by the 0xFF bytes (k_huff_image's fused
// destuff): every byte is kept unless it is an 0xFF or follows one, so the
// lane finds its 0xFF bytes with a word-parallel test and applies the rules
// above only around them (one or two per 16 bytes of entropy-coded data at
// most, usually none) instead of testing all 16 bytes.
__host__ __device__ __forceinline__ uint32_t ds_ff4(uint32_t w) { // bit i: byte i == 0xFF
  const uint32_t t = ~w;
  const uint32_t h = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
  return (((h >> 7) * 0x204081u) >> 21) & 0xFu;
}
// Byte k < 24 of the six words, by bit tests on the word index (a select
// chain over an array's elements is folded into a dynamically indexed load,
// which puts the words in scratch memory)
__host__ __device__ __forceinline__ uint32_t ds_byte(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                                     uint32_t w4, uint32_t w5, int k) {
  const int q = k >> 2;
  const uint32_t a = (q & 1) ? w1 : w0, b = (q & 1) ? w3 : w2, c = (q & 1) ? w5 : w4;
  const uint32_t w = (q & 4) ? c : ((q & 2) ? b : a);
  return (w >> (8 * (k & 3))) & 255u;
}
__host__ __device__ __forceinline__ void ds_classify16_ff(const uint32_t wv[6], int64_t p0, int64_t L,
                                                          uint32_t &keep, uint32_t &rst, int &local_end) {
  // bytes j in [lo, hi) lie in the scan
  const int lo = p0 >= 0 ? 0 : (p0 <= -16 ? 16 : (int)-p0);
  const int64_t room = L - p0;
  const int hi = room <= 0 ? 0 : (room >= 16 ? 16 : (int)room);
  keep = hi > lo ? (((1u << hi) - 1u) & ~((1u << lo) - 1u)) : 0u;
  rst = 0;
  local_end = 16;
  const uint32_t w0 = wv[0], w1 = wv[1], w2 = wv[2], w3 = wv[3], w4 = wv[4], w5 = wv[5];
  const uint32_t ff = ds_ff4(w0) | (ds_ff4(w1) << 4) | (ds_ff4(w2) << 8) | (ds_ff4(w3) << 12) |
                      (ds_ff4(w4) << 16) | (ds_ff4(w5) << 20);
  // 0xFF bytes from the one before the lane's first (bit 0) to its last (16)
  uint32_t m = (ff >> 3) & 0x1FFFFu;
  while (m) {
    const int b = __builtin_ctz(m);
    m &= m - 1u;
    const int j = b - 1; // the 0xFF's byte (-1: the previous lane's last)
    const uint32_t nx_raw = ds_byte(w0, w1, w2, w3, w4, w5, b + 4);
    if (j >= 0) {
      const int64_t p = p0 + j;
      const bool in = p >= 0 && p < L;
      const bool next_in = p + 1 < L;
      const uint32_t nx = next_in ? nx_raw : 0u;
      if (nx != 0u) { // not a stuffed 0xFF: dropped
        keep &= ~(1u << j);
        const bool fill_rst = nx == 0xFFu || (nx >= 0xD0u && nx <= 0xD7u);
        if (!fill_rst && in && next_in && j < local_end) local_end = j; // end-of-scan marker
      }
    }
    // the byte after it, unless that is an 0xFF itself (its own rule)
    const int j1 = j + 1;
    if (j1 <= 15 && nx_raw != 0xFFu && p0 + j1 > 0) {
      if (nx_raw == 0u) {
        keep &= ~(1u << j1); // stuffing zero
      } else if (nx_raw >= 0xD0u && nx_raw <= 0xD7u) {
        keep &= ~(1u << j1); // RSTn code: segment boundary
        const int64_t p1 = p0 + j1;
        if (p1 >= 0 && p1 < L) rst |= 1u << j1;
      }
    }
  }
}

} // namespace ldt

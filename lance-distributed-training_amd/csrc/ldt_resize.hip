// ldt_resize.hip — fused source staging + Pillow BILINEAR Resize((224,224)) +
// ToTensor/Normalize store, banded two-pass form for gfx950.
//
// One 256-thread workgroup = one band of `bh` output rows of one image.
//   Phase A (per wave, no workgroup barrier): the 4 waves take the band's
//     source rows round-robin. A wave stages its row as planar R/G/B bytes in
//     a wave-private LDS buffer — 8 pixels per lane from vectorised plane loads
//     (Y: one 8-byte load; 4:2:0 chroma: three aligned dwords per row and
//     component), with libjpeg's h2v2 fancy upsampling and YCbCr->RGB done in
//     registers — then computes the row's 224x3 horizontal taps (Pillow
//     Resample.c, 22-bit fixed point, clip8) into the band's planar uint8
//     intermediate tmp[c][row][224] in LDS.
//   Phase B: the vertical taps read tmp one dword (4 output columns) per tap,
//     clip8, map through the ToTensor[/Normalize] float32 LUT and store float4
//     (16 B per lane, 896-B rows) into the CHW fp32 output.
// Reference semantics: lance_iterable.py:28-32 (Resize((224,224)), ToTensor),
// :31 (Normalize); jdsample.c h2v2_fancy_upsample, jdcolor.c ycc_rgb_convert,
// Pillow Resample.c ImagingResample (horizontal pass first, uint8 between).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldt_device.hpp"
#include "ldt_kernels.hpp"

namespace ldt {

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t ld32(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }

// 6 chroma samples of one plane row: columns cx0-1 .. cx0+4, edges clamped to
// [0, dw-1] (jdsample.c special first/last columns). cx0 % 4 == 0.
__device__ __forceinline__ void chroma6(const uint8_t *row, int cx0, int dw, int stride, int v[6]) {
  const uint32_t wc = ld32(row + cx0);
  const uint32_t wp = cx0 >= 4 ? ld32(row + cx0 - 4) : 0u;
  const uint32_t wn = (cx0 + 4 < stride) ? ld32(row + cx0 + 4) : 0u;
  int raw[6];
  raw[0] = (int)(wp >> 24);
  raw[1] = (int)(wc & 255);
  raw[2] = (int)((wc >> 8) & 255);
  raw[3] = (int)((wc >> 16) & 255);
  raw[4] = (int)(wc >> 24);
  raw[5] = (int)(wn & 255);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int col = cx0 - 1 + i;
    const int cc = col < 0 ? 0 : (col > dw - 1 ? dw - 1 : col);
    // the clamped column is always inside [cx0, cx0 + 4] here (x0 < W <= 2*dw)
    const int idx = cc - cx0 + 1;
    int val = raw[1];
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if (q == idx) val = raw[q];
    v[i] = val;
  }
}

__device__ __forceinline__ uint32_t pack4(const int *b) {
  return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}

__device__ __forceinline__ uint32_t rgbx(int r, int g, int b) {
  return (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16);
}

// Stage 8 pixels [x0, x0+8) of JPEG row y as RGBx dwords into an LDS row.
__device__ __forceinline__ void stage8_jpeg(const ImgDesc &d, const uint8_t *__restrict__ planes, int y,
                                            int x0, uint32_t *row) {
  const uint8_t *py = planes + d.plane_off[0] + (int64_t)y * d.plane_stride[0];
  const uint2 yy = *reinterpret_cast<const uint2 *>(py + x0);
  int Y[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    Y[j] = (int)((yy.x >> (8 * j)) & 255);
    Y[4 + j] = (int)((yy.y >> (8 * j)) & 255);
  }
  uint32_t px[8];
  if (d.color == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) px[j] = rgbx(Y[j], Y[j], Y[j]);
  } else {
    int Cb[8], Cr[8];
    const bool fast420 = d.hf[1] == 2 && d.vf[1] == 2 && d.hf[2] == 2 && d.vf[2] == 2 &&
                         d.cdw[1] > 2 && d.cdw[2] > 2;
    if (fast420) {
      const int cy = y >> 1;
      const int dh = d.cdh[1], dw = d.cdw[1];
      const int ny = (y & 1) ? min(cy + 1, dh - 1) : max(cy - 1, 0);
      const int cx0 = x0 >> 1;
      const int cs = d.plane_stride[1];
      const bool interior = cx0 >= 4 && cx0 + 4 <= dw - 1;
#pragma unroll
      for (int comp = 1; comp <= 2; ++comp) {
        const uint8_t *pl = planes + d.plane_off[comp];
        int a[6], bb[6], col[6];
        if (interior) {
          const uint8_t *r0 = pl + (int64_t)cy * cs + cx0, *r1 = pl + (int64_t)ny * cs + cx0;
          const uint32_t p0 = ld32(r0 - 4), c0 = ld32(r0), n0 = ld32(r0 + 4);
          const uint32_t p1 = ld32(r1 - 4), c1 = ld32(r1), n1 = ld32(r1 + 4);
          a[0] = (int)(p0 >> 24); bb[0] = (int)(p1 >> 24);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            a[1 + q] = (int)((c0 >> (8 * q)) & 255);
            bb[1 + q] = (int)((c1 >> (8 * q)) & 255);
          }
          a[5] = (int)(n0 & 255); bb[5] = (int)(n1 & 255);
        } else {
          chroma6(pl + (int64_t)cy * cs, cx0, dw, cs, a);
          chroma6(pl + (int64_t)ny * cs, cx0, dw, cs, bb);
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) col[i] = a[i] * 3 + bb[i];
        int *dst = comp == 1 ? Cb : Cr;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ci = (j >> 1) + 1;
          const int thiscol = col[ci];
          const int nextcol = (j & 1) ? col[ci + 1] : col[ci - 1];
          dst[j] = (thiscol * 3 + nextcol + 8 - (j & 1)) >> 4;
        }
      }
    } else {
      const uint8_t *pcb = planes + d.plane_off[1];
      const uint8_t *pcr = planes + d.plane_off[2];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int x = min(x0 + j, d.width - 1);
        Cb[j] = chroma_at(d, pcb, 1, x, y);
        Cr[j] = chroma_at(d, pcr, 2, x, y);
      }
    }
    if (d.color == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) px[j] = rgbx(Y[j], Cb[j], Cr[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int xcr = Cr[j] - 128, xcb = Cb[j] - 128;
        const int R = clampi(Y[j] + ((__mul24(91881, xcr) + 32768) >> 16), 0, 255);
        const int G = clampi(Y[j] + ((__mul24(-22554, xcb) + 32768 + __mul24(-46802, xcr)) >> 16), 0, 255);
        const int B = clampi(Y[j] + ((__mul24(116130, xcb) + 32768) >> 16), 0, 255);
        px[j] = rgbx(R, G, B);
      }
    }
  }
  uint4 *o = reinterpret_cast<uint4 *>(row + x0);
  o[0] = make_uint4(px[0], px[1], px[2], px[3]);
  o[1] = make_uint4(px[4], px[5], px[6], px[7]);
}

// Raw HWC: 16 pixels (48 bytes) per lane.
struct Raw16 {
  uint4 a, b, c;
};

__device__ __forceinline__ Raw16 load16_raw(const uint8_t *__restrict__ src_row, int W, int x0,
                                            bool aligned16) {
  Raw16 r;
  const uint8_t *p = src_row + 3 * x0;
  if (aligned16 && x0 + 16 <= W) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    r.a = q[0];
    r.b = q[1];
    r.c = q[2];
  } else {
    uint32_t w[12];
    const int nb = max(0, min(48, 3 * (W - x0)));
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      uint32_t v = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * i + e < nb) v |= (uint32_t)p[4 * i + e] << (8 * e);
      w[i] = v;
    }
    r.a = make_uint4(w[0], w[1], w[2], w[3]);
    r.b = make_uint4(w[4], w[5], w[6], w[7]);
    r.c = make_uint4(w[8], w[9], w[10], w[11]);
  }
  return r;
}

__device__ __forceinline__ void store16_raw(const Raw16 &r, int x0, uint32_t *row) {
  const uint32_t w[12] = {r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.y, r.b.z, r.b.w,
                          r.c.x, r.c.y, r.c.z, r.c.w};
  uint32_t px[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int o = 3 * j; // byte offset of pixel j within the 48 bytes
    const uint64_t pair = ((uint64_t)w[(o >> 2) + ((o >> 2) < 11 ? 1 : 0)] << 32) | w[o >> 2];
    px[j] = (uint32_t)(pair >> (8 * (o & 3))) & 0xFFFFFFu;
  }
  uint4 *d = reinterpret_cast<uint4 *>(row + x0);
#pragma unroll
  for (int q = 0; q < 4; ++q) d[q] = make_uint4(px[4 * q], px[4 * q + 1], px[4 * q + 2], px[4 * q + 3]);
}

struct Geom3 {
  int nbands, bh;
  int ring;  // power of two, >= ks_v + 8
  int ks_v;
  int wpad;  // staging row pixels (>= max width + KS), multiple of 16
};

// One workgroup = one band of output rows of one image, streaming its source
// rows once: waves take source rows round-robin (stage as RGBx dwords in a
// wave-private LDS row, horizontal taps with register-resident weights),
// intermediate rows go to an LDS ring, and output rows are finished as soon
// as their vertical window is complete.
template <int SRC, int KS>
__global__ void __launch_bounds__(256) k_resize3(const ImgDesc *__restrict__ descs,
                                                 const uint8_t *__restrict__ planes, RawSrc raw,
                                                 const float *__restrict__ lut,
                                                 const int64_t *__restrict__ labels,
                                                 float *__restrict__ out,
                                                 int64_t *__restrict__ out_labels,
                                                 const int32_t *__restrict__ status, int n, Geom3 gm) {
  const int Lb = blockIdx.x;
  const int g = Lb / (8 * gm.nbands), rr = Lb % (8 * gm.nbands);
  const int img = g * 8 + (rr % 8);
  const int band = rr / 8;
  if (img >= n) return;
  if (SRC == 0 && status[img] != 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int W, H;
  if constexpr (SRC == 0) {
    W = descs[img].width;
    H = descs[img].height;
  } else {
    W = raw.w;
    H = raw.h;
  }
  const int bh = gm.bh, ks_v = gm.ks_v, ring = gm.ring;
  const int oy0 = band * bh;
  const int nb_rows = min(bh, kOut - oy0);
  if (nb_rows <= 0) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float *s_lut = reinterpret_cast<float *>(smem);            // 768 f32
  int32_t *s_kv = reinterpret_cast<int32_t *>(smem + 3072);  // bh * ks_v
  int32_t *s_vb = s_kv + bh * ks_v;                          // bh * 2
  int32_t *s_hx = s_vb + 2 * bh;                             // 224 xmin
  uint8_t *s_tmp = reinterpret_cast<uint8_t *>(
      ((uintptr_t)(s_hx + kOut) + 15) & ~(uintptr_t)15);     // 3 * ring * 224
  uint32_t *s_rows = reinterpret_cast<uint32_t *>(s_tmp + 3 * ring * kOut); // 4 * wpad
  int32_t *s_kh = reinterpret_cast<int32_t *>(s_rows);       // setup only: 224 * KS

  for (int i = tid; i < 768; i += 256) s_lut[i] = lut[i];
  if (tid < kOut) {
    int xmin;
    resample_coeffs_one(W, kOut, tid, KS, s_kh + tid * KS, &xmin);
    s_hx[tid] = xmin;
  }
  // vertical coefficients of every band row (bands can be taller than 32 rows)
  for (int j = (tid + 32) & 255; j < nb_rows; j += 256) {
    int ymin;
    const int cnt = resample_coeffs_one(H, kOut, oy0 + j, ks_v, s_kv + j * ks_v, &ymin);
    s_vb[2 * j] = ymin;
    s_vb[2 * j + 1] = cnt;
  }
  if (band == 0 && tid == 0 && labels != nullptr) out_labels[img] = labels[img];
  __syncthreads();
  // horizontal weights of this lane's output columns ox = lane + 64q, in registers
  int32_t wgt[4][KS];
  int xm[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int ox = lane + 64 * q;
    const bool v = ox < kOut;
    xm[q] = v ? s_hx[ox] : 0;
#pragma unroll
    for (int t = 0; t < KS; ++t) wgt[q][t] = v ? s_kh[ox * KS + t] : 0;
  }
  __syncthreads(); // s_kh aliases the staging rows
  const int ya = max(s_vb[0], 0);
  const int yb = min(s_vb[2 * (nb_rows - 1)] + s_vb[2 * (nb_rows - 1) + 1], H);
  const int nrows = yb - ya;
  uint32_t *myrow = s_rows + wave * gm.wpad;

  const ImgDesc *dp = SRC == 0 ? descs + img : nullptr;
  const uint8_t *raw_cell = SRC == 1 ? raw.base + (int64_t)img * raw.cell_stride : nullptr;
  const bool raw_al16 = SRC == 1 && ((((uintptr_t)raw_cell) & 15) == 0) && ((W * 3) & 15) == 0;
  Raw16 pf;  // raw: prefetched first 16-pixel chunk of this wave's next row
  if constexpr (SRC == 1) {
    if (raw_al16 && wave < nrows)
      pf = load16_raw(raw_cell + (int64_t)(ya + wave) * W * 3, W, lane * 16, true);
  }
  int next_oy = 0;
  const int vc = tid / 56, vox4 = (tid % 56) * 4; // vertical-pass mapping (tid < 168)
  for (int r0 = 0; r0 < nrows; r0 += 4) {
    const int r = r0 + wave;
    if (r < nrows) {
      const int y = ya + r;
      if constexpr (SRC == 1) {
        const uint8_t *srow = raw_cell + (int64_t)y * W * 3;
        if (raw_al16) {
          // register prefetch of this wave's next row (aligned fast path)
          const Raw16 cur = pf;
          if (r + 4 < nrows) pf = load16_raw(srow + (int64_t)4 * W * 3, W, lane * 16, true);
          if (lane * 16 < W) store16_raw(cur, lane * 16, myrow);
        } else if (lane * 16 < W) {
          store16_raw(load16_raw(srow, W, lane * 16, false), lane * 16, myrow);
        }
        for (int x0 = lane * 16 + 1024; x0 < W; x0 += 1024)
          store16_raw(load16_raw(srow, W, x0, raw_al16), x0, myrow);
      } else {
        for (int x0 = lane * 8; x0 < W; x0 += 512) stage8_jpeg(*dp, planes, y, x0, myrow);
      }
      wave_sync_lds();
      const int slot = r & (ring - 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ox = lane + 64 * q;
        if (ox < kOut) {
          int32_t a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
          const uint32_t *src = myrow + xm[q];
#pragma unroll
          for (int t = 0; t < KS; ++t) {
            const uint32_t v = src[t];
            const uint32_t kw = (uint32_t)wgt[q][t]; // Pillow weights: 0 <= kw <= 2^22
            a0 += (int32_t)__umul24(v & 255, kw);
            a1 += (int32_t)__umul24((v >> 8) & 255, kw);
            a2 += (int32_t)__umul24((v >> 16) & 255, kw);
          }
          s_tmp[(0 * ring + slot) * kOut + ox] = (uint8_t)clip8(a0);
          s_tmp[(1 * ring + slot) * kOut + ox] = (uint8_t)clip8(a1);
          s_tmp[(2 * ring + slot) * kOut + ox] = (uint8_t)clip8(a2);
        }
      }
    }
    __syncthreads();
    const int done = min(nrows, r0 + 4);
    // finish every output row whose vertical window is complete
    while (next_oy < nb_rows && s_vb[2 * next_oy] - ya + s_vb[2 * next_oy + 1] <= done) {
      const int j = next_oy++;
      if (tid < 168) {
        const int ymin = s_vb[2 * j] - ya, cnt = s_vb[2 * j + 1];
        const int32_t *kv = s_kv + j * ks_v;
        int32_t a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0, a3 = a0;
        for (int t = 0; t < cnt; ++t) {
          const int slot = (ymin + t) & (ring - 1);
          const uint32_t v = *reinterpret_cast<const uint32_t *>(s_tmp + (vc * ring + slot) * kOut + vox4);
          const uint32_t kw = (uint32_t)kv[t];
          a0 += (int32_t)__umul24(v & 255, kw);
          a1 += (int32_t)__umul24((v >> 8) & 255, kw);
          a2 += (int32_t)__umul24((v >> 16) & 255, kw);
          a3 += (int32_t)__umul24(v >> 24, kw);
        }
        const float *lc = s_lut + vc * 256;
        float4 f;
        f.x = lc[clip8(a0)];
        f.y = lc[clip8(a1)];
        f.z = lc[clip8(a2)];
        f.w = lc[clip8(a3)];
        *reinterpret_cast<float4 *>(out + (((int64_t)img * 3 + vc) * kOut + oy0 + j) * kOut + vox4) = f;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Launch geometry. Horizontal taps are compiled per tap count (KS = 3 .. 19,
// sources up to 2016 px wide); wider sources use the streaming k_resize.
// Bands: enough workgroups to fill 256 CUs several times over (>= ~2048).
// ---------------------------------------------------------------------------
static size_t geom3_lds(const Geom3 &g, int ks_h) {
  size_t b = 3072 + 4 * ((size_t)g.bh * g.ks_v + 2 * g.bh + kOut);
  b = (b + 15) & ~(size_t)15;
  size_t rows = 4 * 4 * (size_t)g.wpad;
  const size_t kh = 4 * (size_t)kOut * ks_h;
  if (rows < kh) rows = kh;
  return b + 3 * (size_t)g.ring * kOut + rows;
}

static bool make_geom3(int n, int max_w, int max_h, int ks_h, Geom3 &g) {
  g.ks_v = resample_ksize_host(max_h, kOut);
  int ring = 16;
  while (ring < g.ks_v + 8) ring *= 2;
  g.ring = ring;
  int nb = (2048 + n - 1) / n;
  if (nb < 1) nb = 1;
  if (nb > 28) nb = 28;
  g.bh = (kOut + nb - 1) / nb;
  g.nbands = (kOut + g.bh - 1) / g.bh;
  g.wpad = ((max_w + ks_h + 15) / 16) * 16 + 16;
  return geom3_lds(g, ks_h) <= 128 * 1024;
}

template <int SRC, int KS>
static hipError_t launch3(const ImgDesc *descs, const uint8_t *planes, RawSrc raw, const float *lut,
                          const int64_t *labels, float *out, int64_t *out_labels,
                          const int32_t *status, int n, const Geom3 &g, hipStream_t s) {
  static hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_resize3<SRC, KS>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  const int groups = (n + 7) / 8;
  hipLaunchKernelGGL((k_resize3<SRC, KS>), dim3(groups * 8 * g.nbands), dim3(256), geom3_lds(g, KS),
                     s, descs, planes, raw, lut, labels, out, out_labels, status, n, g);
  return hipGetLastError();
}

template <int SRC>
static bool dispatch3(int ks_h, const ImgDesc *descs, const uint8_t *planes, RawSrc raw,
                      const float *lut, const int64_t *labels, float *out, int64_t *out_labels,
                      const int32_t *status, int n, const Geom3 &g, hipStream_t s, hipError_t *err) {
  switch (ks_h) {
  case 3: *err = launch3<SRC, 3>(descs, planes, raw, lut, labels, out, out_labels, status, n, g, s); return true;
  case 5: *err = launch3<SRC, 5>(descs, planes, raw, lut, labels, out, out_labels, status, n, g, s); return true;
  case 7: *err = launch3<SRC, 7>(descs, planes, raw, lut, labels, out, out_labels, status, n, g, s); return true;
  case 9: *err = launch3<SRC, 9>(descs, planes, raw, lut, labels, out, out_labels, status, n, g, s); return true;
  case 11: *err = launch3<SRC, 11>(descs, planes, raw, lut, labels, out, out_labels, status, n, g, s); return true;
  case 13: *err = launch3<SRC, 13>(descs, planes, raw, lut, labels, out, out_labels, status, n, g, s); return true;
  case 15: *err = launch3<SRC, 15>(descs, planes, raw, lut, labels, out, out_labels, status, n, g, s); return true;
  case 17: *err = launch3<SRC, 17>(descs, planes, raw, lut, labels, out, out_labels, status, n, g, s); return true;
  case 19: *err = launch3<SRC, 19>(descs, planes, raw, lut, labels, out, out_labels, status, n, g, s); return true;
  default: return false;
  }
}

bool launch_resize2_jpeg(const DevPlan &p, const DevWork &w, float *out, int64_t *out_labels,
                         hipStream_t s, hipError_t *err) {
  Geom3 g;
  const int ks_h = resample_ksize_host(p.max_w, kOut);
  if (!make_geom3(p.n, p.max_w, p.max_h, ks_h, g)) return false;
  RawSrc raw{nullptr, 0, 0, 0};
  return dispatch3<0>(ks_h, p.descs, w.planes, raw, p.lut, p.labels, out, out_labels, w.status, p.n,
                      g, s, err);
}

bool launch_resize2_raw(const uint8_t *hwc, int64_t cell_stride, int n, int h, int wd,
                        const float *lut, float *out, hipStream_t s, hipError_t *err) {
  Geom3 g;
  const int ks_h = resample_ksize_host(wd, kOut);
  if (!make_geom3(n, wd, h, ks_h, g)) return false;
  RawSrc raw{hwc, cell_stride, h, wd};
  return dispatch3<1>(ks_h, (const ImgDesc *)nullptr, (const uint8_t *)nullptr, raw, lut,
                      (const int64_t *)nullptr, out, (int64_t *)nullptr, (const int32_t *)nullptr, n,
                      g, s, err);
}

} // namespace ldt

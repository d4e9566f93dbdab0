// ldt_resize4.hip — fused source staging + Pillow BILINEAR Resize((224,224)) +
// ToTensor/Normalize store, one wavefront per band of output rows.
//
// Every wave owns one (image, band) task and runs it alone: it streams the
// band's source rows two at a time, stages them as RGBx dwords in a
// wave-private LDS buffer (raw HWC bytes, or JPEG planes with libjpeg's h2v2
// fancy upsampling and YCbCr->RGB done in registers), computes the rows'
// 224x3 horizontal taps (Pillow Resample.c, 22-bit fixed point, clip8) into a
// wave-private LDS ring of uint8 rows, and finishes every output row whose
// vertical window is complete: vertical taps, clip8, the ToTensor[/Normalize]
// float32 LUT and float4 stores into the CHW fp32 output. There is no
// workgroup barrier after the prologue, so the waves of a CU overlap their
// loads and arithmetic freely; the next row pair is prefetched into registers
// while the current one is computed.
//
// Reference semantics: lance_iterable.py:28-32 (Resize((224,224)), ToTensor),
// :31 (Normalize); jdsample.c h2v2_fancy_upsample, jdcolor.c ycc_rgb_convert,
// Pillow Resample.c ImagingResample (horizontal pass first, uint8 between).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "ldt_device.hpp"
#include "ldt_kernels.hpp"

namespace ldt {

namespace {

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Lane l receives lane l-1's value (lane 0 keeps its own): DPP wave_shr:1.
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xF, 0xF, false);
}
// Lane l receives lane l+1's value (lane 63 keeps its own): DPP wave_shl:1.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x130, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t rgbx(int r, int g, int b) {
  return (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16);
}

// jdcolor.c ycc_rgb_convert (16-bit fixed point, ONE_HALF in the Cb->G term).
// Every factor fits 24 bits, so the products are v_mul_i32_i24 (full rate)
// rather than the quarter-rate v_mul_lo_u32 the compiler would pick.
__device__ __forceinline__ uint32_t ycc_px(int y, int cb, int cr) {
  const int xcr = cr - 128, xcb = cb - 128;
  const int r = y + ((__mul24(91881, xcr) + 32768) >> 16);
  const int g = y + ((__mul24(-22554, xcb) + 32768 + __mul24(-46802, xcr)) >> 16);
  const int b = y + ((__mul24(116130, xcb) + 32768) >> 16);
  return rgbx(clampi(r, 0, 255), clampi(g, 0, 255), clampi(b, 0, 255));
}

struct Raw16 {
  uint4 a, b, c;
};

__device__ __forceinline__ Raw16 load16_aligned(const uint8_t *p) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  Raw16 r;
  r.a = q[0];
  r.b = q[1];
  r.c = q[2];
  return r;
}

// Bytes [3*x0, 3*x0 + 48) of a row, any alignment, zero past the row end.
__device__ __forceinline__ Raw16 load16_any(const uint8_t *row, int W, int x0) {
  const uint8_t *p = row + 3 * x0;
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
  Raw16 r;
  r.a = make_uint4(w[0], w[1], w[2], w[3]);
  r.b = make_uint4(w[4], w[5], w[6], w[7]);
  r.c = make_uint4(w[8], w[9], w[10], w[11]);
  return r;
}

// Staging rows are skewed by 4 dwords per 32 pixels: the horizontal taps of
// neighbouring output columns start ~scale pixels apart, and for 224-wide
// outputs of 512 / 1024 (scale 16/7, 32/7) every 7th lane would otherwise hit
// the same LDS bank (4-5-way conflicts on every tap). Blocks of 8 or 16
// pixels starting at a multiple of 8 stay contiguous and 16-byte aligned.
template <bool SKEW = true> __device__ __forceinline__ int skw(int x) {
  return SKEW ? x + ((x >> 5) << 2) : x;
}

// 16 packed RGB pixels -> 16 RGBx dwords at pixels [x0, x0+16) of a staging
// row. The byte above B is left as whatever follows (the taps read bytes 0..2).
template <bool SKEW>
__device__ __forceinline__ void stage16_raw(const Raw16 &r, uint32_t *row, int x0) {
  const uint32_t w[13] = {r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.y, r.b.z, r.b.w,
                          r.c.x, r.c.y, r.c.z, r.c.w, 0u};
  uint32_t px[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int o = 3 * j;
    px[j] = __builtin_amdgcn_alignbyte(w[(o >> 2) + 1], w[o >> 2], (uint32_t)(o & 3));
  }
  uint4 *d = reinterpret_cast<uint4 *>(row + skw<SKEW>(x0));
#pragma unroll
  for (int q = 0; q < 4; ++q) d[q] = make_uint4(px[4 * q], px[4 * q + 1], px[4 * q + 2], px[4 * q + 3]);
}

// One JPEG row pair's registers for the 4:2:0 fast path (lane = 8 pixels).
struct Jpair {
  uint2 y0, y1;        // luma rows 2cy, 2cy+1 (8 px each)
  uint32_t c[2][3];    // chroma comp (Cb, Cr) x row (cy-1, cy, cy+1), 4 samples each
};

__device__ __forceinline__ void bytes6(uint32_t w, int lane, int rc, int s[6]) {
  const uint32_t p = from_prev_lane(w), n = from_next_lane(w);
  s[0] = (int)(p >> 24);
  s[1] = (int)(w & 255);
  s[2] = (int)((w >> 8) & 255);
  s[3] = (int)((w >> 16) & 255);
  s[4] = (int)(w >> 24);
  s[5] = (int)(n & 255);
  // column -1 -> column 0; columns past downsampled_width - 1 -> that column
  // (jdsample.c special first/last columns, context rows replicated)
  s[0] = lane == 0 ? s[1] : s[0];
  int e = s[1];
#pragma unroll
  for (int i = 2; i <= 5; ++i) e = rc == i ? s[i] : e;
#pragma unroll
  for (int i = 2; i <= 5; ++i) s[i] = i > rc ? e : s[i];
}

// ---- packed 16-bit fancy upsampling (SRC 5) ----
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_pk(uint32_t v) { return __builtin_bit_cast(u16x2, v); }

// A chroma row's upsampling context, columns 4*lane-1 .. 4*lane+4 (jdsample.c
// edge rules: column -1 -> column 0, columns past the last one -> the last),
// as six (cb, cr) u16x2 pairs built by v_perm_b32 from the Cb and Cr dwords
// (4 samples each) and the neighbouring lanes', with per-lane byte selectors
// that encode the edge rules once (0x0C selects a zero byte). The fancy
// upsampling's packed 16-bit arithmetic then covers both components at once,
// and each output pixel's (cb, cr) arrives in one register (round 5: 377 ->
// 348 VALU per staged row pair against one component per register,
// standalone c2 resize 0.149 -> 0.146 ms, profiles/r5/resize_cc_r5.txt). Selectors per lane: q[i]
// for i = 1..4 from (M_hi, M_lo) (own samples, clamped to the last valid
// column), q[0] from (previous lane's M_hi, M_lo) (lane 0: its own column 0),
// q[5] from (next lane's M_lo, M_lo or M_hi) (the last valid lane: its own
// last column).
struct CC6 {
  u16x2 q[6];
};

__device__ __forceinline__ void cc_selectors(int lane, int rc, uint32_t sel[6], bool &x_lo) {
  auto pair = [](uint32_t b) { return b | (0x0Cu << 8) | ((b + 1u) << 16) | (0x0Cu << 24); };
  sel[0] = lane == 0 ? pair(0u) : pair(6u);
#pragma unroll
  for (int i = 1; i <= 4; ++i) sel[i] = pair(2u * (uint32_t)(min(i, rc) - 1));
  // q[5]: next lane's column 0 (bytes 4, 5 of (Mn, X)), or own column rc - 1
  // in X = M_lo (rc <= 2) or M_hi
  x_lo = rc <= 2;
  sel[5] = rc == 5 ? pair(4u) : pair(2u * (uint32_t)((rc - 1) & 1));
}

__device__ __forceinline__ CC6 cc_pairs(uint32_t cbw, uint32_t crw, const uint32_t sel[6], bool x_lo) {
  const uint32_t mlo = __builtin_amdgcn_perm(crw, cbw, 0x05010400u); // cb0 cr0 cb1 cr1
  const uint32_t mhi = __builtin_amdgcn_perm(crw, cbw, 0x07030602u); // cb2 cr2 cb3 cr3
  const uint32_t mp = from_prev_lane(mhi), mn = from_next_lane(mlo);
  CC6 r;
  r.q[0] = as_pk(__builtin_amdgcn_perm(mp, mlo, sel[0]));
#pragma unroll
  for (int i = 1; i <= 4; ++i) r.q[i] = as_pk(__builtin_amdgcn_perm(mhi, mlo, sel[i]));
  r.q[5] = as_pk(__builtin_amdgcn_perm(mn, x_lo ? mlo : mhi, sel[5]));
  return r;
}


} // namespace

struct Geom4 {
  int nbands, bh;  // bands per image, output rows per band
  int ring;        // intermediate ring rows (>= ks_v + 1)
  int ks_v;        // vertical taps (max over the batch)
  int spad;        // staging row stride in dwords (multiple of 4)
  int ntask;       // n * nbands
  int wave_bytes;  // LDS per wave
  int fill;        // JPEG: this launch zero-fills failed images' bands (label -100)
  int wpg;         // waves (tasks) per workgroup
  int rgbx;        // ring rows of RGBx dwords (JPEG sources) instead of three byte planes
};

constexpr int kKvRows = 8; // vertical coefficient rows cached per wave
// Waves (tasks) per workgroup. Raw sources: two. JPEG sources: four, which
// hold 12 waves per CU with the RGBx ring (3 KB LUT + 4 x 11.5 KB at 512 px:
// 3 workgroups; 2-wave workgroups of 26 KB fit only 5 per CU and measured
// 0.183 vs 0.150 ms standalone, profiles/r5/resize_rgbx_wg_r5wg.txt). No
// resize workgroup shares a CU with a k_huff_image workgroup usefully: one
// that fits (1 wave, <= 128 VGPRs) slows the decoder's rounds more than it
// gains (profiles/r5/resize_coresident_ab_r5co.txt).
constexpr int kResizeWaves = 2;
constexpr int kResizeWavesJpeg = 4;

// SRC: 0 JPEG planes, 4:2:0 fast staging (resize_fast420 images only);
// 2 JPEG planes, generic staging (the other images); 1 raw HWC rows, 16-byte
// aligned; 3 raw HWC rows, any alignment. Each variant is its own kernel so
// the waitcnt pass never sees another path's loads pending at the loop's
// merge points (that forced a vmcnt(0) ahead of the horizontal taps and
// serialised the prefetch).
// SRC 5: the 4:2:0 fast path on packed 16-bit pairs (the default).
template <int SRC, int KS>
__device__ __forceinline__ void resize4_body(const ImgDesc *__restrict__ descs,
                                             const uint8_t *__restrict__ planes, RawSrc raw,
                                             const float *__restrict__ lut,
                                             const int64_t *__restrict__ labels,
                                             float *__restrict__ out,
                                             int64_t *__restrict__ out_labels,
                                             const int32_t *__restrict__ status, const Geom4 &g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // Skewed staging for raw rows (c5: 4-5-way tap conflicts otherwise, and the
  // kernel is LDS-bound). JPEG rows stay plain (the
  // skew's per-tap selects took k_resize4<5,7> to 190 VGPRs, 2 waves per
  // SIMD, 0.153 -> 0.175 ms at c2 with half the bank conflicts; blocked rows
  // with a halo copy, 2-way banks at 148 VGPRs, measured 0.155 vs 0.152 ms).
  constexpr bool kJpeg = SRC == 0 || SRC == 2 || SRC == 5;
  constexpr bool kSkew = !kJpeg;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float *s_lut = reinterpret_cast<float *>(smem);
  for (int i = tid; i < 768; i += (int)blockDim.x) s_lut[i] = lut[i];
  __syncthreads(); // the only workgroup barrier
  // wave-uniform task: descriptor loads become scalar loads into SGPRs
  const int task = __builtin_amdgcn_readfirstlane((int)blockIdx.x * g.wpg + wave);
  if (task >= g.ntask) return;
  const int img = task / g.nbands, band = task - img * g.nbands;
  if (kJpeg && status[img] != 0) {
    // a failed image's band: zeros (and label -100), by one of the launches
    const int oy0 = band * g.bh, nb = min(g.bh, kOut - oy0);
    if (!g.fill || nb <= 0) return;
    if (band == 0 && lane == 0 && out_labels != nullptr) out_labels[img] = -100;
    float4 *o = reinterpret_cast<float4 *>(out + (int64_t)img * 3 * kOut * kOut + oy0 * kOut);
    const int per = nb * kOut / 4; // float4s of the band in one channel plane
    for (int c = 0; c < 3; ++c)
      for (int i = lane; i < per; i += 64) o[c * (kOut * kOut / 4) + i] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  if (kJpeg && resize_fast420(descs[img]) != (SRC == 0 || SRC == 5)) return;
  int W, H;
  if constexpr (kJpeg) {
    W = descs[img].width;
    H = descs[img].height;
  } else {
    W = raw.w;
    H = raw.h;
  }
  const int oy0 = band * g.bh;
  const int nb = min(g.bh, kOut - oy0);
  if (nb <= 0) return;
  if (band == 0 && lane == 0 && labels != nullptr) out_labels[img] = labels[img];

  uint8_t *wbase = smem + 3072 + wave * g.wave_bytes;
  uint32_t *stg = reinterpret_cast<uint32_t *>(wbase);               // 2 * spad dwords
  // the intermediate ring: JPEG sources keep RGBx dwords per column (one
  // 4-byte store per column and row, one 16-byte read of 4 columns per
  // vertical tap); raw sources three byte planes (their larger rings would
  // cost a workgroup per CU as dwords)
  constexpr bool kRgbx = kJpeg;
  uint8_t *ring = wbase + 8 * g.spad;                                // (kRgbx ? 4 : 3) * ring * 224
  int32_t *kv = reinterpret_cast<int32_t *>(ring + (kRgbx ? 4 : 3) * g.ring * kOut); // kKvRows * ks_v
  int32_t *vb = kv + kKvRows * g.ks_v;                               // kKvRows * 2
  const int ks_v = g.ks_v, RING = g.ring;

  // horizontal weights of this lane's output columns, in registers:
  // q = 0..2 -> column lane + 64q of both rows; q = 3 -> column 192 + lane%32
  // of row (lane / 32)
  int32_t wgt[4][KS];
  int xm[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int ox = q < 3 ? lane + 64 * q : 192 + (lane & 31);
    int32_t k[KS];
    resample_coeffs_one(W, kOut, ox, KS, k, &xm[q]);
#pragma unroll
    for (int t = 0; t < KS; ++t) wgt[q][t] = k[t];
  }
  // skewed staging address of each window start, and the first tap past a skew step
  int xsk[4], xcr[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    xsk[q] = skw<kSkew>(xm[q]);
    xcr[q] = 32 - (xm[q] & 31);
  }
  // band source rows
  int ya, yb;
  {
    int32_t kk[32];
    int ymin_a, ymin_b;
    resample_coeffs_one(H, kOut, oy0, 0, kk, &ymin_a);
    const int cnt_b = resample_coeffs_one(H, kOut, oy0 + nb - 1, 0, kk, &ymin_b);
    ya = ymin_a;
    yb = ymin_b + cnt_b;
  }
  const int ya0 = kJpeg ? (ya & ~1) : ya;

  // vertical-pass items: 168 dwords (3 channels x 56 groups of 4 columns)
  int vc[3], vo[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int it = min(lane + 64 * i, 167);
    vc[i] = it / 56;
    vo[i] = (it - vc[i] * 56) * 4;
  }

  // JPEG fast path: 4:2:0 with both chroma planes fancy-upsampled, W <= 512
  constexpr bool fast420 = SRC == 0 || SRC == 5;
  constexpr bool kPk = SRC == 5; // packed 16-bit fancy upsampling, (cb, cr) pairs
  int rc = 5, cdh = 1;
  // plane geometry copied to registers once: the wave fences in process()
  // would otherwise make every fetch reload it (a dependent global round trip
  // per plane load, which serialised the prefetch)
  int64_t po0 = 0, po1 = 0, po2 = 0;
  int ps0 = 0, ps1 = 0;
  const ImgDesc *dp = nullptr;
  const uint8_t *raw_cell = nullptr;
  uint32_t csel[6] = {0u, 0u, 0u, 0u, 0u, 0u};
  bool cx_lo = false;
  constexpr bool raw_al16 = SRC == 1;
  if constexpr (kJpeg) {
    dp = descs + img;
    const ImgDesc &d = *dp;
    const int dw = d.cdw[1];
    rc = lane == (dw - 1) / 4 ? (dw - 1) % 4 + 1 : 5;
    cdh = d.cdh[1];
    if constexpr (kPk) cc_selectors(lane, rc, csel, cx_lo);
    po0 = d.plane_off[0];
    po1 = d.plane_off[1];
    po2 = d.plane_off[2];
    ps0 = d.plane_stride[0];
    ps1 = d.plane_stride[1];
  } else {
    raw_cell = raw.base + (int64_t)img * raw.cell_stride;
  }

  // ---- prefetch helpers ----
  struct Pre {
    Jpair jp;
    Raw16 r0, r1;
  } pa;
  auto fetch = [&](Pre &pf, int y) {
    Jpair &jp = pf.jp;
    if constexpr (kJpeg) {
      if constexpr (fast420) {
        const int x0 = lane * 8;
        const uint8_t *py = planes + po0 + (int64_t)y * ps0 + x0;
        jp.y0 = x0 < W ? *reinterpret_cast<const uint2 *>(py) : make_uint2(0, 0);
        jp.y1 = (x0 < W && y + 1 < H) ? *reinterpret_cast<const uint2 *>(py + ps0) : make_uint2(0, 0);
        const int cy = y >> 1;
        const int rows[3] = {max(cy - 1, 0), cy, min(cy + 1, cdh - 1)};
        const int cx0 = lane * 4;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int r = 0; r < 3; ++r)
            jp.c[c][r] = cx0 < ps1 ? *reinterpret_cast<const uint32_t *>(planes + (c ? po2 : po1) +
                                                                         (int64_t)rows[r] * ps1 + cx0)
                                   : 0u;
      }
    } else {
      if constexpr (raw_al16) {
        const int x0 = lane * 16;
        if (x0 < W) {
          pf.r0 = load16_aligned(raw_cell + (int64_t)y * W * 3 + 3 * x0);
          if (y + 1 < H) pf.r1 = load16_aligned(raw_cell + (int64_t)(y + 1) * W * 3 + 3 * x0);
        }
      }
    }
  };

  // ---- staging of one row pair into stg[0..spad) / stg[spad..2 spad) ----
  auto stage = [&](const Pre &pf, int y) {
    const Jpair &jp = pf.jp;
    uint32_t *s0 = stg, *s1 = stg + g.spad;
    if constexpr (kJpeg) {
      const ImgDesc &d = *dp;
      if constexpr (kPk) {
        // h2v2 fancy upsampling on (cb, cr) pairs, then jdcolor.c
        // ycc_rgb_convert with the pair in one register: each channel's value
        // before the >> 16, with Y << 16 and the -128 offsets folded into
        // constants (y + ((91881 (cr - 128) + 32768) >> 16) = (Y16 + 91881 cr
        // + 32768 - 91881 * 128) >> 16, an arithmetic shift), clamped to
        // [0, 2^24) so that byte 2 is the channel; G's two chroma products by
        // one v_dot2_u32_u16
        const int x0 = lane * 8;
        const CC6 U = cc_pairs(jp.c[0][0], jp.c[1][0], csel, cx_lo);
        const CC6 A = cc_pairs(jp.c[0][1], jp.c[1][1], csel, cx_lo);
        const CC6 D = cc_pairs(jp.c[0][2], jp.c[1][2], csel, cx_lo);
        const u16x2 three = {3, 3}, c8 = {8, 8}, c7 = {7, 7};
        const u16x2 wg = {22554, 46802};
        constexpr uint32_t kKg = 32768u + (22554u + 46802u) * 128u;
        constexpr int32_t kKr = 32768 - 91881 * 128 - (int32_t)kKg, kKb = 32768 - 116130 * 128 - (int32_t)kKg;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const CC6 &F = r ? D : U;
          u16x2 T[6];
#pragma unroll
          for (int i = 0; i < 6; ++i) T[i] = A.q[i] * three + F.q[i];
          uint32_t px[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int k = j >> 1;
            const u16x2 P = (j & 1) ? (T[k + 1] * three + T[k + 2] + c7) >> 4 : (T[k + 1] * three + T[k] + c8) >> 4;
            const uint32_t pw = __builtin_bit_cast(uint32_t, P);
            const uint32_t yw = r ? (j < 4 ? jp.y1.x : jp.y1.y) : (j < 4 ? jp.y0.x : jp.y0.y);
            const uint32_t yk = __builtin_amdgcn_perm(0u, yw, 0x0C000C0Cu | ((uint32_t)(j & 3) << 16)) + kKg;
            const int rr = (int)(yk + __umul24(pw >> 16, 91881u) + (uint32_t)kKr);
            const int gg = (int)(yk - __builtin_amdgcn_udot2(P, wg, 0u, false));
            const int bb = (int)(yk + __umul24((uint32_t)(uint16_t)pw, 116130u) + (uint32_t)kKb);
            const uint32_t xr = (uint32_t)min(max(rr, 0), 0xFFFFFF), xg = (uint32_t)min(max(gg, 0), 0xFFFFFF),
                           xb = (uint32_t)min(max(bb, 0), 0xFFFFFF);
            px[j] = __builtin_amdgcn_perm(xb, __builtin_amdgcn_perm(xg, xr, 0x0C0C0602u), 0x0C060100u);
          }
          if (x0 < W) {
            uint4 *dq = reinterpret_cast<uint4 *>((r ? s1 : s0) + x0);
            dq[0] = make_uint4(px[0], px[1], px[2], px[3]);
            dq[1] = make_uint4(px[4], px[5], px[6], px[7]);
          }
        }
      } else if constexpr (fast420) {
        const int x0 = lane * 8;
        int cb[2][8], crr[2][8];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          int A[6], U[6], D[6];
          bytes6(jp.c[c][1], lane, rc, A);
          bytes6(jp.c[c][0], lane, rc, U);
          bytes6(jp.c[c][2], lane, rc, D);
          int T[6], B[6];
#pragma unroll
          for (int i = 0; i < 6; ++i) {
            T[i] = A[i] * 3 + U[i];
            B[i] = A[i] * 3 + D[i];
          }
          int *o0 = c == 0 ? cb[0] : crr[0];
          int *o1 = c == 0 ? cb[1] : crr[1];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int ci = (j >> 1) + 1;
            const int nt = (j & 1) ? T[ci + 1] : T[ci - 1];
            const int nbv = (j & 1) ? B[ci + 1] : B[ci - 1];
            o0[j] = (T[ci] * 3 + nt + 8 - (j & 1)) >> 4;
            o1[j] = (B[ci] * 3 + nbv + 8 - (j & 1)) >> 4;
          }
        }
        uint32_t p0[8], p1[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t ya_ = j < 4 ? jp.y0.x : jp.y0.y, yb_ = j < 4 ? jp.y1.x : jp.y1.y;
          const int sh = 8 * (j & 3);
          p0[j] = ycc_px((int)((ya_ >> sh) & 255), cb[0][j], crr[0][j]);
          p1[j] = ycc_px((int)((yb_ >> sh) & 255), cb[1][j], crr[1][j]);
        }
        if (x0 < W) {
          uint4 *d0 = reinterpret_cast<uint4 *>(s0 + skw<kSkew>(x0));
          uint4 *d1 = reinterpret_cast<uint4 *>(s1 + skw<kSkew>(x0));
          d0[0] = make_uint4(p0[0], p0[1], p0[2], p0[3]);
          d0[1] = make_uint4(p0[4], p0[5], p0[6], p0[7]);
          d1[0] = make_uint4(p1[0], p1[1], p1[2], p1[3]);
          d1[1] = make_uint4(p1[4], p1[5], p1[6], p1[7]);
        }
      } else {
        // generic: any supported sampling, gray, RGB, wide images
        const uint8_t *pl0 = planes + d.plane_off[0];
        for (int r = 0; r < 2; ++r) {
          const int yy = y + r;
          if (yy >= H) break;
          uint32_t *sr = r ? s1 : s0;
          for (int x0 = lane * 8; x0 < W; x0 += 512) {
            uint32_t px[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int x = min(x0 + j, W - 1);
              const int Y = pl0[(int64_t)yy * d.plane_stride[0] + x];
              if (d.color == 2) {
                px[j] = rgbx(Y, Y, Y);
              } else {
                const int cb = chroma_at(d, planes + d.plane_off[1], 1, x, yy);
                const int cr = chroma_at(d, planes + d.plane_off[2], 2, x, yy);
                px[j] = d.color == 1 ? rgbx(Y, cb, cr) : ycc_px(Y, cb, cr);
              }
            }
            uint4 *dd = reinterpret_cast<uint4 *>(sr + skw<kSkew>(x0));
            dd[0] = make_uint4(px[0], px[1], px[2], px[3]);
            dd[1] = make_uint4(px[4], px[5], px[6], px[7]);
          }
        }
      }
    } else {
      if constexpr (raw_al16) {
        if (lane * 16 < W) {
          stage16_raw<kSkew>(pf.r0, s0, lane * 16);
          if (y + 1 < H) stage16_raw<kSkew>(pf.r1, s1, lane * 16);
        }
      } else {
        for (int r = 0; r < 2; ++r) {
          const int yy = y + r;
          if (yy >= H) break;
          const uint8_t *row = raw_cell + (int64_t)yy * W * 3;
          for (int x0 = lane * 16; x0 < W; x0 += 1024) stage16_raw<kSkew>(load16_any(row, W, x0), r ? s1 : s0, x0);
        }
      }
    }
  };

  int next_oy = 0;     // next output row of the band to finish
  int kv_base = -1;    // first band row cached in kv
  int slot = 0;        // ring slot of row y
  // horizontal taps of the staged row pair y, y+1: 7 (q, row) jobs of 64
  // output columns
  auto horizontal = [&](int y) {
    const int slot1 = slot + 1 == RING ? 0 : slot + 1;
#pragma unroll
    for (int job = 0; job < 7; ++job) {
      const int q = job < 6 ? job >> 1 : 3;
      const int r = job < 6 ? (job & 1) : (lane >> 5);
      const int ox = q < 3 ? lane + 64 * q : 192 + (lane & 31);
      const uint32_t *rowp = stg + (r ? g.spad : 0);
      int32_t a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        // Pillow weights are >= 0 and <= 2^22: 24-bit products (v_mul_u32_u24
        // with SDWA byte selects), exact in 32 bits. The window crosses at
        // most one 32-pixel skew step (KS < 32), at tap xcr[q].
        const uint32_t v = kSkew ? (rowp + (t < xcr[q] ? xsk[q] : xsk[q] + 4))[t] : rowp[xm[q] + t];
        const uint32_t kw = (uint32_t)wgt[q][t];
        a0 += (int32_t)__umul24(v & 255, kw);
        a1 += (int32_t)__umul24((v >> 8) & 255, kw);
        a2 += (int32_t)__umul24((v >> 16) & 255, kw);
      }
      const int sl = r ? slot1 : slot;
      if constexpr (kRgbx) {
        reinterpret_cast<uint32_t *>(ring)[sl * kOut + ox] =
            min((uint32_t)a0 >> kPrecisionBits, 255u) | (min((uint32_t)a1 >> kPrecisionBits, 255u) << 8) |
            (min((uint32_t)a2 >> kPrecisionBits, 255u) << 16);
      } else {
        uint8_t *rw = ring + sl * kOut + ox;
        rw[0] = (uint8_t)min((uint32_t)a0 >> kPrecisionBits, 255u);
        rw[RING * kOut] = (uint8_t)min((uint32_t)a1 >> kPrecisionBits, 255u);
        rw[2 * RING * kOut] = (uint8_t)min((uint32_t)a2 >> kPrecisionBits, 255u);
      }
    }
    slot = slot1 + 1 == RING ? 0 : slot1 + 1;
  };
  // finish every output row whose vertical window lies in ring rows [ya0, done)
  auto vertical = [&](int done) {
    while (next_oy < nb) {
      const int j = next_oy;
      if (j >= kv_base + kKvRows || kv_base < 0) {
        kv_base = j;
        if (lane < kKvRows && j + lane < nb) {
          int ymin;
          const int cnt = resample_coeffs_one(H, kOut, oy0 + j + lane, ks_v, kv + lane * ks_v, &ymin);
          vb[2 * lane] = ymin;
          vb[2 * lane + 1] = cnt;
        }
        wave_lds_fence();
      }
      const int jr = j - kv_base;
      const int ymin = __builtin_amdgcn_readfirstlane(vb[2 * jr]);
      const int cnt = __builtin_amdgcn_readfirstlane(vb[2 * jr + 1]);
      if (ymin + cnt > done) break;
      ++next_oy;
      int s0 = (ymin - ya0) % RING;
      if constexpr (kRgbx) {
        // lane g < 56: output columns 4g..4g+3, all three channels, from one
        // 16-byte read of the ring row per tap (lanes 56-63 read group 55)
        const int gq = min(lane, 55);
        int32_t acc[3][4];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][e] = 1 << (kPrecisionBits - 1);
        for (int t = 0; t < cnt; ++t) {
          const uint32_t kw = (uint32_t)__builtin_amdgcn_readfirstlane(kv[jr * ks_v + t]);
          const int sl = s0 + t < RING ? s0 + t : s0 + t - RING;
          const uint4 v4 = *reinterpret_cast<const uint4 *>(ring + (sl * kOut + 4 * gq) * 4);
          const uint32_t w4[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[0][e] += (int32_t)__umul24(w4[e] & 255, kw);
            acc[1][e] += (int32_t)__umul24((w4[e] >> 8) & 255, kw);
            acc[2][e] += (int32_t)__umul24((w4[e] >> 16) & 255, kw);
          }
        }
        if (lane < 56) {
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const float *lc = s_lut + i * 256;
            float4 f;
            f.x = lc[min((uint32_t)acc[i][0] >> kPrecisionBits, 255u)];
            f.y = lc[min((uint32_t)acc[i][1] >> kPrecisionBits, 255u)];
            f.z = lc[min((uint32_t)acc[i][2] >> kPrecisionBits, 255u)];
            f.w = lc[min((uint32_t)acc[i][3] >> kPrecisionBits, 255u)];
            *reinterpret_cast<float4 *>(out + (((int64_t)img * 3 + i) * kOut + oy0 + j) * kOut + 4 * lane) = f;
          }
        }
        continue;
      }
      int32_t acc[3][4];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][e] = 1 << (kPrecisionBits - 1);
      for (int t = 0; t < cnt; ++t) {
        const uint32_t kw = (uint32_t)__builtin_amdgcn_readfirstlane(kv[jr * ks_v + t]);
        const int sl = s0 + t < RING ? s0 + t : s0 + t - RING;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const uint32_t v = *reinterpret_cast<const uint32_t *>(ring + (vc[i] * RING + sl) * kOut + vo[i]);
          acc[i][0] += (int32_t)__umul24(v & 255, kw);
          acc[i][1] += (int32_t)__umul24((v >> 8) & 255, kw);
          acc[i][2] += (int32_t)__umul24((v >> 16) & 255, kw);
          acc[i][3] += (int32_t)__umul24(v >> 24, kw);
        }
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (lane + 64 * i < 168) {
          const float *lc = s_lut + vc[i] * 256;
          float4 f;
          f.x = lc[min((uint32_t)acc[i][0] >> kPrecisionBits, 255u)];
          f.y = lc[min((uint32_t)acc[i][1] >> kPrecisionBits, 255u)];
          f.z = lc[min((uint32_t)acc[i][2] >> kPrecisionBits, 255u)];
          f.w = lc[min((uint32_t)acc[i][3] >> kPrecisionBits, 255u)];
          *reinterpret_cast<float4 *>(out + (((int64_t)img * 3 + vc[i]) * kOut + oy0 + j) * kOut + vo[i]) = f;
        }
      }
    }
  };

  // One row pair in flight while the previous one is computed (a second
  // register set measured no faster and costs a wave per SIMD). The output
  // rows completed by the previous pair are finished BEFORE this pair's
  // horizontal taps: their float4 stores then drain behind the taps instead
  // of being waited for (vmcnt counts loads and stores together) by the next
  // staging's wait for its prefetched rows. The ring size is unchanged: the
  // rows still pending need at most ks_v - 1 earlier rows plus this pair.
  constexpr int kStep = 2;
  fetch(pa, ya0);
  for (int y = ya0; y < yb; y += kStep) {
    stage(pa, y);
    if (y + kStep < yb) fetch(pa, y + kStep);
    wave_lds_fence();
    vertical(y);
    horizontal(y);
    wave_lds_fence();
  }
  vertical(yb + 1);
}

template <int SRC, int KS>
__global__ void __launch_bounds__(256) k_resize4(const ImgDesc *__restrict__ descs,
                                                 const uint8_t *__restrict__ planes, RawSrc raw,
                                                 const float *__restrict__ lut,
                                                 const int64_t *__restrict__ labels,
                                                 float *__restrict__ out,
                                                 int64_t *__restrict__ out_labels,
                                                 const int32_t *__restrict__ status, Geom4 g) {
  resize4_body<SRC, KS>(descs, planes, raw, lut, labels, out, out_labels, status, g);
}

// ---------------------------------------------------------------------------
// Launch geometry.
// ---------------------------------------------------------------------------
static int wave_bytes4(const Geom4 &g) {
  const int b = 8 * g.spad + (g.rgbx ? 4 : 3) * g.ring * kOut + 4 * (kKvRows * g.ks_v + 2 * kKvRows);
  return (b + 15) & ~15;
}

static bool make_geom4(int n, int max_w, int max_h, int ks_h, int waves_target, Geom4 &g,
                       int wpg = kResizeWaves, bool jpeg = false) {
  g.wpg = wpg;
  g.rgbx = jpeg ? 1 : 0;
  g.ks_v = resample_ksize_host(max_h, kOut);
  g.ring = g.ks_v + 1; // an output row is finished within 2 rows of its window end
  const int px = ((max_w + 15) / 16) * 16 + ks_h + 16;
  // raw rows are skewed (skw); JPEG rows are not
  g.spad = (px + (jpeg ? 0 : (px >> 5) << 2) + 4 + 3) & ~3;
  g.wave_bytes = wave_bytes4(g);
  int nb = (waves_target + n - 1) / n;
  if (nb < 1) nb = 1;
  if (nb > 28) nb = 28;
  g.bh = (kOut + nb - 1) / nb;
  g.nbands = (kOut + g.bh - 1) / g.bh;
  g.ntask = n * g.nbands;
  return 3072 + g.wpg * (size_t)g.wave_bytes <= 160 * 1024;
}

template <int SRC, int KS>
static hipError_t launch4(const ImgDesc *descs, const uint8_t *planes, RawSrc raw, const float *lut,
                          const int64_t *labels, float *out, int64_t *out_labels,
                          const int32_t *status, const Geom4 &g, hipStream_t s) {
  static hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_resize4<SRC, KS>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  const int groups = (g.ntask + g.wpg - 1) / g.wpg;
  hipLaunchKernelGGL((k_resize4<SRC, KS>), dim3(groups), dim3(64 * g.wpg),
                     3072 + g.wpg * g.wave_bytes, s, descs,
                     planes, raw, lut, labels, out, out_labels, status, g);
  return hipGetLastError();
}

template <int SRC>
static bool dispatch4(int ks_h, const ImgDesc *descs, const uint8_t *planes, RawSrc raw,
                      const float *lut, const int64_t *labels, float *out, int64_t *out_labels,
                      const int32_t *status, const Geom4 &g, hipStream_t s, hipError_t *err) {
  switch (ks_h) {
  case 3: *err = launch4<SRC, 3>(descs, planes, raw, lut, labels, out, out_labels, status, g, s); return true;
  case 5: *err = launch4<SRC, 5>(descs, planes, raw, lut, labels, out, out_labels, status, g, s); return true;
  case 7: *err = launch4<SRC, 7>(descs, planes, raw, lut, labels, out, out_labels, status, g, s); return true;
  case 9: *err = launch4<SRC, 9>(descs, planes, raw, lut, labels, out, out_labels, status, g, s); return true;
  case 11: *err = launch4<SRC, 11>(descs, planes, raw, lut, labels, out, out_labels, status, g, s); return true;
  default: return false;
  }
}

// Waves to aim for: the CU count times the resident waves per CU the LDS
// allows (at most 12).
static int waves_target4(const Geom4 &g, int pct, int max_waves = 12) {
  const int max_wg = max_waves / g.wpg;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) cus = 256;
    else cus = prop.multiProcessorCount;
  }
  int wg = (160 * 1024) / (3072 + g.wpg * g.wave_bytes);
  if (wg > max_wg) wg = max_wg;
  if (wg < 1) wg = 1;
  // LDT_OPT_RESIZE_WAVES_PCT: more, shorter bands fill the
  // pipeline's CU gaps better but cost the kernel's own efficiency
  return cus * g.wpg * wg * (pct > 0 ? pct : 100) / 100;
}

bool launch_resize4_jpeg(const DevPlan &p, const DevWork &w, float *out, int64_t *out_labels,
                         hipStream_t s, hipError_t *err, int *wpg_used) {
  Geom4 g;
  const int ks_h = resample_ksize_host(p.max_w, kOut);
  if (ks_h > 11) return false;
  // a tall image (large ring) may not fit 4 waves' LDS in one workgroup:
  // fewer waves per workgroup before giving the batch to the streaming kernel
  int wpg = p.resize_wpg > 0 ? p.resize_wpg : kResizeWavesJpeg;
  while (!make_geom4(p.n, p.max_w, p.max_h, ks_h, 1, g, wpg, true)) {
    if (wpg == 1) return false;
    wpg >>= 1;
  }
  if (!make_geom4(p.n, p.max_w, p.max_h, ks_h, waves_target4(g, p.resize_waves_pct), g, wpg, true)) return false;
  if (wpg_used) *wpg_used = wpg;
  RawSrc raw{nullptr, 0, 0, 0};
  // fast-path images and the rest go to separate kernels (each skips the
  // other's images); a batch of one kind launches one kernel. The first
  // launch also writes the failed images (k_fill_failed's job otherwise).
  g.fill = 1;
  if (p.n_fast420 > 0) {
    // 4:2:0 images of width <= 512: the packed 16-bit staging (k_resize4<5>),
    // or the 32-bit one (k_resize4<0>, LDT_OPT_RESIZE_IMPL 1, cross-check)
    const bool ok = p.resize420 == 3
                        ? dispatch4<5>(ks_h, p.descs, w.planes, raw, p.lut, p.labels, out, out_labels, w.status, g, s, err)
                        : dispatch4<0>(ks_h, p.descs, w.planes, raw, p.lut, p.labels, out, out_labels, w.status, g, s, err);
    if (!ok) return false;
    if (*err != hipSuccess || p.n_fast420 == p.n) return true;
    g.fill = 0;
  }
  return dispatch4<2>(ks_h, p.descs, w.planes, raw, p.lut, p.labels, out, out_labels, w.status, g, s,
                      err);
}

bool launch_resize4_raw(const uint8_t *hwc, int64_t cell_stride, int n, int h, int wd,
                        const float *lut, float *out, hipStream_t s, hipError_t *err) {
  Geom4 g;
  const int ks_h = resample_ksize_host(wd, kOut);
  if (ks_h > 11) return false;
  if (!make_geom4(n, wd, h, ks_h, 1, g)) return false;
  if (!make_geom4(n, wd, h, ks_h, waves_target4(g, 100), g)) return false;
  g.fill = 0;
  RawSrc raw{hwc, cell_stride, h, wd};
  const bool al16 = (((uintptr_t)hwc) & 15) == 0 && (cell_stride & 15) == 0 && ((wd * 3) & 15) == 0 &&
                    wd <= 1024;
  if (!al16)
    return dispatch4<3>(ks_h, (const ImgDesc *)nullptr, (const uint8_t *)nullptr, raw, lut,
                        (const int64_t *)nullptr, out, (int64_t *)nullptr, (const int32_t *)nullptr, g,
                        s, err);
  return dispatch4<1>(ks_h, (const ImgDesc *)nullptr, (const uint8_t *)nullptr, raw, lut,
                      (const int64_t *)nullptr, out, (int64_t *)nullptr, (const int32_t *)nullptr, g,
                      s, err);
}

} // namespace ldt

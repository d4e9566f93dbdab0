// ldt_kernels.hip — gfx950 (MI355X / CDNA4) kernels of the batch-decode path.
//
// Pipeline per batch (all device-resident, one HIP stream):
//   k_destuff     one workgroup per image: remove 0xFF00 stuffing, split the
//                 entropy-coded data at RSTn markers into segments, find the
//                 end-of-scan marker (libjpeg jdmarker.c / jdhuff.c semantics).
//   k_huff_*      baseline Huffman decode of each segment into int16 DCT
//                 coefficients, natural order, MCU-major block layout
//                 (jdhuff.c decode_mcu restated; see ldt_huffman.hip).
//   k_idct        dequantise + JDCT_ISLOW 8x8 IDCT (jidctint.c), one lane per
//                 block (both passes in registers), uint8 planes.
//   k_resize<S>   fused chroma fancy-upsampling (jdsample.c) + YCbCr->RGB
//                 (jdcolor.c) + Pillow BILINEAR Resize((224,224)) (Resample.c,
//                 22-bit fixed point, horizontal-then-vertical, uint8
//                 intermediate) + ToTensor/Normalize via a float32 LUT, coalesced
//                 CHW fp32 stores. S = raw HWC source for config 5.
//   k_shard_*     ShardedBatchSampler / ShardedFragmentSampler index ranges.
//
// Reference call sites replaced: lance_iterable.py:38-50, lance_map_style.py:21-44,
// lance_iterable.py:61-69. Nothing here is a dense contraction, so no MFMA: the
// decode stages are VALU/LDS/latency bound and the resize/store is HBM bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldt_device.hpp"
#include "ldt_kernels.hpp"

#pragma clang fp contract(off)

namespace ldt {

// ---------------------------------------------------------------------------
// Destuff: jdhuff.c jpeg_fill_bit_buffer / jdmarker.c semantics over the
// entropy-coded bytes of each cell — FF00 -> FF, FF fill bytes dropped, RSTn
// ends a segment, any other marker ends the scan. Kept bytes are compacted per
// image; every segment is followed by kSegPad zero bytes.
//   k_destuff_count   one workgroup per 4 KB chunk: kept bytes, RSTn markers,
//                     end marker seen;
//   k_destuff_write   one workgroup per chunk: output offset from the image's
//                     earlier chunks, classify again, compact in LDS, copy out;
//   k_destuff_layout  one workgroup per image: segment ends, the final pad, the
//                     parallel decoder's subsequence layout.
// Chunks run over 4-aligned source words (B0 = cell scan start rounded down):
// chunk byte k of chunk c is relative position c * kDsChunk + k - lead.
// ---------------------------------------------------------------------------
constexpr int kDsChunk = kDsChunkBytes;        // 16 bytes per lane
constexpr int kDsWords = kDsChunk / 4 + 2;     // + the words before and after
constexpr int kDsInLds = kDsWords + kDsWords / 8 + 1;
// LDS output of one chunk: kept bytes + kSegPad per RSTn + alignment. Sized for
// kDsRstLds markers per chunk (the workgroup then fits beside a k_huff_image
// workgroup of another batch); a chunk with more writes its bytes straight to
// memory.
constexpr int kDsRstLds = 64;
constexpr int kDsOutLds = (kDsChunk + kSegPad * kDsRstLds) / 4 + 4;

__device__ __forceinline__ int ds_skew(int w) { return w + (w >> 3); }

struct DsChunk {
  const uint8_t *B0;
  int lead;
  int64_t span;  // bytes from B0 to the end of the cell
  int64_t cb;    // chunk start (bytes from B0)
};

__device__ __forceinline__ DsChunk ds_chunk(const uint8_t *data, const ImgDesc &d, int lc) {
  DsChunk k;
  const uint8_t *src = data + d.src_off;
  k.B0 = reinterpret_cast<const uint8_t *>((uintptr_t)src & ~(uintptr_t)3);
  k.lead = (int)(src - k.B0);
  k.span = d.src_len + k.lead;
  k.cb = (int64_t)lc * kDsChunk;
  return k;
}

// Stage the chunk's words (and one on each side) into LDS, zero outside the cell.
__device__ __forceinline__ void ds_stage(const DsChunk &k, uint32_t *s_in, int tid) {
  const uint32_t *wsrc = reinterpret_cast<const uint32_t *>(k.B0 + k.cb) - 1;
  const int64_t nwords_cell = (k.span - k.cb + 3) / 4 + 1; // words touching the cell
  for (int w = tid; w < kDsWords; w += 256) {
    uint32_t v = 0;
    if (w < nwords_cell && (k.cb > 0 || w > 0)) v = wsrc[w];
    s_in[ds_skew(w)] = v;
  }
}

// Classify lane tid's 16 bytes (after the LDS stage and a barrier).
__device__ __forceinline__ void ds_classify(const uint32_t *s_in, const DsChunk &k, int64_t L, int tid,
                                            uint32_t wv[6], uint32_t &keep, uint32_t &rst,
                                            int &local_end) {
#pragma unroll
  for (int i = 0; i < 6; ++i) wv[i] = s_in[ds_skew(4 * tid + i)];
  ds_classify16(wv, k.cb + 16 * tid - k.lead, L, keep, rst, local_end);
}

// Limit the lane's masks to bytes before the chunk's end marker (sh_end).
__device__ __forceinline__ void ds_limit(int cend, int tid, uint32_t &keep, uint32_t &rst) {
  const int my_lo = tid * 16;
  const uint32_t lim = (cend <= my_lo) ? 0u : (cend - my_lo >= 16 ? 0xFFFFu : ((1u << (cend - my_lo)) - 1u));
  keep &= lim;
  rst &= lim;
}

__global__ void __launch_bounds__(256) k_destuff_count(const uint8_t *__restrict__ data,
                                                       const ImgDesc *__restrict__ descs,
                                                       const int32_t *__restrict__ chunk_img,
                                                       int4 *__restrict__ cnt,
                                                       const int32_t *__restrict__ status) {
  __shared__ uint32_t s_in[kDsInLds];
  __shared__ int sh_scan[8];
  __shared__ int sh_end;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int img = chunk_img[c];
  const ImgDesc &d = descs[img];
  const DsChunk k = ds_chunk(data, d, c - d.ds_first);
  if (status[img] != 0 || k.cb >= k.span) {
    if (tid == 0) cnt[c] = make_int4(0, 0, 0, 0);
    return;
  }
  ds_stage(k, s_in, tid);
  if (tid == 0) sh_end = kDsChunk;
  __syncthreads();
  uint32_t wv[6], keep, rst;
  int local_end;
  ds_classify(s_in, k, d.src_len, tid, wv, keep, rst, local_end);
  if (local_end < 16) atomicMin(&sh_end, tid * 16 + local_end);
  __syncthreads();
  const int cend = sh_end;
  ds_limit(cend, tid, keep, rst);
  int ktot, rtot;
  (void)block_excl_scan256(__popc(keep), sh_scan, &ktot);
  (void)block_excl_scan256(__popc(rst), sh_scan, &rtot);
  if (tid == 0) cnt[c] = make_int4(ktot, rtot, cend < kDsChunk ? 1 : 0, 0);
}

__device__ __forceinline__ void lds_put8(uint32_t *buf, int pos, uint32_t v) {
  reinterpret_cast<uint8_t *>(buf)[pos] = (uint8_t)v;
}

__global__ void __launch_bounds__(256) k_destuff_write(const uint8_t *__restrict__ data,
                                                       const ImgDesc *__restrict__ descs,
                                                       Segment *__restrict__ segs,
                                                       const int32_t *__restrict__ chunk_img,
                                                       const int4 *__restrict__ cnt,
                                                       uint8_t *__restrict__ dst,
                                                       const int32_t *__restrict__ status) {
  __shared__ uint32_t s_in[kDsInLds];
  __shared__ __attribute__((aligned(16))) uint32_t s_out[kDsOutLds];
  __shared__ int sh_scan[8];
  __shared__ int sh_end;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int img = chunk_img[c];
  const ImgDesc &d = descs[img];
  const DsChunk k = ds_chunk(data, d, c - d.ds_first);
  if (status[img] != 0 || k.cb >= k.span) return;
  // output offset: kept bytes and RSTn markers of the image's earlier chunks
  int kb = 0, rb = 0, ended = 0;
  for (int q = d.ds_first + tid; q < c; q += 256) {
    const int4 v = cnt[q];
    kb += v.x;
    rb += v.y;
    ended |= v.z;
  }
  int tmp;
  (void)block_excl_scan256(kb, sh_scan, &kb);
  (void)block_excl_scan256(rb, sh_scan, &rb);
  (void)block_excl_scan256(ended, sh_scan, &tmp);
  if (tmp != 0) return; // after the end-of-scan marker
  ds_stage(k, s_in, tid);
  if (tid == 0) sh_end = kDsChunk;
  __syncthreads();
  uint32_t wv[6], keep, rst;
  int local_end;
  ds_classify(s_in, k, d.src_len, tid, wv, keep, rst, local_end);
  if (local_end < 16) atomicMin(&sh_end, tid * 16 + local_end);
  __syncthreads();
  ds_limit(sh_end, tid, keep, rst);
  int ktot, rtot;
  const int kex = block_excl_scan256(__popc(keep), sh_scan, &ktot);
  const int rex = block_excl_scan256(__popc(rst), sh_scan, &rtot);
  // kept byte o of segment r lands at o + kSegPad * r (r clamped so a stream
  // with surplus RSTn markers stays inside the image's region)
  const int last = d.nseg - 1;
  const int64_t g0 = kb + (int64_t)kSegPad * min(rb, last); // chunk output start (image-relative)
  const int64_t gal = g0 & ~(int64_t)3;                      // s_out byte 0
  const int rpads = min(rb + rtot, last) - min(rb, last);
  const int lo_b = (int)(g0 - gal);
  const int gend = lo_b + ktot + kSegPad * rpads;
  int r = rb + rex;
  int o = lo_b + kex + kSegPad * (min(r, last) - min(rb, last));
  uint8_t *out = dst + d.dst_off;
  if (rtot > kDsRstLds) { // marker-dense chunk: bytes straight to memory
    uint8_t *ob = out + gal;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (rst & (1u << j)) {
        if (r < last) {
          for (int q = 0; q < kSegPad; ++q) ob[o + q] = 0;
          o += kSegPad;
        }
        ++r;
        if (r < d.nseg) segs[d.seg_base + r].byte_start = d.dst_off + gal + o;
      }
      if (keep & (1u << j)) ob[o++] = (uint8_t)(wv[(j + 4) >> 2] >> (8 * ((j + 4) & 3)));
    }
    return;
  }
  if (keep == 0xFFFFu) {
    // all 16 bytes kept, no marker: a byte-shifted copy of the input run
    const int a = o & 3, w0 = o >> 2;
    if (a == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) s_out[w0 + q] = wv[1 + q];
    } else {
      for (int q = 0; q < 4 - a; ++q) lds_put8(s_out, o + q, wv[1] >> (8 * q));
#pragma unroll
      for (int q = 0; q < 3; ++q)
        s_out[w0 + 1 + q] = __builtin_amdgcn_alignbyte(wv[2 + q], wv[1 + q], (uint32_t)(4 - a));
      for (int q = 0; q < a; ++q) lds_put8(s_out, 4 * (w0 + 4) + q, wv[4] >> (8 * (4 - a + q)));
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (rst & (1u << j)) {
        if (r < last) {
          for (int q = 0; q < kSegPad; ++q) lds_put8(s_out, o + q, 0u);
          o += kSegPad;
        }
        ++r;
        if (r < d.nseg) segs[d.seg_base + r].byte_start = d.dst_off + gal + o;
      }
      if (keep & (1u << j)) lds_put8(s_out, o++, wv[(j + 4) >> 2] >> (8 * ((j + 4) & 3)));
    }
  }
  __syncthreads();
  for (int w = tid; 4 * w < gend; w += 256) {
    const int b0 = 4 * w;
    if (b0 >= lo_b && b0 + 4 <= gend) {
      *reinterpret_cast<uint32_t *>(out + gal + b0) = s_out[w];
    } else {
      for (int q = 0; q < 4; ++q)
        if (b0 + q >= lo_b && b0 + q < gend)
          out[gal + b0 + q] = reinterpret_cast<const uint8_t *>(s_out)[b0 + q];
    }
  }
}

__global__ void __launch_bounds__(256) k_destuff_layout(const ImgDesc *__restrict__ descs,
                                                        Segment *__restrict__ segs,
                                                        const int4 *__restrict__ cnt,
                                                        uint8_t *__restrict__ dst,
                                                        int32_t *__restrict__ status) {
  __shared__ int sh_scan[8];
  __shared__ int sh_endc;
  const int img = blockIdx.x, tid = threadIdx.x;
  const ImgDesc &d = descs[img];
  // nseg 0: progressive (k_prog); ds_count 0: destuffed by k_huff_image
  if (status[img] != 0 || d.nseg == 0 || d.ds_count == 0) return;
  // chunks up to and including the first one holding the end-of-scan marker
  if (tid == 0) sh_endc = d.ds_count;
  __syncthreads();
  for (int q = tid; q < d.ds_count; q += 256)
    if (cnt[d.ds_first + q].z) atomicMin(&sh_endc, q + 1);
  __syncthreads();
  const int nch = sh_endc;
  int kt = 0, rt = 0;
  for (int q = tid; q < nch; q += 256) {
    kt += cnt[d.ds_first + q].x;
    rt += cnt[d.ds_first + q].y;
  }
  (void)block_excl_scan256(kt, sh_scan, &kt);
  (void)block_excl_scan256(rt, sh_scan, &rt);
  const int64_t out_base = kt;
  const int rst_base = rt;
  uint8_t *out = dst + d.dst_off;
  if (tid == 0) {
    segs[d.seg_base].byte_start = d.dst_off;
    if (rst_base != d.nseg - 1) {
      status[img] = 3; // LDT_IMG_CORRUPT: restart markers do not match the header
    }
    // zero pad after the last segment
    const int64_t tail = out_base + (int64_t)kSegPad * min(rst_base, d.nseg - 1);
    for (int j = 0; j < kSegPad; ++j) out[tail + j] = 0;
  }
  __syncthreads();
  // segment ends: the next segment's start less the pad; last = end of data
  for (int s = tid; s < d.nseg; s += 256) {
    int64_t e = (s + 1 < d.nseg && rst_base == d.nseg - 1)
                    ? segs[d.seg_base + s + 1].byte_start - kSegPad
                    : d.dst_off + out_base + (int64_t)kSegPad * min(rst_base, d.nseg - 1);
    if (rst_base != d.nseg - 1) segs[d.seg_base + s].byte_start = d.dst_off;
    segs[d.seg_base + s].byte_end = e;
  }
  if (d.sub_bits <= 0) return; // serial Huffman decoder
  __syncthreads();
  // subsequence layout for the parallel Huffman decoder: segment s gets
  // max(1, ceil(bits / S)) lanes, numbered from 0 across the image, with the
  // image's own S (the planner sizes it so they fit one workgroup).
  const int S = d.sub_bits;
  int base = 0;
  for (int s0 = 0; s0 < d.nseg; s0 += 256) {
    const int s = s0 + tid;
    int cnt_s = 0;
    if (s < d.nseg) {
      const Segment &sg = segs[d.seg_base + s];
      const int64_t bits = (sg.byte_end - sg.byte_start) * 8;
      cnt_s = (int)((bits + S - 1) / S);
      if (cnt_s < 1) cnt_s = 1;
    }
    int tot;
    const int ex = block_excl_scan256(cnt_s, sh_scan, &tot);
    if (s < d.nseg) {
      segs[d.seg_base + s].sub_first = base + ex;
      segs[d.seg_base + s].sub_count = cnt_s;
    }
    base += tot;
  }
  if (tid == 0 && base > kHuffThreads) status[img] = 3;
}

// ---------------------------------------------------------------------------
// k_idct: jidctint.c jpeg_idct_islow, one lane per 8x8 block (see below).
// ---------------------------------------------------------------------------
#define FIX_0_298631336 2446
#define FIX_0_390180644 3196
#define FIX_0_541196100 4433
#define FIX_0_765366865 6270
#define FIX_0_899976223 7373
#define FIX_1_175875602 9633
#define FIX_1_501321110 12299
#define FIX_1_847759065 15137
#define FIX_1_961570560 16069
#define FIX_2_053119869 16819
#define FIX_2_562915447 20995
#define FIX_3_072711026 25172

// One 1-D ISLOW butterfly on in[0..7] (stride 1), producing the 8 pre-descale
// sums in the order libjpeg stores them. Every multiply is var x FIX_* with
// |var| < 2^23 (pass 1: dequantised 11-bit coefficients x 8-bit quant, sums
// of <= 4; pass 2: int16 workspace values, see k_idct), so the products are
// exact 24-bit multiplies (v_mul_i32_i24, full rate; a plain int multiply
// becomes the quarter-rate v_mul_lo_u32).
struct Islow8 {
  int32_t o[8];
};
__device__ __forceinline__ Islow8 islow_1d(const int32_t *x, int pass1) {
  int32_t tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13, z1, z2, z3, z4, z5;
  z2 = x[2];
  z3 = x[6];
  z1 = __mul24(z2 + z3, FIX_0_541196100);
  tmp2 = z1 + __mul24(z3, -FIX_1_847759065);
  tmp3 = z1 + __mul24(z2, FIX_0_765366865);
  tmp0 = (x[0] + x[4]) * (1 << 13);
  tmp1 = (x[0] - x[4]) * (1 << 13);
  tmp10 = tmp0 + tmp3;
  tmp13 = tmp0 - tmp3;
  tmp11 = tmp1 + tmp2;
  tmp12 = tmp1 - tmp2;
  tmp0 = x[7];
  tmp1 = x[5];
  tmp2 = x[3];
  tmp3 = x[1];
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  z4 = tmp1 + tmp3;
  z5 = __mul24(z3 + z4, FIX_1_175875602);
  tmp0 = __mul24(tmp0, FIX_0_298631336);
  tmp1 = __mul24(tmp1, FIX_2_053119869);
  tmp2 = __mul24(tmp2, FIX_3_072711026);
  tmp3 = __mul24(tmp3, FIX_1_501321110);
  z1 = __mul24(z1, -FIX_0_899976223);
  z2 = __mul24(z2, -FIX_2_562915447);
  z3 = __mul24(z3, -FIX_1_961570560);
  z4 = __mul24(z4, -FIX_0_390180644);
  z3 += z5;
  z4 += z5;
  tmp0 += z1 + z3;
  tmp1 += z2 + z4;
  tmp2 += z2 + z3;
  tmp3 += z1 + z4;
  Islow8 r;
  r.o[0] = tmp10 + tmp3;
  r.o[7] = tmp10 - tmp3;
  r.o[1] = tmp11 + tmp2;
  r.o[6] = tmp11 - tmp2;
  r.o[2] = tmp12 + tmp1;
  r.o[5] = tmp12 - tmp1;
  r.o[3] = tmp13 + tmp0;
  r.o[4] = tmp13 - tmp0;
  (void)pass1;
  return r;
}

// The pass-1 workspace is 16-bit in libjpeg-turbo's SIMD ISLOW (the path
// Pillow runs on x86-64: packssdw after pass 1); for valid data the values fit
// and this is the identity, and it bounds the pass-2 multiplies to 24 bits.
__device__ __forceinline__ int32_t sat16(int32_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

// jdmaster.c prepare_range_limit_table, post-IDCT part, indexed by x & 1023:
// [0,128) -> x + 128, [128,512) -> 255, [512,896) -> 0, [896,1024) -> x - 896,
// i.e. clamp(sext10(x) + 128, 0, 255).
__device__ __forceinline__ uint32_t idct_limit(int32_t x) {
  const int32_t v = (int32_t)__builtin_amdgcn_sbfe(x, 0u, 10u) + 128;
  return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// One lane per 8x8 block: the whole block stays in registers for both
// passes (no transposes, no barriers between them). A workgroup covers
// kIdctBlocksPerWg consecutive blocks of one image; each lane loads its
// block's 16-B groups straight into registers (no LDS tile: occupancy is set
// by registers alone, so more blocks are in flight).
//
// Baseline images: the block record gives the block's nonzero groups (mask)
// and where their packed units start (ldt_kernels.hpp); only those are read,
// the others are zero, and nothing is written back. Progressive images: the
// dense group planes of `pcoef` (one contiguous 1 KB per group and wave), and
// zeros are written back over the groups that were not zero — the all-zero
// contract of that buffer with k_prog (also for failed images), so it needs no
// memset per batch.
constexpr int kIdctBlocksPerWg = 256; // = threads
// jpeg_natural_order: zigzag position -> natural (row-major) index
constexpr int kZigzagNat[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

__global__ void __launch_bounds__(kIdctBlocksPerWg) k_idct(const ImgDesc *__restrict__ descs,
                                              const uint16_t *__restrict__ qtabs,
                                              const int16_t *__restrict__ coef,
                                              const uint32_t *__restrict__ brec,
                                              const uint32_t *__restrict__ bcarry,
                                              int16_t *__restrict__ pcoef,
                                              const int16_t *__restrict__ dcv,
                                              uint8_t *__restrict__ planes,
                                              const int32_t *__restrict__ status) {
  __shared__ __attribute__((aligned(16))) uint16_t s_q[3][64];
  const int img = blockIdx.y;
  const ImgDesc &d = descs[img];
  const int64_t nblk = (int64_t)d.mcux * d.mcuy * d.bpm;
  const int64_t b0 = (int64_t)blockIdx.x * kIdctBlocksPerWg;
  if (b0 >= nblk) return;
  const int tid = threadIdx.x;
  const bool ok = status[img] == 0;
  const bool prog = d.nseg == 0;
  if (!ok && !prog) return; // packed coefficients need no clearing
  const int nb = (int)min((int64_t)kIdctBlocksPerWg, nblk - b0);
  // quant tables in zigzag order, like the coefficients
  for (int i = tid; i < 64 * d.ncomp; i += kIdctBlocksPerWg)
    s_q[i >> 6][i & 63] = qtabs[d.qt[i >> 6] * 64 + kZigzagNat[i & 63]];
  const int64_t blk = b0 + tid;
  uint4 raw[8];
  int32_t dc = 0;
  if (prog) {
    __syncthreads();
    if (tid >= nb) return;
    uint4 *cimg = reinterpret_cast<uint4 *>(pcoef + d.pcoef_off * 64);
    const int npad = coef_npad(d);
#pragma unroll
    for (int r = 0; r < 8; ++r) raw[r] = cimg[coef_piece((int)blk, r, npad)];
#pragma unroll
    for (int r = 0; r < 8; ++r)
      if ((raw[r].x | raw[r].y | raw[r].z | raw[r].w) != 0) cimg[coef_piece((int)blk, r, npad)] = make_uint4(0u, 0u, 0u, 0u);
    if (!ok) return;
    dc = dcv[d.coef_off + blk];
  } else {
    // the block's record; its first unit by a segmented scan over the wave's
    // 64 consecutive blocks: a run start begins at 8 * blk, every other
    // block where its predecessor's groups end, and the wave's first block
    // (unless a run starts there) at its chunk's carry
    const bool in = tid < nb;
    const uint32_t rc = in ? brec[d.coef_off + blk] : 0u;
    const int lane = tid & 63;
    const uint32_t cnt = (uint32_t)__popc(rc & 255u);
    int fl = (rc >> 8) & 1;
    uint32_t v = fl ? 8u * (uint32_t)blk + cnt : cnt; // end of this block's units
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int pf = __shfl_up(fl, off);
      const uint32_t pv = (uint32_t)__shfl_up((int)v, off);
      if (lane >= off && !fl) v += pv;
      fl |= lane >= off ? pf : 0;
    }
    const uint32_t carry = fl ? 0u : bcarry[(d.coef_off + (blk & ~(int64_t)63)) >> 6];
    __syncthreads();
    if (!in) return;
    const uint4 *u = reinterpret_cast<const uint4 *>(coef + d.coef_off * 64) + (carry + v - cnt);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      raw[r] = make_uint4(0u, 0u, 0u, 0u);
      if ((rc >> r) & 1u) raw[r] = *u++;
    }
    dc = (int32_t)rc >> 16;
  }
  const int64_t m = blk / d.bpm;
  const int b = (int)(blk - m * d.bpm);
  const int comp = d.bcomp[b];
  const uint16_t *q = s_q[comp];
  // dequantised block, row-major (jidctint.c DEQUANTIZE); the stored slots
  // are in zigzag order (k_huff_write), placed at their natural index here
  int32_t ws[64];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint4 q4 = *reinterpret_cast<const uint4 *>(q + 8 * r);
    const uint32_t rw[4] = {raw[r].x, raw[r].y, raw[r].z, raw[r].w};
    const uint32_t qw[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t lo = (int32_t)(int16_t)(rw[j] & 0xFFFF), hi = (int32_t)(int16_t)(rw[j] >> 16);
      ws[kZigzagNat[8 * r + 2 * j]] = __mul24(lo, (int32_t)(qw[j] & 0xFFFF));
      ws[kZigzagNat[8 * r + 2 * j + 1]] = __mul24(hi, (int32_t)(qw[j] >> 16));
    }
  }
  ws[0] = dc * (int32_t)q[0]; // DC: absolute value after the predictor scan
  // pass 1: columns (CONST_BITS 13, PASS1_BITS 2). A column whose AC terms are
  // all zero gives DC << 2 exactly (jidctint.c shortcut); the butterfly runs
  // when any lane of the wave needs it.
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const bool nz = (ws[8 + c] | ws[16 + c] | ws[24 + c] | ws[32 + c] | ws[40 + c] | ws[48 + c] |
                     ws[56 + c]) != 0;
    if (__any(nz)) {
      int32_t x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = ws[8 * j + c];
      const Islow8 t = islow_1d(x, 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) ws[8 * j + c] = sat16((t.o[j] + (1 << 10)) >> 11); // DESCALE(, 13-2)
    } else {
      const int32_t dc4 = sat16(ws[c] * 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) ws[8 * j + c] = dc4;
    }
  }
  // pass 2: rows, DESCALE(, 13+2+3) and the range limit
  const int mx = (int)(m % d.mcux), my = (int)(m / d.mcux);
  const int bx = mx * d.ch[comp] + d.bdx[b];
  const int by = my * d.cv[comp] + d.bdy[b];
  uint8_t *dst = planes + d.plane_off[comp] + (int64_t)(by * 8) * d.plane_stride[comp] + bx * 8;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    int32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = ws[8 * r + j];
    const bool nz = (x[1] | x[2] | x[3] | x[4] | x[5] | x[6] | x[7]) != 0;
    uint32_t px[8];
    if (__any(nz)) {
      const Islow8 t = islow_1d(x, 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) px[j] = idct_limit((t.o[j] + (1 << 17)) >> 18);
    } else {
      const uint32_t v = idct_limit((x[0] + (1 << 4)) >> 5); // DESCALE(, PASS1_BITS+3)
#pragma unroll
      for (int j = 0; j < 8; ++j) px[j] = v;
    }
    uint2 packed;
    packed.x = px[0] | (px[1] << 8) | (px[2] << 16) | (px[3] << 24);
    packed.y = px[4] | (px[5] << 8) | (px[6] << 16) | (px[7] << 24);
    *reinterpret_cast<uint2 *>(dst + (int64_t)r * d.plane_stride[comp]) = packed;
  }
}

// Rows whose decode failed, behind the streaming k_resize fallback (k_resize4
// writes them itself): k_resize skips them, so their outputs
// are set here to defined values — zeros for the image and -100 for the label
// (torch.nn.CrossEntropyLoss's default ignore_index) — in case an
// asynchronous consumer (prefetching iterators) uses the batch before the
// per-row status is read. One workgroup per row; rows that decoded return.
__global__ void __launch_bounds__(256) k_fill_failed(const int32_t *__restrict__ status,
                                                     float *__restrict__ out,
                                                     int64_t *__restrict__ out_labels) {
  const int img = blockIdx.x;
  if (status[img] == 0) return;
  float4 *o = reinterpret_cast<float4 *>(out + (int64_t)img * 3 * kOut * kOut);
  for (int i = threadIdx.x; i < 3 * kOut * kOut / 4; i += 256) o[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (threadIdx.x == 0 && out_labels != nullptr) out_labels[img] = -100;
}

hipError_t launch_fill_failed(const DevPlan &p, const DevWork &w, float *out, int64_t *out_labels,
                              hipStream_t s) {
  if (p.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill_failed, dim3(p.n), dim3(256), 0, s, w.status, out, out_labels);
  return hipGetLastError();
}

// Test hook: coefficient tables for one (in, out) pair.
__global__ void k_resample_coeffs(int inSize, int outSize, int ksize, int32_t *bounds,
                                  int32_t *kk) {
  int xx = blockIdx.x * blockDim.x + threadIdx.x;
  if (xx >= outSize) return;
  int xmin;
  int cnt = resample_coeffs_one(inSize, outSize, xx, ksize, kk + (int64_t)xx * ksize, &xmin);
  bounds[2 * xx] = xmin;
  bounds[2 * xx + 1] = cnt;
}

// ---------------------------------------------------------------------------
// k_resize: fused source (JPEG planes or raw HWC) -> Pillow BILINEAR 224x224
// -> LUT (ToTensor [+Normalize]) -> fp32 CHW. One workgroup = kBandRows output
// rows of one image; workgroups of an image share blockIdx % 8 (one XCD under
// the observed round-robin placement, for L2 reuse of overlapping rows).
// Each thread < 224 owns one output column: it computes the horizontal tap
// sum of every needed source row and accumulates the vertical taps in
// registers, so the uint8 intermediate never leaves the thread.
// ---------------------------------------------------------------------------

template <int SRC>
__global__ void __launch_bounds__(kResizeThreads)
    k_resize(const ImgDesc *__restrict__ descs, const uint8_t *__restrict__ planes, RawSrc raw,
             const float *__restrict__ lut, const int64_t *__restrict__ labels,
             float *__restrict__ out, int64_t *__restrict__ out_labels,
             const int32_t *__restrict__ status, int n, int ks_h, int ks_v, int row_bytes) {
  constexpr int NB = kOut / kBandRows;
  const int L = blockIdx.x;
  const int g = L / (8 * NB), rr = L % (8 * NB);
  const int img = g * 8 + (rr % 8);
  const int band = rr / 8;
  if (img >= n) return;
  if (SRC == 0 && status[img] != 0) return;
  const int tid = threadIdx.x;
  int W, H;
  if (SRC == 0) {
    W = descs[img].width;
    H = descs[img].height;
  } else {
    W = raw.w;
    H = raw.h;
  }
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float *s_lut = reinterpret_cast<float *>(smem);                 // 768 floats
  int32_t *s_kh = reinterpret_cast<int32_t *>(smem + 3072);       // 224 * ks_h
  int32_t *s_kv = s_kh + kOut * ks_h;                             // kBandRows * ks_v
  int32_t *s_hb = s_kv + kBandRows * ks_v;                        // 224 * 2
  int32_t *s_vb = s_hb + 2 * kOut;                                // kBandRows * 2
  uint8_t *s_row = reinterpret_cast<uint8_t *>(s_vb + 2 * kBandRows); // 2 * row_bytes

  for (int i = tid; i < 768; i += kResizeThreads) s_lut[i] = lut[i];
  const int oy0 = band * kBandRows;
  if (tid < kOut) {
    int xmin;
    int cnt = resample_coeffs_one(W, kOut, tid, ks_h, s_kh + tid * ks_h, &xmin);
    s_hb[2 * tid] = xmin;
    s_hb[2 * tid + 1] = cnt;
  } else if (tid >= kOut && tid < kOut + kBandRows) {
    const int j = tid - kOut;
    int ymin;
    int cnt = resample_coeffs_one(H, kOut, oy0 + j, ks_v, s_kv + j * ks_v, &ymin);
    s_vb[2 * j] = ymin;
    s_vb[2 * j + 1] = cnt;
  }
  if (band == 0 && tid == 0 && labels != nullptr) out_labels[img] = labels[img];
  __syncthreads();
  const int ya = s_vb[0];
  const int yb = s_vb[2 * (kBandRows - 1)] + s_vb[2 * (kBandRows - 1) + 1];

  int32_t acc[kBandRows][3];
#pragma unroll
  for (int j = 0; j < kBandRows; ++j) acc[j][0] = acc[j][1] = acc[j][2] = 1 << (kPrecisionBits - 1);
  int hxmin = 0, hcnt = 0;
  if (tid < kOut) {
    hxmin = s_hb[2 * tid];
    hcnt = s_hb[2 * tid + 1];
  }

  for (int y = ya; y < yb; ++y) {
    uint8_t *row = s_row + ((y - ya) & 1) * row_bytes;
    // ---- stage source row y as interleaved RGB in LDS ----
    if (SRC == 0) {
      const ImgDesc &d = descs[img];
      const uint8_t *py = planes + d.plane_off[0] + (int64_t)y * d.plane_stride[0];
      if (d.color == 2) {
        for (int x = tid; x < W; x += kResizeThreads) {
          const uint8_t v = py[x];
          row[3 * x] = v;
          row[3 * x + 1] = v;
          row[3 * x + 2] = v;
        }
      } else {
        const uint8_t *pcb = planes + d.plane_off[1];
        const uint8_t *pcr = planes + d.plane_off[2];
        for (int x = tid; x < W; x += kResizeThreads) {
          const int Y = py[x];
          const int cb = chroma_at(d, pcb, 1, x, y);
          const int cr = chroma_at(d, pcr, 2, x, y);
          if (d.color == 1) {
            row[3 * x] = (uint8_t)Y;
            row[3 * x + 1] = (uint8_t)cb;
            row[3 * x + 2] = (uint8_t)cr;
          } else {
            ycc_to_rgb(Y, cb, cr, row + 3 * x);
          }
        }
      }
    } else {
      const uint8_t *src = raw.base + (int64_t)img * raw.cell_stride + (int64_t)y * W * 3;
      const int nbytes = W * 3;
      if ((((uintptr_t)src) & 3) == 0 && (nbytes & 3) == 0) {
        const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src);
        uint32_t *r4 = reinterpret_cast<uint32_t *>(row);
        for (int i = tid; i < nbytes / 4; i += kResizeThreads) r4[i] = s4[i];
      } else {
        for (int i = tid; i < nbytes; i += kResizeThreads) row[i] = src[i];
      }
    }
    __syncthreads();
    // ---- horizontal taps for column tid, then vertical accumulate ----
    if (tid < kOut) {
      int32_t s0 = 1 << (kPrecisionBits - 1), s1 = s0, s2 = s0;
      const int32_t *k = s_kh + tid * ks_h;
      const uint8_t *p = row + 3 * hxmin;
      for (int t = 0; t < hcnt; ++t) {
        const int32_t kw = k[t];
        s0 += (int32_t)p[3 * t] * kw;
        s1 += (int32_t)p[3 * t + 1] * kw;
        s2 += (int32_t)p[3 * t + 2] * kw;
      }
      const int32_t h0 = (int32_t)clip8(s0), h1 = (int32_t)clip8(s1), h2 = (int32_t)clip8(s2);
#pragma unroll
      for (int j = 0; j < kBandRows; ++j) {
        const int jj = y - s_vb[2 * j];
        if (jj >= 0 && jj < s_vb[2 * j + 1]) {
          const int32_t kw = s_kv[j * ks_v + jj];
          acc[j][0] += h0 * kw;
          acc[j][1] += h1 * kw;
          acc[j][2] += h2 * kw;
        }
      }
    }
    // the next iteration writes the other row buffer; one barrier per row suffices
  }
  if (tid < kOut) {
    float *o = out + (int64_t)img * 3 * kOut * kOut;
#pragma unroll
    for (int j = 0; j < kBandRows; ++j) {
      const int oy = oy0 + j;
#pragma unroll
      for (int c = 0; c < 3; ++c) o[((int64_t)c * kOut + oy) * kOut + tid] = s_lut[c * 256 + clip8(acc[j][c])];
    }
  }
}

// ---------------------------------------------------------------------------
// Samplers.
// ---------------------------------------------------------------------------
// ShardedBatchSampler (README.md:257-271): pairs [k*B, min(k*B+B, N)), k = r, r+W, ...
__global__ void k_shard_ranges(int64_t num_rows, int64_t bsz, int rank, int world,
                               int64_t *out, int64_t capacity, int64_t *count) {
  const int64_t nb = (num_rows + bsz - 1) / bsz;
  const int64_t cnt = rank < nb ? (nb - rank + world - 1) / world : 0;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *count = cnt;
  if (i < cnt && i < capacity) {
    const int64_t k = rank + i * world;
    const int64_t s = k * bsz;
    out[2 * i] = s;
    out[2 * i + 1] = min(s + bsz, num_rows);
  }
}

// ShardedFragmentSampler (README.md:140-155) + this build's pad rule.
// Single workgroup: per-fragment batch counts, block scans over fragments
// (global batch ids and own-rank batch ids), then record emission.
__global__ void __launch_bounds__(256) k_shard_fragments(const int64_t *frag_rows, int nfrag,
                                                         int64_t bsz, int rank, int world,
                                                         int64_t pad_to, int64_t *out,
                                                         int64_t capacity, int64_t *count,
                                                         int64_t *local_count) {
  __shared__ long long sh_scan[8];
  __shared__ long long sh_tot[3]; // own batches, global batches, rows
  const int tid = threadIdx.x;
  if (tid == 0) {
    sh_tot[0] = sh_tot[1] = sh_tot[2] = 0;
  }
  __syncthreads();
  // pass 1: own records (64-bit scans: a dataset may hold 2^31 rows or more)
  for (int f0 = 0; f0 < nfrag; f0 += 256) {
    const int f = f0 + tid;
    const int64_t rows = f < nfrag ? frag_rows[f] : 0;
    const int64_t nbf = (rows + bsz - 1) / bsz;
    const int64_t own = (f < nfrag && (f % world) == rank) ? nbf : 0;
    int64_t tot_own, tot_all, tot_rows;
    const int64_t own_ex = block_excl_scan256_i64(own, sh_scan, &tot_own);
    (void)block_excl_scan256_i64(nbf, sh_scan, &tot_all);
    const int64_t row_ex = block_excl_scan256_i64(rows, sh_scan, &tot_rows);
    const int64_t own_base = sh_tot[0] + own_ex;
    const int64_t gstart = sh_tot[2] + row_ex;
    for (int64_t j = 0; j < own; ++j) {
      const int64_t idx = own_base + j;
      if (idx >= capacity) break;
      int64_t *rec = out + idx * 5;
      rec[0] = f;
      rec[1] = j * bsz;
      rec[2] = min((j + 1) * bsz, rows);
      rec[3] = gstart + j * bsz;
      rec[4] = 0;
    }
    __syncthreads();
    if (tid == 0) {
      sh_tot[0] += tot_own;
      sh_tot[1] += tot_all;
      sh_tot[2] += tot_rows;
    }
    __syncthreads();
  }
  const int64_t own_n = sh_tot[0];
  const int64_t all_n = sh_tot[1];
  if (tid == 0) {
    *local_count = own_n;
    *count = pad_to > own_n ? pad_to : own_n;
  }
  if (pad_to <= own_n) return;
  __syncthreads();
  if (own_n > 0) {
    // cycle own records
    for (int64_t i = own_n + tid; i < pad_to; i += 256) {
      if (i >= capacity) break;
      const int64_t srci = (i - own_n) % own_n;
      if (srci >= capacity) continue;
      for (int q = 0; q < 4; ++q) out[i * 5 + q] = out[srci * 5 + q];
      out[i * 5 + 4] = 1;
    }
    return;
  }
  if (all_n == 0) {
    if (tid == 0) *count = 0;
    return;
  }
  // rank owns nothing: cycle the global batch list from index `rank`
  for (int64_t i = tid; i < pad_to; i += 256) {
    if (i >= capacity) break;
    int64_t gidx = (rank + i) % all_n;
    // locate global batch gidx by walking fragments (nfrag small in practice)
    int64_t acc = 0, rowbase = 0;
    for (int f = 0; f < nfrag; ++f) {
      const int64_t rows = frag_rows[f];
      const int64_t nbf = (rows + bsz - 1) / bsz;
      if (gidx < acc + nbf) {
        const int64_t j = gidx - acc;
        int64_t *rec = out + i * 5;
        rec[0] = f;
        rec[1] = j * bsz;
        rec[2] = min((j + 1) * bsz, rows);
        rec[3] = rowbase + j * bsz;
        rec[4] = 1;
        break;
      }
      acc += nbf;
      rowbase += rows;
    }
  }
}

// ---------------------------------------------------------------------------
// Host launchers.
// ---------------------------------------------------------------------------
hipError_t launch_destuff(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n == 0) return hipSuccess;
  if (p.n_chunks > 0) {
    hipLaunchKernelGGL(k_destuff_count, dim3(p.n_chunks), dim3(256), 0, s, w.data, p.descs,
                       p.chunk_img, w.ds_cnt, w.status);
    hipLaunchKernelGGL(k_destuff_write, dim3(p.n_chunks), dim3(256), 0, s, w.data, p.descs, p.segs,
                       p.chunk_img, w.ds_cnt, w.dstuf, w.status);
  }
  if (p.n_ds_img > 0)
    hipLaunchKernelGGL(k_destuff_layout, dim3(p.n), dim3(256), 0, s, p.descs, p.segs, w.ds_cnt,
                       w.dstuf, w.status);
  return hipGetLastError();
}

hipError_t launch_idct(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n == 0 || p.max_blocks == 0) return hipSuccess;
  dim3 grid((unsigned)((p.max_blocks + kIdctBlocksPerWg - 1) / kIdctBlocksPerWg), (unsigned)p.n);
  hipLaunchKernelGGL(k_idct, grid, dim3(kIdctBlocksPerWg), 0, s, p.descs, p.qtabs, w.coef, w.brec, w.bcarry, w.pcoef, w.dcv, w.planes,
                     w.status);
  return hipGetLastError();
}

static size_t resize_lds_bytes(int ks_h, int ks_v, int row_bytes) {
  return 3072 + (size_t)4 * (kOut * ks_h + kBandRows * ks_v + 2 * kOut + 2 * kBandRows) +
         2 * (size_t)row_bytes;
}

static int round_row_bytes(int w) { return ((w * 3 + 15) / 16) * 16; }

// Allow up to the full 160 KiB of LDS for the resize kernels (wide images).
static hipError_t resize_lds_attr() {
  static hipError_t once = [] {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_resize<0>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess)
      e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_resize<1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return e;
  }();
  return once;
}

hipError_t launch_resize_jpeg(const DevPlan &p, const DevWork &w, float *out, int64_t *out_labels,
                              hipStream_t s) {
  if (p.n == 0) return hipSuccess;
  const int nb = kOut / kBandRows;
  const int groups = (p.n + 7) / 8;
  const int row_bytes = round_row_bytes(p.max_w);
  const size_t lds = resize_lds_bytes(p.max_ks_h, p.max_ks_v, row_bytes);
  if (lds > 64 * 1024) {
    hipError_t e = resize_lds_attr();
    if (e != hipSuccess) return e;
  }
  RawSrc raw{nullptr, 0, 0, 0};
  hipLaunchKernelGGL(k_resize<0>, dim3(groups * 8 * nb), dim3(kResizeThreads), lds, s, p.descs,
                     w.planes, raw, p.lut, p.labels, out, out_labels, w.status, p.n, p.max_ks_h,
                     p.max_ks_v, row_bytes);
  return hipGetLastError();
}

hipError_t launch_resize_raw(const uint8_t *hwc, int64_t cell_stride, int n, int h, int w,
                             const float *lut, float *out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const int nb = kOut / kBandRows;
  const int groups = (n + 7) / 8;
  const int ks_h = resample_ksize_host(w, kOut), ks_v = resample_ksize_host(h, kOut);
  const int row_bytes = round_row_bytes(w);
  const size_t lds = resize_lds_bytes(ks_h, ks_v, row_bytes);
  if (lds > 64 * 1024) {
    hipError_t e = resize_lds_attr();
    if (e != hipSuccess) return e;
  }
  RawSrc raw{hwc, cell_stride, h, w};
  hipLaunchKernelGGL(k_resize<1>, dim3(groups * 8 * nb), dim3(kResizeThreads), lds, s,
                     (const ImgDesc *)nullptr, (const uint8_t *)nullptr, raw, lut,
                     (const int64_t *)nullptr, out, (int64_t *)nullptr, (const int32_t *)nullptr, n,
                     ks_h, ks_v, row_bytes);
  return hipGetLastError();
}

hipError_t launch_resample_coeffs(int in_size, int out_size, int ksize, int32_t *bounds,
                                  int32_t *kk, hipStream_t s) {
  hipLaunchKernelGGL(k_resample_coeffs, dim3((out_size + 255) / 256), dim3(256), 0, s, in_size,
                     out_size, ksize, bounds, kk);
  return hipGetLastError();
}

hipError_t launch_shard_ranges(int64_t num_rows, int64_t bsz, int rank, int world, int64_t *out,
                               int64_t capacity, int64_t *count, hipStream_t s) {
  const int64_t nb = bsz > 0 ? (num_rows + bsz - 1) / bsz : 0;
  const int64_t cnt = rank < nb ? (nb - rank + world - 1) / world : 0;
  const int64_t threads = cnt > 0 ? cnt : 1;
  hipLaunchKernelGGL(k_shard_ranges, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                     num_rows, bsz, rank, world, out, capacity, count);
  return hipGetLastError();
}

hipError_t launch_shard_fragments(const int64_t *frag_rows, int nfrag, int64_t bsz, int rank,
                                  int world, int64_t pad_to, int64_t *out, int64_t capacity,
                                  int64_t *count, int64_t *local_count, hipStream_t s) {
  hipLaunchKernelGGL(k_shard_fragments, dim3(1), dim3(256), 0, s, frag_rows, nfrag, bsz, rank,
                     world, pad_to, out, capacity, count, local_count);
  return hipGetLastError();
}

} // namespace ldt

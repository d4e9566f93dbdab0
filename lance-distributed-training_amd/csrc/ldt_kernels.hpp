// ldt_kernels.hpp — host-callable launchers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldt_types.hpp"

namespace ldt {

__host__ __device__ inline int resample_ksize_host(int inSize, int outSize) {
  int s = (inSize + outSize - 1) / outSize;
  if (s < 1) s = 1;
  return s * 2 + 1;
}

struct RawSrc {
  const uint8_t *base;
  int64_t cell_stride;
  int h, w;
};

struct DevPlan {
  const ImgDesc *descs;
  Segment *segs;
  const HuffTab *htabs;
  const uint16_t *qtabs;
  const float *lut;
  const int64_t *labels; // may be null
  int n, nseg;
  int max_ks_h, max_ks_v, max_w, max_h;
  int64_t max_blocks;
  // Huffman decode: k_huff_image (one workgroup per image) and k_huff_serial
  int n_par;              // images on the parallel decoder
  const int32_t *par_img; // its workgroup -> image
  int n_serial;           // images on the serial decoder (sub_bits == 0)
  int win_bytes;          // LDS window of k_huff_image (images needing more read global memory)
  int warm_pct;           // phase-1 warm-up before each range, % of S
  int resize_waves_pct;   // k_resize4 band count, % of one full wave of resize waves
  int resize_wpg;         // k_resize4 waves per workgroup for JPEG sources (0: default 2)
  int resize420;          // 4:2:0 images <= 512 px: 3 k_resize4<5> (packed 16-bit staging), 0 k_resize4<0>
  int32_t *redo;          // debug counters of the parallel decoder (16 ints)
  int max_tabs;           // max distinct Huffman tables of one image (LDS slots)
  int n_fast420;         // images on k_resize4's fast staging path (resize_fast420)
  // progressive images (k_prog, one workgroup each)
  int n_prog;
  const int32_t *prog_img; // -> image index
  const ProgScan *pscans;
  const ProgTab *ptabs;
  // destuff chunks (4 KB of entropy-coded bytes each)
  int n_chunks;
  int n_ds_img;           // baseline images destuffed by k_destuff_* (the others: k_huff_image)
  const int32_t *chunk_img; // chunk -> image
};

// Coefficients of baseline images (the Huffman decoders' output), packed:
// a block's nonzero 16-byte groups (zigzag slots 8g..8g+7, slot 0 unused) in
// increasing g, one 16-byte unit each, in the image's region of `coef`
// (starting at coef_off * 64 int16s, room for 8 units per block). A run (the
// blocks one decoder lane owns, consecutive) writes its blocks' units
// contiguously from unit 8 * (its first block), so its first unit is
// 64-byte aligned and it writes whole 64-byte segments. Per block a 4-byte
// record brec[coef_off + ib] = nonzero-group mask (bits 0-7) | run start
// (bit 8) | DC (bits 16-31: the difference from the decoder, the absolute
// value after the predictor scan), and per 64 blocks a carry
// bcarry[coef_off / 64 + c] = the first unit of block 64c. A block's first
// unit is then 8 * ib at a run start, else its predecessor's first unit plus
// the predecessor's group count: k_idct, whose waves own 64 consecutive
// blocks, gets it with one segmented wave scan from the chunk's carry.
// Nothing is read that was not written in the same batch, so the buffer needs
// no clearing.
//
// Progressive images (k_prog) refine coefficients over many scans, so they
// keep dense per-image group planes in `pcoef`: zigzag slots 8g..8g+7 of block
// ib at piece g * npad + ib of the region at pcoef_off * 64 int16s (npad = the
// block count rounded up to 64), so the 64 lanes of a wave owning 64
// consecutive blocks read group g with one contiguous 1 KB access. That buffer
// is all zero between batches (k_idct clears the groups it read).
constexpr int kCoefAlign = 64;
__host__ __device__ __forceinline__ int coef_npad(const ImgDesc &d) {
  return (int)(((int64_t)d.mcux * d.mcuy * d.bpm + kCoefAlign - 1) & ~(int64_t)(kCoefAlign - 1));
}
// Index of the 16-byte piece (block ib, group g) from the image's dense region.
// npad < 2^24 (LDT_MAX_DIM 8192, 4:4:4), so this is one 24-bit multiply-add.
__host__ __device__ __forceinline__ uint32_t coef_piece(int ib, int g, int npad) {
  return __umul24((unsigned)g, (unsigned)npad) + (unsigned)ib;
}

struct DevWork {
  const uint8_t *data;  // compressed cells
  uint8_t *dstuf;       // destuffed entropy data
  int16_t *coef;        // baseline images: packed nonzero coefficient groups (above)
  uint32_t *brec;       // baseline images: per block group mask | run start << 8 | DC << 16
  uint32_t *bcarry;     // baseline images: per 64 blocks the first unit of the chunk's first block
  int16_t *pcoef;       // progressive images: dense group planes, all zero between batches
  int16_t *dcv;         // progressive images, per block (coef_off): absolute DC (k_prog)
  uint8_t *planes;      // component planes
  int32_t *status;      // per image
  int4 *ds_cnt;         // per destuff chunk: kept bytes, RSTn markers, end marker seen
};

hipError_t launch_destuff(const DevPlan &p, const DevWork &w, hipStream_t s);
hipError_t launch_huff_serial(const DevPlan &p, const DevWork &w, hipStream_t s);
hipError_t launch_huff_parallel(const DevPlan &p, const DevWork &w, hipStream_t s);
hipError_t launch_dc_scan(const DevPlan &p, const DevWork &w, hipStream_t s);
hipError_t launch_idct(const DevPlan &p, const DevWork &w, hipStream_t s);
// Progressive (SOF2) images: serial per-scan decode into coef/dcv (ldt_prog.hip).
hipError_t launch_prog(const DevPlan &p, const DevWork &w, hipStream_t s);
// Failed rows: zero image, label -100 (after the resize kernels).
hipError_t launch_fill_failed(const DevPlan &p, const DevWork &w, float *out, int64_t *out_labels,
                              hipStream_t s);
hipError_t launch_resize_jpeg(const DevPlan &p, const DevWork &w, float *out, int64_t *out_labels,
                              hipStream_t s);
// One-wave-per-band resize (ldt_resize4.hip); false when unsupported (taps
// > 11, i.e. sources wider than 1120 px, or LDS), then the streaming
// workgroup kernel (launch_resize_jpeg / launch_resize_raw) is used.
// *wpg_used: the waves per workgroup the launch took (a tall batch may need
// fewer than the default to fit the LDS); untouched when it returns false
bool launch_resize4_jpeg(const DevPlan &p, const DevWork &w, float *out, int64_t *out_labels,
                         hipStream_t s, hipError_t *err, int *wpg_used = nullptr);
bool launch_resize4_raw(const uint8_t *hwc, int64_t cell_stride, int n, int h, int wd,
                        const float *lut, float *out, hipStream_t s, hipError_t *err);
hipError_t launch_resize_raw(const uint8_t *hwc, int64_t cell_stride, int n, int h, int w,
                             const float *lut, float *out, hipStream_t s);
hipError_t launch_resample_coeffs(int in_size, int out_size, int ksize, int32_t *bounds,
                                  int32_t *kk, hipStream_t s);
hipError_t launch_shard_ranges(int64_t num_rows, int64_t bsz, int rank, int world, int64_t *out,
                               int64_t capacity, int64_t *count, hipStream_t s);
hipError_t launch_shard_fragments(const int64_t *frag_rows, int nfrag, int64_t bsz, int rank,
                                  int world, int64_t pad_to, int64_t *out, int64_t capacity,
                                  int64_t *count, int64_t *local_count, hipStream_t s);
// DistributedSampler indices (ldt_sampler.hip). Shuffled: the rank's
// num_samples entries of torch.randperm(n) strided from rank (H, head, nxt: n
// int32 each of scratch). launch_dist_select: the unshuffled identity.
hipError_t launch_dist_shuffled(uint32_t seed, int64_t n, int rank, int world,
                                int64_t num_samples, int32_t *H, int32_t *head, int32_t *nxt,
                                int64_t *out, hipStream_t s);
hipError_t launch_dist_select(const int32_t *perm, int64_t n, int rank, int world,
                              int64_t num_samples, int64_t *out, hipStream_t s);

} // namespace ldt

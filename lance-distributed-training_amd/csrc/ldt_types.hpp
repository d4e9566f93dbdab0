// ldt_types.hpp — plain-old-data structures shared by the host planner
// (ldt_abi.cpp) and the gfx950 kernels (ldt_kernels.hip). Everything here is
// laid out for one H2D copy of a per-batch "plan" blob into HBM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ldt {

constexpr int kOut = 224;            // transforms.Resize((224, 224)) lance_iterable.py:29
constexpr int kMaxBlocksPerMcu = 10; // T.81 limit for interleaved scans
constexpr int kLookBits = 11;        // first-level Huffman lookup bits (libjpeg HUFF_LOOKAHEAD = 8)
constexpr int kPrecisionBits = 22;   // Pillow Resample.c PRECISION_BITS = 32 - 8 - 2

// Per-image descriptor, one per row of the batch.
struct ImgDesc {
  int32_t width, height;
  int32_t ncomp;     // 1 or 3
  int32_t color;     // 0: YCbCr->RGB, 1: RGB passthrough (Adobe transform 0), 2: gray
  int32_t mcux, mcuy;
  int32_t bpm;       // blocks per MCU
  int32_t restart;   // MCUs per restart interval, 0 = none
  int32_t nseg;      // entropy segments (restart intervals)
  int32_t seg_base;  // first index in the segment table
  int64_t src_off;   // entropy-coded bytes: absolute offset in the device data buffer
  int64_t src_len;   // bytes from src_off to the end of the cell
  int64_t dst_off;   // destuffed bytes: offset in the destuff buffer
  int64_t coef_off;  // first block (x64 coefficients) in the coefficient buffer
  int64_t plane_off[3];
  int32_t plane_stride[3]; // bytes per plane row (blocks_w * 8)
  int32_t cdw[3], cdh[3];  // libjpeg downsampled_width / downsampled_height
  int32_t hf[3], vf[3];    // upsampling factor per component (hmax/h, vmax/v)
  int32_t ch[3], cv[3];    // sampling factors h, v in the MCU
  int32_t qt[3];           // quant table index (plan quant array)
  int32_t dct[3], act[3];  // Huffman table indices (plan table array)
  uint8_t bcomp[kMaxBlocksPerMcu], bdx[kMaxBlocksPerMcu], bdy[kMaxBlocksPerMcu];
  uint8_t pad_[2];
  // destuff: this image's 4 KB chunks are [ds_first, ds_first + ds_count)
  int32_t ds_first, ds_count;
  // parallel Huffman decode (k_huff_image, one workgroup per image): the
  // subsequence length S of this image in bits; 0 = the serial decoder
  int32_t sub_bits;
  int32_t pad1_;
  // progressive (SOF2) images: scans [prog_first, prog_first + prog_count) of
  // the plan's scan table, decoded by k_prog; nseg == 0 (no baseline segments)
  int32_t prog_first, prog_count;
  // progressive images: first block of the image's dense group planes in the
  // progressive coefficient buffer (DevWork::pcoef)
  int64_t pcoef_off;
};

// k_resize4's fast staging path: 4:2:0 YCbCr with both chroma planes
// fancy-upsampled (h2v2), one lane per 8 luma columns (W <= 512). Shared by
// the host dispatch and the kernel so both agree image by image.
__host__ __device__ inline bool resize_fast420(const ImgDesc &d) {
  return d.color == 0 && d.hf[1] == 2 && d.vf[1] == 2 && d.hf[2] == 2 && d.vf[2] == 2 &&
         d.cdw[1] > 2 && d.cdw[2] > 2 && d.cdw[1] == d.cdw[2] && d.cdh[1] == d.cdh[2] &&
         d.plane_stride[1] == d.plane_stride[2] && d.width <= 512;
}

// One entropy-coded segment (a restart interval, or the whole scan).
struct Segment {
  int32_t img;
  int32_t mcu_first;
  int32_t mcu_count;
  int32_t sub_first;  // first subsequence thread (image-local index), set on device
  int64_t byte_start; // destuffed, absolute in the destuff buffer (set on device)
  int64_t byte_end;
  int32_t sub_count;  // subsequences of S bits, set on device
  int32_t pad_[3];
};

// Parallel Huffman decoder (k_huff_image): one workgroup of kHuffThreads
// lanes per image, one subsequence slot per lane. Images with more restart
// segments than kMaxParSegs take the serial decoder (one lane per segment).
constexpr int kHuffThreads = 1024;
constexpr int kMaxParSegs = 256;
constexpr int kMaxParS = 32768;           // larger S (huge images): serial decoder
constexpr int kHuffLdsMax = 160 * 1024;   // LDS per CU (gfx950)
constexpr int kHuffStaticLds = 42 * 1024; // k_huff_image's static LDS (ImgLds) + margin
// Zero bytes after every destuffed segment (restart interval): a bit reader
// may look up to 8 bytes past a segment without a bounds check and reads the
// zeros libjpeg inserts at a marker (jdhuff.c jpeg_fill_bit_buffer).
constexpr int kSegPad = 8;
// Destuffed bytes reserved for an image (all segments, their pads, slack);
// 16-aligned, so every image's region starts 16-aligned.
__host__ __device__ inline int64_t destuff_region_bytes(int64_t src_len, int nseg) {
  return (src_len + 16 + (int64_t)kSegPad * nseg + 15) & ~(int64_t)15;
}
// Destuff work unit: bytes of entropy-coded data per workgroup.
constexpr int kDsChunkBytes = 4096;

// Device Huffman table: jdhuff.c's d_derived_tbl restated as a two-level
// lookup over the next 16 bits: l1 by the next kLookBits bits, l2 (chunks of
// 2^kL2Bits) by the following kL2Bits. Entries are 16 bits:
//   total (bits 0-4)  code length + extra (magnitude) bits, >= 1
//   s     (bits 5-8)  extra bits (jdhuff.c s; DC: the symbol, AC: symbol & 15)
//   adv   (bits 9-15) advance of the coefficient index k: DC 1; AC r + 1 if
//                     s != 0, 16 for ZRL, 64 for EOB (ends the block)
// total == 0 marks an indirect l1 entry: s-field = chunk of l2, or
// 15 = canonical maxcode search (tables
// with more than kL2Chunks long-code prefixes). Unused codes hold the invalid
// entry (libjpeg: warning, 16 bits skipped, symbol 0).
constexpr int kL2Chunks = 8;
constexpr int kL2Bits = 16 - kLookBits;
constexpr uint32_t kHuffCanon = 15u << 5;
// A table in the decoders' LDS: lc (uint32 per kLookBits-bit peek: l1 entry in
// the low half, count-mode entry in the high half), then l2 (uint16).
constexpr int kL2Off = 2 << kLookBits;                      // l2 offset in uint16
constexpr int kTabStride = kL2Off + (kL2Chunks << kL2Bits); // uint16 per table
// LDS bytes of an image's distinct Huffman tables in the decoders
__host__ __device__ inline int huff_tab_lds(int max_tabs) {
  return (max_tabs < 1 ? 1 : max_tabs) * kTabStride * 2;
}
// k_huff_image's table area: the tables as above for phase 1 and the rounds;
// for the write pass each table's lc part is compacted to its l1 halves (4 KB,
// then its 512-byte l2 part), and the rest holds the write pass's coefficient
// groups (kHuffThreads x 16 B, 4 B of padding per 8 lanes). Sized so that both fit for every image
// of the batch (ns <= max_tabs distinct tables).
constexpr int kHuffPlaneBytes = 16 * kHuffThreads + 4 * (kHuffThreads / 8); // + 4 B per 8 lanes
constexpr int kTabCompactBytes = (2 << kLookBits) + 2 * (kL2Chunks << kL2Bits);
__host__ __device__ inline int huff_tab_lds_image(int max_tabs) {
  const int t = max_tabs < 1 ? 1 : max_tabs;
  const int a = huff_tab_lds(t), b = t * kTabCompactBytes + kHuffPlaneBytes;
  return a > b ? a : b;
}
__host__ __device__ inline uint16_t huff_entry(int len, int sym, bool dc) {
  int s, adv;
  if (dc) {
    s = sym;
    adv = 1;
  } else {
    s = sym & 15;
    const int r = sym >> 4;
    adv = s ? r + 1 : (r == 15 ? 16 : 64);
  }
  return (uint16_t)((len + s) | (s << 5) | (adv << 9));
}
// Count-mode entries (the parallel decoder's sync passes only count blocks,
// so one lookup may consume several symbols), per kLookBits-bit peek, laid out
// like the l1 entries (total bits 0-4, advance 9-15):
//   T (bits 0-4)    bits of the longest run of AC symbols of one block whose
//                   codes all lie in the peeked bits (the last symbol's
//                   magnitude may extend past them); DC tables: one symbol
//   PRE (5-8)       advance before the run's last symbol (<= 15): no block
//                   ends inside the run while k + PRE < 64 (the decoder uses
//                   the run entries for k <= 48 only)
//   ADV (9-15)      coefficient advance of the run (an EOB, 64, ends it)
// T == 0: a long code; the entry equals l1's indirect entry.
struct HuffTab {
  uint32_t lc[1 << kLookBits]; // l1 | cnt << 16
  uint16_t l2[kL2Chunks << kL2Bits];
  int32_t maxcode[18]; // [l] largest code of length l (-1 none), [17] sentinel
  int32_t valoff[18];
  uint8_t vals[256];
};

// One scan of a progressive image (jdphuff.c start_pass_phuff_decoder
// parameters), in file order.
struct ProgScan {
  int32_t ss, se, ah, al; // spectral band [ss, se], successive approximation
  int32_t ns;             // components in the scan (> 1 only for DC scans)
  int32_t restart;        // restart interval (MCUs) in force for the scan
  int32_t comp[4];        // frame component index of each scan component
  int32_t tab[4];         // ProgTab index: DC first -> DC table per component,
                          // AC scans -> tab[0] = AC table; -1 if unused
  int64_t data_off;       // entropy-coded bytes: absolute offset in the data buffer
  int64_t data_len;       // bytes up to the marker that ends the scan
};

// Progressive-scan Huffman table for the serial decoder: an 8-bit lookahead
// (jdhuff.c HUFF_LOOKAHEAD) plus the canonical maxcode/valoffset search.
struct ProgTab {
  uint16_t look[256];  // codes <= 8 bits: (length << 8) | symbol; 0 = longer code
  int32_t maxcode[18]; // [l] largest code of length l (-1 none), [17] sentinel
  int32_t valoff[18];
  uint8_t vals[256];
};
constexpr int kMaxProgScans = 64; // per image; more -> LDT_IMG_UNSUPPORTED

// Per-batch plan header; offsets are bytes from the start of the plan blob.
struct PlanHdr {
  int32_t n;
  int32_t nseg;
  int32_t nhuff;
  int32_t nquant;
  int64_t off_desc, off_seg, off_huff, off_quant, off_lut, off_labels;
  int32_t has_labels;
  int32_t max_ks_h;      // max horizontal taps over the batch
  int32_t max_ks_v;
  int32_t max_w;
  int64_t max_blocks;    // max blocks of one image
  int64_t total_blocks;
};

// Resize kernel launch geometry.
constexpr int kBandRows = 8;       // output rows per workgroup
constexpr int kResizeThreads = 256;

} // namespace ldt

// ldt_types.hpp — plain-old-data structures shared by the host planner
// (ldt_abi.cpp) and the gfx950 kernels (ldt_kernels.hip). Everything here is
// laid out for one H2D copy of a per-batch "plan" blob into HBM.
#pragma once
#include <stdint.h>

namespace ldt {

constexpr int kOut = 224;            // transforms.Resize((224, 224)) lance_iterable.py:29
constexpr int kMaxBlocksPerMcu = 10; // T.81 limit for interleaved scans
constexpr int kLookBits = 9;         // Huffman lookahead (libjpeg HUFF_LOOKAHEAD = 8)
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
  // parallel Huffman decode: this image's subsequence threads occupy
  // workgroups [wg_first, wg_first + wg_count) (256 threads each)
  int32_t wg_first, wg_count;
  int32_t sub_cap;   // thread slots reserved (>= sum of segment sub_count)
  int32_t pad2_;
};

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

// Per-subsequence-thread decode state of the parallel Huffman decoder.
struct SubState {
  int32_t exit_p;   // bit position (segment-relative) of the first symbol at/after the range end
  int32_t exit_bk;  // (b << 8) | k at that symbol
  int32_t nblk;     // DC symbols decoded inside the range (blocks started)
  int32_t dc[3];    // sum of DC differences per component inside the range
};

constexpr int kSyncThreads = 256;
// Lane 0 of every decode workgroup is a helper that warms up on the previous
// workgroup's last subsequence; lanes 1..255 own subsequence slots.
constexpr int kSlotsPerWg = kSyncThreads - 1;

// Device Huffman table: jdhuff.c's d_derived_tbl restated as a two-level
// lookup. l1 is indexed by the next 9 bits: (code_len << 8) | symbol for codes
// of <= 9 bits; 0x8000 | chunk for longer codes, whose symbol is l2[chunk]
// indexed by the following 7 bits; 0xFFFF (tables with more than kL2Chunks
// long-code prefixes) falls back to the canonical maxcode search. An l2 entry
// of 0 is an invalid code (libjpeg: warning, 16 bits skipped, value 0).
constexpr int kL2Chunks = 8;
constexpr int kTabU16 = 512 + kL2Chunks * 128; // uint16 entries per table in LDS
struct HuffTab {
  uint16_t l1[512];
  uint16_t l2[kL2Chunks * 128];
  int32_t maxcode[18]; // [l] largest code of length l (-1 none), [17] sentinel
  int32_t valoff[18];
  uint8_t vals[256];
};

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

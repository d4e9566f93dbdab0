// ldt_huffman.hip — baseline JPEG Huffman decode on gfx950.
//
// Restates libjpeg-turbo jdhuff.c decode_mcu (sequential, Huffman, 8-bit):
//   DC: s = HUFF_DECODE(dc_tbl); diff = HUFF_EXTEND(GET_BITS(s), s); pred += diff
//   AC: for k = 1..63: rs = HUFF_DECODE(ac_tbl); r = rs >> 4; s = rs & 15;
//         s != 0: k += r; coef[natural[k]] = HUFF_EXTEND(GET_BITS(s), s)
//         s == 0: r == 15 ? k += 15 (ZRL) : break (EOB)
// Bits past a segment's end read as zero (jdhuff.c inserts zeros at a marker).
// Input: destuffed segments (k_destuff). Output: int16 coefficients, natural
// order, block (mcu, b) at coef_off + mcu * bpm + b.
//
// Two decoders share one inner loop (decode_until):
//   k_huff_serial    one lane per segment (restart interval or whole scan).
//   k_huff_sync_*    self-synchronising parallel decode (Weissenberger &
//                    Schmidt, ICPP 2018): a segment is cut into subsequences
//                    of S bits, every lane decodes one subsequence from a
//                    guessed state, lanes re-decode from their predecessor's
//                    exit state until exit states stop changing (Huffman codes
//                    resynchronise within tens of symbols), then a prefix sum
//                    places each lane's blocks and a final pass writes them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldt_kernels.hpp"

namespace ldt {

__constant__ uint8_t c_natural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// MSB-first bit reader over destuffed bytes [start, end); zeros past `end`.
// Reads aligned 32-bit words (the destuff buffer is padded past every image).
struct BitReader {
  const uint8_t *base;
  int64_t wpos;   // next byte address to load (multiple of 4)
  int64_t end;    // absolute end byte
  uint64_t buf;   // MSB-aligned
  int n;          // valid bits in buf

  __device__ __forceinline__ uint32_t load_word(int64_t a) const {
    if (a >= end) return 0u;
    uint32_t w = *reinterpret_cast<const uint32_t *>(base + a);
    w = __builtin_bswap32(w);
    const int64_t valid = end - a;
    if (valid < 4) w &= ~(0xFFFFFFFFu >> (8 * valid));
    return w;
  }
  // Position `bitpos` = absolute bit address (byte * 8).
  __device__ __forceinline__ void init(const uint8_t *b, int64_t bitpos, int64_t e) {
    base = b;
    end = e;
    const int64_t byte = bitpos >> 3;
    const int64_t a = byte & ~(int64_t)3;
    const int skip = (int)(bitpos - a * 8);
    buf = (uint64_t)load_word(a) << 32;
    buf |= (uint64_t)load_word(a + 4);
    buf <<= skip;
    n = 64 - skip;
    wpos = a + 8;
  }
  __device__ __forceinline__ void refill() {
    if (n <= 32) {
      buf |= (uint64_t)load_word(wpos) << (32 - n);
      n += 32;
      wpos += 4;
    }
  }
  __device__ __forceinline__ int64_t bitpos() const { return wpos * 8 - n; }
  __device__ __forceinline__ uint32_t peek(int k) const { return (uint32_t)(buf >> (64 - k)); }
  __device__ __forceinline__ void skip(int k) {
    buf <<= k;
    n -= k;
  }
};

// jdhuff.c jpeg_huff_decode with a 9-bit lookahead table.
__device__ __forceinline__ int huff_decode(BitReader &br, const HuffTab *__restrict__ t) {
  const uint32_t e = t->lut[br.peek(kLookBits)];
  if (e >> 8) {
    br.skip((int)(e >> 8));
    return (int)(e & 0xFF);
  }
  const uint32_t w = br.peek(16);
  for (int l = kLookBits + 1; l <= 16; ++l) {
    const int code = (int)(w >> (16 - l));
    if (code <= t->maxcode[l]) {
      br.skip(l);
      return t->vals[(t->valoff[l] + code) & 0xFF];
    }
  }
  br.skip(16); // bad code: libjpeg warns and yields 0
  return 0;
}

__device__ __forceinline__ int huff_extend(uint32_t v, int s) {
  return (s == 0) ? 0 : ((int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v);
}

__device__ __forceinline__ uint32_t get_bits(BitReader &br, int s) {
  if (s == 0) return 0;
  const uint32_t v = br.peek(s);
  br.skip(s);
  return v;
}

// Decode `nmcu` MCUs of one segment starting at MCU `mcu0`, writing
// coefficients (DC already prediction-resolved: pred starts at 0 per segment).
__device__ void decode_segment_serial(const ImgDesc &d, const HuffTab *__restrict__ htabs,
                                      BitReader &br, int mcu0, int nmcu,
                                      int16_t *__restrict__ coef) {
  int pred0 = 0, pred1 = 0, pred2 = 0;
  const int bpm = d.bpm;
  for (int m = 0; m < nmcu; ++m) {
    int16_t *mcu_coef = coef + (d.coef_off + (int64_t)(mcu0 + m) * bpm) * 64;
    for (int b = 0; b < bpm; ++b) {
      const int c = d.bcomp[b];
      const HuffTab *dct = htabs + d.dct[c];
      const HuffTab *act = htabs + d.act[c];
      int16_t *blk = mcu_coef + b * 64;
      br.refill();
      int s = huff_decode(br, dct);
      br.refill();
      const int diff = huff_extend(get_bits(br, s), s);
      int p;
      if (c == 0) p = (pred0 += diff);
      else if (c == 1) p = (pred1 += diff);
      else p = (pred2 += diff);
      blk[0] = (int16_t)p;
      for (int k = 1; k < 64; ++k) {
        br.refill();
        const int rs = huff_decode(br, act);
        const int r = rs >> 4;
        s = rs & 15;
        if (s) {
          k += r;
          br.refill();
          blk[c_natural[k]] = (int16_t)huff_extend(get_bits(br, s), s);
        } else {
          if (r != 15) break;
          k += 15;
        }
      }
    }
  }
}

__global__ void __launch_bounds__(64) k_huff_serial(const ImgDesc *__restrict__ descs,
                                                    const Segment *__restrict__ segs, int nseg,
                                                    const HuffTab *__restrict__ htabs,
                                                    const uint8_t *__restrict__ dstuf,
                                                    int16_t *__restrict__ coef,
                                                    int32_t *__restrict__ status) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  const Segment sg = segs[s];
  const ImgDesc &d = descs[sg.img];
  if (status[sg.img] != 0) return;
  BitReader br;
  br.init(dstuf, sg.byte_start * 8, sg.byte_end);
  decode_segment_serial(d, htabs, br, sg.mcu_first, sg.mcu_count, coef);
  if (br.bitpos() > sg.byte_end * 8) status[sg.img] = 3; // ran past the data: truncated
}

hipError_t launch_huff_serial(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.nseg == 0) return hipSuccess;
  hipLaunchKernelGGL(k_huff_serial, dim3((p.nseg + 63) / 64), dim3(64), 0, s, p.descs, p.segs,
                     p.nseg, p.htabs, w.dstuf, w.coef, w.status);
  return hipGetLastError();
}

} // namespace ldt

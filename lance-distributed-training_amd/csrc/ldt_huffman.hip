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

#include "ldt_device.hpp"
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

// ===========================================================================
// Parallel self-synchronising decode.
//
// Threads = subsequences: segment s owns sub_count consecutive image-local
// thread slots starting at sub_first; thread j of a segment owns the bit
// range [j*S, (j+1)*S) of that segment. The decode state at a symbol
// boundary is (p, b, k): bit position, block-in-MCU, coefficient index
// (k == 0: a DC symbol is next). A thread's exit state is the state at the
// first symbol boundary p >= (j+1)*S; the successor's true entry state is
// its predecessor's exit state under the true entry. Equal states decode
// identically from there on, which is what makes the chain converge.
// ===========================================================================

// Bit reader over a workgroup's LDS window of the destuffed stream, falling
// back to global memory outside it.
struct WinReader {
  const uint8_t *g;
  const uint32_t *win; // LDS words for bytes [wbase, wbase + wbytes)
  int64_t wbase;
  int32_t wbytes;
  int64_t wpos, end;
  uint64_t buf;
  int n;

  __device__ __forceinline__ uint32_t load_word(int64_t a) const {
    if (a >= end) return 0u;
    const int64_t o = a - wbase;
    uint32_t w = (o >= 0 && o + 4 <= wbytes) ? win[o >> 2] : *reinterpret_cast<const uint32_t *>(g + a);
    w = __builtin_bswap32(w);
    const int64_t valid = end - a;
    if (valid < 4) w &= ~(0xFFFFFFFFu >> (8 * valid));
    return w;
  }
  __device__ __forceinline__ void init(int64_t bitpos) {
    const int64_t a = (bitpos >> 3) & ~(int64_t)3;
    const int skip = (int)(bitpos - a * 8);
    buf = ((uint64_t)load_word(a) << 32) | (uint64_t)load_word(a + 4);
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

__device__ __forceinline__ int huff_decode_w(WinReader &br, const HuffTab *__restrict__ t) {
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
  br.skip(16);
  return 0;
}

__device__ __forceinline__ int get_extend_w(WinReader &br, int s) {
  if (s == 0) return 0;
  const uint32_t v = br.peek(s);
  br.skip(s);
  return (int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v;
}

struct RunAcc {
  int nblk;
  int dc0, dc1, dc2;
};

// Decode symbols from the reader's position while the segment-relative
// position of the next symbol is < stop. WRITE: also store coefficients
// into block `cursor` (segment-relative), stopping before block `total`.
template <bool WRITE>
__device__ __forceinline__ void decode_run(WinReader &br, int64_t seg_bit0, int64_t stop, int &b,
                                           int &k, const int bpm, const uint8_t *bcomp,
                                           const HuffTab *tabs, RunAcc &acc, int16_t *coef_seg,
                                           int64_t &cursor, int64_t total, int *pred) {
  while (true) {
    const int64_t p = br.bitpos() - seg_bit0;
    if (p >= stop) break;
    br.refill();
    const int c = bcomp[b];
    if (k == 0) {
      if (WRITE) {
        if (cursor + 1 >= total) break;
        ++cursor;
      }
      const int s = huff_decode_w(br, tabs + 2 * c);
      const int v = get_extend_w(br, s);
      acc.nblk += 1;
      if (c == 0) acc.dc0 += v;
      else if (c == 1) acc.dc1 += v;
      else acc.dc2 += v;
      if (WRITE) {
        pred[c] += v;
        coef_seg[cursor * 64] = (int16_t)pred[c];
      }
      k = 1;
    } else {
      const int rs = huff_decode_w(br, tabs + 2 * c + 1);
      const int r = rs >> 4, s = rs & 15;
      if (s) {
        k += r;
        const int v = get_extend_w(br, s);
        if (WRITE && cursor >= 0) coef_seg[cursor * 64 + c_natural[k]] = (int16_t)v;
        ++k;
      } else if (r == 15) {
        k += 16;
      } else {
        k = 64;
      }
      if (k >= 64) {
        k = 0;
        b = (b + 1 == bpm) ? 0 : b + 1;
      }
    }
  }
}

// Locate the segment that owns image-local thread `lt` (sub_first ascending).
__device__ __forceinline__ int find_segment(const Segment *__restrict__ segs, int seg_base, int nseg,
                                            int lt) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[seg_base + mid].sub_first <= lt) lo = mid;
    else hi = mid - 1;
  }
  return seg_base + lo;
}

// Shared workgroup setup of the sync and write kernels: the image's Huffman
// tables (slot 2c = DC, 2c+1 = AC of component c) and the workgroup's window
// of destuffed bytes in LDS.
constexpr int kWinBytes = 36 * 1024;

struct SubCtx {
  int img;
  int seg;        // segment index (global), -1 if inactive
  int j;          // subsequence index within the segment
  int64_t seg_bit0;
  int64_t seg_bits;
  int64_t seg_end; // absolute end byte
  bool active;
};

__device__ __forceinline__ void sub_setup(const ImgDesc &d, const Segment *__restrict__ segs,
                                          const HuffTab *__restrict__ htabs, int S, HuffTab *tabs,
                                          uint32_t *win, int64_t *wbase_out, int *wbytes_out,
                                          long long *sh_lo, long long *sh_hi, const uint8_t *dstuf,
                                          SubCtx &sc, int img) {
  const int tid = threadIdx.x;
  // tables: 6 slots x sizeof(HuffTab) bytes, copied as dwords
  {
    constexpr int kWords = sizeof(HuffTab) / 4;
    for (int i = tid; i < 6 * kWords; i += kSyncThreads) {
      const int slot = i / kWords, o = i - slot * kWords;
      const int c = slot >> 1;
      const int tix = (c < d.ncomp) ? ((slot & 1) ? d.act[c] : d.dct[c]) : 0;
      reinterpret_cast<uint32_t *>(tabs + slot)[o] = reinterpret_cast<const uint32_t *>(htabs + tix)[o];
    }
  }
  const int lt = (int)(blockIdx.x - d.wg_first) * kSyncThreads + tid;
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  const int total_sub = last.sub_first + last.sub_count;
  sc.img = img;
  sc.active = lt < total_sub;
  int64_t lo = INT64_MAX, hi = 0;
  if (sc.active) {
    sc.seg = find_segment(segs, d.seg_base, d.nseg, lt);
    const Segment &sg = segs[sc.seg];
    sc.j = lt - sg.sub_first;
    sc.seg_bit0 = sg.byte_start * 8;
    sc.seg_bits = (sg.byte_end - sg.byte_start) * 8;
    sc.seg_end = sg.byte_end;
    lo = sg.byte_start + ((int64_t)sc.j * S) / 8;
    hi = sg.byte_start + ((int64_t)(sc.j + 1) * S) / 8 + 64;
    if (hi > sg.byte_end + 8) hi = sg.byte_end + 8;
  } else {
    sc.seg = -1;
    sc.j = 0;
    sc.seg_bit0 = sc.seg_bits = sc.seg_end = 0;
  }
  if (tid == 0) {
    *sh_lo = INT64_MAX;
    *sh_hi = 0;
  }
  __syncthreads();
  if (sc.active) {
    atomicMin(sh_lo, (long long)lo);
    atomicMax(sh_hi, (long long)hi);
  }
  __syncthreads();
  int64_t wb = (*sh_lo) & ~(int64_t)3;
  int64_t we = *sh_hi;
  if (we < wb) we = wb;
  int wbytes = (int)((we - wb + 3) & ~(int64_t)3);
  if (wbytes > kWinBytes) wbytes = kWinBytes;
  for (int i = tid; i < wbytes / 4; i += kSyncThreads)
    win[i] = *reinterpret_cast<const uint32_t *>(dstuf + wb + 4 * (int64_t)i);
  *wbase_out = wb;
  *wbytes_out = wbytes;
  __syncthreads();
}

__device__ __forceinline__ void reader_at(WinReader &br, const uint8_t *dstuf, const uint32_t *win,
                                          int64_t wbase, int wbytes, int64_t end, int64_t bitpos) {
  br.g = dstuf;
  br.win = win;
  br.wbase = wbase;
  br.wbytes = wbytes;
  br.end = end;
  br.init(bitpos);
}

// Phase 1 + intra-workgroup convergence.
__global__ void __launch_bounds__(kSyncThreads) k_huff_sync(
    const ImgDesc *__restrict__ descs, const Segment *__restrict__ segs,
    const HuffTab *__restrict__ htabs, const uint8_t *__restrict__ dstuf,
    const int32_t *__restrict__ wg_img, int S, SubState *__restrict__ sub,
    const int32_t *__restrict__ status, int32_t *__restrict__ dbg) {
  __shared__ HuffTab tabs[6];
  __shared__ __attribute__((aligned(16))) uint32_t win[kWinBytes / 4];
  __shared__ int32_t ex_p[kSyncThreads], ex_bk[kSyncThreads];
  __shared__ uint8_t chg[kSyncThreads];
  __shared__ long long sh_lo, sh_hi;
  __shared__ int any_changed;
  __shared__ uint8_t bcomp[kMaxBlocksPerMcu];
  const int img = wg_img[blockIdx.x];
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  if (tid < kMaxBlocksPerMcu) bcomp[tid] = d.bcomp[tid];
  SubCtx sc;
  int64_t wbase;
  int wbytes;
  sub_setup(d, segs, htabs, S, tabs, win, &wbase, &wbytes, &sh_lo, &sh_hi, dstuf, sc, img);
  const int bpm = d.bpm;
  RunAcc acc{0, 0, 0, 0};
  int b = 0, k = 0;
  int64_t cur = 0;
  WinReader br;
  if (sc.active) {
    const int64_t start = (int64_t)sc.j * S;
    const int64_t stop = min((int64_t)(sc.j + 1) * S, sc.seg_bits);
    reader_at(br, dstuf, win, wbase, wbytes, sc.seg_end, sc.seg_bit0 + start);
    decode_run<false>(br, sc.seg_bit0, stop, b, k, bpm, bcomp, tabs, acc, nullptr, cur, 0, nullptr);
    ex_p[tid] = (int32_t)(br.bitpos() - sc.seg_bit0);
    ex_bk[tid] = (b << 8) | k;
  } else {
    ex_p[tid] = 0;
    ex_bk[tid] = 0;
  }
  bool need = sc.active && tid > 0 && sc.j > 0;
  int rounds_done = 0;
  for (int round = 0; round < kSyncThreads + 1; ++round) {
    ++rounds_done;
    __syncthreads();
    if (tid == 0) any_changed = 0;
    bool changed = false;
    int np = 0, nbk = 0;
    if (need) {
      const int ep = ex_p[tid - 1], ebk = ex_bk[tid - 1];
      b = ebk >> 8;
      k = ebk & 255;
      acc = RunAcc{0, 0, 0, 0};
      const int64_t stop = min((int64_t)(sc.j + 1) * S, sc.seg_bits);
      reader_at(br, dstuf, win, wbase, wbytes, sc.seg_end, sc.seg_bit0 + ep);
      decode_run<false>(br, sc.seg_bit0, stop, b, k, bpm, bcomp, tabs, acc, nullptr, cur, 0, nullptr);
      np = (int32_t)(br.bitpos() - sc.seg_bit0);
      nbk = (b << 8) | k;
      changed = (np != ex_p[tid]) || (nbk != ex_bk[tid]);
    }
    __syncthreads();
    chg[tid] = changed ? 1 : 0;
    if (changed) {
      ex_p[tid] = np;
      ex_bk[tid] = nbk;
      any_changed = 1;
    }
    __syncthreads();
    if (!any_changed) break;
    need = sc.active && tid > 0 && sc.j > 0 && chg[tid - 1];
  }
  if (tid == 0 && dbg) {
    atomicAdd(dbg + 1, 1);
    atomicAdd(dbg + 2, rounds_done);
    atomicMax(dbg + 3, rounds_done);
  }
  if (sc.active) {
    SubState st;
    st.exit_p = ex_p[tid];
    st.exit_bk = ex_bk[tid];
    st.nblk = acc.nblk;
    st.dc[0] = acc.dc0;
    st.dc[1] = acc.dc1;
    st.dc[2] = acc.dc2;
    sub[(int64_t)blockIdx.x * kSyncThreads + tid] = st;
  }
}

// Re-decode thread slots from the workgroup boundary at global slot `gt0`
// (image-local `lt0`) until a recomputed exit state equals the stored one.
// bounded = true: stop at the end of the workgroup and raise *redo if the
// chain did not converge (the next workgroup's walk used a stale entry).
__device__ void boundary_walk(const ImgDesc &d, const Segment *__restrict__ segs,
                              const HuffTab *__restrict__ htabs, const uint8_t *__restrict__ dstuf,
                              int S, SubState *__restrict__ sub, int64_t gt0, int lt0, bool bounded,
                              int32_t *redo, int32_t *dbg) {
  const int si = find_segment(segs, d.seg_base, d.nseg, lt0);
  const Segment &sg = segs[si];
  int j = lt0 - sg.sub_first;
  if (j == 0) return;
  const HuffTab *tabs[6];
  for (int c = 0; c < 3; ++c) {
    const int cc = c < d.ncomp ? c : 0;
    tabs[2 * c] = htabs + d.dct[cc];
    tabs[2 * c + 1] = htabs + d.act[cc];
  }
  const int64_t seg_bit0 = sg.byte_start * 8, seg_bits = (sg.byte_end - sg.byte_start) * 8;
  int64_t gt = gt0;
  int ep = sub[gt - 1].exit_p, ebk = sub[gt - 1].exit_bk;
  const int64_t wg_end = (gt0 / kSyncThreads + 1) * kSyncThreads;
  int steps = 0;
  while (true) {
    ++steps;
    int b = ebk >> 8, k = ebk & 255;
    RunAcc acc{0, 0, 0, 0};
    int64_t cur = 0;
    WinReader br;
    br.g = dstuf;
    br.win = nullptr;
    br.wbase = 0;
    br.wbytes = 0;
    br.end = sg.byte_end;
    br.init(seg_bit0 + ep);
    const int64_t stop = min((int64_t)(j + 1) * S, seg_bits);
    // generic-table variant of decode_run (tables in global memory)
    while (true) {
      const int64_t p = br.bitpos() - seg_bit0;
      if (p >= stop) break;
      br.refill();
      const int c = d.bcomp[b];
      if (k == 0) {
        const int s = huff_decode_w(br, tabs[2 * c]);
        const int v = get_extend_w(br, s);
        acc.nblk += 1;
        if (c == 0) acc.dc0 += v;
        else if (c == 1) acc.dc1 += v;
        else acc.dc2 += v;
        k = 1;
      } else {
        const int rs = huff_decode_w(br, tabs[2 * c + 1]);
        const int r = rs >> 4, s = rs & 15;
        if (s) {
          k += r;
          (void)get_extend_w(br, s);
          ++k;
        } else if (r == 15) {
          k += 16;
        } else {
          k = 64;
        }
        if (k >= 64) {
          k = 0;
          b = (b + 1 == d.bpm) ? 0 : b + 1;
        }
      }
    }
    (void)cur;
    const int np = (int)(br.bitpos() - seg_bit0), nbk = (b << 8) | k;
    SubState &st = sub[gt];
    st.nblk = acc.nblk;
    st.dc[0] = acc.dc0;
    st.dc[1] = acc.dc1;
    st.dc[2] = acc.dc2;
    if (np == st.exit_p && nbk == st.exit_bk) {
      if (dbg) {
        atomicAdd(dbg + 4, 1);
        atomicAdd(dbg + 6, steps);
        if (steps == 1) atomicAdd(dbg + 5, 1);
      }
      break; // converged
    }
    st.exit_p = np;
    st.exit_bk = nbk;
    ep = np;
    ebk = nbk;
    ++gt;
    ++j;
    if (j >= sg.sub_count) break; // end of segment: nothing downstream
    if (bounded && gt >= wg_end) {
      atomicExch(redo, 1);
      if (dbg) atomicAdd(dbg + 7, 1);
      break;
    }
  }
}

// One lane per workgroup: walk the chain across its first slot's boundary.
__global__ void __launch_bounds__(64) k_huff_fix(const ImgDesc *__restrict__ descs,
                                                 const Segment *__restrict__ segs,
                                                 const HuffTab *__restrict__ htabs,
                                                 const uint8_t *__restrict__ dstuf,
                                                 const int32_t *__restrict__ wg_img, int n_wg, int S,
                                                 SubState *__restrict__ sub,
                                                 const int32_t *__restrict__ status,
                                                 int32_t *__restrict__ redo) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n_wg) return;
  const int img = wg_img[w];
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const int lt0 = (w - d.wg_first) * kSyncThreads;
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  if (lt0 == 0 || lt0 >= last.sub_first + last.sub_count) return;
  boundary_walk(d, segs, htabs, dstuf, S, sub, (int64_t)w * kSyncThreads, lt0, true, redo, redo);
}

// Fallback when some walk did not converge inside its workgroup: one lane
// per image walks every workgroup boundary in order (always correct).
__global__ void __launch_bounds__(64) k_huff_fix_serial(const ImgDesc *__restrict__ descs,
                                                        const Segment *__restrict__ segs,
                                                        const HuffTab *__restrict__ htabs,
                                                        const uint8_t *__restrict__ dstuf, int n,
                                                        int S, SubState *__restrict__ sub,
                                                        const int32_t *__restrict__ status,
                                                        const int32_t *__restrict__ redo) {
  const int img = blockIdx.x * blockDim.x + threadIdx.x;
  if (img >= n || redo[0] == 0 || status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  const int total = last.sub_first + last.sub_count;
  for (int wl = 1; wl < d.wg_count; ++wl) {
    const int lt0 = wl * kSyncThreads;
    if (lt0 >= total) break;
    boundary_walk(d, segs, htabs, dstuf, S, sub, (int64_t)(d.wg_first + wl) * kSyncThreads, lt0,
                  false, nullptr, nullptr);
  }
}

// Exclusive prefix of (nblk, dc0, dc1, dc2) over each image's thread slots.
__global__ void __launch_bounds__(256) k_huff_scan(const ImgDesc *__restrict__ descs,
                                                   const Segment *__restrict__ segs,
                                                   const SubState *__restrict__ sub,
                                                   int32_t *__restrict__ pre,
                                                   const int32_t *__restrict__ status) {
  __shared__ int sh_scan[8];
  const int img = blockIdx.x;
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  const int total = last.sub_first + last.sub_count;
  const int64_t g0 = (int64_t)d.wg_first * kSyncThreads;
  int run[4] = {0, 0, 0, 0};
  for (int base = 0; base < total; base += 256) {
    const int lt = base + threadIdx.x;
    int v[4] = {0, 0, 0, 0};
    if (lt < total) {
      const SubState &st = sub[g0 + lt];
      v[0] = st.nblk;
      v[1] = st.dc[0];
      v[2] = st.dc[1];
      v[3] = st.dc[2];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int tot;
      const int ex = block_excl_scan256(v[q], sh_scan, &tot);
      if (lt < total) pre[(g0 + lt) * 4 + q] = run[q] + ex;
      run[q] += tot;
    }
  }
}

// Final pass: every slot decodes its range from its true entry state and
// writes coefficients; DC predictors come from the prefix sums.
__global__ void __launch_bounds__(kSyncThreads) k_huff_write(
    const ImgDesc *__restrict__ descs, const Segment *__restrict__ segs,
    const HuffTab *__restrict__ htabs, const uint8_t *__restrict__ dstuf,
    const int32_t *__restrict__ wg_img, int S, const SubState *__restrict__ sub,
    const int32_t *__restrict__ pre, int16_t *__restrict__ coef, int32_t *__restrict__ status) {
  __shared__ HuffTab tabs[6];
  __shared__ __attribute__((aligned(16))) uint32_t win[kWinBytes / 4];
  __shared__ long long sh_lo, sh_hi;
  __shared__ uint8_t bcomp[kMaxBlocksPerMcu];
  const int img = wg_img[blockIdx.x];
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  if (tid < kMaxBlocksPerMcu) bcomp[tid] = d.bcomp[tid];
  SubCtx sc;
  int64_t wbase;
  int wbytes;
  sub_setup(d, segs, htabs, S, tabs, win, &wbase, &wbytes, &sh_lo, &sh_hi, dstuf, sc, img);
  if (!sc.active) return;
  const Segment &sg = segs[sc.seg];
  const int64_t gt = (int64_t)blockIdx.x * kSyncThreads + tid;
  const int64_t gfirst = (int64_t)d.wg_first * kSyncThreads + sg.sub_first;
  int b = 0, k = 0;
  int64_t entry = 0;
  if (sc.j > 0) {
    const SubState &ps = sub[gt - 1];
    entry = ps.exit_p;
    b = ps.exit_bk >> 8;
    k = ps.exit_bk & 255;
  }
  const int32_t *pg = pre + gt * 4, *pf = pre + gfirst * 4;
  int pred[3] = {pg[1] - pf[1], pg[2] - pf[2], pg[3] - pf[3]};
  int64_t cursor = (int64_t)(pg[0] - pf[0]) - 1;
  const int64_t total = (int64_t)sg.mcu_count * d.bpm;
  int16_t *coef_seg = coef + (d.coef_off + (int64_t)sg.mcu_first * d.bpm) * 64;
  const int64_t stop = min((int64_t)(sc.j + 1) * S, sc.seg_bits);
  WinReader br;
  reader_at(br, dstuf, win, wbase, wbytes, sc.seg_end, sc.seg_bit0 + entry);
  RunAcc acc{0, 0, 0, 0};
  decode_run<true>(br, sc.seg_bit0, stop, b, k, d.bpm, bcomp, tabs, acc, coef_seg, cursor, total, pred);
  if (sc.j == sg.sub_count - 1 && cursor + 1 < total) status[img] = 3; // ran out of data
}

hipError_t launch_huff_parallel(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n_wg == 0) return hipSuccess;
  hipLaunchKernelGGL(k_huff_sync, dim3(p.n_wg), dim3(kSyncThreads), 0, s, p.descs, p.segs, p.htabs,
                     w.dstuf, p.wg_img, p.subseq_bits, w.sub, w.status, p.redo);
  hipLaunchKernelGGL(k_huff_fix, dim3((p.n_wg + 63) / 64), dim3(64), 0, s, p.descs, p.segs, p.htabs,
                     w.dstuf, p.wg_img, p.n_wg, p.subseq_bits, w.sub, w.status, p.redo);
  hipLaunchKernelGGL(k_huff_fix_serial, dim3((p.n + 63) / 64), dim3(64), 0, s, p.descs, p.segs,
                     p.htabs, w.dstuf, p.n, p.subseq_bits, w.sub, w.status, p.redo);
  hipLaunchKernelGGL(k_huff_scan, dim3(p.n), dim3(256), 0, s, p.descs, p.segs, w.sub, w.sub_pre,
                     w.status);
  hipLaunchKernelGGL(k_huff_write, dim3(p.n_wg), dim3(kSyncThreads), 0, s, p.descs, p.segs,
                     p.htabs, w.dstuf, p.wg_img, p.subseq_bits, w.sub, w.sub_pre, w.coef, w.status);
  return hipGetLastError();
}

} // namespace ldt

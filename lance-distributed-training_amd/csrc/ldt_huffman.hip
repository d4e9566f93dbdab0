// ldt_huffman.hip — baseline JPEG Huffman decode on gfx950.
//
// Restates libjpeg-turbo jdhuff.c decode_mcu (sequential, Huffman, 8-bit):
//   DC: s = HUFF_DECODE(dc_tbl); diff = HUFF_EXTEND(GET_BITS(s), s); pred += diff
//   AC: for k = 1..63: rs = HUFF_DECODE(ac_tbl); r = rs >> 4; s = rs & 15;
//         s != 0: k += r; coef[natural[k]] = HUFF_EXTEND(GET_BITS(s), s)
//         s == 0: r == 15 ? k += 15 (ZRL) : break (EOB)
// Bits past a segment's end read as zero (jdhuff.c inserts zeros at a marker;
// here k_destuff leaves kSegPad zero bytes after every segment).
// Input: destuffed segments (k_destuff). Output: int16 coefficients, natural
// order, block (mcu, b) at coef_off + mcu * bpm + b (raw, dequantised in k_idct).
//
// The symbol step is uniform for DC and AC: a table entry carries the bits to
// consume (code + magnitude), the magnitude width s and the advance of the
// coefficient index k (DC 1, AC r + 1, ZRL 16, EOB 64), so one lookup, one
// bit-field extract and one add move the state (see ldt_types.hpp).
//
// Two decoders share it:
//   k_huff_serial    one workgroup per image, one lane per segment;
//   k_huff_sync/fix/scan/write   the self-synchronising parallel decoder
//                    (Weissenberger & Schmidt, ICPP 2018), see below.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldt_device.hpp"
#include "ldt_kernels.hpp"

namespace ldt {

// LDS pointers keep their address space so loads compile to ds_read_* (a
// generic pointer becomes flat_load_*, which waits on both vmcnt and lgkmcnt).
#define LDS_AS __attribute__((address_space(3)))
typedef const LDS_AS uint32_t *lds_cu32;
typedef const LDS_AS uint16_t *lds_cu16;
typedef const LDS_AS uint8_t *lds_cu8;
typedef LDS_AS uint16_t *lds_u16;
typedef LDS_AS uint32_t *lds_u32;

__constant__ uint8_t c_natural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// Dynamic LDS of every Huffman kernel: [window words][tables] (sync, write) or
// [tables] (serial, fix). Sizes come from the launcher.
extern __shared__ __attribute__((aligned(16))) uint32_t dyn_lds[];

// ---------------------------------------------------------------------------
// Bit input, MSB first. Words are 32-bit big-endian-as-integer: either the
// workgroup's LDS window (byte-swapped when staged) or global memory. Bit
// positions are relative to word 0 of the source; a lane adds its pbias to
// convert segment-relative positions. No bounds checks: every segment is
// followed by kSegPad zero bytes, and a symbol starting before the segment end
// reads at most 31 bits from its start.
// ---------------------------------------------------------------------------
// The LDS window is stored linearly. Lanes' ranges start S/32 words apart, and
// the planner keeps S/32 odd, so lanes at the same relative position fall in
// distinct banks without a skew (which would cost 3 VALU per symbol on the
// refill address).
struct LdsWords {
  lds_cu32 w;
  __device__ __forceinline__ uint32_t operator()(int32_t i) const { return w[i]; }
};
struct GlobWords {
  const uint32_t *w; // 4-aligned
  __device__ __forceinline__ uint32_t operator()(int32_t i) const { return __builtin_bswap32(w[i]); }
};

// Reader state: words wi-2 (hi), wi-1 (lo) and wi (nxt, prefetched); rs is
// 32 minus the consumed bits of hi (0 <= rs <= 31), so the next 32 bits are
// one alignbit with rs as its shift.
template <class W>
struct Rd {
  W src;
  uint32_t hi, lo, nxt;
  int32_t wi;
  int32_t rs;
  int32_t p;     // source bit position of the next symbol
  __device__ __forceinline__ void seek(int32_t q) {
    const int32_t i = (q - 1) >> 5;
    hi = i >= 0 ? src(i) : 0u; // q == 0: hi is fully consumed
    lo = src(i + 1);
    nxt = src(i + 2);
    wi = i + 2;
    rs = 32 * (i + 1) - q;
    p = q;
    // settle the seek's loads here: the decode loop's header then inherits no
    // pending LDS load and waits only on its own lookup (lgkmcnt(0))
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  __device__ __forceinline__ uint32_t peek() const {
    return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)rs);
  }
  __device__ __forceinline__ void consume(int t) { // t <= 31
    p += t;
    rs -= t;
    const bool m = rs < 0;
    hi = m ? lo : hi;
    lo = m ? nxt : lo;
    rs = m ? rs + 32 : rs;
    wi += m ? 1 : 0;
    nxt = src(wi);
  }
};

// ---------------------------------------------------------------------------
// Decode constants of one image and the lookup. The state between symbols is
// (b3, k): 3 * (block within the MCU) and the coefficient index (0: DC next).
// ---------------------------------------------------------------------------
struct Dec {
  lds_cu16 tabs;     // the image's distinct tables, kTabU16 entries per slot
  uint32_t dcseq;    // LDS table slot of MCU block b's DC table at bits 3b
  uint32_t acseq;    // ... AC table
  int b3end;         // 3 * blocks per MCU
  const HuffTab *g;  // plan tables (canonical fallback)
  const ImgDesc *d;
};

struct St {
  int b3, k;
  __device__ __forceinline__ int bk() const { return (b3 << 8) | k; }
};

__device__ __forceinline__ St make_state(int bk) {
  St st;
  st.b3 = bk >> 8;
  st.k = bk & 255;
  return st;
}

// Distinct tables of an image's six contexts (2 * component + AC), first
// come first slot; slotmap holds 3 bits per context.
__device__ __forceinline__ int image_slots(const ImgDesc &d, uint32_t &slotmap, int *slot_tab) {
  int ns = 0;
  slotmap = 0;
  for (int x = 0; x < 6; ++x) {
    const int c = x >> 1;
    const int cc = c < d.ncomp ? c : 0;
    const int tix = (x & 1) ? d.act[cc] : d.dct[cc];
    int found = -1;
    for (int q = 0; q < ns; ++q)
      if (slot_tab[q] == tix) found = q;
    if (found < 0) {
      found = ns;
      slot_tab[ns++] = tix;
    }
    slotmap |= (uint32_t)found << (3 * x);
  }
  return ns;
}

// Copy an image's distinct tables into LDS and return the decode constants.
__device__ __forceinline__ Dec load_dec(const ImgDesc &d, const HuffTab *__restrict__ htabs,
                                        lds_u16 tabs, int tid, int nthreads) {
  int slot_tab[6];
  uint32_t slotmap;
  const int ns = image_slots(d, slotmap, slot_tab);
  constexpr int kWords = kTabU16 / 2;
  for (int i = tid; i < ns * kWords; i += nthreads) {
    const int q = i / kWords, o = i - q * kWords;
    int tix = slot_tab[0];
#pragma unroll
    for (int x = 1; x < 6; ++x)
      if (q == x) tix = slot_tab[x];
    ((LDS_AS uint32_t *)(tabs + q * kTabU16))[o] = reinterpret_cast<const uint32_t *>(htabs + tix)[o];
  }
  Dec dec;
  dec.tabs = tabs;
  dec.dcseq = dec.acseq = 0;
  for (int b = 0; b < d.bpm; ++b) {
    const int c = d.bcomp[b] & 3;
    dec.dcseq |= ((slotmap >> (6 * c)) & 7) << (3 * b);
    dec.acseq |= ((slotmap >> (6 * c + 3)) & 7) << (3 * b);
  }
  dec.b3end = 3 * d.bpm;
  dec.g = htabs;
  dec.d = &d;
  return dec;
}

// Tables with more than kL2Chunks long-code prefixes: jdhuff.c
// jpeg_huff_decode's canonical search (first length l with code <= maxcode[l]).
__device__ __attribute__((noinline)) uint32_t lookup_canon(const HuffTab *__restrict__ g,
                                                           const ImgDesc *__restrict__ d, int b,
                                                           bool ac, uint32_t pk) {
  const int c = d->bcomp[b];
  const HuffTab *cn = g + (ac ? d->act[c] : d->dct[c]);
  const uint32_t w16 = pk >> 16;
  for (int l = kLookBits + 1; l <= 16; ++l) {
    const int code = (int)(w16 >> (16 - l));
    if (code <= cn->maxcode[l]) return huff_entry(l, cn->vals[(cn->valoff[l] + code) & 0xFF], !ac);
  }
  return huff_entry(16, 0, !ac);
}

// Entry of the symbol whose code starts at the top bit of pk.
__device__ __forceinline__ uint32_t lookup(const Dec &dec, const St &st, uint32_t pk) {
  const bool ac = st.k != 0;
  const uint32_t slot = __builtin_amdgcn_ubfe(ac ? dec.acseq : dec.dcseq, (uint32_t)st.b3, 3u);
  const lds_cu16 t = dec.tabs + slot * kTabU16;
  uint32_t e = t[pk >> (32 - kLookBits)];
  if (__builtin_expect((e & 31) == 0, 0)) {
    if (e != kHuffCanon)
      e = t[(1 << kLookBits) + ((e >> 5) << kL2Bits) + ((pk >> 16) & ((1u << kL2Bits) - 1))];
    else
      e = lookup_canon(dec.g, dec.d, st.b3 / 3, ac, pk);
  }
  return e;
}

// HUFF_EXTEND of the s magnitude bits following the code.
__device__ __forceinline__ int ext_value(uint32_t pk, uint32_t e) {
  const uint32_t total = e & 31, s = (e >> 5) & 15;
  const int raw = (int)__builtin_amdgcn_ubfe(pk, 32 - total, s);
  const int half = (1 << s) >> 1;
  return raw < half ? raw - 2 * half + 1 : raw;
}

// k += adv; k >= 64 ends the block (EOB advances by 64).
__device__ __forceinline__ void advance(St &st, const Dec &dec, int adv) {
  const int k2 = st.k + adv;
  const bool end = k2 >= 64;
  int nb = st.b3 + 3;
  nb = nb == dec.b3end ? 0 : nb;
  st.b3 = end ? nb : st.b3;
  st.k = end ? 0 : k2;
}

// Count-only symbol: blocks started.
template <class W>
__device__ __forceinline__ void count_step(Rd<W> &R, St &st, const Dec &dec, int &nblk) {
  const uint32_t pk = R.peek();
  const uint32_t e = lookup(dec, st, pk);
  nblk += st.k == 0 ? 1 : 0;
  R.consume((int)(e & 31));
  advance(st, dec, (int)(e >> 9));
}

// Coefficients of a block are stored in zigzag (decode) order, int16 slots
// 1..63 (DC lives in dcv); k_idct de-zigzags while dequantising. Slots are
// combined 8 at a time (16 bytes) in registers and written with one store per
// touched group instead of one 2-byte scatter per coefficient: a block's
// coefficient indices only grow, so a group is complete once the index leaves
// it or the block ends. Groups a neighbouring range may also write (a block
// straddling the range boundary) are written slot by slot.
__device__ __forceinline__ void store_group(int16_t *__restrict__ p, uint64_t lo, uint64_t hi) {
  *reinterpret_cast<uint4 *>(p) =
      make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

// Coefficient-writing decode of one range: from the reader's position until
// it reaches `stop` or the segment's `total` blocks are complete. cursor is
// the current block (segment-relative, -1 before the first DC). DC symbols
// store their difference in dcv_seg[cursor] (k_dc_scan adds the predictors);
// nonzero AC coefficients go to coef_seg, which is all zero beforehand
// (k_idct clears every block it reads). The loop body is straight-line: every
// store is predicated, so a wave branches only around stores no lane makes.
template <class W>
__device__ __forceinline__ void write_run(Rd<W> &R, St &st, const Dec &dec, int32_t stop,
                                          int &cursor, int total, int16_t *__restrict__ coef_seg,
                                          int16_t *__restrict__ dcv_seg) {
  uint64_t lo = 0, hi = 0; // buffered group: slots 0-3, 4-7
  int grp = -1;            // its index (slot >> 3), -1 = empty
  // entered mid-block: the previous range may have written this group of it
  const int shared_g = st.k != 0 ? (st.k >> 3) : -1;
  bool first = true;       // still in the block the range entered
  bool go = R.p < stop && !(st.k == 0 && cursor + 1 >= total);
  while (go) {
    const bool dc = st.k == 0;
    cursor += dc ? 1 : 0;
    // corrupt streams can count more blocks than the segment has, so a range
    // may enter mid-block with its cursor outside [0, total): no stores then
    const bool inb = (uint32_t)cursor < (uint32_t)total;
    const uint32_t pk = R.peek();
    const uint32_t e = lookup(dec, st, pk);
    const int v = ext_value(pk, e);
    const int adv = (int)(e >> 9);
    const bool nz = !dc && ((e >> 5) & 15) != 0;
    const int slot = st.k + adv - 1;
    const int g = slot >> 3;
    int16_t *__restrict__ blk = coef_seg + (int64_t)cursor * 64;
    if (dc) dcv_seg[cursor] = (int16_t)v;
    const bool direct = nz && first && g == shared_g;
    if (direct && inb) blk[slot] = (int16_t)v;
    const bool buf = nz && !direct;
    const bool newg = buf && g != grp;
    if (newg && grp >= 0 && inb) store_group(blk + 8 * grp, lo, hi);
    lo = newg ? 0ull : lo;
    hi = newg ? 0ull : hi;
    grp = newg ? g : grp;
    const uint64_t x = buf ? (uint64_t)((uint32_t)v & 0xFFFFu) << (16 * (slot & 3)) : 0ull;
    lo |= (slot & 4) ? 0ull : x;
    hi |= (slot & 4) ? x : 0ull;
    R.consume((int)(e & 31));
    const bool end = st.k + adv >= 64;
    if (end && grp >= 0 && inb) store_group(blk + 8 * grp, lo, hi);
    grp = end ? -1 : grp;
    first = first && !end;
    advance(st, dec, adv);
    go = R.p < stop && !(st.k == 0 && cursor + 1 >= total);
  }
  if (grp >= 0 && (uint32_t)cursor < (uint32_t)total) { // the open block continues in the next range
    int16_t *p = coef_seg + (int64_t)cursor * 64 + 8 * grp;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint16_t x = (uint16_t)(((j & 4) ? hi : lo) >> (16 * (j & 3)));
      if (x) p[j] = (int16_t)x;
    }
  }
}

// ---------------------------------------------------------------------------
// Serial decoder: one 64-lane workgroup per image, one lane per segment.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_huff_serial(const ImgDesc *__restrict__ descs,
                                                    const Segment *__restrict__ segs,
                                                    const HuffTab *__restrict__ htabs,
                                                    const uint8_t *__restrict__ dstuf,
                                                    int16_t *__restrict__ coef,
                                                    int16_t *__restrict__ dcv,
                                                    int32_t *__restrict__ status) {
  const int img = blockIdx.x;
  if (status[img] != 0 || descs[img].nseg == 0) return;
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  const Dec dec = load_dec(d, htabs, (lds_u16)dyn_lds, tid, 64);
  __syncthreads();
  for (int si = d.seg_base + tid; si < d.seg_base + d.nseg; si += 64) {
    const Segment sg = segs[si];
    const int32_t seg_bits = (int32_t)((sg.byte_end - sg.byte_start) * 8);
    Rd<GlobWords> R;
    R.src.w = reinterpret_cast<const uint32_t *>(dstuf + (sg.byte_start & ~(int64_t)3));
    const int32_t pbias = (int32_t)(sg.byte_start & 3) * 8;
    R.seek(pbias);
    St st = make_state(0);
    const int total = sg.mcu_count * d.bpm;
    int cursor = -1;
    const int64_t blk0 = d.coef_off + (int64_t)sg.mcu_first * d.bpm;
    // a valid segment ends inside its bits; 64 bits of slack bound a corrupt one
    write_run(R, st, dec, pbias + seg_bits + 64, cursor, total, coef + blk0 * 64, dcv + blk0);
    if (R.p - pbias > seg_bits || cursor + 1 < total || st.k != 0) status[img] = 3; // truncated
  }
}

hipError_t launch_huff_serial(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n == 0) return hipSuccess;
  const size_t tab_lds = (size_t)(p.max_tabs < 1 ? 1 : p.max_tabs) * kTabU16 * 2;
  hipLaunchKernelGGL(k_huff_serial, dim3(p.n), dim3(64), tab_lds, s, p.descs, p.segs, p.htabs,
                     w.dstuf, w.coef, w.dcv, w.status);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_dc_scan: DC predictors (jdhuff.c: last_dc_val[ci] += diff, reset to 0 at
// every restart marker, process_restart). One workgroup per image; thread t
// owns a run of consecutive blocks; a segmented scan over the threads carries
// the per-component sums. Stores the absolute DC (JCOEF, truncated) in place.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dc_scan(const ImgDesc *__restrict__ descs,
                                                 int16_t *__restrict__ dcv,
                                                 const int32_t *__restrict__ status) {
  __shared__ int s_f[256];
  __shared__ int s_v[3][256];
  const int img = blockIdx.x;
  if (status[img] != 0 || descs[img].nseg == 0) return; // progressive: dcv holds final DC
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  const int bpm = d.bpm;
  const int64_t nblk = (int64_t)d.mcux * d.mcuy * bpm;
  const int64_t seglen = d.restart ? (int64_t)d.restart * bpm : nblk;
  uint32_t compmap = 0;
  for (int b = 0; b < bpm; ++b) compmap |= (uint32_t)(d.bcomp[b] & 3) << (2 * b);
  const int64_t K = (nblk + 255) / 256;
  const int64_t lo = (int64_t)tid * K, hi = min(lo + K, nblk);
  int16_t *v = dcv + d.coef_off;
  int s0 = 0, s1 = 0, s2 = 0, flag = 0;
  int b0 = 0;
  int64_t sp0 = 0;
  if (lo < hi) {
    b0 = (int)(lo % bpm);
    sp0 = lo % seglen;
  }
  {
    int b = b0;
    int64_t sp = sp0;
    for (int64_t x = lo; x < hi; ++x) {
      if (sp == 0) {
        s0 = s1 = s2 = 0;
        flag = 1;
      }
      const int c = (int)((compmap >> (2 * b)) & 3);
      const int dv = v[x];
      s0 += c == 0 ? dv : 0;
      s1 += c == 1 ? dv : 0;
      s2 += c == 2 ? dv : 0;
      b = b + 1 == bpm ? 0 : b + 1;
      sp = sp + 1 == seglen ? 0 : sp + 1;
    }
  }
  // inclusive segmented scan of (flag, s0, s1, s2) over the threads
  s_f[tid] = flag;
  s_v[0][tid] = s0;
  s_v[1][tid] = s1;
  s_v[2][tid] = s2;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    int pf = 0, p0 = 0, p1 = 0, p2 = 0;
    if (tid >= off) {
      pf = s_f[tid - off];
      p0 = s_v[0][tid - off];
      p1 = s_v[1][tid - off];
      p2 = s_v[2][tid - off];
    }
    __syncthreads();
    if (tid >= off && !flag) {
      s0 += p0;
      s1 += p1;
      s2 += p2;
      s_v[0][tid] = s0;
      s_v[1][tid] = s1;
      s_v[2][tid] = s2;
    }
    flag |= pf;
    s_f[tid] = flag;
    __syncthreads();
  }
  int r0 = tid > 0 ? s_v[0][tid - 1] : 0;
  int r1 = tid > 0 ? s_v[1][tid - 1] : 0;
  int r2 = tid > 0 ? s_v[2][tid - 1] : 0;
  int b = b0;
  int64_t sp = sp0;
  for (int64_t x = lo; x < hi; ++x) {
    if (sp == 0) r0 = r1 = r2 = 0;
    const int c = (int)((compmap >> (2 * b)) & 3);
    const int dv = v[x];
    r0 += c == 0 ? dv : 0;
    r1 += c == 1 ? dv : 0;
    r2 += c == 2 ? dv : 0;
    v[x] = (int16_t)(c == 0 ? r0 : c == 1 ? r1 : r2);
    b = b + 1 == bpm ? 0 : b + 1;
    sp = sp + 1 == seglen ? 0 : sp + 1;
  }
}

hipError_t launch_dc_scan(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_dc_scan, dim3(p.n), dim3(256), 0, s, p.descs, w.dcv, w.status);
  return hipGetLastError();
}

// ===========================================================================
// Parallel self-synchronising decode.
//
// A segment's bits are cut into subsequences of S bits; image-local slot lt
// of segment s (sub_first <= lt < sub_first + sub_count) owns subsequence
// j = lt - sub_first, i.e. bits [j*S, (j+1)*S). The decode state at a symbol
// boundary is (p, b, k): bit position, block within the MCU, coefficient
// index (k == 0: a DC symbol is next). A slot's exit state is the state at
// the first symbol boundary p >= (j+1)*S; under its true entry state that is
// its successor's true entry state. Two decoders in the same state decode
// identically from there on — which is why chains started from a guessed
// state converge (Huffman codes resynchronise).
//
// Workgroup w = 256 lanes: lanes kHelpers..255 own slots
// (w - wg_first) * kSlotsPerWg + lane - kHelpers; lanes 0..kHelpers-1 are
// helpers that decode the kHelpers subsequences before the first slot, so its
// entry state is right unless no chain resynchronised within kHelpers * S bits.
// Inside the workgroup, lanes re-decode from their predecessor's exit until no
// exit changes; each lane keeps two checkpoint states of its last trajectory
// so a re-decode stops as soon as it merges with it. Across workgroups,
// k_huff_fix compares the last helper's exit with the previous workgroup's
// last exit and walks (one lane, LDS tables) only on a mismatch. The sync pass
// only counts blocks per range; k_huff_write then decodes every range from its
// true entry and k_dc_scan adds the DC predictors.
//
// LDS window: the workgroup's destuffed bytes, byte-swapped. Without
// restart markers they span 256 * S/8 + 76 bytes; a workgroup whose ranges
// span more (many small restart segments, kSegPad apart) reads global memory
// instead. LDS per workgroup stays under a third of the CU's 160 KB at S = 1024
// with four tables, so three decode workgroups share a CU.
// ===========================================================================

__host__ __device__ inline int window_bytes(int S) { return 256 * (S / 8) + 128; }
__host__ __device__ inline int window_lds_bytes(int S) {
  const int words = window_bytes(S) / 4 + 1;
  return (words * 4 + 15) & ~15;
}

// Locate the segment that owns image-local slot `lt` (sub_first ascending).
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

// Global state index of image-local slot lt.
__device__ __forceinline__ int64_t slot_gt(const ImgDesc &d, int lt) {
  return (int64_t)(d.wg_first + lt / kSlotsPerWg) * kSyncThreads + kHelpers + lt % kSlotsPerWg;
}

struct SubCtx {
  int seg;        // segment index (global), -1 if idle
  int j;          // subsequence index within the segment
  int32_t seg_bits;
  int32_t pbias;  // source bit of the segment's bit 0
  bool active;    // a real slot
  bool helper;    // a helper lane with a subsequence to decode
  bool in_lds;    // the workgroup's window is in LDS (else global words)
  const uint32_t *gw; // global words at the window base
};

// Workgroup setup shared by the sync and write kernels: the image's tables
// and the LDS window.
__device__ __forceinline__ Dec sub_setup(const ImgDesc &d, const Segment *__restrict__ segs,
                                         const HuffTab *__restrict__ htabs, int S, int Smax,
                                         const uint8_t *__restrict__ dstuf, lds_u32 win,
                                         lds_u16 tabs, unsigned long long *sh_lohi, SubCtx &sc) {
  const int tid = threadIdx.x;
  const Dec dec = load_dec(d, htabs, tabs, tid, kSyncThreads);
  const int lt0 = ((int)blockIdx.x - d.wg_first) * kSlotsPerWg;
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  const int total_sub = last.sub_first + last.sub_count;
  sc.active = false;
  sc.helper = false;
  sc.seg = -1;
  sc.j = 0;
  sc.seg_bits = 0;
  sc.pbias = 0;
  int64_t seg0 = 0;
  uint64_t lo = ~0ull, hi = 0;
  const int lt = tid >= kHelpers ? lt0 + tid - kHelpers : lt0;
  if (lt < total_sub) {
    const int si = find_segment(segs, d.seg_base, d.nseg, lt);
    const Segment &sg = segs[si];
    int j = lt - sg.sub_first;
    if (tid >= kHelpers) {
      sc.active = true;
    } else {
      j -= kHelpers - tid;
      sc.helper = j >= 0;
    }
    if (sc.active || sc.helper) {
      sc.seg = si;
      sc.j = j;
      seg0 = sg.byte_start;
      sc.seg_bits = (int32_t)((sg.byte_end - sg.byte_start) * 8);
      lo = (uint64_t)(sg.byte_start + ((int64_t)j * S) / 8);
      int64_t h = sg.byte_start + ((int64_t)(j + 1) * S) / 8 + 64;
      if (h > sg.byte_end + kSegPad) h = sg.byte_end + kSegPad;
      hi = (uint64_t)h;
    }
  }
  if (tid == 0) {
    sh_lohi[0] = ~0ull;
    sh_lohi[1] = 0;
  }
  __syncthreads();
  if (hi > 0) {
    atomicMin(&sh_lohi[0], (unsigned long long)lo);
    atomicMax(&sh_lohi[1], (unsigned long long)hi);
  }
  __syncthreads();
  int64_t wb = 0, nbytes = 0;
  if (sh_lohi[1] > 0) {
    wb = (int64_t)sh_lohi[0] & ~(int64_t)3;
    nbytes = (((int64_t)sh_lohi[1] - wb) + 3) & ~(int64_t)3;
  }
  sc.in_lds = nbytes <= window_bytes(Smax);
  sc.gw = reinterpret_cast<const uint32_t *>(dstuf + wb);
  if (sc.in_lds)
    for (int i = tid; i < (int)nbytes / 4; i += kSyncThreads) win[i] = __builtin_bswap32(sc.gw[i]);
  sc.pbias = (int32_t)(seg0 - wb) * 8;
  __syncthreads();
  return dec;
}

// Checkpoints: the state at the first symbol boundary at/after
// range_start + S/3 and + 2S/3, with the blocks counted up to it.
struct Cp {
  int p0, bk0, p1, bk1;
  int a0, a1;
  int n;
};

template <class W>
__device__ __forceinline__ void count_until(Rd<W> &R, int32_t lim, St &st, const Dec &dec,
                                            int &nblk) {
  while (R.p < lim) count_step(R, st, dec, nblk);
}

// COUNT decode from the reader's position to the first boundary >= stop
// (positions in reader coordinates), recording the checkpoints. COMPARE: stop
// at the first checkpoint equal to prev's (merge) and adopt prev's tail.
// Returns true on a merge.
template <bool COMPARE, class W>
__device__ __forceinline__ bool count_run(Rd<W> &R, int32_t range_start, int32_t stop, int S,
                                          St &st, const Dec &dec, int &nblk, Cp &cp,
                                          const Cp &prev, int prev_total) {
  cp.n = 0;
  count_until(R, min(range_start + S / 3, stop), st, dec, nblk);
  if (R.p >= stop) return false;
  {
    const int p = R.p, bk = st.bk();
    if (COMPARE && prev.n > 0 && prev.p0 == p && prev.bk0 == bk) {
      const int delta = nblk - prev.a0;
      cp = prev;
      cp.a0 = nblk;
      cp.a1 = prev.a1 + delta;
      nblk = prev_total + delta;
      return true;
    }
    cp.p0 = p;
    cp.bk0 = bk;
    cp.a0 = nblk;
    cp.n = 1;
  }
  count_until(R, min(range_start + (2 * S) / 3, stop), st, dec, nblk);
  if (R.p >= stop) return false;
  {
    const int p = R.p, bk = st.bk();
    if (COMPARE && prev.n > 1 && prev.p1 == p && prev.bk1 == bk) {
      const int delta = nblk - prev.a1;
      cp.p1 = p;
      cp.bk1 = bk;
      cp.a1 = nblk;
      cp.n = 2;
      nblk = prev_total + delta;
      return true;
    }
    cp.p1 = p;
    cp.bk1 = bk;
    cp.a1 = nblk;
    cp.n = 2;
  }
  count_until(R, stop, st, dec, nblk);
  return false;
}

struct SyncLds {
  int32_t ex_p[kSyncThreads];
  uint16_t ex_bk[kSyncThreads]; // (3b << 8) | k <= 27 * 256 + 63
  int any_changed;
};

// Phase 1 + intra-workgroup convergence for one lane; returns its block count.
//
// Phase 1 starts `warm` bits before the lane's range (never before its segment
// or the window) from a guessed state (b = 0, k = 0), so the trajectory has
// usually resynchronised by the range start; the lane records its entry state
// (first symbol boundary at/after the range start) and its exit. A lane then
// re-decodes only while its entry differs from its predecessor's exit, and a
// re-decode stops at the first checkpoint where it merges with the lane's own
// previous trajectory. The warm-up trades one extra range of decoding in phase
// 1 for chains of wrong exits that are much rarer (they need a resync distance
// above warm + S instead of S), which cuts the rounds of the slowest
// workgroup, and with them the kernel's latency.
template <class W>
__device__ __forceinline__ int sync_lane(W src, const SubCtx &sc, const Dec &dec, int S, int warm,
                                         SyncLds &sh, int32_t *__restrict__ dbg) {
  const int tid = threadIdx.x;
  int nblk = 0;
  Cp cp, none;
  cp.n = 0;
  none.n = 0;
  St st = make_state(0);
  Rd<W> R;
  R.src = src;
  const int32_t rstart = sc.pbias + sc.j * S;
  const int32_t stop = sc.pbias + min((sc.j + 1) * S, sc.seg_bits);
  const bool live = sc.active || sc.helper;
  int en_p = 0, en_bk = 0; // state at the range start (segment-relative position)
  if (live) {
    const int32_t w0 = max(rstart - warm, max(sc.pbias, 0));
    R.seek(w0);
    if (w0 < rstart) {
      int skipped = 0;
      count_until(R, rstart, st, dec, skipped);
    }
    en_p = R.p - sc.pbias;
    en_bk = st.bk();
    count_run<false>(R, rstart, stop, S, st, dec, nblk, cp, none, 0);
    sh.ex_p[tid] = R.p - sc.pbias;
    sh.ex_bk[tid] = (uint16_t)st.bk();
  } else {
    sh.ex_p[tid] = 0;
    sh.ex_bk[tid] = 0;
  }
  int rounds = 0;
  for (int round = 0; round < kSyncThreads + 1; ++round) {
    ++rounds;
    __syncthreads();
    if (tid == 0) sh.any_changed = 0;
    bool changed = false;
    int np = 0, nbk = 0;
    const bool need = live && sc.j > 0 && tid > 0 &&
                      (sh.ex_p[tid - 1] != en_p || sh.ex_bk[tid - 1] != en_bk);
    if (need) {
      en_p = sh.ex_p[tid - 1];
      en_bk = sh.ex_bk[tid - 1];
      st = make_state(en_bk);
      const int prev_total = nblk;
      const Cp prev = cp;
      nblk = 0;
      R.seek(sc.pbias + en_p);
      if (count_run<true>(R, rstart, stop, S, st, dec, nblk, cp, prev, prev_total)) {
        np = sh.ex_p[tid];
        nbk = sh.ex_bk[tid];
      } else {
        np = R.p - sc.pbias;
        nbk = st.bk();
      }
      changed = (np != sh.ex_p[tid]) || (nbk != sh.ex_bk[tid]);
    }
    __syncthreads();
    if (changed) {
      sh.ex_p[tid] = np;
      sh.ex_bk[tid] = (uint16_t)nbk;
      sh.any_changed = 1;
    }
    __syncthreads();
    if (!sh.any_changed) break;
  }
  if (dbg && tid == 0) {
    atomicAdd(dbg + 1, 1);
    atomicAdd(dbg + 2, rounds);
    atomicMax(dbg + 3, rounds);
  }
  return nblk;
}

__global__ void __launch_bounds__(kSyncThreads) k_huff_sync(
    const ImgDesc *__restrict__ descs, const Segment *__restrict__ segs,
    const HuffTab *__restrict__ htabs, const uint8_t *__restrict__ dstuf,
    const int32_t *__restrict__ wg_img, int Smax, int warm_pct, SubState *__restrict__ sub,
    const int32_t *__restrict__ status, int32_t *__restrict__ dbg) {
  __shared__ SyncLds sh;
  __shared__ unsigned long long sh_lohi[2];
  const int img = wg_img[blockIdx.x];
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  SubCtx sc;
  const lds_u32 win = (lds_u32)dyn_lds;
  const int S = d.sub_bits;
  const Dec dec = sub_setup(d, segs, htabs, S, Smax, dstuf, win,
                            (lds_u16)(dyn_lds + window_lds_bytes(Smax) / 4), sh_lohi, sc);
  int nblk;
  const int warm = (S * warm_pct) / 100;
  if (sc.in_lds) nblk = sync_lane(LdsWords{(lds_cu32)win}, sc, dec, S, warm, sh, dbg);
  else nblk = sync_lane(GlobWords{sc.gw}, sc, dec, S, warm, sh, dbg);
  if (sc.active || tid == kHelpers - 1) {
    SubState s;
    s.exit_p = sh.ex_p[tid];
    s.exit_bk = sh.ex_bk[tid];
    s.nblk = nblk;
    s.pad = 0;
    sub[(int64_t)blockIdx.x * kSyncThreads + tid] = s;
  }
}

// Lane 0 of the calling wave walks slots from lt0 (true entry = the stored
// exit of slot lt0 - 1) until a recomputed exit equals the stored one. The
// image's tables must already be in LDS (dec). bounded = true stops at the end
// of lt0's workgroup and raises *redo (the next boundary then compared against
// a stale exit).
__device__ void boundary_walk(const ImgDesc &d, const Dec &dec, const Segment *__restrict__ segs,
                              const uint8_t *__restrict__ dstuf, int S,
                              SubState *__restrict__ sub, int lt0, bool bounded, int32_t *redo,
                              int32_t *dbg) {
  const int si = find_segment(segs, d.seg_base, d.nseg, lt0);
  const Segment &sg = segs[si];
  int j = lt0 - sg.sub_first;
  if (j == 0) return;
  const int32_t seg_bits = (int32_t)((sg.byte_end - sg.byte_start) * 8);
  const SubState &pv = sub[slot_gt(d, lt0 - 1)];
  int ep = pv.exit_p, ebk = pv.exit_bk;
  int lt = lt0;
  const int wg_next = (lt0 / kSlotsPerWg + 1) * kSlotsPerWg;
  Rd<GlobWords> R;
  R.src.w = reinterpret_cast<const uint32_t *>(dstuf + (sg.byte_start & ~(int64_t)3));
  const int32_t pbias = (int32_t)(sg.byte_start & 3) * 8;
  int steps = 0;
  Cp cp, none;
  none.n = 0;
  while (true) {
    ++steps;
    St st = make_state(ebk);
    int nblk = 0;
    R.seek(pbias + ep);
    count_run<false>(R, pbias + j * S, pbias + min((j + 1) * S, seg_bits), S, st, dec, nblk, cp,
                     none, 0);
    const int np = R.p - pbias, nbk = st.bk();
    SubState &s = sub[slot_gt(d, lt)];
    s.nblk = nblk;
    if (np == s.exit_p && nbk == s.exit_bk) break; // converged
    s.exit_p = np;
    s.exit_bk = nbk;
    ep = np;
    ebk = nbk;
    ++lt;
    ++j;
    if (j >= sg.sub_count) break; // end of segment: nothing downstream
    if (bounded && lt >= wg_next) {
      atomicExch(redo, 1);
      if (dbg) atomicAdd(dbg + 7, 1);
      break;
    }
  }
  if (dbg) {
    atomicAdd(dbg + 4, 1);
    atomicAdd(dbg + 6, steps);
    if (steps == 1) atomicAdd(dbg + 5, 1);
  }
}

// One wave per decode workgroup: compare the last helper's candidate entry
// for the workgroup's first slot with the true predecessor exit; walk on a
// mismatch.
__global__ void __launch_bounds__(64) k_huff_fix(const ImgDesc *__restrict__ descs,
                                                 const Segment *__restrict__ segs,
                                                 const HuffTab *__restrict__ htabs,
                                                 const uint8_t *__restrict__ dstuf,
                                                 const int32_t *__restrict__ wg_img, int Smax,
                                                 SubState *__restrict__ sub,
                                                 const int32_t *__restrict__ status,
                                                 int32_t *__restrict__ redo) {
  const int w = blockIdx.x;
  const int img = wg_img[w];
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const int wl = w - d.wg_first;
  const int lt0 = wl * kSlotsPerWg;
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  if (wl == 0 || lt0 >= last.sub_first + last.sub_count) return;
  const int si = find_segment(segs, d.seg_base, d.nseg, lt0);
  if (lt0 == segs[si].sub_first) return; // the first slot starts a segment: exact entry
  const SubState &pv = sub[slot_gt(d, lt0 - 1)];
  const SubState &cand = sub[(int64_t)w * kSyncThreads + kHelpers - 1];
  if (threadIdx.x == 0) atomicAdd(redo + 8, 1); // boundaries checked
  if (pv.exit_p == cand.exit_p && pv.exit_bk == cand.exit_bk) return; // helpers were right
  const Dec dec = load_dec(d, htabs, (lds_u16)dyn_lds, threadIdx.x, 64);
  __syncthreads();
  if (threadIdx.x == 0) boundary_walk(d, dec, segs, dstuf, d.sub_bits, sub, lt0, true, redo, redo);
  (void)Smax;
}

// Fallback when a walk did not converge inside its workgroup: one lane per
// image walks every workgroup boundary in order (always correct).
__global__ void __launch_bounds__(64) k_huff_fix_serial(const ImgDesc *__restrict__ descs,
                                                        const Segment *__restrict__ segs,
                                                        const HuffTab *__restrict__ htabs,
                                                        const uint8_t *__restrict__ dstuf, int Smax,
                                                        SubState *__restrict__ sub,
                                                        const int32_t *__restrict__ status,
                                                        const int32_t *__restrict__ redo) {
  const int img = blockIdx.x;
  if (redo[0] == 0 || status[img] != 0 || descs[img].nseg == 0) return;
  const ImgDesc &d = descs[img];
  const Dec dec = load_dec(d, htabs, (lds_u16)dyn_lds, threadIdx.x, 64);
  __syncthreads();
  if (threadIdx.x != 0) return;
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  const int total = last.sub_first + last.sub_count;
  for (int wl = 1; wl < d.wg_count; ++wl) {
    const int lt0 = wl * kSlotsPerWg;
    if (lt0 >= total) break;
    boundary_walk(d, dec, segs, dstuf, d.sub_bits, sub, lt0, false, nullptr, nullptr);
  }
}

// Exclusive prefix of nblk over each image's slots.
__global__ void __launch_bounds__(256) k_huff_scan(const ImgDesc *__restrict__ descs,
                                                   const Segment *__restrict__ segs,
                                                   const SubState *__restrict__ sub,
                                                   int32_t *__restrict__ pre,
                                                   const int32_t *__restrict__ status) {
  __shared__ int sh_scan[8];
  const int img = blockIdx.x;
  if (status[img] != 0 || descs[img].nseg == 0) return;
  const ImgDesc &d = descs[img];
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  const int total = last.sub_first + last.sub_count;
  int run = 0;
  for (int base = 0; base < total; base += 256) {
    const int lt = base + threadIdx.x;
    int v = 0;
    int64_t gt = 0;
    if (lt < total) {
      gt = slot_gt(d, lt);
      v = sub[gt].nblk;
    }
    int tot;
    const int ex = block_excl_scan256(v, sh_scan, &tot);
    if (lt < total) pre[gt] = run + ex;
    run += tot;
  }
}

template <class W>
__device__ __forceinline__ void write_lane(W src, const SubCtx &sc, const Dec &dec, int S,
                                           const ImgDesc &d, const Segment &sg, int entry, int bk,
                                           int cursor, int16_t *__restrict__ coef,
                                           int16_t *__restrict__ dcv,
                                           int32_t *__restrict__ status, int img) {
  St st = make_state(bk);
  const int total = sg.mcu_count * d.bpm;
  const int64_t blk0 = d.coef_off + (int64_t)sg.mcu_first * d.bpm;
  Rd<W> R;
  R.src = src;
  R.seek(sc.pbias + entry);
  write_run(R, st, dec, sc.pbias + min((sc.j + 1) * S, sc.seg_bits), cursor, total,
            coef + blk0 * 64, dcv + blk0);
  if (sc.j == sg.sub_count - 1 && cursor + 1 < total) status[img] = 3; // ran out of data
}

// Final pass: every slot decodes its range from its true entry state and
// writes coefficients (DC differences to dcv).
__global__ void __launch_bounds__(kSyncThreads) k_huff_write(
    const ImgDesc *__restrict__ descs, const Segment *__restrict__ segs,
    const HuffTab *__restrict__ htabs, const uint8_t *__restrict__ dstuf,
    const int32_t *__restrict__ wg_img, int Smax, const SubState *__restrict__ sub,
    const int32_t *__restrict__ pre, int16_t *__restrict__ coef,
    int16_t *__restrict__ dcv, int32_t *__restrict__ status) {
  __shared__ unsigned long long sh_lohi[2];
  const int img = wg_img[blockIdx.x];
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  SubCtx sc;
  const lds_u32 win = (lds_u32)dyn_lds;
  const int S = d.sub_bits;
  const Dec dec = sub_setup(d, segs, htabs, S, Smax, dstuf, win,
                            (lds_u16)(dyn_lds + window_lds_bytes(Smax) / 4), sh_lohi, sc);
  if (!sc.active) return;
  const Segment &sg = segs[sc.seg];
  const int64_t gt = (int64_t)blockIdx.x * kSyncThreads + tid;
  int entry = 0, bk = 0;
  if (sc.j > 0) {
    const int64_t pg = (tid == kHelpers) ? (int64_t)blockIdx.x * kSyncThreads - 1 : gt - 1;
    const SubState &ps = sub[pg];
    entry = ps.exit_p;
    bk = ps.exit_bk;
  }
  const int cursor = pre[gt] - pre[slot_gt(d, sg.sub_first)] - 1;
  if (sc.in_lds)
    write_lane(LdsWords{(lds_cu32)win}, sc, dec, S, d, sg, entry, bk, cursor, coef, dcv,
               status, img);
  else
    write_lane(GlobWords{sc.gw}, sc, dec, S, d, sg, entry, bk, cursor, coef, dcv,
               status, img);
}

hipError_t launch_huff_parallel(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n_wg == 0) return hipSuccess;
  const size_t tab_lds = (size_t)(p.max_tabs < 1 ? 1 : p.max_tabs) * kTabU16 * 2;
  const size_t dec_lds = (size_t)window_lds_bytes(p.subseq_bits) + tab_lds;
  hipLaunchKernelGGL(k_huff_sync, dim3(p.n_wg), dim3(kSyncThreads), dec_lds, s, p.descs, p.segs,
                     p.htabs, w.dstuf, p.wg_img, p.subseq_bits, p.warm_pct, w.sub, w.status, p.redo);
  hipLaunchKernelGGL(k_huff_fix, dim3(p.n_wg), dim3(64), tab_lds, s, p.descs, p.segs, p.htabs,
                     w.dstuf, p.wg_img, p.subseq_bits, w.sub, w.status, p.redo);
  hipLaunchKernelGGL(k_huff_fix_serial, dim3(p.n), dim3(64), tab_lds, s, p.descs, p.segs, p.htabs,
                     w.dstuf, p.subseq_bits, w.sub, w.status, p.redo);
  hipLaunchKernelGGL(k_huff_scan, dim3(p.n), dim3(256), 0, s, p.descs, p.segs, w.sub, w.sub_pre,
                     w.status);
  hipLaunchKernelGGL(k_huff_write, dim3(p.n_wg), dim3(kSyncThreads), dec_lds, s, p.descs, p.segs,
                     p.htabs, w.dstuf, p.wg_img, p.subseq_bits, w.sub, w.sub_pre, w.coef,
                     w.dcv, w.status);
  return hipGetLastError();
}

} // namespace ldt

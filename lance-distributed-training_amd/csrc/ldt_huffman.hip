// ldt_huffman.hip — baseline JPEG Huffman decode on gfx950.
//
// Restates libjpeg-turbo jdhuff.c decode_mcu (sequential, Huffman, 8-bit):
//   DC: s = HUFF_DECODE(dc_tbl); diff = HUFF_EXTEND(GET_BITS(s), s); pred += diff
//   AC: for k = 1..63: rs = HUFF_DECODE(ac_tbl); r = rs >> 4; s = rs & 15;
//         s != 0: k += r; coef[natural[k]] = HUFF_EXTEND(GET_BITS(s), s)
//         s == 0: r == 15 ? k += 15 (ZRL) : break (EOB)
// Bits past a segment's end read as zero (jdhuff.c inserts zeros at a marker;
// here k_destuff leaves kSegPad zero bytes after every segment).
// Input: destuffed segments (k_destuff). Output: int16 coefficients in zigzag
// order, image-relative block (mcu, b) = mcu * bpm + b, as packed nonzero
// 16-byte groups plus a 4-byte record per block (ldt_kernels.hpp; raw,
// dequantised in k_idct), and the absolute DC values in the records.
//
// The symbol step is uniform for DC and AC: a table entry carries the bits to
// consume (code + magnitude), the magnitude width s and the advance of the
// coefficient index k (DC 1, AC r + 1, ZRL 16, EOB 64), so one lookup, one
// bit-field extract and one add move the state (see ldt_types.hpp).
//
// Two decoders share it:
//   k_huff_serial    one workgroup per image, one lane per segment (images
//                    with many restart segments, or LDT_OPT_HUFF_MODE 1);
//   k_huff_image     the self-synchronising parallel decoder (Weissenberger &
//                    Schmidt, ICPP 2018), one 1024-lane workgroup per image.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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
    const int32_t r2 = rs - t;
    const bool m = r2 < 0;
    hi = m ? lo : hi;
    lo = m ? nxt : lo;
    rs = r2 & 31;
    wi += m ? 1 : 0;
    nxt = src(wi);
  }
  // consume() without the refill: the caller reloads nxt with refill() at the
  // top of its next step, next to the lookup, so that both LDS loads share
  // one wait (a refill at the end of a loop body with branches is waited for
  // on the spot to merge its value)
  __device__ __forceinline__ void consume_nl(int t) {
    p += t;
    const int32_t r2 = rs - t;
    const bool m = r2 < 0;
    hi = m ? lo : hi;
    lo = m ? nxt : lo;
    rs = r2 & 31;
    wi += m ? 1 : 0;
  }
  __device__ __forceinline__ void refill() { nxt = src(wi); }
  __device__ __forceinline__ int32_t pos() const { return p; }
};

// ---------------------------------------------------------------------------
// Decode constants of one image and the lookup. The state between symbols is
// (b3, k): 3 * (block within the MCU) and the coefficient index (0: DC next).
// ---------------------------------------------------------------------------
struct Dec {
  lds_cu8 tabs;      // the image's distinct tables: lc of slot s at byte s << 13,
                     // l2 of slot s at byte (ns << 13) + s * kL2Bytes
  uint32_t dcseq;    // LDS table slot of MCU block b's DC table at bits 3b
  uint32_t acseq;    // ... AC table
  int b3end;         // 3 * blocks per MCU
  int ns;            // distinct tables (slots)
  uint32_t acmask;   // slots holding AC tables
  const HuffTab *g;  // plan tables (canonical fallback)
  const ImgDesc *d;
};

constexpr int kLcBytes = 4 << kLookBits;              // lc part of a table in LDS
constexpr int kL2Bytes = 2 * (kL2Chunks << kL2Bits);  // l2 part
static_assert(kLcBytes == 1 << 13, "lc slot stride is a shift by 13");

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
// Constant indices only (fully unrolled selects), so slot_tab stays in
// registers instead of a scratch array.
__device__ __forceinline__ int image_slots(const ImgDesc &d, uint32_t &slotmap, int *slot_tab) {
  int t[6], sl[6];
#pragma unroll
  for (int x = 0; x < 6; ++x) {
    const int c = x >> 1;
    const int cc = c < d.ncomp ? c : 0;
    t[x] = (x & 1) ? d.act[cc] : d.dct[cc];
    slot_tab[x] = 0;
  }
  int ns = 0;
  slotmap = 0;
#pragma unroll
  for (int x = 0; x < 6; ++x) {
    int found = -1;
#pragma unroll
    for (int y = 0; y < x; ++y)
      if (found < 0 && t[y] == t[x]) found = sl[y];
    const bool fresh = found < 0;
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if (fresh && q == ns) slot_tab[q] = t[x];
    sl[x] = fresh ? ns : found;
    ns += fresh ? 1 : 0;
    slotmap |= (uint32_t)sl[x] << (3 * x);
  }
  return ns;
}

// An image's distinct tables in LDS: lc parts at an 8 KB stride (the slot's
// offset is one shift), l2 parts after them. Piece i (16 bytes) of the copy:
// its source in the plan tables and its LDS byte offset.
constexpr int kTabPieces = (kLcBytes + kL2Bytes) / 16; // HuffTab: lc then l2
typedef uint32_t v4u __attribute__((ext_vector_type(4))); // 16-byte piece (LDS-storable)
static_assert(sizeof(HuffTab) % 16 == 0, "16-byte table pieces");
// The plan-table index of each of an image's (at most 6) slots, 16 bits
// each, packed into integers: picking one by a variable slot is shifts, where
// an int[6] picked by a select chain is folded into a dynamically indexed
// load that puts the array in scratch memory.
struct SlotTabs {
  uint64_t lo; // slots 0-3
  uint32_t hi; // slots 4-5
  __device__ __forceinline__ int get(int q) const {
    return (int)(q < 4 ? (lo >> (16 * q)) & 0xFFFFu : (hi >> (16 * (q - 4))) & 0xFFFFu);
  }
};
__device__ __forceinline__ SlotTabs pack_slots(const int *slot_tab) {
  SlotTabs t;
  t.lo = 0;
  t.hi = 0;
#pragma unroll
  for (int x = 0; x < 4; ++x) t.lo |= (uint64_t)(slot_tab[x] & 0xFFFF) << (16 * x);
  t.hi = (uint32_t)(slot_tab[4] & 0xFFFF) | ((uint32_t)(slot_tab[5] & 0xFFFF) << 16);
  return t;
}
__device__ __forceinline__ const v4u *tab_piece_src(const HuffTab *__restrict__ htabs,
                                                      const SlotTabs &st, int i, int &dst, int ns) {
  const int q = i / kTabPieces, o = i - q * kTabPieces;
  const int tix = st.get(q);
  dst = o < kLcBytes / 16 ? (q << 13) + 16 * o : (ns << 13) + q * kL2Bytes + 16 * o - kLcBytes;
  return reinterpret_cast<const v4u *>(htabs + tix) + o;
}

// The decode constants of an image; with `copy`, also its tables into LDS
// (k_huff_image stages them itself, together with the stream window).
__device__ __forceinline__ Dec load_dec(const ImgDesc &d, const HuffTab *__restrict__ htabs,
                                        LDS_AS uint8_t *tabs, int tid, int nthreads,
                                        bool copy = true, SlotTabs *slot_tab_out = nullptr) {
  int slot_tab[6];
  uint32_t slotmap;
  const int ns = image_slots(d, slotmap, slot_tab);
  const SlotTabs stp = pack_slots(slot_tab);
  if (copy) {
    for (int i = tid; i < ns * kTabPieces; i += nthreads) {
      int dst;
      const v4u v = *tab_piece_src(htabs, stp, i, dst, ns);
      *(LDS_AS v4u *)(tabs + dst) = v;
    }
  }
  if (slot_tab_out) *slot_tab_out = stp;
  Dec dec;
  dec.tabs = tabs;
  dec.dcseq = dec.acseq = 0;
  // constant indices into dword loads of bcomp (4-aligned in ImgDesc): scalar
  // loads of the descriptor, no loop of dependent byte loads
  static_assert(offsetof(ImgDesc, bcomp) % 4 == 0, "bcomp dword loads");
  const uint32_t *bcw = reinterpret_cast<const uint32_t *>(d.bcomp);
  const uint32_t bw[3] = {bcw[0], bcw[1], bcw[2]};
#pragma unroll
  for (int b = 0; b < kMaxBlocksPerMcu; ++b) {
    if (b < d.bpm) {
      const int c = (int)(bw[b >> 2] >> (8 * (b & 3))) & 3;
      dec.dcseq |= ((slotmap >> (6 * c)) & 7) << (3 * b);
      dec.acseq |= ((slotmap >> (6 * c + 3)) & 7) << (3 * b);
    }
  }
  dec.ns = ns;
  dec.acmask = 0;
  for (int x = 1; x < 6; x += 2) dec.acmask |= 1u << ((slotmap >> (3 * x)) & 7);
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

// Second level of a long code (l1 entry e1: total == 0).
__device__ __forceinline__ uint32_t lookup_long(const Dec &dec, uint32_t slot, uint32_t e1, uint32_t pk,
                                                int b3, bool ac) {
  if (e1 == kHuffCanon) return lookup_canon(dec.g, dec.d, b3 / 3, ac, pk);
  const lds_cu16 l2 = (lds_cu16)(dec.tabs + (dec.ns << 13) + slot * kL2Bytes);
  return l2[((e1 >> 5) << kL2Bits) + ((pk >> 16) & ((1u << kL2Bits) - 1))];
}

// Entry of the symbol whose code starts at the top bit of pk.
__device__ __forceinline__ uint32_t lookup(const Dec &dec, const St &st, uint32_t pk) {
  const bool ac = st.k != 0;
  const uint32_t slot = __builtin_amdgcn_ubfe(ac ? dec.acseq : dec.dcseq, (uint32_t)st.b3, 3u);
  // the l1 entry: the low 16-bit half of the lc word, read on its own
  uint32_t e = *(lds_cu16)(dec.tabs + (slot << 13) + ((pk >> (32 - kLookBits)) << 2));
  // long codes are rare: a wave-uniform test keeps the exec mask untouched
  if (__builtin_expect(__any((e & 31) == 0), 0))
    if ((e & 31) == 0) e = lookup_long(dec, slot, e, pk, st.b3, ac);
  return e;
}

// HUFF_EXTEND of the s magnitude bits following the code.
// raw < 2^(s-1) (top magnitude bit clear) is negative: raw - (2^s - 1); the
// s-bit mask is one bit-field extract of all ones (s = 0: raw = mask = 0,
// value 0).
__device__ __forceinline__ int ext_value(uint32_t pk, uint32_t e) {
  const uint32_t total = e & 31, s = (e >> 5) & 15;
  const int raw = (int)__builtin_amdgcn_ubfe(pk, 32 - total, s);
  const int mask = (int)__builtin_amdgcn_ubfe(0xFFFFFFFFu, 0u, s);
  return raw <= (mask >> 1) ? raw - mask : raw;
}

// k += adv; k >= 64 ends the block (EOB advances by 64).
__device__ __forceinline__ void advance(St &st, int b3end, int adv) {
  const int k2 = st.k + adv;
  const bool end = k2 >= 64;
  int nb = st.b3 + 3;
  nb = nb == b3end ? 0 : nb;
  st.b3 = end ? nb : st.b3;
  st.k = end ? 0 : k2;
}
__device__ __forceinline__ void advance(St &st, const Dec &dec, int adv) { advance(st, dec.b3end, adv); }

// Count-only step (blocks started) on the count-mode entries (HuffTab.lc
// high half, see ldt_types.hpp): one lookup consumes a run of AC symbols of
// one block. A run's symbols before its last advance k by at most 15, so with
// k <= 48 no block ends inside it; from k = 49 on, the l1 entry (low half:
// the first symbol alone) is used. Both halves keep total bits at 0-4 and the
// coefficient advance at 9-15.
template <class W>
__device__ __forceinline__ void count_step(Rd<W> &R, St &st, const Dec &dec, int &nblk) {
  const uint32_t pk = R.peek();
  const bool dcs = st.k == 0;
  const uint32_t slot = __builtin_amdgcn_ubfe(dcs ? dec.dcseq : dec.acseq, (uint32_t)st.b3, 3u);
  // the entry's 16-bit half straight from LDS (no shift/select after the
  // load, which is on the bit-position dependency chain): the count-mode
  // half (high) while k <= 48, the l1 half (low) from k = 49
  // (table offset and half come from the state, off the chain)
  const uint32_t soff = (slot << 13) + (st.k >= 49 ? 0u : 2u);
  const uint32_t idx4 = (pk >> (32 - kLookBits)) << 2;
  const uint32_t e = *(lds_cu16)(dec.tabs + soff + idx4);
  uint32_t t = e & 31u;
  uint32_t adv = e >> 9;
  if (__builtin_expect(__any(t == 0), 0)) {
    if (t == 0) { // long code: the first symbol alone
      const uint32_t e2 = lookup_long(dec, slot, *(lds_cu16)(dec.tabs + (slot << 13) + idx4), pk, st.b3, !dcs);
      t = e2 & 31;
      adv = e2 >> 9;
    }
  }
  nblk += dcs ? 1 : 0;
  R.consume((int)t);
  advance(st, dec, (int)adv);
}

// Coefficients of a block are stored in zigzag (decode) order, int16 slots
// 1..63 (the DC difference goes into the block record; k_idct de-zigzags while
// dequantising). Slots are combined 8 at a time (a 16-byte group) in
// registers: a block's coefficient indices only grow, so a group is complete
// once the decode moves to another group or block. Only nonzero groups are
// stored, packed (ldt_kernels.hpp): one 16-byte unit each, consecutive for the
// run's consecutive blocks. (Holding four units back in registers so that a
// run's 64-byte segments leave as one burst cut the kernel's HBM writes from
// ~210 to 132 MB per c2 batch but made the write pass 20 us per image slower:
// the extra store instructions issue for the whole wave)

// Where a run's block records and chunk carries go: the workgroup's LDS
// (k_huff_image, copied out coalesced after the DC scan) or global memory.
struct RecLds {
  LDS_AS uint32_t *rec, *carry;
  __device__ __forceinline__ void put(int ib, uint32_t v) const { rec[ib] = v; }
  __device__ __forceinline__ void put_carry(int c, uint32_t u) const { carry[c] = u; }
};
struct RecGlob {
  uint32_t *rec, *carry;
  __device__ __forceinline__ void put(int ib, uint32_t v) const { rec[ib] = v; }
  __device__ __forceinline__ void put_carry(int c, uint32_t u) const { carry[c] = u; }
};

// Coefficient-writing decode of one range, with block ownership: a block
// belongs to the range that decodes its DC symbol. The run starts at the
// reader's position with cursor -1; a block it enters mid-way (k != 0) is
// decoded without stores (the previous range writes it), and the run goes on
// past `stop` until its last block is complete (k back to 0), so every block
// is written by one lane. Blocks are base + cursor of the image for cursor in
// [0, lim) (lim: the segment's blocks not started before the range); the run
// ends before a block beyond lim. Its nonzero groups are packed from unit
// 8 * base of the image's coefficient region (at most 8 per block, so a run
// never reaches the next run's units). Each block's record (gmask | run
// start << 8 | DC difference << 16, see ldt_kernels.hpp) is stored when the
// next block starts or the run ends, and a block at a multiple of 64
// publishes its first unit as its chunk's carry. The loop has one group store
// site: the buffered group is stored when a nonzero AC value opens another
// group or a block starts.
// Returns the symbols decoded (loop iterations; a diagnostic).
template <class W, class RS>
__device__ __forceinline__ int write_run(Rd<W> &R, St &st, const Dec &dec, int32_t stop,
                                          int &cursor, int lim, uint4 *__restrict__ coef_img,
                                          const RS &rs, int base) {
  uint64_t lo = 0, hi = 0;           // buffered group: slots 0-3, 4-7
  int cg = -1;                       // its group index; < 0: none
  // units leave in pairs (one 32-byte store per two units: the Huffman stage
  // writes 166 MB per c2 batch instead of 235 MB unpaired at the same speed;
  // a 4-unit queue, 132 MB, cost 2%: profiles/r4/write_queue_ab_r4.txt)
  uint4 q2 = make_uint4(0u, 0u, 0u, 0u), q3 = q2;
  uint32_t wu = (uint32_t)base * 8u; // units stored
  uint32_t gmask = 0;                // groups of the current block
  uint32_t dcd = 0;                  // its DC difference (16 bits)
  bool go = (R.p < stop || st.k != 0) && !(st.k == 0 && cursor + 1 >= lim);
  int iters = 0;
  while (go) {
    ++iters;
    R.refill();
    const bool first = st.k == 0; // a block starts: its DC symbol
    const uint32_t pk = R.peek();
    const uint32_t e = lookup(dec, st, pk);
    const int v = ext_value(pk, e);
    const int adv = (int)(e >> 9);
    // a corrupt stream can run k past 63 (a run or ZRL from k > 48): jdhuff.c
    // then stores into natural[k >= 64] = position 63; so does this clamp.
    const int slot = min(st.k + adv - 1, 63);
    const int g = slot >> 3;
    const bool opens = !first && v != 0 && g != cg && cursor >= 0;
    const bool flush = cg >= 0 && (first || opens);
    const uint4 cur = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
    if (flush) {
      q2 = q3;
      q3 = cur;
      gmask |= 1u << cg;
      ++wu;
      if ((wu & 1u) == 0) {
        coef_img[wu - 2] = q2;
        coef_img[wu - 1] = q3;
      }
    }
    // a block starts: the previous one's record, then this block's state
    if (first) {
      if (cursor >= 0) rs.put(base + cursor, gmask | (cursor == 0 ? 256u : 0u) | (dcd << 16));
      ++cursor;
      if (((base + cursor) & 63) == 0) rs.put_carry((base + cursor) >> 6, wu);
    }
    gmask = first ? 0u : gmask;
    dcd = first ? (uint32_t)v & 0xFFFFu : dcd;
    lo = (first || opens) ? 0ull : lo;
    hi = (first || opens) ? 0ull : hi;
    cg = first ? -1 : (opens ? g : cg);
    // cg < 0: the partial block the run entered (not owned) or a DC symbol
    const uint64_t x = cg >= 0 ? (uint64_t)((uint32_t)v & 0xFFFFu) << (16 * (slot & 3)) : 0ull;
    lo |= (slot & 4) ? 0ull : x;
    hi |= (slot & 4) ? x : 0ull;
    R.consume_nl((int)(e & 31));
    advance(st, dec, adv);
    go = (R.p < stop || st.k != 0) && !(st.k == 0 && cursor + 1 >= lim);
  }
  if (cursor >= 0) {
    if (cg >= 0) {
      const uint4 cur = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
      if (wu & 1u) coef_img[wu - 1] = q3;
      coef_img[wu] = cur;
      gmask |= 1u << cg;
      ++wu;
    } else if (wu & 1u) {
      coef_img[wu - 1] = q3;
    }
    rs.put(base + cursor, gmask | (cursor == 0 ? 256u : 0u) | (dcd << 16));
  }
  return iters;
}

// ---------------------------------------------------------------------------
// k_huff_image's write pass (round 6): the same output as write_run, with the
// open coefficient group staged in LDS instead of registers.
//
// The write pass is bound by VALU issue (16 waves), and with
// the lanes at different points of their decodes every path of the loop body
// issues in nearly every iteration. write_run's register group (two 64-bit
// halves: a 64-bit shift, selects and ORs to place each value, and selects to
// clear it) and its unit pairing cost ~20 of its ~100 VALU per iteration.
// Here the lane's open group lives in 16 bytes of LDS (group_at), so a value
// lands with one ds_write_b16 at an address of two VALU; a flush reads the 16
// bytes back (two 64-bit LDS reads), stores the unit and writes zeros behind
// it. The l1 lookup reads the compacted tables (compact_tables).
// ---------------------------------------------------------------------------
struct DecW {
  lds_cu8 l1;        // compacted l1 entries: slot s at byte s << 12
  lds_cu8 l2;        // l2 parts: slot s at byte s * kL2Bytes
  uint32_t dcseq, acseq;
  int b3end;
  const HuffTab *g;
  const ImgDesc *d;
};

// The write pass's lookup (l1 entry, as lookup()).
__device__ __forceinline__ uint32_t lookup_w(const DecW &dec, const St &st, uint32_t pk) {
  const bool ac = st.k != 0;
  const uint32_t slot = __builtin_amdgcn_ubfe(ac ? dec.acseq : dec.dcseq, (uint32_t)st.b3, 3u);
  uint32_t e = *(lds_cu16)(dec.l1 + (slot << 12) + ((pk >> (32 - kLookBits)) << 1));
  if (__builtin_expect(__any((e & 31) == 0), 0)) {
    if ((e & 31) == 0) {
      if (e == kHuffCanon)
        e = lookup_canon(dec.g, dec.d, st.b3 / 3, ac, pk);
      else
        e = ((lds_cu16)(dec.l2 + slot * kL2Bytes))[((e >> 5) << kL2Bits) + ((pk >> 16) & ((1u << kL2Bits) - 1))];
    }
  }
  return e;
}

// A lane's open group: 16 bytes at planes + 16 t + 4 (t >> 3). The 4-byte step
// every 8 lanes spreads a wave's 16-bit value stores over the banks (lanes 8
// apart would otherwise hit the same one); the group is read and zeroed as
// two 64-bit halves of 4-byte alignment (ds_read2 / ds_write2). An earlier
// layout rotated each lane's dwords instead and spent 8 selects per flush
// undoing the rotation (write phase 83 vs 79 us per c2 image,
// profiles/r6/write_group_ab_r6wxy.txt).
typedef uint32_t v4ua __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ LDS_AS v4ua *group_at(LDS_AS uint8_t *planes, int t) {
  return (LDS_AS v4ua *)(planes + 16 * t + 4 * (t >> 3));
}

// After the rounds (no lane reads the count-mode halves any more): each
// table's l1 halves become a 4 KB u16 array at slot << 12, its l2 part moves
// to (ns << 12) + slot * kL2Bytes, and the lanes' groups at ns *
// kTabCompactBytes (kHuffPlaneBytes, within huff_tab_lds_image) are zeroed.
// Entries are moved in chunks of 4 per lane in increasing order, each read
// before a barrier and written after it: entry j moves from byte 4j to 2j, so
// a chunk's writes stay below every later chunk's sources. Contains
// __syncthreads (two per chunk).
__device__ __forceinline__ DecW compact_tables(const Dec &dec, LDS_AS uint8_t *tabs, int tid,
                                              LDS_AS uint8_t *&planes) {
  const int ns = dec.ns;
  const int nw = ns << (kLookBits); // lc words (2048 per table)
  const int nl2 = ns * (kL2Bytes / 4);
  const uint32_t l2w = tid < nl2 ? ((lds_cu32)(tabs + (ns << 13)))[tid] : 0u;
  for (int c0 = 0; c0 < nw; c0 += 4 * kHuffThreads) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = c0 + tid + i * kHuffThreads;
      w[i] = j < nw ? ((lds_cu32)tabs)[j] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = c0 + tid + i * kHuffThreads;
      if (j < nw) ((LDS_AS uint16_t *)tabs)[j] = (uint16_t)w[i];
    }
    __syncthreads();
  }
  // the l2 parts (read above, before any write) below the groups
  if (tid < nl2) ((LDS_AS uint32_t *)(tabs + (ns << 12)))[tid] = l2w;
  planes = tabs + ns * kTabCompactBytes;
  static_assert(kHuffPlaneBytes == 16 * kHuffThreads + 4 * (kHuffThreads / 8), "16 bytes per lane, 4 per 8 lanes");
  *group_at(planes, tid) = (v4ua)(0u);
  __syncthreads();
  DecW dw;
  dw.l1 = tabs;
  dw.l2 = tabs + (ns << 12);
  dw.dcseq = dec.dcseq;
  dw.acseq = dec.acseq;
  dw.b3end = dec.b3end;
  dw.g = dec.g;
  dw.d = dec.d;
  return dw;
}

typedef v4ua GroupT;
template <class RD, class RS>
__device__ __forceinline__ int write_run_lds(RD &R, St &st, const DecW &dec, int32_t stop,
                                              int &cursor, int lim, uint4 *__restrict__ coef_img,
                                              const RS &rs, int base, LDS_AS GroupT *gp) {
  // the lane's open group (group_at: 16 contiguous bytes, one read and one
  // zeroing write per flush instead of 8 + 8 16-bit ones)
  auto unit = [&]() {
    const v4ua sv = *gp;
    return make_uint4(sv.x, sv.y, sv.z, sv.w);
  };
  int cg = -1;                       // the open group's index; < 0: none
  uint32_t wu = (uint32_t)base * 8u; // units stored
  uint32_t gmask = 0;                // groups of the current block
  uint32_t dcd = 0;                  // its DC difference (16 bits)
  int bcur = base + cursor;          // image block of the current block (base - 1: none owned yet)
  const int blast = base + lim - 1;  // the last block the run may own
  bool go = (R.pos() < stop || st.k != 0) && !(st.k == 0 && bcur >= blast);
  int iters = 0;
  while (go) {
    ++iters;
    R.refill();
    const bool first = st.k == 0; // a block starts: its DC symbol
    const uint32_t pk = R.peek();
    const uint32_t e = lookup_w(dec, st, pk);
    const int v = ext_value(pk, e);
    const int adv = (int)(e >> 9);
    // a corrupt stream can run k past 63 (a run or ZRL from k > 48): jdhuff.c
    // then stores into natural[k >= 64] = position 63; so does this clamp.
    const int slot = min(st.k + adv - 1, 63);
    const int g = slot >> 3;
    // a nonzero AC value of an owned block (an AC value is nonzero iff s != 0)
    const bool put = !first && (e & (15u << 5)) != 0 && bcur >= base;
    const bool opens = put && g != cg;
    if (cg >= 0 && (first || opens)) {
      // the open group is complete: its unit, then zeros behind it
      const uint4 u = unit();
      *gp = (GroupT)(0u);
      coef_img[wu] = u;
      ++wu;
      gmask |= 1u << cg;
    }
    if (put) ((LDS_AS uint16_t *)gp)[slot & 7] = (uint16_t)v;
    // a block starts: the previous one's record, then this block's state
    if (first) {
      if (bcur >= base) rs.put(bcur, gmask | (bcur == base ? 256u : 0u) | (dcd << 16));
      ++bcur;
      if ((bcur & 63) == 0) rs.put_carry(bcur >> 6, wu);
    }
    gmask = first ? 0u : gmask;
    dcd = first ? (uint32_t)v & 0xFFFFu : dcd;
    cg = first ? -1 : (opens ? g : cg);
    R.consume_nl((int)(e & 31));
    advance(st, dec.b3end, adv);
    go = (R.pos() < stop || st.k != 0) && !(st.k == 0 && bcur >= blast);
  }
  if (bcur >= base) {
    if (cg >= 0) {
      coef_img[wu] = unit();
      gmask |= 1u << cg;
      ++wu;
    }
    rs.put(bcur, gmask | (bcur == base ? 256u : 0u) | (dcd << 16));
  }
  cursor = bcur - base;
  return iters;
}

// ---------------------------------------------------------------------------
// Serial decoder: one 64-lane workgroup per image, one lane per segment.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_huff_serial(const ImgDesc *__restrict__ descs,
                                                    const Segment *__restrict__ segs,
                                                    const HuffTab *__restrict__ htabs,
                                                    const uint8_t *__restrict__ dstuf,
                                                    int16_t *__restrict__ coef,
                                                    uint32_t *__restrict__ brec,
                                                    uint32_t *__restrict__ bcarry,
                                                    int32_t *__restrict__ status) {
  const int img = blockIdx.x;
  // nseg 0: progressive (k_prog); sub_bits > 0: the parallel decoder
  if (status[img] != 0 || descs[img].nseg == 0 || descs[img].sub_bits > 0) return;
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  const Dec dec = load_dec(d, htabs, (LDS_AS uint8_t *)dyn_lds, tid, 64);
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
    const int blk0 = sg.mcu_first * d.bpm; // image-relative
    // a valid segment ends inside its bits; 64 bits of slack bound a corrupt one
    write_run(R, st, dec, pbias + seg_bits + 64, cursor, total, reinterpret_cast<uint4 *>(coef + d.coef_off * 64),
              RecGlob{brec + d.coef_off, bcarry + d.coef_off / 64}, blk0);
    if (R.p - pbias > seg_bits || cursor + 1 < total || st.k != 0) status[img] = 3; // truncated
  }
}

hipError_t launch_huff_serial(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n_serial == 0) return hipSuccess;
  const size_t tab_lds = (size_t)huff_tab_lds(p.max_tabs);
  hipLaunchKernelGGL(k_huff_serial, dim3(p.n), dim3(64), tab_lds, s, p.descs, p.segs, p.htabs,
                     w.dstuf, w.coef, w.brec, w.bcarry, w.status);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// DC predictors (jdhuff.c: last_dc_val[ci] += diff, reset to 0 at every
// restart marker, process_restart) of one image, by its NT-thread workgroup:
// thread t owns a run of consecutive blocks; a segmented scan over the threads
// carries the per-component sums. The DC differences are read from the block
// records (bits 16-31, write_run) and replaced there by the absolute DC
// (JCOEF, truncated) in place: each record is read and written by one thread.
// REC is the records' pointer type (LDS or global). `scr` is 4*NT/64 ints of
// LDS; contains __syncthreads.
template <int NT, class REC>
__device__ __forceinline__ void dc_scan_image(const ImgDesc &d, REC rec, LDS_AS int32_t *scr) {
  static_assert(NT % 64 == 0, "whole waves");
  const int tid = threadIdx.x;
  const int bpm = d.bpm;
  const int64_t nblk = (int64_t)d.mcux * d.mcuy * bpm;
  const int64_t seglen = d.restart ? (int64_t)d.restart * bpm : nblk;
  uint32_t compmap = 0;
  for (int b = 0; b < bpm; ++b) compmap |= (uint32_t)(d.bcomp[b] & 3) << (2 * b);
  const int64_t K = (nblk + NT - 1) / NT;
  const int64_t lo = (int64_t)tid * K, hi = min(lo + K, nblk);
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
      const int dv = (int)rec[x] >> 16;
      s0 += c == 0 ? dv : 0;
      s1 += c == 1 ? dv : 0;
      s2 += c == 2 ? dv : 0;
      b = b + 1 == bpm ? 0 : b + 1;
      sp = sp + 1 == seglen ? 0 : sp + 1;
    }
  }
  // segmented scan of (flag, s0, s1, s2) over the threads: within each wave
  // by lane shifts, then across the NT/64 wave totals (one barrier)
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int pf = __shfl_up(flag, off), p0 = __shfl_up(s0, off), p1 = __shfl_up(s1, off),
              p2 = __shfl_up(s2, off);
    if (lane >= off && !flag) {
      s0 += p0;
      s1 += p1;
      s2 += p2;
    }
    flag |= lane >= off ? pf : 0;
  }
  if (lane == 63) {
    scr[4 * wave] = flag;
    scr[4 * wave + 1] = s0;
    scr[4 * wave + 2] = s1;
    scr[4 * wave + 3] = s2;
  }
  __syncthreads();
  // the carry into this wave: the segmented sum of the earlier waves' totals
  int r0 = 0, r1 = 0, r2 = 0;
  for (int w = 0; w < wave; ++w) {
    const bool f = scr[4 * w] != 0;
    r0 = (f ? 0 : r0) + scr[4 * w + 1];
    r1 = (f ? 0 : r1) + scr[4 * w + 2];
    r2 = (f ? 0 : r2) + scr[4 * w + 3];
  }
  {
    // exclusive within the wave: the previous lane's inclusive value
    const int pf = __shfl_up(flag, 1), p0 = __shfl_up(s0, 1), p1 = __shfl_up(s1, 1),
              p2 = __shfl_up(s2, 1);
    if (lane > 0) {
      r0 = (pf ? 0 : r0) + p0;
      r1 = (pf ? 0 : r1) + p1;
      r2 = (pf ? 0 : r2) + p2;
    }
  }
  int b = b0;
  int64_t sp = sp0;
  for (int64_t x = lo; x < hi; ++x) {
    if (sp == 0) r0 = r1 = r2 = 0;
    const int c = (int)((compmap >> (2 * b)) & 3);
    const uint32_t rv = rec[x];
    const int dv = (int)rv >> 16;
    r0 += c == 0 ? dv : 0;
    r1 += c == 1 ? dv : 0;
    r2 += c == 2 ? dv : 0;
    const int dc = c == 0 ? r0 : c == 1 ? r1 : r2;
    rec[x] = (rv & 0xFFFFu) | ((uint32_t)dc << 16);
    b = b + 1 == bpm ? 0 : b + 1;
    sp = sp + 1 == seglen ? 0 : sp + 1;
  }
}

// k_dc_scan: the DC predictors of the serial decoder's images (the parallel
// decoder's workgroups scan their own image after the write pass).
__global__ void __launch_bounds__(256) k_dc_scan(const ImgDesc *__restrict__ descs,
                                                 uint32_t *__restrict__ brec,
                                                 const int32_t *__restrict__ status) {
  __shared__ int32_t scr[4 * 256 / 64];
  const int img = blockIdx.x;
  // progressive: dcv holds the final DC; sub_bits > 0: k_huff_image
  if (status[img] != 0 || descs[img].nseg == 0 || descs[img].sub_bits > 0) return;
  dc_scan_image<256>(descs[img], brec + descs[img].coef_off, (LDS_AS int32_t *)scr);
}

hipError_t launch_dc_scan(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n_serial == 0) return hipSuccess;
  hipLaunchKernelGGL(k_dc_scan, dim3(p.n), dim3(256), 0, s, p.descs, w.brec, w.status);
  return hipGetLastError();
}

// ===========================================================================
// Parallel self-synchronising decode: one 1024-lane workgroup per image.
//
// A segment's bits are cut into subsequences of S bits; lane t of the image's
// workgroup owns slot t, subsequence j = t - sub_first of the segment that
// holds it, i.e. bits [j*S, (j+1)*S). The decode state at a symbol boundary is
// (p, b, k): bit position, block within the MCU, coefficient index (k == 0: a
// DC symbol is next). A slot's exit state is the state at the first symbol
// boundary p >= (j+1)*S; under its true entry state that is its successor's
// true entry state. Two decoders in the same state decode identically from
// there on, which is why chains started from a guessed state converge (Huffman
// codes resynchronise).
//
// The planner gives every image an S that fits all its slots in one workgroup
// (S >= bits / (1024 - nseg)), so an image converges inside its workgroup:
// no helper lanes, no walks across workgroup boundaries, and the block prefix
// that places each range's coefficients is a workgroup scan. Per image:
//   setup    the image's distinct tables and its whole destuffed stream
//            (byte-swapped) into LDS; a stream larger than the window is read
//            from global memory instead;
//   phase 1  every lane decodes its range from a guessed state (b = 0, k = 0;
//            exact at a segment start), counting blocks, and records its entry,
//            exit and two checkpoints;
//   rounds   a lane re-decodes only while its entry differs from its
//            predecessor's exit; a re-decode stops at the first checkpoint
//            where it merges with its own previous trajectory. The rounds end
//            when no exit changed (at most one per slot: the true state only
//            flows to the right);
//   prefix   exclusive scan of the block counts: each range's first block;
//   write    every lane decodes its range again from its true entry and stores
//            its blocks' nonzero coefficient groups (packed) and their records
//            (into LDS when the image has <= kRecCap blocks);
//   dc       the workgroup adds the DC predictors in the records
//            (dc_scan_image), which then leave in coalesced stores.
// An image with more than kMaxParSegs restart segments takes k_huff_serial
// instead: one lane per segment is already parallel there.
// ===========================================================================

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

// Static LDS of k_huff_image (the window and the tables are dynamic): the
// decode state of every slot, so that a round's re-decodes can be packed into
// the first waves of the workgroup (any lane may work on any slot).
constexpr int kRecCap = 8192; // block records an image keeps in LDS during the write pass
struct ImgLds {
  int32_t ex_p[kHuffThreads];  // exit position (segment-relative)
  union {
    // decode state of the slots (phase 1 and the rounds)
    struct {
      // entry of the slot's current trajectory and its checkpoint positions,
      // relative to the range start j*S (< S + 32 <= kMaxParS + 32)
      uint16_t en_p[kHuffThreads];
      uint16_t cp_p0[kHuffThreads], cp_p1[kHuffThreads];
      uint16_t ex_bk[kHuffThreads], en_bk[kHuffThreads]; // (3b << 8) | k
      uint16_t cp_bk0[kHuffThreads], cp_bk1[kHuffThreads];
      uint16_t cp_a0[kHuffThreads], cp_a1[kHuffThreads]; // blocks counted up to the checkpoints
      uint16_t nblk[kHuffThreads]; // blocks started in the range (S <= kMaxParS bounds it)
      uint16_t work[kHuffThreads]; // this round's slots to re-decode
      // the slot's previous trajectory (memo): entry, exit (relative to the
      // range start) and block count; m_en_bk = 0xFFFF: none
      uint16_t m_en_p[kHuffThreads], m_en_bk[kHuffThreads];
      uint16_t m_ex_p[kHuffThreads], m_ex_bk[kHuffThreads], m_nblk[kHuffThreads];
      uint8_t cp_n[kHuffThreads];
    };
    // write pass (images of <= kRecCap blocks): the block records and chunk
    // carries (ldt_kernels.hpp), copied out coalesced after the DC scan
    struct {
      uint32_t rec[kRecCap];
      uint32_t carry[kRecCap / 64];
    };
  };
  int32_t seg_first[kMaxParSegs + 1]; // sub_first of the image's segments; [nseg] = slots
  int32_t seg_pb[kMaxParSegs];        // segment start: bit position in the window
  int32_t seg_nb[kMaxParSegs];        // segment length in bits
  int32_t scan[kHuffThreads / 64];
  int32_t nwork;          // the rounds' work list length
  int32_t any_changed[2]; // a round's exits changed (alternating words)
  // fused destuff: per wave, the scan position of the first end-of-scan
  // marker in its lanes' bytes of the current tile (written every tile by
  // every wave, so no initialisation has to be ordered before other waves'
  // writes)
  alignas(16) int32_t ds_endw[kHuffThreads / 64];
  int32_t need_lanes, need_waves, memo_hits; // diagnostic counters (summed over rounds)
  int32_t w_syms, w_wmax;                      // ... and of the write pass
};
static_assert(sizeof(ImgLds) + 512 <= kHuffStaticLds, "k_huff_image static LDS");
static_assert(sizeof(ImgLds) >= 4 * (kHuffThreads / 64) * sizeof(int32_t), "dc_scan_image scratch");

// Exclusive prefix of v over the 1024-lane workgroup; contains __syncthreads.
__device__ __forceinline__ int block_excl_scan1024(int v, int32_t *scratch, int *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int inc = wave_incl_scan(v);
  if (lane == 63) scratch[wave] = inc;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kHuffThreads / 64; ++w) {
    const int s = scratch[w];
    base += w < wave ? s : 0;
    tot += s;
  }
  *total = tot;
  __syncthreads();
  return base + inc - v;
}

// Where slot q of the image lies: its segment, subsequence index, window bit
// position of the segment start, segment length and the range [rstart, stop).
struct SlotGeom {
  int si, j;
  int32_t pbias, seg_bits, rstart, stop;
};
__device__ __forceinline__ SlotGeom slot_geom(const ImgLds &sh, int nseg, int S, int q) {
  int lo = 0, hi = nseg - 1; // last segment with seg_first <= q
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (sh.seg_first[mid] <= q) lo = mid;
    else hi = mid - 1;
  }
  SlotGeom g;
  g.si = lo;
  g.j = q - sh.seg_first[lo];
  g.pbias = sh.seg_pb[lo];
  g.seg_bits = sh.seg_nb[lo];
  g.rstart = g.pbias + g.j * S;
  g.stop = g.pbias + min((g.j + 1) * S, g.seg_bits);
  return g;
}

// checkpoint positions are reader positions; stored relative to the range start
__device__ __forceinline__ void put_cp(ImgLds &sh, int q, const Cp &cp, int32_t rstart) {
  sh.cp_p0[q] = (uint16_t)(cp.p0 - rstart);
  sh.cp_p1[q] = (uint16_t)(cp.p1 - rstart);
  sh.cp_bk0[q] = (uint16_t)cp.bk0;
  sh.cp_bk1[q] = (uint16_t)cp.bk1;
  sh.cp_a0[q] = (uint16_t)cp.a0;
  sh.cp_a1[q] = (uint16_t)cp.a1;
  sh.cp_n[q] = (uint8_t)cp.n;
}

__device__ __forceinline__ Cp get_cp(const ImgLds &sh, int q, int32_t rstart) {
  Cp cp;
  cp.p0 = rstart + sh.cp_p0[q];
  cp.p1 = rstart + sh.cp_p1[q];
  cp.bk0 = sh.cp_bk0[q];
  cp.bk1 = sh.cp_bk1[q];
  cp.a0 = sh.cp_a0[q];
  cp.a1 = sh.cp_a1[q];
  cp.n = sh.cp_n[q];
  return cp;
}

template <class W>
__device__ __forceinline__ void image_decode(W src, const ImgDesc &d,
                                             const Segment *__restrict__ segs, const Dec &dec,
                                             int warm, uint64_t t_setup, ImgLds &sh,
                                             int16_t *__restrict__ coef,
                                             uint32_t *__restrict__ brec,
                                             uint32_t *__restrict__ bcarry,
                                             int32_t *__restrict__ status, int img,
                                             int32_t *__restrict__ dbg) {
  const int tid = threadIdx.x;
  const int S = d.sub_bits;
  const int nseg = d.nseg;
  const bool live = tid < sh.seg_first[nseg];
  const SlotGeom g = slot_geom(sh, nseg, S, live ? tid : 0);

  // ---- phase 1: every lane decodes its own range from a guess ----
  {
    int nblk = 0;
    Cp cp, none;
    cp.n = 0;
    none.n = 0;
    St st = make_state(0);
    Rd<W> R;
    R.src = src;
    if (live) {
      const int32_t w0 = max(g.rstart - warm, g.pbias);
      R.seek(w0);
      if (w0 < g.rstart) {
        int skipped = 0;
        count_until(R, g.rstart, st, dec, skipped);
      }
      sh.en_p[tid] = (uint16_t)(R.p - g.rstart);
      sh.en_bk[tid] = (uint16_t)st.bk();
      count_run<false>(R, g.rstart, g.stop, S, st, dec, nblk, cp, none, 0);
      sh.ex_p[tid] = R.p - g.pbias;
      sh.ex_bk[tid] = (uint16_t)st.bk();
    } else {
      sh.en_p[tid] = 0;
      sh.ex_p[tid] = 0;
      sh.en_bk[tid] = sh.ex_bk[tid] = 0;
    }
    sh.nblk[tid] = (uint16_t)nblk;
    sh.m_en_bk[tid] = 0xFFFF;
    put_cp(sh, tid, cp, g.rstart);
  }

  // ---- rounds: re-decode every slot whose entry differs from its
  // predecessor's exit, packed into the first waves ----
  int rounds = 0;
  uint64_t t_ph1 = 0;
  const int wave = tid >> 6, lane = tid & 63;
  for (int round = 0; round <= kHuffThreads; ++round) {
    ++rounds;
    // phase 1's states published (a later round's are, by the barrier that
    // ends the round before it)
    if (round == 0) __syncthreads();
    if (dbg && round == 0 && tid == 0) t_ph1 = wall_clock64();
    // this round's work-list length and changed flag start at zero (their
    // last readers, in the rounds before, are past the barrier that ended
    // the previous round; the flag alternates between two words, so no lane
    // still reading the previous round's can see this one's reset)
    if (tid == 0) {
      sh.nwork = 0;
      sh.any_changed[round & 1] = 0;
    }
    // A slot whose predecessor's exit equals the entry of its previous
    // trajectory (its memo) adopts that trajectory again (exits flip between
    // two values while an unsynchronised stretch converges), so a run of such
    // slots resolves without decoding. Round 6 resolves the runs in one pass
    // instead of repeating the test until no slot adopts (~3 passes of two
    // barriers per round): a slot keeps its trajectory C or adopts its memo M,
    // and which one is a function of the predecessor's choice: C if the
    // predecessor's exit equals C's entry, else M if it equals M's entry,
    // else C (the slot is needy). These maps over {C, M} compose along the
    // slots, so an inclusive scan (wave shifts, then the waves' totals after
    // one barrier) gives every slot its choice. A map is 2 bits: bit 0 the
    // choice after a predecessor on C, bit 1 after one on M (1: M). A
    // segment's first slot (and an idle lane) is the constant C.
    uint32_t map = 0u;
    int pc_rel = 0, pc_bk = 0, pm_rel = 0, pm_bk = 0; // the predecessor's C and M exits, range-relative
    int ec_p = 0, ec_bk = 0, em_p = 0, em_bk = 0;      // this slot's C and M entries
    if (live && g.j > 0) {
      ec_p = sh.en_p[tid];
      ec_bk = sh.en_bk[tid];
      em_p = sh.m_en_p[tid];
      em_bk = sh.m_en_bk[tid]; // 0xFFFF: no memo (no exit has that block phase)
      pc_rel = sh.ex_p[tid - 1] - g.j * S;
      pc_bk = sh.ex_bk[tid - 1];
      pm_rel = (int)sh.m_ex_p[tid - 1] - S;
      pm_bk = sh.m_ex_bk[tid - 1];
      // (a predecessor without a memo never chooses M: bit 1 is then unused)
      const bool c_c = pc_rel == ec_p && pc_bk == ec_bk, c_m = pc_rel == em_p && pc_bk == em_bk;
      const bool m_c = pm_rel == ec_p && pm_bk == ec_bk, m_m = pm_rel == em_p && pm_bk == em_bk;
      map = ((!c_c && c_m) ? 1u : 0u) | ((!m_c && m_m) ? 2u : 0u);
    }
    // f o g on 2-bit maps: image of x under f o g is f's bit at g's image of x
    auto compose = [](uint32_t f, uint32_t g2) -> uint32_t {
      return ((f >> (g2 & 1u)) & 1u) | (((f >> ((g2 >> 1) & 1u)) & 1u) << 1);
    };
    uint32_t F = map; // the composition over this wave's slots up to this lane
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t pf = (uint32_t)__shfl_up((int)F, off);
      if (lane >= off) F = compose(F, pf);
    }
    if (lane == 63) sh.scan[wave] = (int32_t)F;
    __syncthreads(); // the waves' maps; also: every read of the slot states is done
    uint32_t G = 2u;  // identity: the composition over the earlier waves
    for (int w = 0; w < wave; ++w) G = compose((uint32_t)sh.scan[w], G);
    const bool on_m = (compose(F, G) & 1u) != 0; // this slot's choice (from C at the image start)
    bool pred_m = (uint32_t)__shfl_up((int)on_m, 1) != 0;
    if (lane == 0) pred_m = (G & 1u) != 0;
    bool need = false;
    if (live && g.j > 0 && !on_m)
      need = pred_m ? (pm_rel != ec_p || pm_bk != ec_bk) : (pc_rel != ec_p || pc_bk != ec_bk);
    const uint64_t bal = __ballot(need);
    const uint64_t hbal = __ballot(on_m);
    // the work list: each wave reserves its needy slots' places with one LDS
    // atomic (any order serves: lane i re-decodes the list's i-th slot)
    int wbase = 0;
    if (lane == 0) {
      if (bal) wbase = atomicAdd(&sh.nwork, (int)__popcll(bal));
      if (hbal) atomicAdd(&sh.memo_hits, (int)__popcll(hbal));
    }
    wbase = __shfl(wbase, 0);
    if (need) {
      sh.work[wbase + __popcll(bal & ((1ull << lane) - 1))] = (uint16_t)tid;
      // the slot's trajectory becomes its memo now, and its entry the
      // predecessor's exit, so that the lane re-decoding it reads only this
      // slot's state (no barrier between the re-decodes and the updates)
      sh.m_en_p[tid] = (uint16_t)ec_p;
      sh.m_en_bk[tid] = (uint16_t)ec_bk;
      sh.m_ex_p[tid] = (uint16_t)(sh.ex_p[tid] - g.j * S);
      sh.m_ex_bk[tid] = sh.ex_bk[tid];
      sh.m_nblk[tid] = sh.nblk[tid];
      sh.en_p[tid] = (uint16_t)(pred_m ? pm_rel : pc_rel);
      sh.en_bk[tid] = (uint16_t)(pred_m ? pm_bk : pc_bk);
    }
    if (on_m) {
      const uint16_t ep = sh.en_p[tid], ebk = sh.en_bk[tid], nb = sh.nblk[tid], xbk = sh.ex_bk[tid];
      const int xp = sh.ex_p[tid];
      sh.en_p[tid] = sh.m_en_p[tid];
      sh.en_bk[tid] = sh.m_en_bk[tid];
      sh.ex_p[tid] = (int)sh.m_ex_p[tid] + g.j * S;
      sh.ex_bk[tid] = sh.m_ex_bk[tid];
      sh.nblk[tid] = sh.m_nblk[tid];
      sh.m_en_p[tid] = ep;
      sh.m_en_bk[tid] = ebk;
      sh.m_ex_p[tid] = (uint16_t)(xp - g.j * S);
      sh.m_ex_bk[tid] = xbk;
      sh.m_nblk[tid] = nb;
      sh.cp_n[tid] = 0; // the adopted trajectory's checkpoints are not kept
    }
    __syncthreads(); // adoptions, the work list and the needy slots' entries published
    const int tot = sh.nwork;
    if (tid == 0) {
      sh.need_lanes += tot;
      sh.need_waves += (tot + 63) >> 6;
    }
    if (tot == 0) break;
    if (tid < tot) {
      // re-decode slot q from its new entry; it merges at the first
      // checkpoint where it meets its previous trajectory (now its memo)
      const int q = sh.work[tid];
      const SlotGeom h = slot_geom(sh, nseg, S, q);
      const int qj = h.j * S;
      const int ep = (int)sh.en_p[q] + qj, ebk = sh.en_bk[q];
      const Cp prev = get_cp(sh, q, h.rstart);
      const int prev_total = sh.m_nblk[q];
      St st = make_state(ebk);
      Rd<W> R;
      R.src = src;
      R.seek(h.pbias + ep);
      int np, nbk, nb = 0;
      Cp cp;
      cp.n = 0;
      if (count_run<true>(R, h.rstart, h.stop, S, st, dec, nb, cp, prev, prev_total)) {
        np = sh.ex_p[q];
        nbk = sh.ex_bk[q];
      } else {
        np = R.p - h.pbias;
        nbk = st.bk();
      }
      sh.nblk[q] = (uint16_t)nb;
      put_cp(sh, q, cp, h.rstart);
      if (np != sh.ex_p[q] || nbk != sh.ex_bk[q]) {
        sh.ex_p[q] = np;
        sh.ex_bk[q] = (uint16_t)nbk;
        sh.any_changed[round & 1] = 1;
      }
    }
    __syncthreads(); // the round's new states published
    if (!sh.any_changed[round & 1]) break;
  }
  const uint64_t t_rounds = dbg ? wall_clock64() : 0;
  if (dbg && tid == 0) {
    atomicAdd(dbg + 1, 1);
    atomicAdd(dbg + 2, rounds);
    atomicMax(dbg + 3, rounds);
  }

  // ---- prefix of the block counts; the true entry is the predecessor's exit ----
  int wp = 0, wbk = 0;
  if (live && g.j > 0) {
    wp = sh.ex_p[tid - 1];
    wbk = sh.ex_bk[tid - 1];
  }
  const Segment &sg = segs[d.seg_base + g.si];
  // the write pass ends where the next range starts: this lane's exit (a
  // count step may run past the range end); a segment's last range at its end
  const int sub_count = sh.seg_first[g.si + 1] - sh.seg_first[g.si];
  const int32_t wstop = g.j == sub_count - 1 ? g.stop : g.pbias + sh.ex_p[tid];
  int tot;
  const int pre = block_excl_scan1024(live ? (int)sh.nblk[tid] : 0, sh.scan, &tot);
  sh.ex_p[tid] = pre;
  __syncthreads();
  const uint64_t t_scan = dbg ? wall_clock64() : 0;
  // the count-mode halves are dead: compact the tables, zero the group planes
  LDS_AS uint8_t *planes;
  const DecW decw = compact_tables(dec, (LDS_AS uint8_t *)dec.tabs, tid, planes);

  // ---- write pass from the true entry ----
  // block records into LDS (the slot state is dead from here) when they fit
  const int64_t nblk_img = (int64_t)d.mcux * d.mcuy * d.bpm;
  const bool rec_lds = nblk_img <= kRecCap;
  bool trunc = false;
  int witers = 0;
  if (live) {
    // blocks of the segment started before this range: the first block whose
    // DC this range decodes is the segment's block `bstart`
    const int bstart = pre - sh.ex_p[sh.seg_first[g.si]];
    const int total = sg.mcu_count * d.bpm;
    const int base = sg.mcu_first * d.bpm + bstart; // image-relative
    int cursor = -1;
    St st = make_state(wbk);
    Rd<W> R;
    R.src = src;
    R.seek(g.pbias + wp);
    uint4 *cimg = reinterpret_cast<uint4 *>(coef + d.coef_off * 64);
    LDS_AS GroupT *gp = group_at(planes, tid); // the lane's open group
    const RecLds rl{(LDS_AS uint32_t *)sh.rec, (LDS_AS uint32_t *)sh.carry};
    const RecGlob rg{brec + d.coef_off, bcarry + d.coef_off / 64};
    if (rec_lds)
      witers = write_run_lds(R, st, decw, wstop, cursor, total - bstart, cimg, rl, base, gp);
    else
      witers = write_run_lds(R, st, decw, wstop, cursor, total - bstart, cimg, rg, base, gp);
    if (g.j == sub_count - 1 && bstart + cursor + 1 < total) {
      status[img] = 3; // ran out of data
      trunc = true;
    }
  }
  // the image's records are complete. The barrier's workgroup-scope fence
  // publishes them to the other waves (one CU, one vector L1 and the LDS); an
  // agent-scope fence would write back and invalidate the XCD's whole L2.
  trunc = __syncthreads_or(trunc);
  if (dbg) {
    // diagnostics (LDT_OPT_DEBUG_COUNTERS): phase times in 10 ns ticks and
    // write-pass symbols (summed over the lanes, and the waves' slowest
    // lanes), summed over images; per wave into LDS, one global atomic per
    // counter and workgroup (same-address atomics of every wave cost the
    // kernel ~20% when they were global)
    const uint64_t t_end = wall_clock64();
    int wsum = witers, wmax = witers;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      wsum += __shfl_xor(wsum, o);
      wmax = max(wmax, __shfl_xor(wmax, o));
    }
    if ((tid & 63) == 0) {
      atomicAdd(&sh.w_syms, wsum);
      atomicAdd(&sh.w_wmax, wmax);
    }
    __syncthreads();
    if (tid == 0) {
      atomicAdd(dbg + 5, sh.w_syms);
      atomicAdd(dbg + 6, sh.w_wmax);
      atomicAdd(dbg + 9, (int)(t_ph1 - t_setup));
      atomicAdd(dbg + 10, (int)(t_rounds - t_ph1));
      atomicAdd(dbg + 11, (int)(t_scan - t_rounds));
      atomicAdd(dbg + 12, (int)(t_end - t_scan));
      atomicAdd(dbg + 13, sh.need_lanes);
      atomicAdd(dbg + 14, sh.need_waves);
      atomicAdd(dbg + 4, sh.memo_hits);
    }
  }
  if (trunc) return; // a failed image's records are never read
  // ---- DC predictors (the serial path runs k_dc_scan instead), in the
  // records; then the LDS records and carries leave in coalesced stores ----
  // (sh's first 256 bytes, ex_p, are the scan scratch)
  if (rec_lds) {
    dc_scan_image<kHuffThreads>(d, (LDS_AS uint32_t *)sh.rec, (LDS_AS int32_t *)&sh);
    __syncthreads();
    uint32_t *gr = brec + d.coef_off;
    for (int ib = tid; ib < (int)nblk_img; ib += kHuffThreads) gr[ib] = sh.rec[ib];
    uint32_t *gc = bcarry + d.coef_off / 64;
    for (int c = tid; c < (int)((nblk_img + 63) >> 6); c += kHuffThreads) gc[c] = sh.carry[c];
  } else {
    dc_scan_image<kHuffThreads>(d, brec + d.coef_off, (LDS_AS int32_t *)&sh);
  }
}

// ---------------------------------------------------------------------------
// Fused destuff (images the planner gave no destuff chunks: ds_count == 0,
// their destuffed stream fits the LDS window). The workgroup classifies the
// cell's scan bytes itself, 16 per lane per 16 KB tile and the tiles in order,
// with the rules of k_destuff_count/_write/_layout (ldt_kernels.hip;
// ds_classify16), and compacts the kept bytes, the kSegPad zero pads and the
// segment starts straight into the window (byte-swapped words, as the copy of
// a destuffed stream leaves them), then lays out the segments' subsequences
// in sh. No destuffed bytes go through memory. Returns false (workgroup-
// uniform) for a corrupt image, with status 3 as k_destuff_layout sets it.
// ---------------------------------------------------------------------------
constexpr int kFuseTile = 16 * kHuffThreads;
__device__ __forceinline__ bool destuff_into_window(const uint8_t *__restrict__ data, const ImgDesc &d,
                                                    LDS_AS uint8_t *win, ImgLds &sh, int tid,
                                                    int32_t *__restrict__ status, int img) {
  // B0: the scan start rounded down to a word (pointer arithmetic on `data`
  // only, so the loads stay global loads rather than flat ones, which an LDS
  // wait would also wait for)
  const int lead = (int)((uintptr_t)(data + d.src_off) & 3);
  const uint32_t *W = reinterpret_cast<const uint32_t *>(data + (d.src_off - lead));
  const int64_t L = d.src_len;
  const int64_t span = L + lead;         // bytes from B0 to the end of the cell
  const int64_t nwords = (span + 3) / 4; // words from B0 that touch the cell
  const int last = d.nseg - 1;
  // lane words of the tile at cb: the 16 bytes at B0 + cb + 16 tid and one
  // word on either side, zero outside the words touching the cell (ds_stage).
  // The loads are unconditional (clamped indices): a conditional load would
  // make the next tile's prefetch be waited for at once.
  auto load = [&](int64_t cb, uint32_t wv[6]) {
    const int64_t w0 = cb / 4 + 4 * tid - 1;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int64_t wi = w0 + i;
      const uint32_t v = W[min(max(wi, (int64_t)0), nwords - 1)];
      wv[i] = (wi >= 0 && wi < nwords) ? v : 0u;
    }
  };
  auto put = [&](int o, uint32_t v) { win[o ^ 3] = (uint8_t)v; };
  int K = 0, R = 0; // kept bytes and RSTn markers of the earlier tiles
  // One tile: classify the lane's 16 bytes, find the tile's first end-of-scan
  // marker, compact the kept bytes into the window. Returns true at the end
  // of the scan (workgroup-uniform).
  auto tile = [&](int64_t cb, const uint32_t wv[6]) __attribute__((always_inline)) -> bool {
    const int64_t p0 = cb + 16 * tid - lead;
    uint32_t keep, rst;
    int le;
    ds_classify16_ff(wv, p0, L, keep, rst, le);
    // a lane's 16 bytes precede the next lane's, so a wave's first marker is
    // its lowest lane's with one, and the tile's is the lowest wave's
    const uint64_t em = __ballot(le < 16);
    if (em != 0ull) {
      const int first = __shfl((int)(p0 + le), __ffsll((unsigned long long)em) - 1);
      if ((tid & 63) == 0) sh.ds_endw[tid >> 6] = first;
    } else if ((tid & 63) == 0) {
      sh.ds_endw[tid >> 6] = 0x7FFFFFFF;
    }
    __syncthreads();
    // the first end-of-scan marker ends the stream (it lies in this tile:
    // an earlier one would have ended the loop)
    int E = 0x7FFFFFFF;
#pragma unroll
    for (int q = 0; q < kHuffThreads / 64; ++q) E = min(E, sh.ds_endw[q]);
    const bool ended = E != 0x7FFFFFFF;
    if (ended) {
      const int64_t c = (int64_t)E - p0;
      const uint32_t lim = c <= 0 ? 0u : (c >= 16 ? 0xFFFFu : ((1u << c) - 1u));
      keep &= lim;
      rst &= lim;
    }
    int tot;
    const int ex = block_excl_scan1024(__popc(keep) | (__popc(rst) << 16), sh.scan, &tot);
    // kept byte o of segment r lands at o + kSegPad * min(r, last)
    int r = R + (ex >> 16);
    int o = K + (ex & 0xFFFF) + kSegPad * min(r, last);
    if (rst == 0u) {
      // kept byte j goes to o + (kept bytes before it)
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if ((keep >> j) & 1u) put(o + __popc(keep & ((1u << j) - 1u)), wv[(j + 4) >> 2] >> (8 * ((j + 4) & 3)));
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if ((rst >> j) & 1u) {
          if (r < last) {
#pragma unroll
            for (int q = 0; q < kSegPad; ++q) put(o + q, 0u);
            o += kSegPad;
          }
          ++r;
          if (r < d.nseg) sh.seg_pb[r] = o * 8;
        }
        if ((keep >> j) & 1u) put(o++, wv[(j + 4) >> 2] >> (8 * ((j + 4) & 3)));
      }
    }
    K += tot & 0xFFFF;
    R += tot >> 16;
    return ended;
  };
  // one tile's loads in flight while the one before it is compacted (issuing
  // two or three tiles at a time saved 3 of the ~25 us of a c2 image's setup
  // but raised the kernel to 110-128 VGPRs, and the pipeline lost more than
  // that: profiles/r4/huffvar_r4hv.txt)
  uint32_t wv[6], nx[6];
  load(0, wv);
  for (int64_t cb = 0; cb < span; cb += kFuseTile) {
    load(cb + kFuseTile, nx); // the next tile (clamped past the end)
    if (tile(cb, wv)) break;
#pragma unroll
    for (int i = 0; i < 6; ++i) wv[i] = nx[i];
  }
  if (R != last) { // restart markers do not match the header
    if (tid == 0) status[img] = 3;
    return false;
  }
  // zero pad after the last segment; segment bit ranges and subsequences
  const int tail = K + kSegPad * last;
  // zero pad after the last segment, then zeros over the rest of the window
  // the decoders may read ahead into (up to 16 KB past it, capped at the
  // window): nothing of an earlier workgroup's LDS is read, as with the
  // k_destuff_* kernels' padded stream
  if (tid < kSegPad + 16) put(tail + tid, 0u);
  {
    const int z = ((tail + kSegPad + 16) & ~15) + 16 * tid;
    if (z + 16 <= (int)(destuff_region_bytes(L, d.nseg) + 16)) *(LDS_AS v4u *)(win + z) = (v4u)(0u);
  }
  if (tid == 0) sh.seg_pb[0] = 0;
  __syncthreads(); // segment starts published
  const int S = d.sub_bits;
  int cnt_s = 0, pb = 0, nb = 0;
  if (tid < d.nseg) {
    pb = sh.seg_pb[tid];
    const int end = tid + 1 < d.nseg ? sh.seg_pb[tid + 1] - 8 * kSegPad : 8 * tail;
    nb = end - pb;
    cnt_s = max(1, (nb + S - 1) / S);
  }
  int nsub;
  const int first = block_excl_scan1024(cnt_s, sh.scan, &nsub);
  if (tid < d.nseg) {
    sh.seg_first[tid] = first;
    sh.seg_nb[tid] = nb;
  }
  if (tid == 0) sh.seg_first[d.nseg] = nsub;
  if (nsub > kHuffThreads) {
    if (tid == 0) status[img] = 3;
    return false;
  }
  return true;
}

// The image's distinct tables into LDS by LDS-DMA (global_load_lds_dwordx4:
// each wave instruction moves 64 x 16 B to one contiguous KB of LDS and holds
// no VGPRs while in flight): the lc part of a slot is 8 such chunks, the l2
// parts of two slots one chunk (their LDS areas are adjacent). The caller
// waits (vmcnt 0) before the barrier that publishes them.
__device__ __forceinline__ void stage_tables_dma(const HuffTab *__restrict__ htabs, const SlotTabs &st, int ns,
                                                 LDS_AS uint8_t *tabs, int wave, int lane) {
  const int nlc = ns * (kLcBytes / 1024);
  const int nch = nlc + (ns + 1) / 2;
  for (int c = wave; c < nch; c += kHuffThreads / 64) {
    if (c < nlc) {
      const int sl = c / (kLcBytes / 1024), k = c % (kLcBytes / 1024);
      const uint8_t *src = reinterpret_cast<const uint8_t *>(htabs + st.get(sl)) + k * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds(src, (LDS_AS void *)(tabs + (sl << 13) + k * 1024), 16, 0, 0);
    } else {
      static_assert(kL2Bytes == 512, "two slots' l2 parts per KB chunk");
      const int sl = 2 * (c - nlc) + (lane >> 5);
      if (sl < ns) {
        const uint8_t *src = reinterpret_cast<const uint8_t *>(htabs + st.get(sl)) + kLcBytes + (lane & 31) * 16;
        __builtin_amdgcn_global_load_lds(src, (LDS_AS void *)(tabs + (ns << 13) + 2 * (c - nlc) * kL2Bytes), 16, 0,
                                         0);
      }
    }
  }
}

// At most 80 VGPRs (6 waves per SIMD's worth): the decoder's 16 waves then
// hold 4 x 80 of a SIMD's 512 registers, and two waves of k_idct (82) from
// the other batches in flight fit beside them instead of one. k_idct uses no
// LDS, so it shares the CU without slowing the decoder's LDS-bound rounds
// (the resize does not: DESIGN.md §4), and the pipeline gains 4-5%
// (profiles/r5/huff_vgpr_ab_r5h80.txt). The cap costs only SGPR spills to
// VGPR lanes; at 72 VGPRs scratch spills begin, and a third k_idct wave per
// SIMD bought with them (decoder 72 or 64 VGPRs) measured slower
// (profiles/r5/huff_tabdma_ab_r5dma.txt).
__global__ void __launch_bounds__(kHuffThreads) __attribute__((amdgpu_waves_per_eu(6, 8))) k_huff_image(
    const ImgDesc *__restrict__ descs, const Segment *__restrict__ segs,
    const HuffTab *__restrict__ htabs, const uint8_t *__restrict__ data,
    const uint8_t *__restrict__ dstuf, const int32_t *__restrict__ par_img, int win_bytes, int warm_pct,
    int16_t *__restrict__ coef, uint32_t *__restrict__ brec, uint32_t *__restrict__ bcarry,
    int32_t *__restrict__ status, int32_t *__restrict__ dbg) {
  __shared__ ImgLds sh;
  const int img = par_img[blockIdx.x];
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  const uint64_t t_start = dbg ? wall_clock64() : 0;
  // dynamic LDS: [window win_bytes][tables]
  LDS_AS uint8_t *tabs = (LDS_AS uint8_t *)(dyn_lds + win_bytes / 4);
  SlotTabs slot_tab;
  const Dec dec = load_dec(d, htabs, tabs, tid, kHuffThreads, false, &slot_tab);
  const bool fused = d.ds_count == 0;
  for (int s = tid; s < d.nseg && !fused; s += kHuffThreads) {
    const Segment &sg = segs[d.seg_base + s];
    sh.seg_first[s] = sg.sub_first;
    sh.seg_pb[s] = (int32_t)(sg.byte_start - d.dst_off) * 8; // window word 0 = dst_off
    sh.seg_nb[s] = (int32_t)((sg.byte_end - sg.byte_start) * 8);
  }
  if (tid == 0) {
    if (!fused) {
      const Segment &l = segs[d.seg_base + d.nseg - 1];
      sh.seg_first[d.nseg] = l.sub_first + l.sub_count;
    }
    sh.need_lanes = 0;
    sh.nwork = 0;
    sh.need_waves = 0;
    sh.memo_hits = 0;
    sh.w_syms = 0;
    sh.w_wmax = 0;
  }
  const int64_t need = destuff_region_bytes(d.src_len, d.nseg) + 16;
  const bool in_lds = need <= win_bytes;
  const uint8_t *base = dstuf + d.dst_off; // 16-aligned
  if (fused) {
    // the planner fuses only images whose stream fits the window
    if (!in_lds) {
      if (tid == 0) status[img] = 3;
      return;
    }
    // the tables stream into LDS while the stream's tiles are destuffed
    stage_tables_dma(htabs, slot_tab, dec.ns, tabs, tid >> 6, tid & 63);
    if (!destuff_into_window(data, d, (LDS_AS uint8_t *)dyn_lds, sh, tid, status, img)) return;
  } else {
    // Tables (LDS-DMA) and, when it fits, the whole destuffed stream,
    // byte-swapped, into LDS, a lane's 16-byte pieces kWinPer at a time in
    // flight. Every load is unconditional (clamped indices) so that no branch
    // merge makes the compiler wait for the loads before it. (Only images the
    // fused destuff does not take come here; the four pieces in flight keep
    // this path's registers below the kernel's cap.)
    constexpr int kWinPer = 4;
    stage_tables_dma(htabs, slot_tab, dec.ns, tabs, tid >> 6, tid & 63);
    const v4u *gsrc = reinterpret_cast<const v4u *>(base);
    LDS_AS v4u *wl = (LDS_AS v4u *)dyn_lds;
    const int nwin = in_lds ? (int)(need / 16) : 0;
    for (int r0 = 0; r0 == 0 || r0 < nwin; r0 += kWinPer * kHuffThreads) {
      v4u v[kWinPer];
#pragma unroll
      for (int k = 0; k < kWinPer; ++k) v[k] = gsrc[max(min(r0 + k * kHuffThreads + tid, nwin - 1), 0)];
#pragma unroll
      for (int k = 0; k < kWinPer; ++k) {
        const int i = r0 + k * kHuffThreads + tid;
        if (i < nwin) {
          v4u o;
          o.x = __builtin_bswap32(v[k].x);
          o.y = __builtin_bswap32(v[k].y);
          o.z = __builtin_bswap32(v[k].z);
          o.w = __builtin_bswap32(v[k].w);
          wl[i] = o;
        }
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0); // this wave's table DMAs have landed
  __syncthreads();
  const uint64_t t_setup = dbg ? wall_clock64() : 0;
  if (dbg && tid == 0) atomicAdd(dbg + 8, (int)(t_setup - t_start));
  const int warm = (d.sub_bits * warm_pct) / 100;
  if (in_lds)
    image_decode(LdsWords{(lds_cu32)dyn_lds}, d, segs, dec, warm, t_setup, sh, coef, brec, bcarry,
                 status, img, dbg);
  else
    image_decode(GlobWords{reinterpret_cast<const uint32_t *>(base)}, d, segs, dec, warm, t_setup,
                 sh, coef, brec, bcarry, status, img, dbg);
}

hipError_t launch_huff_parallel(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n_par == 0) return hipSuccess;
  static hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_huff_image),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               kHuffLdsMax - kHuffStaticLds);
  if (attr != hipSuccess) return attr;
  const size_t lds = (size_t)p.win_bytes + huff_tab_lds_image(p.max_tabs);
  hipLaunchKernelGGL(k_huff_image, dim3(p.n_par), dim3(kHuffThreads), lds, s, p.descs, p.segs,
                     p.htabs, w.data, w.dstuf, p.par_img, p.win_bytes, p.warm_pct, w.coef, w.brec, w.bcarry,
                     w.status, p.redo);
  return hipGetLastError();
}

} // namespace ldt

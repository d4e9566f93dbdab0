// ldt_huffman.hip — baseline JPEG Huffman decode on gfx950.
//
// Restates libjpeg-turbo jdhuff.c decode_mcu (sequential, Huffman, 8-bit):
//   DC: s = HUFF_DECODE(dc_tbl); diff = HUFF_EXTEND(GET_BITS(s), s); pred += diff
//   AC: for k = 1..63: rs = HUFF_DECODE(ac_tbl); r = rs >> 4; s = rs & 15;
//         s != 0: k += r; coef[natural[k]] = HUFF_EXTEND(GET_BITS(s), s)
//         s == 0: r == 15 ? k += 15 (ZRL) : break (EOB)
// Bits past a segment's end read as zero (jdhuff.c inserts zeros at a marker).
// Input: destuffed segments (k_destuff). Output: int16 coefficients, natural
// order, block (mcu, b) at coef_off + mcu * bpm + b (raw, dequantised in k_idct).
//
// Two decoders share the symbol step (sym_step):
//   k_huff_serial    one lane per segment (restart interval or whole scan);
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
typedef LDS_AS uint16_t *lds_u16;

__constant__ uint8_t c_natural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// ---------------------------------------------------------------------------
// Bit input: MSB-first over the destuffed bytes of ONE segment, positions are
// segment-relative 32-bit. Words come from the workgroup's LDS window when
// inside it, else from global memory; bytes at/after the segment end read 0.
// ---------------------------------------------------------------------------
struct Bits {
  const uint8_t *g;     // destuffed buffer (global)
  lds_cu32 win;         // LDS window (wbytes == 0: none)
  int64_t wbase;        // absolute byte address of win[0] (4-aligned)
  int32_t wbytes;
  int64_t seg0;         // absolute byte address of the segment start
  int32_t endrel;       // segment length in bytes
  uint64_t buf;         // MSB-aligned
  int32_t n;            // valid bits in buf
  int32_t wrel;         // next word to load, bytes relative to seg0 (seg0 + wrel 4-aligned)

  __device__ __forceinline__ uint32_t word(int32_t rel) const {
    if (rel >= endrel) return 0u;
    const int64_t a = seg0 + rel;
    const int64_t o = a - wbase;
    uint32_t w = (o >= 0 && o + 4 <= wbytes) ? win[o >> 2] : *reinterpret_cast<const uint32_t *>(g + a);
    w = __builtin_bswap32(w);
    const int32_t valid = endrel - rel;
    if (valid < 4) w &= ~(0xFFFFFFFFu >> (8 * valid));
    return w;
  }
  // Position the reader at segment-relative bit `p`.
  __device__ __forceinline__ void seek(int32_t p) {
    const int64_t abit = seg0 * 8 + p;
    const int64_t a = (abit >> 3) & ~(int64_t)3;
    const int32_t rel = (int32_t)(a - seg0);
    const int skip = (int)(abit - a * 8);
    buf = (((uint64_t)word(rel) << 32) | (uint64_t)word(rel + 4)) << skip;
    n = 64 - skip;
    wrel = rel + 8;
  }
  __device__ __forceinline__ void refill() {
    if (n <= 32) {
      buf |= (uint64_t)word(wrel) << (32 - n);
      n += 32;
      wrel += 4;
    }
  }
  __device__ __forceinline__ int32_t pos() const { return wrel * 8 - n; }
};

// Table addressing for a context ctx = 2 * component + (AC ? 1 : 0).
//   LdsTabs: the image's distinct tables copied into LDS (slot per context).
//   GlobTabs: the plan's tables in global memory.
// canon() is the global table for the rare canonical-search fallback.
struct LdsTabs {
  lds_cu16 base;
  uint32_t slotmap; // 3 bits per context
  const HuffTab *g;
  const ImgDesc *d;
  __device__ __forceinline__ lds_cu16 t(int ctx) const {
    return base + ((slotmap >> (3 * ctx)) & 7) * kTabU16;
  }
  __device__ __forceinline__ const HuffTab *canon(int ctx) const {
    const int c = ctx >> 1, cc = c < d->ncomp ? c : 0;
    return g + ((ctx & 1) ? d->act[cc] : d->dct[cc]);
  }
};
struct GlobTabs {
  const HuffTab *g;
  const ImgDesc *d;
  __device__ __forceinline__ const HuffTab *canon(int ctx) const {
    const int c = ctx >> 1, cc = c < d->ncomp ? c : 0;
    return g + ((ctx & 1) ? d->act[cc] : d->dct[cc]);
  }
  __device__ __forceinline__ const uint16_t *t(int ctx) const { return canon(ctx)->l1; }
};

// jdhuff.c jpeg_huff_decode, two-level lookup (l1 and l2 are contiguous).
template <class T>
__device__ __forceinline__ uint32_t huff_lookup(const T &tabs, int ctx, uint32_t w16) {
  const auto t = tabs.t(ctx);
  uint32_t e = t[w16 >> 7];
  if (e & 0x8000) {
    if (e != 0xFFFF) {
      e = t[512 + ((e & 0x7F) << 7) + (w16 & 127)];
    } else {
      const HuffTab *cn = tabs.canon(ctx);
      e = 0;
#pragma unroll
      for (int l = 16; l > kLookBits; --l)
        if ((int)(w16 >> (16 - l)) <= cn->maxcode[l])
          e = ((uint32_t)l << 8) | cn->vals[(cn->valoff[l] + (int)(w16 >> (16 - l))) & 0xFF];
    }
  }
  return e == 0 ? (16u << 8) : e; // invalid code: skip 16 bits, symbol 0
}

struct RunAcc {
  int nblk;
  int dc0, dc1, dc2;
};
__device__ __forceinline__ RunAcc acc_add(RunAcc a, RunAcc b) {
  return RunAcc{a.nblk + b.nblk, a.dc0 + b.dc0, a.dc1 + b.dc1, a.dc2 + b.dc2};
}
__device__ __forceinline__ RunAcc acc_sub(RunAcc a, RunAcc b) {
  return RunAcc{a.nblk - b.nblk, a.dc0 - b.dc0, a.dc1 - b.dc1, a.dc2 - b.dc2};
}

// Per-image constants: component of block b, 2 bits each; blocks per MCU.
struct DecConst {
  uint32_t compmap;
  int bpm;
};
__device__ __forceinline__ DecConst dec_const(const ImgDesc &d) {
  DecConst dc;
  dc.compmap = 0;
  for (int b = 0; b < d.bpm; ++b) dc.compmap |= (uint32_t)(d.bcomp[b] & 3) << (2 * b);
  dc.bpm = d.bpm;
  return dc;
}

// One symbol (DC if k == 0, else AC) and its extra bits; updates (b, k).
// Returns the coefficient value; zz = zig-zag index written (0 = DC, -1 none),
// cc = component.
template <class T>
__device__ __forceinline__ int sym_step(Bits &B, int &b, int &k, const DecConst &dcn, const T &tabs,
                                        RunAcc &acc, int &zz, int &cc) {
  B.refill();
  const int c = (int)((dcn.compmap >> (2 * b)) & 3);
  const int ac = k != 0 ? 1 : 0;
  const uint32_t w16 = (uint32_t)(B.buf >> 48);
  const uint32_t e = huff_lookup(tabs, 2 * c + ac, w16);
  const int len = (int)(e >> 8), sym = (int)(e & 0xFF);
  const int s = ac ? (sym & 15) : sym;
  const int r = ac ? (sym >> 4) : 0;
  const uint64_t t = B.buf << len;
  const uint32_t raw = s ? (uint32_t)(t >> (64 - s)) : 0u;
  B.buf = t << s;
  B.n -= len + s;
  const int v = (s != 0 && (int)raw < (1 << (s - 1))) ? (int)raw - (1 << s) + 1 : (int)raw;
  cc = c;
  if (!ac) {
    acc.nblk += 1;
    acc.dc0 += c == 0 ? v : 0;
    acc.dc1 += c == 1 ? v : 0;
    acc.dc2 += c == 2 ? v : 0;
    zz = 0;
    k = 1;
  } else {
    if (s) {
      k += r;
      zz = k;
      ++k;
    } else {
      zz = -1;
      k = (r == 15) ? k + 16 : 64;
    }
    if (k >= 64) {
      k = 0;
      b = (b + 1 == dcn.bpm) ? 0 : b + 1;
    }
  }
  return v;
}

// Distinct Huffman tables of an image's six contexts, first come first slot.
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

// ---------------------------------------------------------------------------
// Serial decoder: one lane per segment, tables read from global memory.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_huff_serial(const ImgDesc *__restrict__ descs,
                                                    const Segment *__restrict__ segs, int nseg,
                                                    const HuffTab *__restrict__ htabs,
                                                    const uint8_t *__restrict__ dstuf,
                                                    int16_t *__restrict__ coef,
                                                    int32_t *__restrict__ status) {
  const int si = blockIdx.x * blockDim.x + threadIdx.x;
  if (si >= nseg) return;
  const Segment sg = segs[si];
  const ImgDesc &d = descs[sg.img];
  if (status[sg.img] != 0) return;
  const GlobTabs tabs{htabs, &d};
  const DecConst dcn = dec_const(d);
  Bits B;
  B.g = dstuf;
  B.win = (lds_cu32)0;
  B.wbase = 0;
  B.wbytes = 0;
  B.seg0 = sg.byte_start;
  B.endrel = (int32_t)(sg.byte_end - sg.byte_start);
  B.seek(0);
  int pred0 = 0, pred1 = 0, pred2 = 0;
  int b = 0, k = 0;
  const int64_t total = (int64_t)sg.mcu_count * d.bpm;
  int64_t cursor = -1;
  int16_t *coef_seg = coef + (d.coef_off + (int64_t)sg.mcu_first * d.bpm) * 64;
  RunAcc acc{0, 0, 0, 0};
  while (true) {
    if (k == 0) {
      if (cursor + 1 >= total) break;
      ++cursor;
    }
    int zz, cc;
    const int v = sym_step(B, b, k, dcn, tabs, acc, zz, cc);
    if (zz == 0) {
      const int pv = (cc == 0 ? pred0 : cc == 1 ? pred1 : pred2) + v;
      pred0 = cc == 0 ? pv : pred0;
      pred1 = cc == 1 ? pv : pred1;
      pred2 = cc == 2 ? pv : pred2;
      coef_seg[cursor * 64] = (int16_t)pv;
    } else if (zz > 0) {
      coef_seg[cursor * 64 + c_natural[zz]] = (int16_t)v;
    }
  }
  if (B.pos() > B.endrel * 8) status[sg.img] = 3; // ran past the data: truncated
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
// Workgroup w = 256 lanes: lanes 1..255 own slots (w - wg_first)*255 + lane-1;
// lane 0 is a helper that decodes the subsequence just before lane 1's from a
// guessed state, giving lane 1 a (usually correct) entry state. Inside the
// workgroup, lanes re-decode from their predecessor's exit until no exit
// changes; each lane keeps two checkpoint states of its last trajectory so a
// re-decode stops as soon as it merges with it. Across workgroups, k_huff_fix
// compares the helper's candidate with the previous workgroup's last exit and
// walks (one wave, LDS tables) only on a mismatch.
// ===========================================================================

constexpr int kWinBytes = 34 * 1024;

// Copy an image's distinct tables (l1 + l2 = kTabU16 entries each) into LDS.
__device__ __forceinline__ void load_tabs(const HuffTab *__restrict__ htabs, const int *slot_tab,
                                          int ns, lds_u16 tabs, int tid, int nthreads) {
  constexpr int kWords = kTabU16 / 2;
  for (int i = tid; i < ns * kWords; i += nthreads) {
    const int q = i / kWords, o = i - q * kWords;
    ((LDS_AS uint32_t *)(tabs + q * kTabU16))[o] = reinterpret_cast<const uint32_t *>(htabs + slot_tab[q])[o];
  }
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
  return (int64_t)(d.wg_first + lt / kSlotsPerWg) * kSyncThreads + 1 + lt % kSlotsPerWg;
}

struct SubCtx {
  int seg;      // segment index (global), -1 if inactive
  int j;        // subsequence index within the segment (helper: lane 1's j - 1)
  int32_t seg_bits;
  int64_t seg0, seg_end;
  bool active;  // real slot
  bool helper;  // lane 0 with something to warm up on
};

struct WgShared {
  uint32_t win[kWinBytes / 4];
  unsigned long long lo, hi;
};

// Huffman tables: dynamic LDS, (max distinct tables of the batch) x kTabU16.
extern __shared__ __attribute__((aligned(16))) uint16_t dyn_tabs[];
#define TABS_LDS ((lds_u16)(dyn_tabs))

// Workgroup setup shared by the sync and write kernels: distinct tables and
// the workgroup's LDS window of destuffed bytes.
__device__ __forceinline__ void sub_setup(const ImgDesc &d, const Segment *__restrict__ segs,
                                          const HuffTab *__restrict__ htabs, int S, WgShared &sh,
                                          int64_t &wbase, int &wbytes, const uint8_t *dstuf,
                                          SubCtx &sc, const int *slot_tab, int ns) {
  const int tid = threadIdx.x;
  load_tabs(htabs, slot_tab, ns, TABS_LDS, tid, kSyncThreads);
  const int wl = (int)blockIdx.x - d.wg_first;
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  const int total_sub = last.sub_first + last.sub_count;
  const int lt = wl * kSlotsPerWg + (tid == 0 ? 0 : tid - 1);
  sc.active = tid > 0 && lt < total_sub;
  sc.helper = false;
  sc.seg = -1;
  sc.j = 0;
  sc.seg_bits = 0;
  sc.seg0 = sc.seg_end = 0;
  uint64_t lo = ~0ull, hi = 0;
  if (lt < total_sub) {
    const int si = find_segment(segs, d.seg_base, d.nseg, lt);
    const Segment &sg = segs[si];
    int j = lt - sg.sub_first;
    bool use = sc.active;
    if (tid == 0) {
      sc.helper = j > 0;
      use = sc.helper;
      j -= 1;
    }
    if (use) {
      sc.seg = si;
      sc.j = j;
      sc.seg0 = sg.byte_start;
      sc.seg_end = sg.byte_end;
      sc.seg_bits = (int32_t)((sg.byte_end - sg.byte_start) * 8);
      lo = (uint64_t)(sg.byte_start + ((int64_t)j * S) / 8);
      int64_t h = sg.byte_start + ((int64_t)(j + 1) * S) / 8 + 64;
      if (h > sg.byte_end + 8) h = sg.byte_end + 8;
      hi = (uint64_t)h;
    }
  }
  if (tid == 0) {
    sh.lo = ~0ull;
    sh.hi = 0;
  }
  __syncthreads();
  if (hi > 0) {
    atomicMin(&sh.lo, (unsigned long long)lo);
    atomicMax(&sh.hi, (unsigned long long)hi);
  }
  __syncthreads();
  int64_t wb = 0, wl_bytes = 0;
  if (sh.hi > 0) {
    wb = (int64_t)sh.lo & ~(int64_t)3;
    wl_bytes = (((int64_t)sh.hi - wb) + 3) & ~(int64_t)3;
    if (wl_bytes > kWinBytes) wl_bytes = kWinBytes;
  }
  for (int i = tid; i < (int)wl_bytes / 4; i += kSyncThreads)
    sh.win[i] = *reinterpret_cast<const uint32_t *>(dstuf + wb + 4 * (int64_t)i);
  wbase = wb;
  wbytes = (int)wl_bytes;
  __syncthreads();
}

__device__ __forceinline__ void bits_init(Bits &B, const uint8_t *dstuf, lds_cu32 win,
                                          int64_t wbase, int wbytes, int64_t seg0, int64_t seg_end) {
  B.g = dstuf;
  B.win = win;
  B.wbase = wbase;
  B.wbytes = wbytes;
  B.seg0 = seg0;
  B.endrel = (int32_t)(seg_end - seg0);
}

// Checkpoints: the state at the first symbol boundary at/after
// range_start + S/3 and + 2S/3, with the counts accumulated up to it.
struct Cp {
  int p0, bk0, p1, bk1;
  RunAcc a0, a1;
  int n;
};

// COUNT decode from the reader's position to the first boundary >= stop.
// COMPARE: stop at the first checkpoint equal to prev's (merge) and adopt
// prev's tail. Returns true on a merge.
template <bool COMPARE, class T>
__device__ __forceinline__ bool count_run(Bits &B, int32_t range_start, int32_t stop, int S, int &b,
                                          int &k, const DecConst &dcn, const T &tabs, RunAcc &acc,
                                          Cp &cp, const Cp &prev, const RunAcc &prev_total) {
  cp.n = 0;
  int32_t next_cp = range_start + S / 3;
  while (true) {
    const int32_t p = B.pos();
    if (p >= stop) break;
    if (p >= next_cp) {
      const int bk = (b << 8) | k;
      if (cp.n == 0) {
        if (COMPARE && prev.n > 0 && prev.p0 == p && prev.bk0 == bk) {
          const RunAcc delta = acc_sub(acc, prev.a0);
          cp = prev;
          cp.a0 = acc;
          cp.a1 = acc_add(prev.a1, delta);
          acc = acc_add(prev_total, delta);
          return true;
        }
        cp.p0 = p;
        cp.bk0 = bk;
        cp.a0 = acc;
        cp.n = 1;
        next_cp = range_start + (2 * S) / 3;
      } else {
        if (COMPARE && prev.n > 1 && prev.p1 == p && prev.bk1 == bk) {
          const RunAcc delta = acc_sub(acc, prev.a1);
          cp.p1 = p;
          cp.bk1 = bk;
          cp.a1 = acc;
          cp.n = 2;
          acc = acc_add(prev_total, delta);
          return true;
        }
        cp.p1 = p;
        cp.bk1 = bk;
        cp.a1 = acc;
        cp.n = 2;
        next_cp = 0x7FFFFFFF;
      }
    }
    int zz, cc;
    (void)sym_step(B, b, k, dcn, tabs, acc, zz, cc);
  }
  return false;
}

// Phase 1 + intra-workgroup convergence.
__global__ void __launch_bounds__(kSyncThreads) k_huff_sync(
    const ImgDesc *__restrict__ descs, const Segment *__restrict__ segs,
    const HuffTab *__restrict__ htabs, const uint8_t *__restrict__ dstuf,
    const int32_t *__restrict__ wg_img, int S, SubState *__restrict__ sub,
    const int32_t *__restrict__ status, int32_t *__restrict__ dbg) {
  __shared__ __attribute__((aligned(16))) WgShared sh;
  __shared__ int32_t ex_p[kSyncThreads], ex_bk[kSyncThreads];
  __shared__ uint8_t chg[kSyncThreads];
  __shared__ int any_changed;
  const int img = wg_img[blockIdx.x];
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  int slot_tab[6];
  uint32_t slotmap;
  const int ns = image_slots(d, slotmap, slot_tab);
  const DecConst dcn = dec_const(d);
  SubCtx sc;
  int64_t wbase;
  int wbytes;
  sub_setup(d, segs, htabs, S, sh, wbase, wbytes, dstuf, sc, slot_tab, ns);
  const LdsTabs tabs{TABS_LDS, slotmap, htabs, &d};
  RunAcc acc{0, 0, 0, 0};
  Cp cp, none;
  cp.n = 0;
  none.n = 0;
  int b = 0, k = 0;
  Bits B;
  bits_init(B, dstuf, (lds_cu32)sh.win, wbase, wbytes, sc.seg0, sc.seg_end);
  const int32_t rstart = sc.j * S;
  const int32_t stop = min((sc.j + 1) * S, sc.seg_bits);
  // phase 1: every slot (and the helper) decodes its range from a guessed
  // state (b = 0, k = 0 at the range start); j == 0 starts exactly.
  if (sc.active || sc.helper) {
    B.seek(rstart);
    count_run<false>(B, rstart, stop, S, b, k, dcn, tabs, acc, cp, none, acc);
    ex_p[tid] = B.pos();
    ex_bk[tid] = (b << 8) | k;
  } else {
    ex_p[tid] = 0; // helper of a workgroup whose lane 1 starts a segment: exact (0, 0, 0)
    ex_bk[tid] = 0;
  }
  // every slot with an in-workgroup predecessor (lane 1's is the helper) re-decodes
  bool need = sc.active && sc.j > 0;
  int rounds = 0;
  for (int round = 0; round < kSyncThreads + 1; ++round) {
    ++rounds;
    __syncthreads();
    if (tid == 0) any_changed = 0;
    bool changed = false;
    int np = 0, nbk = 0;
    if (need) {
      const int ep = ex_p[tid - 1], ebk = ex_bk[tid - 1];
      b = ebk >> 8;
      k = ebk & 255;
      const RunAcc prev_total = acc;
      const Cp prev = cp;
      acc = RunAcc{0, 0, 0, 0};
      B.seek(ep);
      if (count_run<true>(B, rstart, stop, S, b, k, dcn, tabs, acc, cp, prev, prev_total)) {
        np = ex_p[tid];
        nbk = ex_bk[tid];
      } else {
        np = B.pos();
        nbk = (b << 8) | k;
      }
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
    need = sc.active && sc.j > 0 && chg[tid > 0 ? tid - 1 : 0] && tid > 0;
  }
  if (dbg && tid == 0) {
    atomicAdd(dbg + 1, 1);
    atomicAdd(dbg + 2, rounds);
    atomicMax(dbg + 3, rounds);
  }
  if (sc.active || tid == 0) {
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

// One wave per workgroup boundary that needs it: load the tables into LDS,
// then lane 0 walks slots from lt0 (true entry = the stored exit of slot
// lt0 - 1) until a recomputed exit equals the stored one. bounded = true
// stops at the end of lt0's workgroup and raises *redo (the next boundary
// then compared against a stale exit).
__device__ void boundary_walk_wave(const ImgDesc &d, const Segment *__restrict__ segs,
                                   const HuffTab *__restrict__ htabs,
                                   const uint8_t *__restrict__ dstuf, int S,
                                   SubState *__restrict__ sub, int lt0, bool bounded, int32_t *redo,
                                   int32_t *dbg) {
  const int lane = threadIdx.x & 63;
  int slot_tab[6];
  uint32_t slotmap;
  const int ns = image_slots(d, slotmap, slot_tab);
  load_tabs(htabs, slot_tab, ns, TABS_LDS, lane, 64);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (lane != 0) return;
  const LdsTabs tabs{TABS_LDS, slotmap, htabs, &d};
  const DecConst dcn = dec_const(d);
  const int si = find_segment(segs, d.seg_base, d.nseg, lt0);
  const Segment &sg = segs[si];
  int j = lt0 - sg.sub_first;
  if (j == 0) return;
  const int32_t seg_bits = (int32_t)((sg.byte_end - sg.byte_start) * 8);
  const SubState &pv = sub[slot_gt(d, lt0 - 1)];
  int ep = pv.exit_p, ebk = pv.exit_bk;
  int lt = lt0;
  const int wg_next = (lt0 / kSlotsPerWg + 1) * kSlotsPerWg;
  Bits B;
  bits_init(B, dstuf, (lds_cu32)0, 0, 0, sg.byte_start, sg.byte_end);
  int steps = 0;
  Cp cp, none;
  none.n = 0;
  while (true) {
    ++steps;
    int b = ebk >> 8, k = ebk & 255;
    RunAcc acc{0, 0, 0, 0};
    B.seek(ep);
    count_run<false>(B, j * S, min((j + 1) * S, seg_bits), S, b, k, dcn, tabs, acc, cp, none, acc);
    const int np = B.pos(), nbk = (b << 8) | k;
    SubState &st = sub[slot_gt(d, lt)];
    st.nblk = acc.nblk;
    st.dc[0] = acc.dc0;
    st.dc[1] = acc.dc1;
    st.dc[2] = acc.dc2;
    if (np == st.exit_p && nbk == st.exit_bk) break; // converged
    st.exit_p = np;
    st.exit_bk = nbk;
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

// One wave per decode workgroup: compare the helper's candidate entry for the
// workgroup's first slot with the true predecessor exit; walk on a mismatch.
__global__ void __launch_bounds__(64) k_huff_fix(const ImgDesc *__restrict__ descs,
                                                 const Segment *__restrict__ segs,
                                                 const HuffTab *__restrict__ htabs,
                                                 const uint8_t *__restrict__ dstuf,
                                                 const int32_t *__restrict__ wg_img, int S,
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
  if (lt0 == segs[si].sub_first) return; // lane 1 starts a segment: exact entry
  const SubState &pv = sub[slot_gt(d, lt0 - 1)];
  const SubState &cand = sub[(int64_t)w * kSyncThreads];
  if (threadIdx.x == 0) atomicAdd(redo + 8, 1); // boundaries checked
  if (pv.exit_p == cand.exit_p && pv.exit_bk == cand.exit_bk) return; // helper was right
  boundary_walk_wave(d, segs, htabs, dstuf, S, sub, lt0, true, redo, redo);
}

// Fallback when a walk did not converge inside its workgroup: one wave per
// image walks every workgroup boundary in order (always correct).
__global__ void __launch_bounds__(64) k_huff_fix_serial(const ImgDesc *__restrict__ descs,
                                                        const Segment *__restrict__ segs,
                                                        const HuffTab *__restrict__ htabs,
                                                        const uint8_t *__restrict__ dstuf, int S,
                                                        SubState *__restrict__ sub,
                                                        const int32_t *__restrict__ status,
                                                        const int32_t *__restrict__ redo) {
  const int img = blockIdx.x;
  if (redo[0] == 0 || status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const Segment &last = segs[d.seg_base + d.nseg - 1];
  const int total = last.sub_first + last.sub_count;
  for (int wl = 1; wl < d.wg_count; ++wl) {
    const int lt0 = wl * kSlotsPerWg;
    if (lt0 >= total) break;
    boundary_walk_wave(d, segs, htabs, dstuf, S, sub, lt0, false, nullptr, nullptr);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __builtin_amdgcn_wave_barrier();
  }
}

// Exclusive prefix of (nblk, dc0, dc1, dc2) over each image's slots.
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
  int run[4] = {0, 0, 0, 0};
  for (int base = 0; base < total; base += 256) {
    const int lt = base + threadIdx.x;
    int v[4] = {0, 0, 0, 0};
    int64_t gt = 0;
    if (lt < total) {
      gt = slot_gt(d, lt);
      const SubState &st = sub[gt];
      v[0] = st.nblk;
      v[1] = st.dc[0];
      v[2] = st.dc[1];
      v[3] = st.dc[2];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int tot;
      const int ex = block_excl_scan256(v[q], sh_scan, &tot);
      if (lt < total) pre[gt * 4 + q] = run[q] + ex;
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
  __shared__ __attribute__((aligned(16))) WgShared sh;
  __shared__ uint8_t s_nat[80];
  const int img = wg_img[blockIdx.x];
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  const int tid = threadIdx.x;
  if (tid < 80) s_nat[tid] = c_natural[tid];
  int slot_tab[6];
  uint32_t slotmap;
  const int ns = image_slots(d, slotmap, slot_tab);
  const DecConst dcn = dec_const(d);
  SubCtx sc;
  int64_t wbase;
  int wbytes;
  sub_setup(d, segs, htabs, S, sh, wbase, wbytes, dstuf, sc, slot_tab, ns);
  if (!sc.active) return;
  const LDS_AS uint8_t *nat = (const LDS_AS uint8_t *)s_nat;
  const LdsTabs tabs{TABS_LDS, slotmap, htabs, &d};
  const Segment &sg = segs[sc.seg];
  const int64_t gt = (int64_t)blockIdx.x * kSyncThreads + tid;
  const int64_t gfirst = slot_gt(d, sg.sub_first);
  int b = 0, k = 0;
  int32_t entry = 0;
  if (sc.j > 0) {
    const int64_t pg = (tid == 1) ? (int64_t)(blockIdx.x - 1) * kSyncThreads + kSyncThreads - 1 : gt - 1;
    const SubState &ps = sub[pg];
    entry = ps.exit_p;
    b = ps.exit_bk >> 8;
    k = ps.exit_bk & 255;
  }
  const int32_t *pg4 = pre + gt * 4, *pf4 = pre + gfirst * 4;
  int pred0 = pg4[1] - pf4[1], pred1 = pg4[2] - pf4[2], pred2 = pg4[3] - pf4[3];
  int64_t cursor = (int64_t)(pg4[0] - pf4[0]) - 1;
  const int64_t total = (int64_t)sg.mcu_count * d.bpm;
  int16_t *coef_seg = coef + (d.coef_off + (int64_t)sg.mcu_first * d.bpm) * 64;
  const int32_t stop = min((sc.j + 1) * S, sc.seg_bits);
  Bits B;
  bits_init(B, dstuf, (lds_cu32)sh.win, wbase, wbytes, sc.seg0, sc.seg_end);
  B.seek(entry);
  RunAcc acc{0, 0, 0, 0};
  while (true) {
    if (B.pos() >= stop) break;
    if (k == 0) {
      if (cursor + 1 >= total) break;
      ++cursor;
    }
    int zz, cc;
    const int v = sym_step(B, b, k, dcn, tabs, acc, zz, cc);
    if (zz == 0) {
      const int pv = (cc == 0 ? pred0 : cc == 1 ? pred1 : pred2) + v;
      pred0 = cc == 0 ? pv : pred0;
      pred1 = cc == 1 ? pv : pred1;
      pred2 = cc == 2 ? pv : pred2;
      coef_seg[cursor * 64] = (int16_t)pv;
    } else if (zz > 0 && cursor >= 0) {
      coef_seg[cursor * 64 + nat[zz]] = (int16_t)v;
    }
  }
  if (sc.j == sg.sub_count - 1 && cursor + 1 < total) status[img] = 3; // ran out of data
}

hipError_t launch_huff_parallel(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n_wg == 0) return hipSuccess;
  const size_t tab_lds = (size_t)(p.max_tabs < 1 ? 1 : p.max_tabs) * kTabU16 * 2;
  hipLaunchKernelGGL(k_huff_sync, dim3(p.n_wg), dim3(kSyncThreads), tab_lds, s, p.descs, p.segs,
                     p.htabs, w.dstuf, p.wg_img, p.subseq_bits, w.sub, w.status, p.redo);
  hipLaunchKernelGGL(k_huff_fix, dim3(p.n_wg), dim3(64), tab_lds, s, p.descs, p.segs, p.htabs,
                     w.dstuf, p.wg_img, p.subseq_bits, w.sub, w.status, p.redo);
  hipLaunchKernelGGL(k_huff_fix_serial, dim3(p.n), dim3(64), tab_lds, s, p.descs, p.segs, p.htabs,
                     w.dstuf, p.subseq_bits, w.sub, w.status, p.redo);
  hipLaunchKernelGGL(k_huff_scan, dim3(p.n), dim3(256), 0, s, p.descs, p.segs, w.sub, w.sub_pre,
                     w.status);
  hipLaunchKernelGGL(k_huff_write, dim3(p.n_wg), dim3(kSyncThreads), tab_lds, s, p.descs, p.segs,
                     p.htabs, w.dstuf, p.wg_img, p.subseq_bits, w.sub, w.sub_pre, w.coef, w.status);
  return hipGetLastError();
}

} // namespace ldt

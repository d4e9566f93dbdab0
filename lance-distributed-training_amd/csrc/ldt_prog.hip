// ldt_prog.hip — entropy decode of progressive JPEG (SOF2) images.
//
// jdphuff.c restated (decode_mcu_DC_first / DC_refine / AC_first / AC_refine,
// EOB runs, restart intervals) with jdcoefct.c's full-image coefficient
// buffer: every scan updates the image's blocks in dense group planes
// (zigzag slots 1..63 in `pcoef`, the final DC value in `dcv`), which k_idct
// reads (and clears) instead of the baseline decoders' packed groups; the
// resize kernels run unchanged.
//
// Four 64-lane workgroups per progressive image, one per independent scan
// chain (DC scans; each component's AC scans). A scan's Huffman decode is a
// serial bit stream: the wave decodes it with wave-uniform (scalar) state
// (lane 0 stores) between chunks in which all lanes stage its
// inputs: the scan's bytes in an LDS window, and the coefficients of the next
// 64 blocks (one block per lane, coalesced 16-byte loads) which lane 0 then
// reads and refines in LDS before the wave writes them back. A chain's scans
// run in file order (a refinement scan depends on the earlier scans of its band).
//
// Reference semantics: libjpeg-turbo jdphuff.c (Pillow 12.2.0's decoder),
// jdhuff.c jpeg_fill_bit_buffer (byte stuffing, zero bits at a marker),
// process_restart. The host (ldt_abi.cpp plan_progressive) has already
// checked the progression parameters, found each scan's byte range and
// rejected files that libjpeg would block-smooth.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldt_device.hpp"
#include "ldt_kernels.hpp"

namespace ldt {

namespace {

#ifndef LDT_PROG_WIN
#define LDT_PROG_WIN 512
#endif
#ifndef LDT_PROG_CHUNK
#define LDT_PROG_CHUNK 32
#endif
constexpr int kWin = LDT_PROG_WIN;     // scan bytes staged in LDS (per wave)
constexpr int kChunk = LDT_PROG_CHUNK; // blocks staged per round (one per lane)
constexpr int kWaves = 4;   // scans of one chain in flight (one wave each)
// 7 waves per SIMD (72 VGPRs): seven chain workgroups per CU, as many as the
// pipeline's 7 batches in flight can supply. Since the symbol walk left the
// scalar unit, more resident chains raise the rate (profiles/r6/prog_salu_ab_r6p.txt).
#ifndef LDT_PROG_WAVES_EU
#define LDT_PROG_WAVES_EU 7
#endif

struct ProgLds {
  union {
    uint8_t win[kWin];
    uint32_t win32[kWin / 4];
  };
  __attribute__((aligned(16))) int16_t blk[kChunk][64]; // zigzag slots; [0] unused
  int16_t dc[kChunk];
  int16_t sink[64]; // the other lanes' half of lane 0's coefficient stores
  int64_t bidx[kChunk]; // coefficient-buffer block index of each staged slot
  int win_base, win_lim; // scan offsets of win[0] and one past its last valid byte
  int pos;               // the reader position (for window refills)
};
// The DC chain runs on wave 0 alone; its Huffman tables (one per component of
// an interleaved DC scan) live in the LDS of the idle waves 1..3.
static_assert(sizeof(ProgLds) * 3 >= sizeof(ProgTab) * 4, "DC tables do not fit");

// An AC scan's Huffman table held in the wave's registers (all 64 lanes hold a
// piece), so a symbol decode makes no LDS access:
//   lane l in 1..16: lim = (maxcode[l] + 1) << (16 - l), the 16-bit
//   left-aligned limit of the length-l codes (0 when there are none), and
//   voff = valoffset[l];
//   every lane: 4 of the 256 symbol bytes.
// jdhuff.c jpeg_huff_decode's search (the smallest l with code <= maxcode[l])
// is the smallest l with peek16 < lim[l]: one compare across the lanes, a
// ballot and a find-first-set. Meanwhile every lane l decodes the peek as if
// its code were l bits long (shr, voff, the symbol byte fetched from the lane
// holding it), and one readlane of lane l gives the length and the symbol.
// The scalar unit, which the serial decode saturates, issues only the
// find-first-set and the buffer update.
struct RegTab {
  uint32_t lim;
  int32_t voff;
  uint32_t vals;
  uint32_t shr;  // lane l in 1..16: 16 - l
  uint32_t lenb; // lane l: its code length << 8 (lane 17: 16 << 8 | the corrupt symbol)
  uint32_t symw; // lane l in 1..16: 8 (the symbol byte's width), else 0
};

// The wave's bit reader: jdhuff.c semantics (MSB first, FF00 -> FF, FF fill
// bytes skipped, zero bits once a marker is reached). Offsets are relative to
// the scan's first entropy-coded byte (the planner keeps scans below 2 GB).
struct PReader {
  const uint8_t *data;
  int pos, lim; // lim: one past the marker that ends the scan
  int wb, wl;   // the LDS window's scan range (copied from ProgLds)
  uint64_t buf;
  int bits;
  int marker; // 0: none yet; else the marker code reached
};

// The whole wave runs the decoder with identical values; every value the
// decoder's state or control flow takes from LDS or memory passes through
// readfirstlane, so the compiler keeps the reader state in SGPRs and the
// control flow on scalar branches (no exec-mask bookkeeping per branch, SALU
// 64-bit shifts). Results that only lanes consume (stored values, correction
// and new-value masks, the fill's byte assembly) are computed on the VALU
// (vu / vv below): the kernel is bound by the CUs' scalar issue.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

// A lane-held copy of a wave-uniform value: arithmetic on it runs on the
// VALU, beside the scalar unit that the serial decode saturates. For results
// that only lanes consume (stored values, masks); the decoder's own state and
// control flow stay scalar.
__device__ __forceinline__ uint32_t vu(uint32_t x) {
  uint32_t r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
  return r;
}
// The same for a value already in a VGPR (an LDS read): kept there.
__device__ __forceinline__ uint32_t vv(uint32_t x) {
  uint32_t r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

__device__ __forceinline__ int pbyte(const PReader &r, const ProgLds &L, int p) {
  int v;
  if (p < r.wl) v = L.win[p - r.wb];
  else v = __builtin_nontemporal_load(r.data + p);
  return (int)uni((uint32_t)v);
}

// Appends whole bytes while at most 56 bits are buffered. Fast path: the next
// 8 window bytes hold no 0xFF (no stuffing, no marker) -> one read of three
// aligned LDS words instead of a dependent read per byte.
__device__ __forceinline__ void pfill(PReader &r, const ProgLds &L) {
  if (r.marker == 0 && r.pos + 12 <= r.wl) {
    const int o = r.pos - r.wb;
    // on the VALU: the 8 bytes, the 0xFF test, their big-endian placement
    // below the buffered bits; the wave then reads the 64-bit result back
    const uint32_t a = vv(L.win32[o >> 2]), b = vv(L.win32[(o >> 2) + 1]), c = vv(L.win32[(o >> 2) + 2]);
    const uint32_t sh = (uint32_t)(o & 3) * 8;
    const uint32_t lo = __builtin_amdgcn_alignbit(b, a, sh), hi = __builtin_amdgcn_alignbit(c, b, sh);
    const uint32_t xl = ~lo, xh = ~hi;
    const uint32_t ffm = ((xl - 0x01010101u) & ~xl & 0x80808080u) | ((xh - 0x01010101u) & ~xh & 0x80808080u);
    if (__builtin_amdgcn_ballot_w64(ffm != 0) == 0) {
      const int nb = (64 - r.bits) >> 3; // bytes that fit
      const int cut = 64 - 8 * nb;        // bits of the 8 bytes that do not
      const uint64_t be = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
      r.buf |= uni64(((be >> cut) << cut) >> r.bits);
      r.bits += 8 * nb;
      r.pos += nb;
      return;
    }
  }
  while (r.bits <= 56) {
    int c = 0;
    if (r.marker == 0 && r.pos < r.lim) {
      c = pbyte(r, L, r.pos++);
      if (c == 0xFF) {
        int c2;
        do {
          c2 = r.pos < r.lim ? pbyte(r, L, r.pos++) : 0x100;
        } while (c2 == 0xFF);
        if (c2 == 0) {
          c = 0xFF;
        } else {
          r.marker = c2; // RSTn or the marker that ends the scan
          c = 0;
        }
      }
    }
    r.buf |= (uint64_t)c << (56 - r.bits);
    r.bits += 8;
  }
}

__device__ __forceinline__ int pget(PReader &r, const ProgLds &L, int n) {
  if (n == 0) return 0;
  if (r.bits < n) pfill(r, L);
  const int v = (int)(r.buf >> (64 - n));
  r.buf <<= n;
  r.bits -= n;
  return v;
}

// jdhuff.c jpeg_huff_decode on an LDS table (DC scans): 8-bit lookahead, then
// the canonical search.
__device__ __forceinline__ int phuff(PReader &r, const ProgLds &L, const ProgTab &t) {
  if (r.bits < 16) pfill(r, L);
  const uint32_t e = uni(t.look[r.buf >> 56]);
  if (e) {
    const int l = (int)(e >> 8);
    r.buf <<= l;
    r.bits -= l;
    return (int)(e & 255);
  }
  const int w = (int)(r.buf >> 48);
  for (int l = 9; l <= 16; ++l) {
    const int code = w >> (16 - l);
    if (code <= (int)uni((uint32_t)t.maxcode[l])) {
      r.buf <<= l;
      r.bits -= l;
      return (int)uni(t.vals[((int)uni((uint32_t)t.valoff[l]) + code) & 0xFF]);
    }
  }
  r.buf <<= 16; // corrupt data: libjpeg warns and returns symbol 0
  r.bits -= 16;
  return 0;
}

// Lane 17 matches every peek (lim = all ones): the ballot is never empty,
// and l = 17 stands for a code no table entry matches (libjpeg: warning,
// symbol 0, 16 bits consumed). For a refinement scan the symbol bytes are
// stored as classes: r | 0x10 when the size is nonzero (a sign bit follows) |
// 0x20 for EOBr (size 0, r < 15), so the decoder tests bits instead of
// comparing r and the size; corrupt codes then read as 0x20 (EOB0).
__device__ __forceinline__ RegTab reg_tab(const ProgTab &t, int lane, bool refine) {
  RegTab r;
  const bool has = lane >= 1 && lane <= 16;
  const int mc = has ? t.maxcode[lane] : -1;
  r.lim = lane == 17 ? ~0u : (mc < 0 ? 0u : (uint32_t)(mc + 1) << (16 - lane));
  r.voff = has ? t.valoff[lane] : 0;
  uint32_t v = reinterpret_cast<const uint32_t *>(t.vals)[lane];
  if (refine) {
    uint32_t c = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t sym = (v >> (8 * b)) & 0xFF, rr = sym >> 4, sz = sym & 15;
      const uint32_t cls = rr | (sz ? 0x10u : 0u) | (sz == 0 && rr != 15 ? 0x20u : 0u);
      c |= cls << (8 * b);
    }
    v = c;
  }
  r.vals = v;
  r.shr = has ? (uint32_t)(16 - lane) : 0u;
  r.lenb = has ? (uint32_t)lane << 8 : (lane == 17 ? (16u << 8) | (refine ? 0x20u : 0u) : 0u);
  r.symw = has ? 8u : 0u;
  return r;
}

// The symbol (or class) at the front of the buffer, which holds at least 16
// bits (the caller has filled it); consumes its code. Branch-free: a ballot
// of peek16 < lim[l] over the lanes, its lowest lane l, one readlane.
__device__ __forceinline__ int sym_reg(PReader &r, const RegTab &t) {
  const uint32_t w = (uint32_t)(r.buf >> 48);
  const uint64_t hit = __builtin_amdgcn_ballot_w64(w < t.lim);
  const int l = (int)__builtin_ctzll(hit); // 1..17 (lane 17 always matches)
  // Every lane l decodes the peek as if its code were l bits long, on the
  // VALU (the scalar unit is the kernel's bound): its symbol index, the
  // symbol byte fetched from the lane that holds it (one ds_bpermute), and
  // length << 8 | symbol; the wave then reads lane l's.
  const uint32_t idx = (uint32_t)(t.voff + (int)(w >> t.shr));
  const uint32_t word = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(idx & 0xFCu), (int)t.vals);
  const uint32_t cand = t.lenb | __builtin_amdgcn_ubfe(word, idx << 3, t.symw);
  const uint32_t cs = (uint32_t)__builtin_amdgcn_readlane((int)cand, l);
  const int clen = (int)(cs >> 8);
  r.buf <<= clen;
  r.bits -= clen;
  return (int)(cs & 0xFFu);
}

// Lane i's count of the set bits of m below bit i.
__device__ __forceinline__ uint32_t rank_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int pextend(int v, int s) {
  return s == 0 ? 0 : (v < (1 << (s - 1)) ? v - (1 << s) + 1 : v);
}

// jdphuff.c process_restart: drop the buffered bits and consume RSTn.
__device__ __forceinline__ void prestart(PReader &r, const ProgLds &L) {
  r.buf = 0;
  r.bits = 0;
  if (r.marker >= 0xD0 && r.marker <= 0xD7) {
    r.marker = 0;
    return;
  }
  if (r.marker != 0) return; // another marker: zero bits for the rest of the scan
  while (r.pos + 1 < r.lim) {
    const int a = pbyte(r, L, r.pos), b = pbyte(r, L, r.pos + 1);
    if (a == 0xFF && b >= 0xD0 && b <= 0xD7) {
      r.pos += 2;
      return;
    }
    if (a == 0xFF && b != 0x00 && b != 0xFF) return;
    ++r.pos;
  }
}

__device__ __forceinline__ uint64_t mask_from(int k) { return k >= 64 ? 0ull : (~0ull << k); }
__device__ __forceinline__ uint64_t mask_below(int k) { return k >= 64 ? ~0ull : ((1ull << k) - 1); }

// jdphuff.c process_restart's caller side: every `restart` units the reader
// drops its bits and consumes RSTn; the DC predictors and the EOB run reset.
__device__ __forceinline__ bool restart_due(PReader &R, const ProgLds &L, int restart, int &togo) {
  if (!restart) return false;
  bool did = false;
  if (togo == 0) {
    prestart(R, L);
    togo = restart;
    did = true;
  }
  --togo;
  return did;
}

// decode_mcu_AC_first over the chunk's nu blocks (single-component scan).
// EOBr is size 0 with r < 15, i.e. ((c + 0x10) & 0x10F) == 0; ZRL (r = 15,
// size 0) advances k by 16 like a value of size 0 that is not stored.
__device__ __forceinline__ void ac_first_chunk(PReader &R, ProgLds &L, const RegTab &rt, int nu, int Ss, int Se,
                                               int Al, int &eobrun, int &togo, int restart, bool w0) {
  for (int slot = 0; slot < nu; ++slot) {
    if (restart_due(R, L, restart, togo)) eobrun = 0;
    if (eobrun > 0) {
      --eobrun;
      continue;
    }
    int16_t *blk = L.blk[slot];
    for (int k = Ss; k <= Se; ++k) { // one loop exit: an EOBr moves k past 63
      if (R.bits < 32) pfill(R, L); // the code (<= 16 bits) and its value bits (<= 15)
      const int c = sym_reg(R, rt);
      if (((c + 0x10) & 0x10F) == 0) { // EOBr
        const int r = c >> 4;
        eobrun = 1 << r;
        if (r) eobrun += pget(R, L, r);
        --eobrun;
        k = 64;
        continue;
      }
      const int t = c & 15;
      k += c >> 4;
      if (t) {
        // the value on the VALU (t <= 15 bits, all in the buffer's high word);
        // lane 0 stores it, the other lanes into their sink halves
        const uint32_t vt = vu((uint32_t)t), vk = vu((uint32_t)min(k, 63));
        const int v = pextend((int)((uint32_t)(R.buf >> 32) >> (32u - vt)), (int)vt) * (1 << Al);
        int16_t *dst = w0 ? blk + vk : L.sink + (threadIdx.x & 63);
        *dst = (int16_t)v;
        R.buf <<= t;
        R.bits -= t;
      }
    }
  }
}

// decode_mcu_AC_refine over the chunk's nu blocks, on bit masks. jdphuff.c
// walks k one coefficient at a time: a nonzero (history) coefficient takes a
// correction bit, the (r+1)-th zero stops the walk and receives the new value.
// Here the walk is indexed by zero rank: per block the lanes tabulate, for
// each rank q, the band's q-th zero position P(q) and the count C(q) of
// history nonzeros below it (one forward permute), so a symbol with run r
// moves the rank q by r + 1, reads its stop P(q) with one readlane, and takes
// C(q) - C(previous stop) correction bits. The correction bits (which are in
// position order over the block), the ranks given a new value and the sign
// bits collect on the lanes as they are read (lane = rank, VALU) and are
// gathered to positions at the block's end as the masks corr / newm / negm;
// lane 0 stores them and the lanes apply them after the chunk (corrections
// first, then the new values, the order jdphuff.c's walk gives).
__device__ __forceinline__ uint64_t pget64(PReader &r, const ProgLds &L, int n) {
  if (n <= 32) return (uint32_t)pget(r, L, n);
  const uint64_t hi = (uint32_t)pget(r, L, n - 32);
  return (hi << 32) | (uint32_t)pget(r, L, 32);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

// nzv (lane j): block j's positions nonzero before the scan; corr_v / newm_v /
// negm_v (lane j): block j's correction / new-value / negative masks out.
__device__ __forceinline__ void ac_refine_chunk(PReader &R, ProgLds &L, const RegTab &rt, int nu, int Ss, int Se,
                                                int &eobrun, int &togo, int restart, uint64_t nzv,
                                                uint64_t &corr_v, uint64_t &newm_v, uint64_t &negm_v) {
  const int lane = (int)(threadIdx.x & 63);
  const uint64_t band = mask_from(Ss) & mask_below(Se + 1);
  for (int slot = 0; slot < nu; ++slot) {
    if (restart_due(R, L, restart, togo)) eobrun = 0;
    const uint64_t nzh = readlane64(nzv, slot);
    const uint64_t N = nzh & band;  // history nonzeros of the band
    const uint64_t Z = ~nzh & band; // positions of the band still zero
    const int ntot = __popcll(N);
    const int nz0 = __popcll(Z);
    const uint32_t jz = rank_below(Z), jn = rank_below(N);
    const bool in_z = (Z >> lane) & 1;
    // The walk's results collect on the lanes (VALU, off the scalar unit that
    // the serial decode saturates): lane r = the band's r-th nonzero takes its
    // correction bit (cbv), lane q = the q-th zero gets 1 | 2 * positive when a
    // new value lands on it (rbv).
    int ccons = 0;        // corrections read: the first ccons nonzeros of N
    uint32_t cbv = 0;
    uint32_t rbv = 0;
    int ovf = -1;         // a value placed past the band's last zero (jdphuff.c
    int ovf_pos = 0;      // natural_order[Se + 1]; corrupt data only), its sign
    // n (<= 32) correction bits, the first read most significant, for the
    // nonzeros of ranks ccons .. ccons + n - 1
    auto deposit = [&](uint32_t bits, int n) {
      const uint32_t d = (uint32_t)lane - (uint32_t)ccons;
      cbv = d < (uint32_t)n ? ((bits >> (((uint32_t)n - 1u - d) & 31u)) & 1u) : cbv;
      ccons += n;
    };
    if (eobrun == 0) {
      // lane q <- (P(q) | C(q) << 8); ranks q >= nz0: (Se + 1, ntot). Each lane
      // sends to a distinct rank: zero positions to their rank, the others to
      // nz0 + their rank among the non-zero positions.
      const uint32_t dst = in_z ? jz : (uint32_t)nz0 + ((uint32_t)lane - jz);
      const uint32_t val = in_z ? ((uint32_t)lane | (jn << 8)) : ((uint32_t)(Se + 1) | ((uint32_t)ntot << 8));
      const int pc = __builtin_amdgcn_ds_permute((int)(dst * 4), (int)val);
      int rn = 0;   // the rank of the next zero
      int last = 0; // the walk's last stop (64 after an EOBr): one loop exit
      do {
        if (R.bits < 17) pfill(R, L); // the code (<= 16 bits) and the sign bit
        const int c = sym_reg(R, rt);
        if (c & 0x20) { // EOBr
          const int r = c & 15;
          eobrun = 1 << r;
          if (r) eobrun += pget(R, L, r);
          last = 64;
        } else {
          // a nonzero size takes a sign bit (1: +p1), then the corrections
          const int t1 = (c >> 4) & 1;
          const uint32_t shi = (uint32_t)(R.buf >> 32); // the sign bit is its bit 31
          const int q = rn + (c & 15); // the stop's zero rank (ZRL: the 16th zero)
          const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(pc, min(q, 63));
          const int stop = (int)(e & 0xFF);
          int nc = (int)(e >> 8) - ccons; // nonzeros passed: one correction bit each
          R.buf <<= t1;
          R.bits -= t1;
          if ((uint32_t)nc > (uint32_t)min(32, R.bits)) { // rare: long corrections or a low buffer
            while (nc > 32) {
              deposit((uint32_t)pget(R, L, 32), 32);
              nc -= 32;
            }
            if (nc > R.bits) pfill(R, L);
          }
          // lane ccons + j takes correction bit j, the buffer's bit 63 - j
          // (nc <= 32: all in its high word), on the VALU
          const uint32_t d = (uint32_t)lane - (uint32_t)ccons;
          cbv = d < (uint32_t)nc ? ((uint32_t)(R.buf >> 32) >> ((31u - d) & 31u)) & 1u : cbv;
          ccons += nc;
          R.buf <<= nc;
          R.bits -= nc;
          // the new value's rank, sign and (corrupt data) overflow, on the VALU
          const uint32_t vq = vu((uint32_t)q), vt1 = vu((uint32_t)t1);
          const uint32_t vsgn = vu(shi) >> 31;
          const uint32_t t1i = vq < (uint32_t)nz0 ? vt1 : 0u;
          rbv = (uint32_t)lane == vq ? (t1i | ((t1i & vsgn) << 1)) : rbv;
          const bool past = vt1 > t1i;
          const int vstop = (int)vu((uint32_t)min(stop, 63));
          ovf = past ? vstop : ovf;
          ovf_pos = past ? (int)vsgn : ovf_pos;
          rn = q + 1;
          last = stop;
        }
      } while (last < Se); // past Se: the walk's next k is outside the band
    }
    if (eobrun > 0) { // the rest of the band's nonzeros take correction bits
      int nc = ntot - ccons;
      while (nc > 32) {
        deposit((uint32_t)pget(R, L, 32), 32);
        nc -= 32;
      }
      if (nc) deposit((uint32_t)pget(R, L, nc), nc);
      --eobrun;
    }
    // to the positions (lane j = zigzag position j): gather by rank
    const uint32_t cb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(jn * 4u), (int)cbv);
    const uint32_t rb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((jz & 63u) * 4u), (int)rbv);
    const bool in_n = (N >> lane) & 1;
    const uint64_t corr = __builtin_amdgcn_ballot_w64(in_n && (cb & 1u));
    uint64_t newm = __builtin_amdgcn_ballot_w64(in_z && (rb & 1u));
    uint64_t negm = __builtin_amdgcn_ballot_w64(in_z && (rb & 1u) && !(rb & 2u));
    ovf = (int)uni((uint32_t)ovf);
    ovf_pos = (int)uni((uint32_t)ovf_pos);
    if (ovf >= 0) {
      newm |= 1ull << ovf;
      negm = ovf_pos ? (negm & ~(1ull << ovf)) : (negm | (1ull << ovf));
    }
    if (lane == slot) {
      corr_v = corr;
      newm_v = newm;
      negm_v = negm;
    }
  }
}

// Stage scan bytes [base, min(base + kWin, lim)) into the window (all lanes).
__device__ void load_window(ProgLds &L, const uint8_t *data, int base, int lim) {
  const int lane = threadIdx.x & 63;
  const int n = min(kWin, lim - base);
  // all loads in flight before the first LDS write (one memory latency per refill)
  uint8_t v[kWin / 64];
#pragma unroll
  for (int i = 0; i < kWin / 64; ++i) {
    const int o = lane + 64 * i;
    v[i] = o < n ? data[base + o] : (uint8_t)0;
  }
#pragma unroll
  for (int i = 0; i < kWin / 64; ++i) {
    const int o = lane + 64 * i;
    if (o < n) L.win[o] = v[i];
  }
  if (lane == 0) {
    L.win_base = base;
    L.win_lim = base + n;
  }
}

// Orders a wave's LDS accesses across lanes (the wave's LDS operations
// execute in order; this keeps the compiler from moving them across).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

} // namespace

__global__ void __launch_bounds__(64 * kWaves, LDT_PROG_WAVES_EU) k_prog(const ImgDesc *__restrict__ descs,
                                             const int32_t *__restrict__ prog_img,
                                             const ProgScan *__restrict__ scans,
                                             const ProgTab *__restrict__ ptabs,
                                             const uint8_t *__restrict__ data,
                                             int16_t *__restrict__ pcoef,
                                             int16_t *__restrict__ dcv,
                                             const int32_t *__restrict__ status) {
  __shared__ ProgLds Lw[kWaves];
  __shared__ int progress[kMaxProgScans]; // chunks of each chain scan written back
  // chain 0: the DC scans (dcv only); chain 1 + c: component c's AC scans
  // (coef slots 1..63 of its blocks). JPEG AC scans are single-component, so
  // the chains touch disjoint data and run as independent workgroups; within
  // a chain, scans keep file order (refinements follow their first scans).
  // chain-major grid: consecutive workgroups are different images, so the
  // long luma chains spread round-robin over all 8 XCDs; luma AC first
  const int nimg = (int)(gridDim.x >> 2);
  const int img = prog_img[blockIdx.x % nimg];
  const int q = (int)(blockIdx.x / nimg);
  const int chain = q == 0 ? 1 : (q == 1 ? 0 : q);
  if (status[img] != 0) return;
  const ImgDesc &d = descs[img];
  if (chain > d.ncomp) return;
  for (int i = threadIdx.x; i < kMaxProgScans; i += 64 * kWaves) progress[i] = 0;
  __syncthreads(); // the only workgroup barrier: waves run independently from here
  // AC chains are pipelined: the chain's j-th scan runs on wave j % kWaves and
  // processes its chunk c once scan j-1 has written chunk c back (all AC scans
  // of a component walk the same block order in the same chunks). The DC chain
  // (interleaved and per-component DC scans chunk differently) runs on wave 0.
  const int wave = (int)(threadIdx.x >> 6);
  const int lane = (int)(threadIdx.x & 63);
  if (chain == 0 && wave != 0) return;
  ProgLds &L = Lw[wave];
  ProgTab *dctabs = reinterpret_cast<ProgTab *>(&Lw[1]); // DC chain only
  const int64_t nblk = (int64_t)d.mcux * d.mcuy * d.bpm;
  // DC values start at zero: blocks no DC scan covers (the padding blocks of
  // non-interleaved DC scans) must not keep an earlier batch's value
  if (chain == 0)
    for (int64_t b = lane; b < nblk; b += 64) dcv[d.coef_off + b] = 0;
  int b0[3] = {0, 0, 0}, hmax = 1, vmax = 1;
  for (int c = 0; c < d.ncomp; ++c) {
    hmax = max(hmax, d.ch[c]);
    vmax = max(vmax, d.cv[c]);
    for (int b = d.bpm - 1; b >= 0; --b)
      if (d.bcomp[b] == c) b0[c] = b;
  }
  const bool w0 = lane == 0; // the lane that stores
  int nchain = 0; // the chain's scans (the last one publishes no progress)
  for (int si = 0; si < d.prog_count; ++si) {
    const ProgScan &sc = scans[d.prog_first + si];
    nchain += (sc.ss == 0 ? chain == 0 : chain == 1 + sc.comp[0]) ? 1 : 0;
  }
  int jc = -1; // index of the scan within the chain
  for (int si = 0; si < d.prog_count; ++si) {
    const ProgScan &sc = scans[d.prog_first + si];
    const int ns = sc.ns, Ss = sc.ss, Se = sc.se, Ah = sc.ah, Al = sc.al;
    const bool dcband = Ss == 0;
    if (dcband ? chain != 0 : chain != 1 + sc.comp[0]) continue; // another chain's scan
    ++jc;
    const bool piped = chain != 0;
    if (piped && jc % kWaves != wave) continue; // another wave's scan
    const bool wait_prev = piped && jc > 0;
    wave_sync();
    RegTab rt{};
    if (dcband) {
      for (int k = 0; k < 4; ++k) {
        if (sc.tab[k] < 0) continue;
        const uint32_t *src = reinterpret_cast<const uint32_t *>(ptabs + sc.tab[k]);
        uint32_t *dst = reinterpret_cast<uint32_t *>(&dctabs[k]);
        for (int o = lane; o < (int)(sizeof(ProgTab) / 4); o += 64) dst[o] = src[o];
      }
    } else {
      rt = reg_tab(ptabs[sc.tab[0]], lane, Ah != 0);
    }
    PReader R;
    R.data = data + sc.data_off;
    R.lim = (int)sc.data_len + 2; // through the ending marker
    load_window(L, R.data, 0, R.lim);
    wave_sync();
    // units: MCUs of the interleaved grid, or the component's own blocks
    int ux, uy, bpu = 0;
    if (ns == 1) {
      const int c = sc.comp[0];
      ux = (int)(((int64_t)d.width * d.ch[c] + 8 * hmax - 1) / (8 * hmax));
      uy = (int)(((int64_t)d.height * d.cv[c] + 8 * vmax - 1) / (8 * vmax));
      if (d.ncomp == 1) {
        ux = d.mcux;
        uy = d.mcuy;
      }
      bpu = 1;
    } else {
      ux = d.mcux;
      uy = d.mcuy;
      for (int i = 0; i < ns; ++i) bpu += d.ch[sc.comp[i]] * d.cv[sc.comp[i]];
    }
    const int64_t units = (int64_t)ux * uy;
    const int upc = kChunk / bpu;
    // the component (scan order) of each block of a unit, 2 bits per block
    uint32_t cmap = 0;
    for (int i = 0, b = 0; i < ns; ++i) {
      const int nb = ns == 1 ? 1 : d.ch[sc.comp[i]] * d.cv[sc.comp[i]];
      for (int q = 0; q < nb; ++q, ++b) cmap |= (uint32_t)i << (2 * b);
    }
    R.pos = 0;
    R.buf = 0;
    R.bits = 0;
    R.marker = 0;
    int pred[4] = {0, 0, 0, 0};
    int eobrun = 0;
    int togo = sc.restart;
    const int p1 = 1 << Al, m1 = -(1 << Al);
    for (int64_t u0 = 0, ci = 0; u0 < units; u0 += upc, ++ci) {
      const int nu = (int)min((int64_t)upc, units - u0);
      const int nbk = nu * bpu;
      if (wait_prev) // scan jc-1 has written this chunk back
        while (__hip_atomic_load(&progress[jc - 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= ci)
          __builtin_amdgcn_s_sleep(1);
      // stage the chunk's blocks: lane j -> block j of the chunk, scan order
      uint64_t nzv = 0; // lane j: block j's nonzero positions (AC scans)
      if (lane < nbk) {
        const int64_t u = u0 + lane / bpu;
        int64_t blk;
        if (ns == 1) {
          const int c = sc.comp[0];
          const int bx = (int)(u % ux), by = (int)(u / ux);
          const int64_t m = (int64_t)(by / d.cv[c]) * d.mcux + bx / d.ch[c];
          blk = m * d.bpm + b0[c] + (by % d.cv[c]) * d.ch[c] + (bx % d.ch[c]);
        } else {
          int j = lane % bpu, b = 0;
          for (int i = 0; i < ns; ++i) {
            const int c = sc.comp[i], nb = d.ch[c] * d.cv[c];
            if (j >= 0 && j < nb) b = b0[c] + j;
            j -= nb;
          }
          blk = u * d.bpm + b;
        }
        const int64_t gb = d.coef_off + blk;
        L.bidx[lane] = gb;
        if (dcband) {
          L.dc[lane] = dcv[gb];
        } else {
          int4 *dst = reinterpret_cast<int4 *>(L.blk[lane]);
          uint64_t nz = 0;
#pragma unroll 4 // (8 would hold 32 VGPRs of loads: spills under the 72-VGPR cap)
          for (int q = 0; q < 8; ++q) {
            const int4 v = reinterpret_cast<const int4 *>(pcoef + d.pcoef_off * 64)[coef_piece((int)blk, q, coef_npad(d))];
            dst[q] = v;
            const uint32_t w[4] = {(uint32_t)v.x, (uint32_t)v.y, (uint32_t)v.z, (uint32_t)v.w};
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              nz |= (uint64_t)((w[h] & 0xFFFFu) != 0) << (8 * q + 2 * h);
              nz |= (uint64_t)((w[h] >> 16) != 0) << (8 * q + 2 * h + 1);
            }
          }
          nzv = nz;
        }
      }
      wave_sync();

      uint64_t corr_v = 0, newm_v = 0, negm_v = 0;
      R.wb = (int)uni((uint32_t)L.win_base);
      R.wl = (int)uni((uint32_t)L.win_lim);
      if (!dcband) {
        if (Ah == 0)
          ac_first_chunk(R, L, rt, nu, Ss, Se, Al, eobrun, togo, sc.restart, w0);
        else
          ac_refine_chunk(R, L, rt, nu, Ss, Se, eobrun, togo, sc.restart, nzv, corr_v, newm_v, negm_v);
      } else if (Ah != 0 && sc.restart == 0) {
        // decode_mcu_DC_refine without restarts: one bit per block, in the
        // chunk's block order, so the chunk's nbk (<= 32) bits are read at
        // once and each lane takes its block's bit
        const uint32_t bits = (uint32_t)pget(R, L, nbk);
        if (lane < nbk && ((bits >> (nbk - 1 - lane)) & 1u)) L.dc[lane] = (int16_t)(L.dc[lane] | p1);
      } else {
        int slot = 0;
        for (int ui = 0; ui < nu; ++ui) {
          if (restart_due(R, L, sc.restart, togo)) pred[0] = pred[1] = pred[2] = pred[3] = 0;
          {
            for (int b = 0; b < bpu; ++b, ++slot) {
              const int i = (int)(cmap >> (2 * b)) & 3;
              if (Ah == 0) { // decode_mcu_DC_first (size <= 15: the planner's check)
                const int t = phuff(R, L, dctabs[i]);
                pred[i] += pextend(pget(R, L, t), t);
                if (w0) L.dc[slot] = (int16_t)(pred[i] * (1 << Al));
              } else { // decode_mcu_DC_refine (with restarts)
                if (pget(R, L, 1) && w0) L.dc[slot] = (int16_t)(L.dc[slot] | p1);
              }
            }
          }
        }
      }
      if (w0) L.pos = R.pos;
      wave_sync();
      if (lane < nbk) {
        const int64_t gb = L.bidx[lane];
        if (!dcband && Ah != 0) { // apply this block's refinement: corrections, then new values
          int16_t *blk = L.blk[lane];
          for (uint64_t cm = corr_v; cm; cm &= cm - 1) {
            const int pos = __ffsll((unsigned long long)cm) - 1;
            const int c = blk[pos];
            if ((c & p1) == 0) blk[pos] = (int16_t)(c >= 0 ? c + p1 : c + m1);
          }
          const uint64_t ng = negm_v;
          for (uint64_t nm = newm_v; nm; nm &= nm - 1) {
            const int pos = __ffsll((unsigned long long)nm) - 1;
            blk[pos] = (int16_t)(((ng >> pos) & 1) ? m1 : p1);
          }
        }
        if (dcband) {
          dcv[gb] = L.dc[lane];
        } else {
          const int4 *src = reinterpret_cast<const int4 *>(L.blk[lane]);
#pragma unroll
          for (int q = 0; q < 8; ++q)
            reinterpret_cast<int4 *>(pcoef + d.pcoef_off * 64)[coef_piece((int)(gb - d.coef_off), q, coef_npad(d))] = src[q];
        }
      }
      if (piped && jc + 1 < nchain) { // publish chunk ci once the wave's stores are done
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0)
          __hip_atomic_store(&progress[jc], (int)(ci + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // keep at least half a window of bytes ahead of the reader
      wave_sync();

      const int pos = L.pos;
      if (pos - L.win_base > kWin / 2 && L.win_lim < R.lim) {
        wave_sync();
        load_window(L, R.data, pos, R.lim);
      }
      wave_sync();

    }
  }
}

hipError_t launch_prog(const DevPlan &p, const DevWork &w, hipStream_t s) {
  if (p.n_prog == 0) return hipSuccess;
  hipLaunchKernelGGL(k_prog, dim3(4 * p.n_prog), dim3(64 * kWaves), 0, s, p.descs, p.prog_img, p.pscans, p.ptabs,
                     w.data, w.pcoef, w.dcv, w.status);
  return hipGetLastError();
}

} // namespace ldt

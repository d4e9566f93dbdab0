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

constexpr int kWin = 4096;  // scan bytes staged in LDS (per wave)
constexpr int kChunk = 32;  // blocks staged per round (one per lane)
constexpr int kWaves = 4;   // scans of one chain in flight (one wave each)

struct ProgLds {
  union {
    uint8_t win[kWin];
    uint32_t win32[kWin / 4];
  };
  __attribute__((aligned(16))) int16_t blk[kChunk][64]; // zigzag slots; [0] unused
  int16_t dc[kChunk];
  int64_t bidx[kChunk]; // coefficient-buffer block index of each staged slot
  uint64_t nzm[kChunk];  // AC refinement: zigzag positions nonzero before the scan
  uint64_t corr[kChunk]; // AC refinement: positions whose correction bit is 1
  ProgTab tabs[4];
  int64_t win_base, win_lim; // data offsets of win[0] and one past its last valid byte
  int64_t pos;               // lane 0's reader position (for window refills)
};

// Lane 0's bit reader: jdhuff.c semantics (MSB first, FF00 -> FF, FF fill
// bytes skipped, zero bits once a marker is reached).
struct PReader {
  const uint8_t *data;
  int64_t pos, lim; // lim: one past the marker that ends the scan
  int64_t wb, wl;   // the LDS window's data range (copied from ProgLds)
  uint64_t buf;
  int bits;
  int marker; // 0: none yet; else the marker code reached
};

// The whole wave runs the decoder with identical values; every value read
// from LDS or memory passes through readfirstlane, so the compiler keeps the
// reader state in SGPRs and the control flow on scalar branches (no exec-mask
// bookkeeping per branch, SALU 64-bit shifts). Stores are made by lane 0.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

__device__ __forceinline__ int pbyte(const PReader &r, const ProgLds &L, int64_t p) {
  int v;
  if (p < r.wl) v = L.win[(int)(p - r.wb)];
  else v = __builtin_nontemporal_load(r.data + p);
  return (int)uni((uint32_t)v);
}

// Appends whole bytes while at most 56 bits are buffered. Fast path: the next
// 8 window bytes hold no 0xFF (no stuffing, no marker) -> one read of three
// aligned LDS words instead of a dependent read per byte.
__device__ __forceinline__ void pfill(PReader &r, const ProgLds &L) {
  if (r.marker == 0 && r.pos + 12 <= r.wl) {
    const int o = (int)(r.pos - r.wb);
    const uint32_t a = uni(L.win32[o >> 2]), b = uni(L.win32[(o >> 2) + 1]),
                   c = uni(L.win32[(o >> 2) + 2]);
    const uint32_t sh = (uint32_t)(o & 3) * 8;
    // bytes pos..pos+7 in memory order, little-endian words
    const uint32_t lo = sh ? (a >> sh) | (b << (32 - sh)) : a;
    const uint32_t hi = sh ? (b >> sh) | (c << (32 - sh)) : b;
    // any 0xFF byte among the 8?
    const uint32_t xl = ~lo, xh = ~hi;
    const uint32_t ffm = ((xl - 0x01010101u) & ~xl & 0x80808080u) | ((xh - 0x01010101u) & ~xh & 0x80808080u);
    if (ffm == 0) {
      const int nb = (64 - r.bits) >> 3; // bytes that fit
      // big-endian bit order: byte i of memory goes to bits 56-8i of the word
      const uint64_t be = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
      const uint64_t keep = nb == 8 ? ~0ull : ~(~0ull >> (8 * nb));
      r.buf |= (be & keep) >> r.bits;
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

// jdhuff.c jpeg_huff_decode: 8-bit lookahead, then the canonical search.
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

// AC refinement correction bits for the already-nonzero positions in `seg`
// (ascending zigzag order, one bit each, read 16 at a time): returns the
// positions whose bit is 1. The corrections themselves (jdphuff.c: c += p1 or
// m1 when (c & p1) == 0) are applied lane-parallel after the chunk.
__device__ __forceinline__ uint64_t pcorr(PReader &r, const ProgLds &L, uint64_t seg) {
  uint64_t res = 0;
  while (seg) {
    const int cnt = min(__popcll(seg), 16);
    const int bits = pget(r, L, cnt);
    for (int j = cnt - 1; j >= 0; --j) {
      const uint64_t low = seg & (0ull - seg);
      res |= ((bits >> j) & 1) ? low : 0ull;
      seg ^= low;
    }
  }
  return res;
}

__device__ __forceinline__ uint64_t mask_from(int k) { return k >= 64 ? 0ull : (~0ull << k); }
__device__ __forceinline__ uint64_t mask_below(int k) { return k >= 64 ? ~0ull : ((1ull << k) - 1); }

// Stage scan bytes [base, min(base + kWin, lim)) into the window (all lanes).
__device__ void load_window(ProgLds &L, const uint8_t *data, int64_t base, int64_t lim) {
  const int lane = threadIdx.x & 63;
  const int64_t n = min((int64_t)kWin, lim - base);
  for (int64_t o = lane; o < n; o += 64) L.win[o] = data[base + o];
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

__global__ void __launch_bounds__(64 * kWaves) k_prog(const ImgDesc *__restrict__ descs,
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
  PReader R;
  R.data = data;
  int pred[4] = {0, 0, 0, 0};
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
    for (int k = 0; k < 4; ++k) {
      if (sc.tab[k] < 0) continue;
      const uint32_t *src = reinterpret_cast<const uint32_t *>(ptabs + sc.tab[k]);
      uint32_t *dst = reinterpret_cast<uint32_t *>(&L.tabs[k]);
      for (int o = lane; o < (int)(sizeof(ProgTab) / 4); o += 64) dst[o] = src[o];
    }
    const int64_t lim = sc.data_off + sc.data_len + 2; // through the ending marker
    load_window(L, data, sc.data_off, lim);
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
    R.pos = sc.data_off;
    R.lim = lim;
    R.buf = 0;
    R.bits = 0;
    R.marker = 0;
    pred[0] = pred[1] = pred[2] = pred[3] = 0;
    int64_t eobrun = 0;
    int togo = sc.restart;
    const int p1 = 1 << Al, m1 = -(1 << Al);
    for (int64_t u0 = 0, ci = 0; u0 < units; u0 += upc, ++ci) {
      const int nu = (int)min((int64_t)upc, units - u0);
      const int nbk = nu * bpu;
      if (wait_prev) // scan jc-1 has written this chunk back
        while (__hip_atomic_load(&progress[jc - 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= ci)
          __builtin_amdgcn_s_sleep(1);
      // stage the chunk's blocks: lane j -> block j of the chunk, scan order
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
#pragma unroll
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
          L.nzm[lane] = nz;
          L.corr[lane] = 0;
        }
      }
      wave_sync();
      const bool w0 = lane == 0; // the lane that stores
      {
        R.wb = (int64_t)uni64((uint64_t)L.win_base);
        R.wl = (int64_t)uni64((uint64_t)L.win_lim);
        int slot = 0;
        for (int ui = 0; ui < nu; ++ui) {
          if (sc.restart) {
            if (togo == 0) {
              prestart(R, L);
              pred[0] = pred[1] = pred[2] = pred[3] = 0;
              eobrun = 0;
              togo = sc.restart;
            }
            --togo;
          }
          for (int i = 0; i < ns; ++i) {
            const int nb = ns == 1 ? 1 : d.ch[sc.comp[i]] * d.cv[sc.comp[i]];
            for (int q = 0; q < nb; ++q, ++slot) {
              if (dcband && Ah == 0) { // decode_mcu_DC_first
                const int t = phuff(R, L, L.tabs[i]);
                pred[i] += pextend(pget(R, L, t), t);
                if (w0) L.dc[slot] = (int16_t)(pred[i] * (1 << Al));
              } else if (dcband) { // decode_mcu_DC_refine
                if (pget(R, L, 1) && w0) L.dc[slot] = (int16_t)(L.dc[slot] | p1);
              } else if (Ah == 0) { // decode_mcu_AC_first
                if (eobrun > 0) {
                  --eobrun;
                  continue;
                }
                int16_t *blk = L.blk[slot];
                for (int k = Ss; k <= Se; ++k) {
                  const int rs = phuff(R, L, L.tabs[0]);
                  const int r = rs >> 4, t = rs & 15;
                  if (t) {
                    k += r;
                    const int v = pextend(pget(R, L, t), t) * (1 << Al);
                    if (w0) blk[min(k, 63)] = (int16_t)v;
                  } else if (r == 15) {
                    k += 15;
                  } else {
                    eobrun = (int64_t)1 << r;
                    if (r) eobrun += pget(R, L, r);
                    --eobrun;
                    break;
                  }
                }
              } else { // decode_mcu_AC_refine, on bit masks of the block
                // jdphuff.c walks k one coefficient at a time: a nonzero
                // (history) coefficient takes a correction bit, the (r+1)-th
                // zero stops the walk and receives the new value. Here the
                // history is the 64-bit mask nzh, the stop is found by
                // clearing r zero bits, and the correction bits of the
                // nonzeros passed are read in bulk (pcorr).
                int16_t *blk = L.blk[slot];
                const uint64_t nzh = uni64(L.nzm[slot]);
                const uint64_t band = mask_below(Se + 1);
                uint64_t corr = 0;
                int k = Ss;
                if (eobrun == 0) {
                  for (; k <= Se; ++k) {
                    const int rs = phuff(R, L, L.tabs[0]);
                    const int r = rs >> 4;
                    const int t = rs & 15;
                    int sv = 0;
                    if (t) {
                      sv = pget(R, L, 1) ? p1 : m1;
                    } else if (r != 15) {
                      eobrun = (int64_t)1 << r;
                      if (r) eobrun += pget(R, L, r);
                      break;
                    }
                    uint64_t z = ~nzh & mask_from(k) & band;
                    for (int q = 0; q < r && z; ++q) z &= z - 1;
                    const int stop = z ? __ffsll((unsigned long long)z) - 1 : Se + 1;
                    corr |= pcorr(R, L, nzh & mask_from(k) & mask_below(stop));
                    k = stop;
                    if (sv && w0) blk[min(k, 63)] = (int16_t)sv;
                  }
                }
                if (eobrun > 0) {
                  corr |= pcorr(R, L, nzh & mask_from(k) & band);
                  --eobrun;
                }
                if (w0) L.corr[slot] = corr;
              }
            }
          }
        }
        if (w0) L.pos = R.pos;
      }
      wave_sync();
      if (lane < nbk) {
        const int64_t gb = L.bidx[lane];
        if (!dcband && Ah != 0) { // apply this block's refinement corrections
          int16_t *blk = L.blk[lane];
          for (uint64_t cm = L.corr[lane]; cm; cm &= cm - 1) {
            const int pos = __ffsll((unsigned long long)cm) - 1;
            const int c = blk[pos];
            if ((c & p1) == 0) blk[pos] = (int16_t)(c >= 0 ? c + p1 : c + m1);
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
      if (piped) { // publish chunk ci once the wave's stores are done
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0)
          __hip_atomic_store(&progress[jc], (int)(ci + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // keep at least half a window of bytes ahead of the reader
      wave_sync();
      const int64_t pos = L.pos;
      if (pos - L.win_base > kWin / 2 && L.win_lim < lim) {
        wave_sync();
        load_window(L, data, pos, lim);
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

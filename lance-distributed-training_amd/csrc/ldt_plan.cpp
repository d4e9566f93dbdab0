// ldt_plan.cpp — host JPEG header planner (see ldt_plan.hpp). Restates
// libjpeg-turbo jdmarker.c (marker parsing), jdhuff.c
// jpeg_make_d_derived_tbl and jdphuff.c's progression checks for the subset
// the device kernels decode. No HIP calls: built into libldt.so and, for the
// fuzz test, alone with -fsanitize=address,undefined.
#include "ldt_plan.hpp"

#include <stdint.h>
#include <string.h>
#include <emmintrin.h>

#include "../../include/ldt.h"

namespace ldt {

namespace {

const uint8_t kZigzagToNatural[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

inline int be16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

} // namespace

// Returns an LDT_IMG_* code.
int walk_markers(const uint8_t *cell, int64_t len, Header &H) {
  for (int i = 0; i < 4; ++i) H.dc[i].present = H.ac[i].present = false;
  if (len < 4 || cell[0] != 0xFF || cell[1] != 0xD8) return LDT_IMG_NOT_JPEG;
  int64_t i = 2;
  bool sof = false;
  while (true) {
    if (i + 1 >= len) return LDT_IMG_NOT_JPEG;
    if (cell[i] != 0xFF) return LDT_IMG_NOT_JPEG;
    while (i + 1 < len && cell[i + 1] == 0xFF) ++i; // fill bytes
    if (i + 1 >= len) return LDT_IMG_NOT_JPEG;
    const int m = cell[i + 1];
    i += 2;
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (m == 0xD9) return LDT_IMG_NOT_JPEG;
    if (i + 2 > len) return LDT_IMG_NOT_JPEG;
    const int seglen = be16(cell + i);
    if (seglen < 2 || i + seglen > len) return LDT_IMG_NOT_JPEG;
    const uint8_t *s = cell + i + 2;
    const uint8_t *e = cell + i + seglen;
    switch (m) {
    case 0xC0:
    case 0xC1:
    case 0xC2: {
      if (sof) return LDT_IMG_NOT_JPEG; // two SOF markers
      H.progressive = m == 0xC2;
      if (e - s < 6) return LDT_IMG_NOT_JPEG;
      if (s[0] != 8) return LDT_IMG_UNSUPPORTED;
      H.height = be16(s + 1);
      H.width = be16(s + 3);
      H.ncomp = s[5];
      if (H.width == 0 || H.height == 0) return LDT_IMG_NOT_JPEG;
      if (H.ncomp != 1 && H.ncomp != 3) return LDT_IMG_UNSUPPORTED;
      if (e - s < 6 + 3 * H.ncomp) return LDT_IMG_NOT_JPEG;
      for (int c = 0; c < H.ncomp; ++c) {
        H.cid[c] = s[6 + 3 * c];
        H.h[c] = s[7 + 3 * c] >> 4;
        H.v[c] = s[7 + 3 * c] & 15;
        H.tq[c] = s[8 + 3 * c];
        if (H.h[c] < 1 || H.h[c] > 4 || H.v[c] < 1 || H.v[c] > 4 || H.tq[c] > 3)
          return LDT_IMG_NOT_JPEG;
      }
      sof = true;
      break;
    }
    case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA:
    case 0xCB: case 0xCD: case 0xCE: case 0xCF:
      return LDT_IMG_UNSUPPORTED;
    case 0xC4: {
      while (s < e) {
        const int tc = s[0] >> 4, th = s[0] & 15;
        if (tc > 1 || th > 3 || e - s < 17) return LDT_IMG_NOT_JPEG;
        RawHuff &t = tc ? H.ac[th] : H.dc[th];
        int n = 0;
        for (int l = 0; l < 16; ++l) {
          t.counts[l] = s[1 + l];
          n += s[1 + l];
        }
        if (n > 256 || e - s < 17 + n) return LDT_IMG_NOT_JPEG;
        memcpy(t.syms, s + 17, n);
        t.nsym = n;
        t.present = true;
        s += 17 + n;
      }
      break;
    }
    case 0xDB: {
      while (s < e) {
        const int pq = s[0] >> 4, tq = s[0] & 15;
        if (tq > 3 || pq > 1) return LDT_IMG_NOT_JPEG;
        const int need = pq ? 129 : 65;
        if (e - s < need) return LDT_IMG_NOT_JPEG;
        for (int k = 0; k < 64; ++k)
          H.q[tq][kZigzagToNatural[k]] = pq ? (uint16_t)be16(s + 1 + 2 * k) : s[1 + k];
        H.qpresent[tq] = true;
        s += need;
      }
      break;
    }
    case 0xDD:
      if (seglen != 4) return LDT_IMG_NOT_JPEG;
      H.restart = be16(s);
      break;
    case 0xE0:
      if (e - s >= 5 && memcmp(s, "JFIF\0", 5) == 0) H.jfif = true;
      break;
    case 0xEE:
      if (e - s >= 12 && memcmp(s, "Adobe", 5) == 0) {
        H.adobe = true;
        H.adobe_transform = s[11];
      }
      break;
    case 0xDA: {
      if (!sof) return LDT_IMG_NOT_JPEG;
      if (H.progressive) { // every scan is walked by plan_progressive
        H.scan_pos = i - 2;
        return LDT_IMG_OK;
      }
      if (e - s < 1) return LDT_IMG_NOT_JPEG;
      const int ns = s[0];
      if (ns < 1 || ns > 4 || e - s < 4 + 2 * ns) return LDT_IMG_NOT_JPEG;
      if (ns != H.ncomp) return LDT_IMG_UNSUPPORTED; // multi-scan sequential
      bool seen[4] = {false, false, false, false};
      for (int k = 0; k < ns; ++k) {
        int idx = -1;
        for (int c = 0; c < H.ncomp; ++c)
          if (H.cid[c] == s[1 + 2 * k]) idx = c;
        // jdmarker.c get_sos: unknown or repeated component -> JERR_BAD_COMPONENT_ID
        if (idx < 0 || seen[idx]) return LDT_IMG_NOT_JPEG;
        seen[idx] = true;
        H.td[idx] = s[2 + 2 * k] >> 4;
        H.ta[idx] = s[2 + 2 * k] & 15;
        if (H.td[idx] > 3 || H.ta[idx] > 3) return LDT_IMG_NOT_JPEG;
      }
      if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0)
        return LDT_IMG_UNSUPPORTED;
      H.scan_pos = i + seglen;
      return LDT_IMG_OK;
    }
    default:
      break;
    }
    i += seglen;
  }
}

// jdhuff.c jpeg_make_d_derived_tbl restated into the device table layout
// (canonical code assignment, then the two-level lookup of ldt_types.hpp).
bool build_huff(const RawHuff &r, bool is_dc, HuffTab &t) {
  memset(&t, 0, sizeof(t));
  int code = 0, k = 0;
  int lens[256];
  int codes[256];
  for (int l = 1; l <= 16; ++l) {
    const int cnt = r.counts[l - 1];
    if (cnt) {
      t.valoff[l] = k - code;
      for (int j = 0; j < cnt; ++j) {
        lens[k] = l;
        codes[k] = code;
        ++k;
        ++code;
      }
      t.maxcode[l] = code - 1;
    } else {
      t.maxcode[l] = -1;
    }
    if (cnt && code >= (1 << l)) return false; // all-ones code: JERR_BAD_HUFF_TABLE
    code <<= 1;
  }
  t.maxcode[17] = 0x7FFFFFFF;
  for (int j = 0; j < r.nsym; ++j) {
    t.vals[j] = r.syms[j];
    if (is_dc && r.syms[j] > 15) return false;
  }
  // level 1 (unused codes: the invalid entry)
  const uint16_t invalid = huff_entry(16, 0, is_dc);
  static thread_local uint16_t l1[1 << kLookBits];
  for (int q = 0; q < (1 << kLookBits); ++q) l1[q] = invalid;
  for (int q = 0; q < (kL2Chunks << kL2Bits); ++q) t.l2[q] = invalid;
  for (int j = 0; j < r.nsym; ++j) {
    if (lens[j] <= kLookBits) {
      const int shift = kLookBits - lens[j];
      const int base = codes[j] << shift;
      for (int q = 0; q < (1 << shift); ++q) l1[base + q] = huff_entry(lens[j], r.syms[j], is_dc);
    }
  }
  // level 2: one chunk per distinct kLookBits-bit prefix of a longer code
  int prefix_chunk[1 << kLookBits];
  for (int q = 0; q < (1 << kLookBits); ++q) prefix_chunk[q] = -1;
  int nchunks = 0;
  bool overflow = false;
  for (int j = 0; j < r.nsym; ++j) {
    if (lens[j] <= kLookBits) continue;
    const int pre = codes[j] >> (lens[j] - kLookBits);
    if (prefix_chunk[pre] < 0) {
      if (nchunks < kL2Chunks) prefix_chunk[pre] = nchunks++;
      else overflow = true;
    }
  }
  for (int j = 0; j < r.nsym && !overflow; ++j) {
    if (lens[j] <= kLookBits) continue;
    const int pre = codes[j] >> (lens[j] - kLookBits);
    const int rest = lens[j] - kLookBits; // 1..kL2Bits bits after the prefix
    const int sub = (codes[j] & ((1 << rest) - 1)) << (kL2Bits - rest);
    for (int q = 0; q < (1 << (kL2Bits - rest)); ++q)
      t.l2[(prefix_chunk[pre] << kL2Bits) + sub + q] = huff_entry(lens[j], r.syms[j], is_dc);
  }
  for (int q = 0; q < (1 << kLookBits); ++q)
    if (prefix_chunk[q] >= 0) l1[q] = overflow ? (uint16_t)kHuffCanon : (uint16_t)(prefix_chunk[q] << 5);
  if (overflow) // every long-code prefix takes the canonical search
    for (int j = 0; j < r.nsym; ++j)
      if (lens[j] > kLookBits) l1[codes[j] >> (lens[j] - kLookBits)] = (uint16_t)kHuffCanon;
  // count-mode entries (ldt_types.hpp HuffTab): runs of AC symbols whose
  // codes all lie in the kLookBits peeked bits
  const uint32_t mask = (1u << kLookBits) - 1;
  for (uint32_t x = 0; x <= mask; ++x) {
    const uint32_t e = l1[x];
    uint32_t T = e & 31;
    if (T == 0) {
      t.lc[x] = e | (e << 16); // long code: the count entry is l1's indirect entry
      continue;
    }
    uint32_t adv = e >> 9, pre = 0;
    while (!is_dc && adv < 64 && adv <= 15 && T < (uint32_t)kLookBits) {
      const uint32_t e2 = l1[(x << T) & mask];
      const uint32_t t2 = e2 & 31;
      if (t2 == 0 || T + (t2 - ((e2 >> 5) & 15)) > (uint32_t)kLookBits) break; // code past the peek
      pre = adv;
      adv += e2 >> 9;
      T += t2;
    }
    t.lc[x] = e | ((T | (pre << 5) | (adv << 9)) << 16);
  }
  return true;
}

std::string huff_key(const RawHuff &r, bool dc) {
  std::string k(1, dc ? 'D' : 'A');
  k.append(reinterpret_cast<const char *>(r.counts), 16);
  k.append(reinterpret_cast<const char *>(r.syms), r.nsym);
  return k;
}

// ---- progressive (SOF2) planning ----------------------------------------
// The end of a scan's entropy-coded data: the first j >= start (j + 1 < len)
// with cell[j] == 0xFF and cell[j + 1] not 0x00 (stuffing), 0xFF (fill) or
// RSTn; len when there is none. 16 positions per step with SSE2 (the host
// planner cost 5.8 ms per 256-image c2p batch with a byte loop, ~1.5 ms with
// memchr hopping from one stuffed 0xFF to the next).
static int64_t scan_end(const uint8_t *cell, int64_t start, int64_t len) {
  int64_t j = start;
  const __m128i ff = _mm_set1_epi8((char)0xFF), zero = _mm_setzero_si128();
  const __m128i f8 = _mm_set1_epi8((char)0xF8), d0 = _mm_set1_epi8((char)0xD0);
  for (; j + 17 <= len; j += 16) {
    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i *>(cell + j));
    const __m128i y = _mm_loadu_si128(reinterpret_cast<const __m128i *>(cell + j + 1));
    const __m128i keep = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(y, zero), _mm_cmpeq_epi8(y, ff)),
                                      _mm_cmpeq_epi8(_mm_and_si128(y, f8), d0));
    const int m = _mm_movemask_epi8(_mm_andnot_si128(keep, _mm_cmpeq_epi8(x, ff)));
    if (m) return j + __builtin_ctz((unsigned)m);
  }
  for (; j + 1 < len; ++j) {
    const int nx = cell[j + 1];
    if (cell[j] == 0xFF && nx != 0x00 && nx != 0xFF && !(nx >= 0xD0 && nx <= 0xD7)) return j;
  }
  return len;
}

// Table for k_prog: canonical codes as jdhuff.c jpeg_make_d_derived_tbl
// (same validity checks as build_huff), plus the 8-bit lookahead.
bool build_prog_tab(const RawHuff &r, bool is_dc, ProgTab &t) {
  memset(&t, 0, sizeof(t));
  int code = 0, k = 0;
  int lens[256], codes[256];
  for (int l = 1; l <= 16; ++l) {
    const int cnt = r.counts[l - 1];
    if (cnt) {
      t.valoff[l] = k - code;
      for (int j = 0; j < cnt; ++j, ++k, ++code) {
        lens[k] = l;
        codes[k] = code;
      }
      t.maxcode[l] = code - 1;
    } else {
      t.maxcode[l] = -1;
    }
    if (cnt && code >= (1 << l)) return false; // all-ones code: JERR_BAD_HUFF_TABLE
    code <<= 1;
  }
  t.maxcode[17] = 0x7FFFFFFF;
  for (int j = 0; j < r.nsym; ++j) {
    t.vals[j] = r.syms[j];
    if (is_dc && r.syms[j] > 15) return false;
    if (lens[j] <= 8) {
      const int base = codes[j] << (8 - lens[j]);
      for (int x = 0; x < (1 << (8 - lens[j])); ++x)
        t.look[base + x] = (uint16_t)((lens[j] << 8) | r.syms[j]);
    }
  }
  return true;
}



// Walks every scan of a progressive image from its first SOS (H.scan_pos):
// jdmarker.c between scans (DHT / DQT / DRI), jdphuff.c
// start_pass_phuff_decoder's progression checks, jdinput.c's quant table
// latch at a component's first scan, and the byte range of each scan's
// entropy-coded data (up to the first marker that is not RSTn). Files whose
// coefficients 0..9 are not fully refined after the last scan would take
// libjpeg's block-smoothing path (jdcoefct.c smoothing_ok): unsupported.
// Returns an LDT_IMG_* code.
int plan_progressive(const uint8_t *cell, int64_t len, const Header &H0, ProgPlan &P) {
  Header H = H0;
  int coef_bits[4][10];
  bool latched[4] = {false, false, false, false};
  for (int c = 0; c < 4; ++c)
    for (int k = 0; k < 10; ++k) coef_bits[c][k] = -1;
  int64_t i = H0.scan_pos;
  while (true) {
    if (i + 1 >= len || cell[i] != 0xFF) return LDT_IMG_CORRUPT; // data ended before EOI
    while (i + 1 < len && cell[i + 1] == 0xFF) ++i;
    if (i + 1 >= len) return LDT_IMG_CORRUPT;
    const int m = cell[i + 1];
    i += 2;
    if (m == 0xD9) break;
    if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (i + 2 > len) return LDT_IMG_CORRUPT;
    const int seglen = be16(cell + i);
    if (seglen < 2 || i + seglen > len) return LDT_IMG_CORRUPT;
    const uint8_t *s = cell + i + 2;
    const uint8_t *e = cell + i + seglen;
    if (m == 0xC4) {
      while (s < e) {
        const int tc = s[0] >> 4, th = s[0] & 15;
        if (tc > 1 || th > 3 || e - s < 17) return LDT_IMG_NOT_JPEG;
        RawHuff &t = tc ? H.ac[th] : H.dc[th];
        int n = 0;
        for (int l = 0; l < 16; ++l) {
          t.counts[l] = s[1 + l];
          n += s[1 + l];
        }
        if (n > 256 || e - s < 17 + n) return LDT_IMG_NOT_JPEG;
        memcpy(t.syms, s + 17, n);
        t.nsym = n;
        t.present = true;
        s += 17 + n;
      }
    } else if (m == 0xDB) {
      while (s < e) {
        const int pq = s[0] >> 4, tq = s[0] & 15;
        if (tq > 3 || pq > 1) return LDT_IMG_NOT_JPEG;
        const int need = pq ? 129 : 65;
        if (e - s < need) return LDT_IMG_NOT_JPEG;
        for (int k = 0; k < 64; ++k)
          H.q[tq][kZigzagToNatural[k]] = pq ? (uint16_t)be16(s + 1 + 2 * k) : s[1 + k];
        H.qpresent[tq] = true;
        s += need;
      }
    } else if (m == 0xDD) {
      if (seglen != 4) return LDT_IMG_NOT_JPEG;
      H.restart = be16(s);
    } else if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return LDT_IMG_NOT_JPEG; // a second frame header
    } else if (m == 0xDA) {
      if (e - s < 1) return LDT_IMG_NOT_JPEG;
      const int ns = s[0];
      if (ns < 1 || ns > 4 || e - s < 4 + 2 * ns) return LDT_IMG_NOT_JPEG;
      ProgScan sc;
      memset(&sc, 0, sizeof(sc));
      sc.ns = ns;
      sc.ss = s[1 + 2 * ns];
      sc.se = s[2 + 2 * ns];
      sc.ah = s[3 + 2 * ns] >> 4;
      sc.al = s[3 + 2 * ns] & 15;
      sc.restart = H.restart;
      const bool dcband = sc.ss == 0;
      bool bad = dcband ? sc.se != 0 : (sc.ss > sc.se || sc.se > 63 || ns != 1);
      if (sc.ah != 0 && sc.al != sc.ah - 1) bad = true;
      if (sc.al > 13) bad = true;
      if (bad) return LDT_IMG_CORRUPT; // JERR_BAD_PROGRESSION
      for (int k = 0; k < 4; ++k) sc.tab[k] = -1;
      bool seen[4] = {false, false, false, false};
      for (int k = 0; k < ns; ++k) {
        int idx = -1;
        for (int c = 0; c < H.ncomp; ++c)
          if (H.cid[c] == s[1 + 2 * k]) idx = c;
        if (idx < 0 || seen[idx]) return LDT_IMG_NOT_JPEG; // JERR_BAD_COMPONENT_ID
        seen[idx] = true;
        sc.comp[k] = idx;
        const int td = s[2 + 2 * k] >> 4, ta = s[2 + 2 * k] & 15;
        if (td > 3 || ta > 3) return LDT_IMG_NOT_JPEG;
        if (!latched[idx]) {
          if (!H.qpresent[H.tq[idx]]) return LDT_IMG_NOT_JPEG;
          memcpy(P.q[idx], H.q[H.tq[idx]], sizeof(P.q[idx]));
          latched[idx] = true;
        }
        const RawHuff *t = nullptr;
        bool is_dc = false;
        if (dcband && sc.ah == 0) {
          t = &H.dc[td];
          is_dc = true;
        } else if (!dcband && k == 0) {
          t = &H.ac[ta];
        }
        if (t) {
          if (!t->present) return LDT_IMG_NOT_JPEG;
          sc.tab[k] = (int32_t)P.tabs.size();
          P.tabs.emplace_back(*t, is_dc);
        }
        for (int q = sc.ss; q <= sc.se && q < 10; ++q) coef_bits[idx][q] = sc.al;
      }
      const int64_t start = i + seglen;
      const int64_t j = scan_end(cell, start, len);
      if (j + 1 >= len) return LDT_IMG_CORRUPT; // truncated inside the scan
      if (j - start > (int64_t)INT32_MAX - 64) return LDT_IMG_UNSUPPORTED; // k_prog's offsets are int32
      sc.data_off = start;
      sc.data_len = j - start;
      P.scans.push_back(sc);
      if ((int)P.scans.size() > kMaxProgScans) return LDT_IMG_UNSUPPORTED;
      i = j;
      continue;
    }
    i += seglen;
  }
  for (int c = 0; c < H.ncomp; ++c) {
    if (!latched[c]) return LDT_IMG_NOT_JPEG;
    for (int k = 0; k < 10; ++k)
      if (coef_bits[c][k] != 0) return LDT_IMG_UNSUPPORTED; // would be block-smoothed
  }
  return LDT_IMG_OK;
}


} // namespace ldt

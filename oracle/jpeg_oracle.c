/*
 * oracle/jpeg_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot path's arithmetic, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.
 * Nothing in the product (lance-distributed-training_amd/) links, loads or
 * calls this file; the product fails loudly without its HIP library.
 *
 * What it restates (reference call sites in /root/reference):
 *   lance_iterable.py:42 / lance_map_style.py:36
 *       Image.open(io.BytesIO(b)).convert("RGB")
 *       -> Pillow 12.2.0 JpegDecode -> libjpeg-turbo 3.1.4.1 defaults:
 *          jdhuff.c   (baseline Huffman decode, DC prediction, restart markers)
 *          jdphuff.c  (progressive SOF2: DC/AC first and refinement scans,
 *                      EOB runs; jdcoefct.c buffers all scans, then one IDCT)
 *          jidctint.c (JDCT_ISLOW, CONST_BITS 13, PASS1_BITS 2, range-limit table)
 *          jdsample.c (h2v2 / h2v1 fancy upsampling, box when width <= 2)
 *          jdmainct.c (context rows: replicated first/last chroma rows)
 *          jdcolor.c  (YCbCr->RGB, 16-bit fixed-point tables)
 *   lance_iterable.py:29 / lance_map_style.py:30  transforms.Resize((224,224))
 *       -> PIL.Image.resize((224,224), BILINEAR) -> Pillow Resample.c
 *          (precompute_coeffs, normalize_coeffs_8bpc, PRECISION_BITS 22,
 *           horizontal pass then vertical pass with a uint8 intermediate)
 *   lance_iterable.py:30 / lance_map_style.py:31  transforms.ToTensor()
 *       -> HWC uint8 -> CHW float32, IEEE x / 255.0f
 *   lance_iterable.py:31 (commented out) transforms.Normalize(mean, std)
 *       -> (x - mean_c) / std_c in float32
 *   lance_iterable.py:46-48 torch.stack / torch.tensor(labels, long)
 *
 * The third-party sources are not in the container; this is a
 * restatement of their published algorithms, pinned bit-exact against the
 * Pillow/libjpeg-turbo binaries present here by tests/golden (see
 * tests/golden/make_golden.py and tests/test_oracle.py).
 *
 * Plain C99, scalar, single-threaded.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_ERR_FORMAT -1      /* not a JPEG / malformed marker structure */
#define ORC_ERR_UNSUPPORTED -2 /* arithmetic, lossless, 12-bit, CMYK ...    */
#define ORC_ERR_TRUNCATED -3   /* entropy data ends before the last MCU     */
#define ORC_ERR_NOMEM -4

/* ------------------------------------------------------------------------ */
/* Marker parsing (libjpeg jdmarker.c semantics for the baseline subset).    */
/* ------------------------------------------------------------------------ */

typedef struct {
  uint8_t bits[17];    /* bits[l] = number of codes of length l          */
  uint8_t vals[256];
  int present;
  /* derived (jdhuff.c jpeg_make_d_derived_tbl) */
  int32_t maxcode[18]; /* largest code of length l, -1 if none; [17] sentinel */
  int32_t valoffset[18];
} orc_huff;

typedef struct {
  int id, h, v, tq, td, ta;
  int bw, bh;            /* blocks per row / column in the (padded) plane */
  int dw, dh;            /* downsampled_width / downsampled_height         */
  uint8_t *plane;        /* bw*8 x bh*8 samples                            */
} orc_comp;

typedef struct {
  int width, height, ncomp;
  orc_comp comp[4];
  uint16_t qt[4][64];    /* natural order */
  int qt_present[4];
  orc_huff dc[4], ac[4];
  int restart_interval;
  int hmax, vmax;
  int saw_jfif, saw_adobe, adobe_transform;
  const uint8_t *scan;   /* first byte of entropy-coded data */
  const uint8_t *end;
  int scan_ncomp, scan_comp[4];
  int progressive;       /* SOF2 */
  const uint8_t *sos;    /* progressive: the first SOS marker (FF DA) */
} orc_jpeg;

/* jpeg_natural_order (jutils.c): zigzag index -> natural index */
static const int orc_natural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    /* extra entries for safety in decoder (run past 63) */
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

static int rd16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

static void orc_derive_huff(orc_huff *t) {
  /* Canonical code assignment (ITU T.81 Annex C; jdhuff.c make_d_derived_tbl) */
  int code = 0, k = 0;
  for (int l = 1; l <= 16; l++) {
    if (t->bits[l]) {
      t->valoffset[l] = k - code;
      code += t->bits[l];
      k += t->bits[l];
      t->maxcode[l] = code - 1;
    } else {
      t->maxcode[l] = -1;
    }
    code <<= 1;
  }
  t->maxcode[17] = 0x7FFFFFFF; /* sentinel: ensures termination */
}

static int orc_parse(const uint8_t *d, size_t len, orc_jpeg *j) {
  memset(j, 0, sizeof(*j));
  const uint8_t *p = d, *e = d + len;
  if (len < 4 || p[0] != 0xFF || p[1] != 0xD8) return ORC_ERR_FORMAT;
  p += 2;
  int have_sof = 0;
  for (;;) {
    /* skip fill bytes */
    if (p + 2 > e) return ORC_ERR_FORMAT;
    if (p[0] != 0xFF) return ORC_ERR_FORMAT;
    while (p < e && p[0] == 0xFF && p + 1 < e && p[1] == 0xFF) p++;
    if (p + 2 > e) return ORC_ERR_FORMAT;
    int m = p[1];
    p += 2;
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) return ORC_ERR_FORMAT; /* EOI before SOS */
    if (p + 2 > e) return ORC_ERR_FORMAT;
    int L = rd16(p);
    if (L < 2 || p + L > e) return ORC_ERR_FORMAT;
    const uint8_t *s = p + 2, *se = p + L;
    switch (m) {
    case 0xC0: case 0xC1: case 0xC2: { /* SOF0 baseline / SOF1 extended / SOF2 progressive */
      j->progressive = m == 0xC2;
      if (se - s < 6) return ORC_ERR_FORMAT;
      if (s[0] != 8) return ORC_ERR_UNSUPPORTED; /* 12-bit */
      j->height = rd16(s + 1);
      j->width = rd16(s + 3);
      j->ncomp = s[5];
      if (j->width <= 0 || j->height <= 0) return ORC_ERR_FORMAT;
      if (j->ncomp != 1 && j->ncomp != 3) return ORC_ERR_UNSUPPORTED;
      if (se - s < 6 + 3 * j->ncomp) return ORC_ERR_FORMAT;
      for (int c = 0; c < j->ncomp; c++) {
        j->comp[c].id = s[6 + 3 * c];
        j->comp[c].h = s[7 + 3 * c] >> 4;
        j->comp[c].v = s[7 + 3 * c] & 15;
        j->comp[c].tq = s[8 + 3 * c];
        if (j->comp[c].h < 1 || j->comp[c].h > 4 || j->comp[c].v < 1 ||
            j->comp[c].v > 4 || j->comp[c].tq > 3)
          return ORC_ERR_FORMAT;
      }
      have_sof = 1;
      break;
    }
    case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9:
    case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
      return ORC_ERR_UNSUPPORTED; /* progressive / lossless / arithmetic */
    case 0xC4: { /* DHT */
      while (s < se) {
        int tc = s[0] >> 4, th = s[0] & 15;
        if (tc > 1 || th > 3 || se - s < 17) return ORC_ERR_FORMAT;
        orc_huff *t = tc ? &j->ac[th] : &j->dc[th];
        int count = 0;
        t->bits[0] = 0;
        for (int l = 1; l <= 16; l++) { t->bits[l] = s[l]; count += s[l]; }
        if (count > 256 || se - s < 17 + count) return ORC_ERR_FORMAT;
        memcpy(t->vals, s + 17, count);
        t->present = 1;
        orc_derive_huff(t);
        s += 17 + count;
      }
      break;
    }
    case 0xDB: { /* DQT */
      while (s < se) {
        int pq = s[0] >> 4, tq = s[0] & 15;
        if (tq > 3) return ORC_ERR_FORMAT;
        if (pq == 0) {
          if (se - s < 65) return ORC_ERR_FORMAT;
          for (int k = 0; k < 64; k++) j->qt[tq][orc_natural[k]] = s[1 + k];
          s += 65;
        } else {
          if (se - s < 129) return ORC_ERR_FORMAT;
          for (int k = 0; k < 64; k++) j->qt[tq][orc_natural[k]] = (uint16_t)rd16(s + 1 + 2 * k);
          s += 129;
        }
        j->qt_present[tq] = 1;
      }
      break;
    }
    case 0xDD: /* DRI */
      if (L != 4) return ORC_ERR_FORMAT;
      j->restart_interval = rd16(s);
      break;
    case 0xE0: /* APP0: JFIF? (jdmarker.c examine_app0) */
      if (se - s >= 5 && memcmp(s, "JFIF\0", 5) == 0) j->saw_jfif = 1;
      break;
    case 0xEE: /* APP14: Adobe? (examine_app14) */
      if (se - s >= 12 && memcmp(s, "Adobe", 5) == 0) {
        j->saw_adobe = 1;
        j->adobe_transform = s[11];
      }
      break;
    case 0xDA: { /* SOS */
      if (!have_sof) return ORC_ERR_FORMAT;
      if (j->progressive) { /* every scan is parsed by orc_decode_prog */
        j->sos = p - 2;
        j->end = e;
        return ORC_OK;
      }
      int ns = s[0];
      if (ns < 1 || ns > 4 || se - s < 1 + 2 * ns + 3) return ORC_ERR_FORMAT;
      j->scan_ncomp = ns;
      for (int i = 0; i < ns; i++) {
        int cid = s[1 + 2 * i], ci = -1;
        for (int c = 0; c < j->ncomp; c++)
          if (j->comp[c].id == cid) ci = c;
        if (ci < 0) return ORC_ERR_FORMAT;
        j->scan_comp[i] = ci;
        j->comp[ci].td = s[2 + 2 * i] >> 4;
        j->comp[ci].ta = s[2 + 2 * i] & 15;
        if (j->comp[ci].td > 3 || j->comp[ci].ta > 3) return ORC_ERR_FORMAT;
      }
      int Ss = s[1 + 2 * ns], Se = s[2 + 2 * ns], AhAl = s[3 + 2 * ns];
      if (Ss != 0 || Se != 63 || AhAl != 0) return ORC_ERR_UNSUPPORTED;
      /* Only single-scan images (all components in one scan) are baseline-
       * sequential as Pillow writes them; multi-scan sequential -> unsupported. */
      if (ns != j->ncomp) return ORC_ERR_UNSUPPORTED;
      j->scan = se;
      j->end = e;
      return ORC_OK;
    }
    default:
      break; /* APPn, COM, ... skipped */
    }
    p += L;
  }
}

/* ------------------------------------------------------------------------ */
/* Entropy decoding (jdhuff.c): bit buffer with byte stuffing; at a marker   */
/* the reader inserts zero bits (jdhuff.c jpeg_fill_bit_buffer).             */
/* ------------------------------------------------------------------------ */

typedef struct {
  const uint8_t *p, *e;
  uint64_t buf;
  int bits;
  int hit_marker;
  int marker;
  long zero_fill_bits; /* bits synthesised past a marker / end of data */
} orc_br;

static void orc_fill(orc_br *b) {
  while (b->bits <= 56) {
    int c = 0;
    if (!b->hit_marker) {
      if (b->p >= b->e) {
        b->hit_marker = 1;
        b->marker = -1;
      } else {
        c = *b->p++;
        if (c == 0xFF) {
          /* skip FF fill bytes */
          int c2;
          do {
            c2 = (b->p < b->e) ? *b->p++ : -1;
          } while (c2 == 0xFF);
          if (c2 == 0) {
            c = 0xFF;
          } else {
            b->hit_marker = 1;
            b->marker = c2;
            c = 0;
          }
        }
      }
    }
    if (b->hit_marker) {
      c = 0;
      b->zero_fill_bits += 8;
    }
    b->buf |= (uint64_t)c << (56 - b->bits);
    b->bits += 8;
  }
}

static unsigned orc_peek(orc_br *b, int n) {
  if (b->bits < n) orc_fill(b);
  return (unsigned)(b->buf >> (64 - n));
}
static void orc_skip(orc_br *b, int n) {
  b->buf <<= n;
  b->bits -= n;
}
static unsigned orc_get(orc_br *b, int n) {
  if (n == 0) return 0;
  unsigned v = orc_peek(b, n);
  orc_skip(b, n);
  return v;
}

static int orc_huff_decode(orc_br *b, const orc_huff *t) {
  /* jdhuff.c jpeg_huff_decode: code lengths 1..16, canonical codes */
  unsigned w = orc_peek(b, 16);
  for (int l = 1; l <= 16; l++) {
    int code = (int)(w >> (16 - l));
    if (code <= t->maxcode[l]) {
      orc_skip(b, l);
      return t->vals[(t->valoffset[l] + code) & 0xFF];
    }
  }
  /* corrupt data: libjpeg warns "Corrupt JPEG data: bad Huffman code" and
   * returns 0; we do the same, skipping 16 bits. */
  orc_skip(b, 16);
  return 0;
}

/* HUFF_EXTEND (jdhuff.h) */
static int orc_extend(unsigned v, int s) {
  return (s == 0) ? 0 : ((int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v);
}

/* libjpeg process_restart: discard to byte boundary, consume RSTn marker. */
static void orc_restart(orc_br *b) {
  b->buf = 0;
  b->bits = 0;
  if (b->hit_marker && b->marker >= 0xD0 && b->marker <= 0xD7) {
    b->hit_marker = 0;
    b->marker = 0;
    return;
  }
  /* Find the next marker in the raw stream (valid streams: next bytes). */
  while (b->p + 1 < b->e) {
    if (b->p[0] == 0xFF && b->p[1] >= 0xD0 && b->p[1] <= 0xD7) {
      b->p += 2;
      return;
    }
    if (b->p[0] == 0xFF && b->p[1] != 0x00 && b->p[1] != 0xFF) return;
    b->p++;
  }
}

/* ------------------------------------------------------------------------ */
/* Inverse DCT: jidctint.c jpeg_idct_islow (libjpeg 6b / libjpeg-turbo).     */
/* ------------------------------------------------------------------------ */
#define CONST_BITS 13
#define PASS1_BITS 2
#define FIX_0_298631336 2446
#define FIX_0_390180644 3196
#define FIX_0_541196100 4433
#define FIX_0_765366865 6270
#define FIX_0_899976223 7373
#define FIX_1_175875602 9633
#define FIX_1_501321110 12299
#define FIX_1_847759065 15137
#define FIX_1_961570560 16069
#define FIX_2_053119869 16819
#define FIX_2_562915447 20995
#define FIX_3_072711026 25172
#define DESCALE(x, n) (((x) + (1L << ((n)-1))) >> (n))

/* jdmaster.c prepare_range_limit_table, post-IDCT half: index (x & 1023). */
static uint8_t orc_idct_limit(int32_t x) {
  int i = x & 1023;
  if (i < 128) return (uint8_t)(i + 128);
  if (i < 512) return 255;
  if (i < 896) return 0;
  return (uint8_t)(i - 896);
}

static void orc_idct_islow(const int16_t *coef, const uint16_t *q, uint8_t *out, int stride) {
  int32_t ws[64];
  for (int c = 0; c < 8; c++) {
    const int16_t *in = coef + c;
    const uint16_t *qp = q + c;
    int32_t tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13, z1, z2, z3, z4, z5;
    if (in[8] == 0 && in[16] == 0 && in[24] == 0 && in[32] == 0 && in[40] == 0 &&
        in[48] == 0 && in[56] == 0) {
      int32_t dc = ((int32_t)in[0] * qp[0]) * (1 << PASS1_BITS);
      for (int r = 0; r < 8; r++) ws[r * 8 + c] = dc;
      continue;
    }
    z2 = (int32_t)in[16] * qp[16];
    z3 = (int32_t)in[48] * qp[48];
    z1 = (z2 + z3) * FIX_0_541196100;
    tmp2 = z1 + z3 * (-FIX_1_847759065);
    tmp3 = z1 + z2 * FIX_0_765366865;
    z2 = (int32_t)in[0] * qp[0];
    z3 = (int32_t)in[32] * qp[32];
    tmp0 = (z2 + z3) * (1 << CONST_BITS);
    tmp1 = (z2 - z3) * (1 << CONST_BITS);
    tmp10 = tmp0 + tmp3;
    tmp13 = tmp0 - tmp3;
    tmp11 = tmp1 + tmp2;
    tmp12 = tmp1 - tmp2;
    tmp0 = (int32_t)in[56] * qp[56];
    tmp1 = (int32_t)in[40] * qp[40];
    tmp2 = (int32_t)in[24] * qp[24];
    tmp3 = (int32_t)in[8] * qp[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    z4 = tmp1 + tmp3;
    z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 = tmp0 * FIX_0_298631336;
    tmp1 = tmp1 * FIX_2_053119869;
    tmp2 = tmp2 * FIX_3_072711026;
    tmp3 = tmp3 * FIX_1_501321110;
    z1 = z1 * (-FIX_0_899976223);
    z2 = z2 * (-FIX_2_562915447);
    z3 = z3 * (-FIX_1_961570560);
    z4 = z4 * (-FIX_0_390180644);
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    ws[0 * 8 + c] = (int32_t)DESCALE(tmp10 + tmp3, CONST_BITS - PASS1_BITS);
    ws[7 * 8 + c] = (int32_t)DESCALE(tmp10 - tmp3, CONST_BITS - PASS1_BITS);
    ws[1 * 8 + c] = (int32_t)DESCALE(tmp11 + tmp2, CONST_BITS - PASS1_BITS);
    ws[6 * 8 + c] = (int32_t)DESCALE(tmp11 - tmp2, CONST_BITS - PASS1_BITS);
    ws[2 * 8 + c] = (int32_t)DESCALE(tmp12 + tmp1, CONST_BITS - PASS1_BITS);
    ws[5 * 8 + c] = (int32_t)DESCALE(tmp12 - tmp1, CONST_BITS - PASS1_BITS);
    ws[3 * 8 + c] = (int32_t)DESCALE(tmp13 + tmp0, CONST_BITS - PASS1_BITS);
    ws[4 * 8 + c] = (int32_t)DESCALE(tmp13 - tmp0, CONST_BITS - PASS1_BITS);
  }
  for (int r = 0; r < 8; r++) {
    const int32_t *w = ws + r * 8;
    uint8_t *o = out + r * stride;
    int32_t tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13, z1, z2, z3, z4, z5;
    if (w[1] == 0 && w[2] == 0 && w[3] == 0 && w[4] == 0 && w[5] == 0 && w[6] == 0 &&
        w[7] == 0) {
      uint8_t dc = orc_idct_limit((int32_t)DESCALE(w[0], PASS1_BITS + 3));
      for (int c = 0; c < 8; c++) o[c] = dc;
      continue;
    }
    z2 = w[2];
    z3 = w[6];
    z1 = (z2 + z3) * FIX_0_541196100;
    tmp2 = z1 + z3 * (-FIX_1_847759065);
    tmp3 = z1 + z2 * FIX_0_765366865;
    tmp0 = (w[0] + w[4]) * (1 << CONST_BITS);
    tmp1 = (w[0] - w[4]) * (1 << CONST_BITS);
    tmp10 = tmp0 + tmp3;
    tmp13 = tmp0 - tmp3;
    tmp11 = tmp1 + tmp2;
    tmp12 = tmp1 - tmp2;
    tmp0 = w[7];
    tmp1 = w[5];
    tmp2 = w[3];
    tmp3 = w[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    z4 = tmp1 + tmp3;
    z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 = tmp0 * FIX_0_298631336;
    tmp1 = tmp1 * FIX_2_053119869;
    tmp2 = tmp2 * FIX_3_072711026;
    tmp3 = tmp3 * FIX_1_501321110;
    z1 = z1 * (-FIX_0_899976223);
    z2 = z2 * (-FIX_2_562915447);
    z3 = z3 * (-FIX_1_961570560);
    z4 = z4 * (-FIX_0_390180644);
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    const int sh = CONST_BITS + PASS1_BITS + 3;
    o[0] = orc_idct_limit((int32_t)DESCALE(tmp10 + tmp3, sh));
    o[7] = orc_idct_limit((int32_t)DESCALE(tmp10 - tmp3, sh));
    o[1] = orc_idct_limit((int32_t)DESCALE(tmp11 + tmp2, sh));
    o[6] = orc_idct_limit((int32_t)DESCALE(tmp11 - tmp2, sh));
    o[2] = orc_idct_limit((int32_t)DESCALE(tmp12 + tmp1, sh));
    o[5] = orc_idct_limit((int32_t)DESCALE(tmp12 - tmp1, sh));
    o[3] = orc_idct_limit((int32_t)DESCALE(tmp13 + tmp0, sh));
    o[4] = orc_idct_limit((int32_t)DESCALE(tmp13 - tmp0, sh));
  }
}

/* ------------------------------------------------------------------------ */
/* Progressive decode (SOF2): jdphuff.c restated. Every scan updates one      */
/* coefficient array per component (jdcoefct.c full-image buffer); the IDCT  */
/* runs once after the last scan. Block smoothing (jdcoefct.c                */
/* decompress_smooth_data) only applies while coefficients 1..9 are not      */
/* fully refined; such files are reported unsupported.                       */
/* ------------------------------------------------------------------------ */

typedef struct {
  int16_t *coef[4];        /* per component: bw*bh blocks x 64, natural order */
  int coef_bits[4][64];    /* jdphuff.c cinfo->coef_bits: Al of the last scan, -1 never */
} orc_prog;

/* One AC refinement correction bit on an already-nonzero coefficient. */
static void orc_refine_bit(orc_br *b, int16_t *c, int p1, int m1) {
  if (orc_get(b, 1)) {
    if ((*c & p1) == 0) *c = (int16_t)(*c >= 0 ? *c + p1 : *c + m1);
  }
}

/* One scan: header at sos (FF DA), entropy data after it. Returns the first
 * byte after the scan's data (the next marker) or NULL on error. */
static const uint8_t *orc_prog_scan(orc_jpeg *j, orc_prog *pg, const uint8_t *sos, int *err) {
  const uint8_t *e = j->end;
  if (sos + 4 > e) { *err = ORC_ERR_FORMAT; return NULL; }
  int L = rd16(sos + 2);
  const uint8_t *s = sos + 4, *se = sos + 2 + L;
  if (L < 2 || se > e) { *err = ORC_ERR_FORMAT; return NULL; }
  int ns = s[0];
  if (ns < 1 || ns > 4 || se - s < 1 + 2 * ns + 3) { *err = ORC_ERR_FORMAT; return NULL; }
  int comp[4];
  for (int i = 0; i < ns; i++) {
    int cid = s[1 + 2 * i], ci = -1;
    for (int c = 0; c < j->ncomp; c++)
      if (j->comp[c].id == cid) ci = c;
    if (ci < 0) { *err = ORC_ERR_FORMAT; return NULL; }
    comp[i] = ci;
    j->comp[ci].td = s[2 + 2 * i] >> 4;
    j->comp[ci].ta = s[2 + 2 * i] & 15;
    if (j->comp[ci].td > 3 || j->comp[ci].ta > 3) { *err = ORC_ERR_FORMAT; return NULL; }
  }
  int Ss = s[1 + 2 * ns], Se = s[2 + 2 * ns], Ah = s[3 + 2 * ns] >> 4, Al = s[3 + 2 * ns] & 15;
  /* jdphuff.c start_pass_phuff_decoder: JERR_BAD_PROGRESSION cases */
  int dcband = Ss == 0, bad = 0;
  if (dcband) { if (Se != 0) bad = 1; }
  else if (Ss > Se || Se > 63 || ns != 1) bad = 1;
  if (Ah != 0 && Al != Ah - 1) bad = 1;
  if (Al > 13) bad = 1;
  if (bad) { *err = ORC_ERR_FORMAT; return NULL; }
  for (int i = 0; i < ns; i++) {
    orc_comp *cp = &j->comp[comp[i]];
    if (dcband && Ah == 0 && !j->dc[cp->td].present) { *err = ORC_ERR_FORMAT; return NULL; }
    if (!dcband && !j->ac[cp->ta].present) { *err = ORC_ERR_FORMAT; return NULL; }
    for (int k = Ss; k <= Se; k++) pg->coef_bits[comp[i]][k] = Al;
  }
  int mcux, mcuy;
  if (ns == 1) { /* non-interleaved: the component's own block grid */
    orc_comp *cp = &j->comp[comp[0]];
    mcux = (int)(((long)j->width * cp->h + 8L * j->hmax - 1) / (8L * j->hmax));
    mcuy = (int)(((long)j->height * cp->v + 8L * j->vmax - 1) / (8L * j->vmax));
  } else {
    mcux = (j->width + 8 * j->hmax - 1) / (8 * j->hmax);
    mcuy = (j->height + 8 * j->vmax - 1) / (8 * j->vmax);
  }
  orc_br br;
  memset(&br, 0, sizeof(br));
  br.p = se;
  br.e = e;
  int pred[4] = {0, 0, 0, 0};
  long eobrun = 0, total = (long)mcux * mcuy, left = j->restart_interval;
  const int p1 = 1 << Al, m1 = -1 * (1 << Al);
  for (long m = 0; m < total; m++) {
    if (j->restart_interval) {
      if (left == 0) {
        orc_restart(&br);
        pred[0] = pred[1] = pred[2] = pred[3] = 0;
        eobrun = 0;
        left = j->restart_interval;
      }
      left--;
    }
    int mx = (int)(m % mcux), my = (int)(m / mcux);
    for (int i = 0; i < ns; i++) {
      orc_comp *cp = &j->comp[comp[i]];
      int nbh = ns == 1 ? 1 : cp->h, nbv = ns == 1 ? 1 : cp->v;
      for (int by = 0; by < nbv; by++)
        for (int bx = 0; bx < nbh; bx++) {
          int gx = ns == 1 ? mx : mx * cp->h + bx, gy = ns == 1 ? my : my * cp->v + by;
          int16_t *blk = pg->coef[comp[i]] + ((size_t)gy * cp->bw + gx) * 64;
          if (dcband && Ah == 0) { /* decode_mcu_DC_first */
            int t = orc_huff_decode(&br, &j->dc[cp->td]);
            int diff = orc_extend(orc_get(&br, t), t);
            pred[i] += diff;
            blk[0] = (int16_t)(pred[i] * (1 << Al));
          } else if (dcband) { /* decode_mcu_DC_refine */
            if (orc_get(&br, 1)) blk[0] = (int16_t)(blk[0] | p1);
          } else if (Ah == 0) { /* decode_mcu_AC_first */
            if (eobrun > 0) {
              eobrun--;
              continue;
            }
            for (int k = Ss; k <= Se; k++) {
              int rs = orc_huff_decode(&br, &j->ac[cp->ta]);
              int r = rs >> 4, t = rs & 15;
              if (t) {
                k += r;
                int v = orc_extend(orc_get(&br, t), t);
                blk[orc_natural[k]] = (int16_t)(v * (1 << Al));
              } else if (r == 15) {
                k += 15;
              } else {
                eobrun = 1L << r;
                if (r) eobrun += orc_get(&br, r);
                eobrun--;
                break;
              }
            }
          } else { /* decode_mcu_AC_refine */
            int k = Ss;
            if (eobrun == 0) {
              for (; k <= Se; k++) {
                int rs = orc_huff_decode(&br, &j->ac[cp->ta]);
                int r = rs >> 4, t = rs & 15, sv = 0;
                if (t) {
                  sv = orc_get(&br, 1) ? p1 : m1; /* t != 1: libjpeg warns, same decode */
                } else if (r != 15) {
                  eobrun = 1L << r;
                  if (r) eobrun += orc_get(&br, r);
                  break;
                }
                do {
                  int16_t *c = &blk[orc_natural[k]];
                  if (*c != 0) orc_refine_bit(&br, c, p1, m1);
                  else if (--r < 0) break;
                  k++;
                } while (k <= Se);
                if (sv) blk[orc_natural[k]] = (int16_t)sv;
              }
            }
            if (eobrun > 0) {
              for (; k <= Se; k++) {
                int16_t *c = &blk[orc_natural[k]];
                if (*c != 0) orc_refine_bit(&br, c, p1, m1);
              }
              eobrun--;
            }
          }
        }
    }
  }
  if (br.hit_marker && br.marker == -1 && br.zero_fill_bits > 64) { *err = ORC_ERR_TRUNCATED; return NULL; }
  /* next marker: the first FF xx after the data that is not stuffing or RSTn */
  const uint8_t *q = se;
  while (q + 1 < e) {
    if (q[0] == 0xFF && q[1] != 0x00 && q[1] != 0xFF && !(q[1] >= 0xD0 && q[1] <= 0xD7)) return q;
    q++;
  }
  *err = ORC_ERR_TRUNCATED;
  return NULL;
}

static int orc_decode_prog(orc_jpeg *j) {
  orc_prog pg;
  memset(&pg, 0, sizeof(pg));
  int rc = ORC_OK;
  for (int c = 0; c < j->ncomp; c++) {
    orc_comp *cp = &j->comp[c];
    pg.coef[c] = (int16_t *)calloc((size_t)cp->bw * cp->bh * 64, sizeof(int16_t));
    if (!pg.coef[c]) { rc = ORC_ERR_NOMEM; goto done; }
    for (int k = 0; k < 64; k++) pg.coef_bits[c][k] = -1;
  }
  /* quant tables latch at a component's first scan (jdinput.c latch_quant_tables) */
  uint16_t qlatch[4][64];
  int latched[4] = {0, 0, 0, 0};
  const uint8_t *p = j->sos, *e = j->end;
  for (;;) {
    if (p + 2 > e || p[0] != 0xFF) { rc = ORC_ERR_TRUNCATED; goto done; }
    while (p + 1 < e && p[1] == 0xFF) p++;
    if (p + 2 > e) { rc = ORC_ERR_TRUNCATED; goto done; }
    int m = p[1];
    if (m == 0xD9) break; /* EOI */
    if (m == 0xDA) {
      /* which components does this scan name? latch their tables first */
      if (p + 5 > e) { rc = ORC_ERR_FORMAT; goto done; }
      int ns = p[4];
      for (int i = 0; i < ns && p + 5 + 2 * i < e; i++)
        for (int c = 0; c < j->ncomp; c++)
          if (j->comp[c].id == p[5 + 2 * i] && !latched[c]) {
            if (!j->qt_present[j->comp[c].tq]) { rc = ORC_ERR_FORMAT; goto done; }
            memcpy(qlatch[c], j->qt[j->comp[c].tq], sizeof(qlatch[c]));
            latched[c] = 1;
          }
      int err = ORC_OK;
      const uint8_t *nx = orc_prog_scan(j, &pg, p, &err);
      if (!nx) { rc = err; goto done; }
      p = nx;
      continue;
    }
    if (p + 4 > e) { rc = ORC_ERR_TRUNCATED; goto done; }
    int L = rd16(p + 2);
    if (L < 2 || p + 2 + L > e) { rc = ORC_ERR_FORMAT; goto done; }
    const uint8_t *s = p + 4, *se = p + 2 + L;
    if (m == 0xC4) {
      while (s < se) {
        int tc = s[0] >> 4, th = s[0] & 15;
        if (tc > 1 || th > 3 || se - s < 17) { rc = ORC_ERR_FORMAT; goto done; }
        orc_huff *t = tc ? &j->ac[th] : &j->dc[th];
        int count = 0;
        for (int l = 1; l <= 16; l++) { t->bits[l] = s[l]; count += s[l]; }
        if (count > 256 || se - s < 17 + count) { rc = ORC_ERR_FORMAT; goto done; }
        memcpy(t->vals, s + 17, count);
        t->present = 1;
        orc_derive_huff(t);
        s += 17 + count;
      }
    } else if (m == 0xDD) {
      if (L != 4) { rc = ORC_ERR_FORMAT; goto done; }
      j->restart_interval = rd16(s);
    } else if (m == 0xDB) {
      while (s < se) {
        int pq = s[0] >> 4, tq = s[0] & 15, need = pq ? 129 : 65;
        if (tq > 3 || se - s < need) { rc = ORC_ERR_FORMAT; goto done; }
        for (int k = 0; k < 64; k++)
          j->qt[tq][orc_natural[k]] = pq ? (uint16_t)rd16(s + 1 + 2 * k) : s[1 + k];
        j->qt_present[tq] = 1;
        s += need;
      }
    }
    p = se;
  }
  for (int c = 0; c < j->ncomp; c++) {
    if (!latched[c]) { rc = ORC_ERR_FORMAT; goto done; }
    for (int k = 0; k < 10; k++)
      if (pg.coef_bits[c][k] != 0) { rc = ORC_ERR_UNSUPPORTED; goto done; } /* would smooth */
  }
  for (int c = 0; c < j->ncomp; c++) {
    orc_comp *cp = &j->comp[c];
    int stride = cp->bw * 8;
    for (int by = 0; by < cp->bh; by++)
      for (int bx = 0; bx < cp->bw; bx++)
        orc_idct_islow(pg.coef[c] + ((size_t)by * cp->bw + bx) * 64, qlatch[c],
                       cp->plane + (size_t)by * 8 * stride + bx * 8, stride);
  }
done:
  for (int c = 0; c < 4; c++) free(pg.coef[c]);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* Full decode to component planes.                                          */
/* ------------------------------------------------------------------------ */

static int orc_decode_planes(orc_jpeg *j) {
  int hmax = 1, vmax = 1;
  for (int c = 0; c < j->ncomp; c++) {
    if (j->comp[c].h > hmax) hmax = j->comp[c].h;
    if (j->comp[c].v > vmax) vmax = j->comp[c].v;
  }
  j->hmax = hmax;
  j->vmax = vmax;
  int mcux, mcuy;
  if (j->ncomp == 1) {
    /* non-interleaved single-component scan: MCU = one block, component dims */
    j->comp[0].h = j->comp[0].v = 1;
    hmax = vmax = 1;
    j->hmax = j->vmax = 1;
    mcux = (j->width + 7) / 8;
    mcuy = (j->height + 7) / 8;
  } else {
    mcux = (j->width + 8 * hmax - 1) / (8 * hmax);
    mcuy = (j->height + 8 * vmax - 1) / (8 * vmax);
  }
  for (int c = 0; c < j->ncomp; c++) {
    orc_comp *cp = &j->comp[c];
    if (!j->progressive) {
      if (!j->qt_present[cp->tq]) return ORC_ERR_FORMAT;
      if (!j->dc[cp->td].present || !j->ac[cp->ta].present) return ORC_ERR_FORMAT;
    }
    cp->bw = mcux * cp->h;
    cp->bh = mcuy * cp->v;
    cp->dw = (int)(((long)j->width * cp->h + hmax - 1) / hmax);
    cp->dh = (int)(((long)j->height * cp->v + vmax - 1) / vmax);
    cp->plane = (uint8_t *)malloc((size_t)cp->bw * 8 * cp->bh * 8);
    if (!cp->plane) return ORC_ERR_NOMEM;
  }
  if (j->progressive) return orc_decode_prog(j);
  orc_br br;
  memset(&br, 0, sizeof(br));
  br.p = j->scan;
  br.e = j->end;
  int pred[4] = {0, 0, 0, 0};
  int16_t blk[64];
  long total = (long)mcux * mcuy, left_in_interval = j->restart_interval;
  for (long m = 0; m < total; m++) {
    if (j->restart_interval) {
      if (left_in_interval == 0) {
        orc_restart(&br);
        pred[0] = pred[1] = pred[2] = pred[3] = 0;
        left_in_interval = j->restart_interval;
      }
      left_in_interval--;
    }
    int mx = (int)(m % mcux), my = (int)(m / mcux);
    for (int c = 0; c < j->ncomp; c++) {
      orc_comp *cp = &j->comp[c];
      for (int by = 0; by < cp->v; by++)
        for (int bx = 0; bx < cp->h; bx++) {
          memset(blk, 0, sizeof(blk));
          int s = orc_huff_decode(&br, &j->dc[cp->td]);
          int diff = orc_extend(orc_get(&br, s), s);
          pred[c] += diff;
          blk[0] = (int16_t)pred[c];
          for (int k = 1; k < 64; k++) {
            int rs = orc_huff_decode(&br, &j->ac[cp->ta]);
            int r = rs >> 4;
            s = rs & 15;
            if (s) {
              k += r;
              int v = orc_extend(orc_get(&br, s), s);
              blk[orc_natural[k]] = (int16_t)v;
            } else {
              if (r != 15) break;
              k += 15;
            }
          }
          int px = (mx * cp->h + bx) * 8, py = (my * cp->v + by) * 8;
          int stride = cp->bw * 8;
          orc_idct_islow(blk, j->qt[cp->tq], cp->plane + (size_t)py * stride + px, stride);
        }
    }
  }
  /* Truncation: libjpeg zero-fills and warns; Pillow then reports the image
   * as truncated (OSError). Treat fill past a non-EOI end as truncation.
   * The trailing partial byte of a valid stream is padded with 1-bits and
   * never read past; >= 8 synthesized bits means the data ran out. */
  if (br.hit_marker && br.marker == -1 && br.zero_fill_bits > 64) return ORC_ERR_TRUNCATED;
  return ORC_OK;
}

static void orc_free(orc_jpeg *j) {
  for (int c = 0; c < 4; c++) {
    free(j->comp[c].plane);
    j->comp[c].plane = NULL;
  }
}

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* jdsample.c: fancy upsampling of one chroma sample position (x, y) in the
 * full-resolution grid. Edge columns/rows replicate (equivalent to the special
 * first/last column cases and jdmainct.c's duplicated context rows). */
static int orc_upsample(const orc_comp *cp, int hmax, int vmax, int x, int y) {
  const uint8_t *pl = cp->plane;
  int stride = cp->bw * 8;
  int hf = hmax / cp->h, vf = vmax / cp->v;
  if (hf == 1 && vf == 1) return pl[(size_t)y * stride + x];
  if (hf == 2 && vf == 2) {
    int cx = x >> 1, cy = y >> 1;
    if (cp->dw <= 2) /* h2v2_upsample (box) */
      return pl[(size_t)cy * stride + cx];
    int ny = (y & 1) ? clampi(cy + 1, 0, cp->dh - 1) : clampi(cy - 1, 0, cp->dh - 1);
    int nx = (x & 1) ? clampi(cx + 1, 0, cp->dw - 1) : clampi(cx - 1, 0, cp->dw - 1);
    const uint8_t *r0 = pl + (size_t)cy * stride, *r1 = pl + (size_t)ny * stride;
    int thiscol = r0[cx] * 3 + r1[cx];
    int nextcol = r0[nx] * 3 + r1[nx];
    return (x & 1) ? (thiscol * 3 + nextcol + 7) >> 4 : (thiscol * 3 + nextcol + 8) >> 4;
  }
  if (hf == 2 && vf == 1) {
    int cx = x >> 1;
    const uint8_t *r0 = pl + (size_t)y * stride;
    if (cp->dw <= 2) return r0[cx]; /* h2v1_upsample (box) */
    if (x & 1) {
      int nx = clampi(cx + 1, 0, cp->dw - 1);
      return (r0[cx] * 3 + r0[nx] + 2) >> 2;
    } else {
      int nx = clampi(cx - 1, 0, cp->dw - 1);
      return (r0[cx] * 3 + r0[nx] + 1) >> 2;
    }
  }
  /* other ratios: generic box replication (int_upsample) */
  return pl[(size_t)(y / vf) * stride + (x / hf)];
}

/* jdcolor.c build_ycc_rgb_table */
#define SCALEBITS 16
#define ONE_HALF ((int32_t)1 << (SCALEBITS - 1))
#define FIXC(x) ((int32_t)((x) * (1L << SCALEBITS) + 0.5))

static uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

static int orc_is_rgb(const orc_jpeg *j) {
  /* jdapimin.c default_decompress_parms for 3 components */
  if (j->saw_jfif) return 0;
  if (j->saw_adobe) return j->adobe_transform == 0;
  return j->comp[0].id == 82 && j->comp[1].id == 71 && j->comp[2].id == 66;
}

/* Decode a baseline JPEG to interleaved RGB (H*W*3), as
 * Image.open(BytesIO(b)).convert("RGB") does. */
int orc_jpeg_info(const uint8_t *data, size_t len, int *w, int *h, int *ncomp) {
  orc_jpeg j;
  int rc = orc_parse(data, len, &j);
  if (rc) return rc;
  *w = j.width;
  *h = j.height;
  *ncomp = j.ncomp;
  return ORC_OK;
}

int orc_decode_rgb(const uint8_t *data, size_t len, uint8_t *rgb, int cap_pixels) {
  orc_jpeg j;
  int rc = orc_parse(data, len, &j);
  if (rc) return rc;
  if ((long)j.width * j.height > cap_pixels) return ORC_ERR_NOMEM;
  rc = orc_decode_planes(&j);
  if (rc) {
    orc_free(&j);
    return rc;
  }
  int W = j.width, H = j.height;
  if (j.ncomp == 1) {
    const orc_comp *cp = &j.comp[0];
    for (int y = 0; y < H; y++)
      for (int x = 0; x < W; x++) {
        uint8_t v = cp->plane[(size_t)y * cp->bw * 8 + x];
        uint8_t *o = rgb + ((size_t)y * W + x) * 3;
        o[0] = o[1] = o[2] = v;
      }
  } else {
    int rgbmode = orc_is_rgb(&j);
    for (int y = 0; y < H; y++)
      for (int x = 0; x < W; x++) {
        int Y = orc_upsample(&j.comp[0], j.hmax, j.vmax, x, y);
        int cb = orc_upsample(&j.comp[1], j.hmax, j.vmax, x, y);
        int cr = orc_upsample(&j.comp[2], j.hmax, j.vmax, x, y);
        uint8_t *o = rgb + ((size_t)y * W + x) * 3;
        if (rgbmode) {
          o[0] = (uint8_t)Y; o[1] = (uint8_t)cb; o[2] = (uint8_t)cr;
          continue;
        }
        int xcr = cr - 128, xcb = cb - 128;
        int cr_r = (FIXC(1.40200) * xcr + ONE_HALF) >> SCALEBITS;
        int cb_b = (FIXC(1.77200) * xcb + ONE_HALF) >> SCALEBITS;
        int32_t cr_g = (-FIXC(0.71414)) * xcr;
        int32_t cb_g = (-FIXC(0.34414)) * xcb + ONE_HALF;
        o[0] = clamp255(Y + cr_r);
        o[1] = clamp255(Y + (int)((cb_g + cr_g) >> SCALEBITS));
        o[2] = clamp255(Y + cb_b);
      }
  }
  orc_free(&j);
  return ORC_OK;
}

/* Raw coefficient/plane access for kernel-level parity tests: decode and
 * return the component planes (padded bw*8 x bh*8) concatenated. */
int orc_decode_planes_out(const uint8_t *data, size_t len, uint8_t *out, long cap, int *dims) {
  orc_jpeg j;
  int rc = orc_parse(data, len, &j);
  if (rc) return rc;
  rc = orc_decode_planes(&j);
  if (rc) {
    orc_free(&j);
    return rc;
  }
  long off = 0;
  for (int c = 0; c < j.ncomp; c++) {
    long n = (long)j.comp[c].bw * 8 * j.comp[c].bh * 8;
    dims[2 * c] = j.comp[c].bw * 8;
    dims[2 * c + 1] = j.comp[c].bh * 8;
    if (off + n <= cap) memcpy(out + off, j.comp[c].plane, n);
    off += n;
  }
  orc_free(&j);
  return off <= cap ? ORC_OK : ORC_ERR_NOMEM;
}

/* ------------------------------------------------------------------------ */
/* Pillow Resample.c (bilinear, 8 bpc).                                      */
/* ------------------------------------------------------------------------ */
#define PRECISION_BITS (32 - 8 - 2)

static double orc_bilinear_filter(double x) {
  if (x < 0.0) x = -x;
  if (x < 1.0) return 1.0 - x;
  return 0.0;
}

/* precompute_coeffs + normalize_coeffs_8bpc. Returns ksize; bounds has
 * 2*outSize ints (xmin, xcount); kk has outSize*ksize int32. */
int orc_resample_coeffs(int inSize, int outSize, int *bounds, int32_t *kk, int kcap) {
  double in0 = 0.0, in1 = (double)inSize;
  double scale = (in1 - in0) / outSize, filterscale = scale;
  if (filterscale < 1.0) filterscale = 1.0;
  double support = 1.0 * filterscale; /* bilinear support = 1.0 */
  int ksize = (int)ceil(support) * 2 + 1;
  if ((long)ksize * outSize > kcap) return -1;
  double *pre = (double *)malloc(sizeof(double) * ksize);
  for (int xx = 0; xx < outSize; xx++) {
    double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0, ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > inSize) xmax = inSize;
    xmax -= xmin;
    int x;
    for (x = 0; x < xmax; x++) {
      double w = orc_bilinear_filter((x + xmin - center + 0.5) * ss);
      pre[x] = w;
      ww += w;
    }
    for (x = 0; x < xmax; x++)
      if (ww != 0.0) pre[x] /= ww;
    for (; x < ksize; x++) pre[x] = 0;
    for (x = 0; x < ksize; x++) {
      double v = pre[x] * (1 << PRECISION_BITS);
      kk[xx * ksize + x] = (int32_t)(pre[x] < 0 ? (-0.5 + v) : (0.5 + v));
    }
    bounds[xx * 2 + 0] = xmin;
    bounds[xx * 2 + 1] = xmax;
  }
  free(pre);
  return ksize;
}

static uint8_t orc_clip8(int32_t in) {
  if (in >= (1 << PRECISION_BITS << 8)) return 255;
  if (in <= 0) return 0;
  return (uint8_t)(in >> PRECISION_BITS);
}

/* ImagingResample(imIn, xsize, ysize, BILINEAR, box=(0,0,w,h)) on RGB.
 * need_horizontal / need_vertical skip identity passes (Resample.c
 * ImagingResampleInner); an identical size returns a copy. */
int orc_resize_rgb(const uint8_t *in, int w, int h, uint8_t *out, int ow, int oh) {
  int ksh_cap = ow * (2 * ((w + ow - 1) / ow) + 3) + 64;
  int ksv_cap = oh * (2 * ((h + oh - 1) / oh) + 3) + 64;
  int *bh = (int *)malloc(sizeof(int) * 2 * ow), *bv = (int *)malloc(sizeof(int) * 2 * oh);
  int32_t *kh = (int32_t *)malloc(sizeof(int32_t) * ksh_cap);
  int32_t *kv = (int32_t *)malloc(sizeof(int32_t) * ksv_cap);
  int ksh = orc_resample_coeffs(w, ow, bh, kh, ksh_cap);
  int ksv = orc_resample_coeffs(h, oh, bv, kv, ksv_cap);
  if (ksh < 0 || ksv < 0) return ORC_ERR_NOMEM;
  int need_h = (ow != w), need_v = (oh != h);
  int yfirst = bv[0], ylast = bv[oh * 2 - 2] + bv[oh * 2 - 1];
  const uint8_t *src = in;
  int src_h = h, y0 = 0;
  uint8_t *tmp = NULL;
  if (need_h) {
    if (need_v) {
      for (int i = 0; i < oh; i++) bv[i * 2] -= yfirst;
    } else {
      yfirst = 0;
      ylast = h;
    }
    int th = ylast - yfirst;
    tmp = (uint8_t *)malloc((size_t)th * ow * 3);
    for (int yy = 0; yy < th; yy++) {
      const uint8_t *row = in + (size_t)(yy + yfirst) * w * 3;
      for (int xx = 0; xx < ow; xx++) {
        int xmin = bh[xx * 2], xcnt = bh[xx * 2 + 1];
        const int32_t *k = kh + xx * ksh;
        int32_t s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
        for (int x = 0; x < xcnt; x++) {
          const uint8_t *p = row + (size_t)(x + xmin) * 3;
          s0 += p[0] * k[x];
          s1 += p[1] * k[x];
          s2 += p[2] * k[x];
        }
        uint8_t *o = tmp + ((size_t)yy * ow + xx) * 3;
        o[0] = orc_clip8(s0);
        o[1] = orc_clip8(s1);
        o[2] = orc_clip8(s2);
      }
    }
    src = tmp;
    src_h = th;
    y0 = 0;
    w = ow;
  }
  (void)y0;
  (void)src_h;
  if (need_v) {
    for (int yy = 0; yy < oh; yy++) {
      int ymin = bv[yy * 2], ycnt = bv[yy * 2 + 1];
      const int32_t *k = kv + yy * ksv;
      for (int xx = 0; xx < ow; xx++) {
        int32_t s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
        for (int y = 0; y < ycnt; y++) {
          const uint8_t *p = src + ((size_t)(y + ymin) * w + xx) * 3;
          s0 += p[0] * k[y];
          s1 += p[1] * k[y];
          s2 += p[2] * k[y];
        }
        uint8_t *o = out + ((size_t)yy * ow + xx) * 3;
        o[0] = orc_clip8(s0);
        o[1] = orc_clip8(s1);
        o[2] = orc_clip8(s2);
      }
    }
  } else {
    memcpy(out, src, (size_t)oh * ow * 3);
  }
  free(tmp);
  free(bh);
  free(bv);
  free(kh);
  free(kv);
  return ORC_OK;
}

/* torchvision to_tensor (+ optional Normalize): HWC uint8 -> CHW float32.
 * float32 IEEE: v / 255.0f, then (x - mean) / std (float32 ops). */
void orc_to_tensor(const uint8_t *hwc, int h, int w, const float *mean, const float *std,
                   float *out) {
  for (int c = 0; c < 3; c++)
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) {
        volatile float v = (float)hwc[((size_t)y * w + x) * 3 + c] / 255.0f;
        if (mean) {
          volatile float t = v - mean[c];
          v = t / std[c];
        }
        out[((size_t)c * h + y) * w + x] = v;
      }
}

/* End-to-end per image: decode -> resize(oh, ow) -> to_tensor[normalize]. */
int orc_jpeg_to_tensor(const uint8_t *data, size_t len, int oh, int ow, const float *mean,
                       const float *std, float *out) {
  int w, h, nc;
  int rc = orc_jpeg_info(data, len, &w, &h, &nc);
  if (rc) return rc;
  uint8_t *rgb = (uint8_t *)malloc((size_t)w * h * 3);
  uint8_t *small = (uint8_t *)malloc((size_t)ow * oh * 3);
  if (!rgb || !small) return ORC_ERR_NOMEM;
  rc = orc_decode_rgb(data, len, rgb, w * h);
  if (!rc) rc = orc_resize_rgb(rgb, w, h, small, ow, oh);
  if (!rc) orc_to_tensor(small, oh, ow, mean, std, out);
  free(rgb);
  free(small);
  return rc;
}

/* Raw HWC uint8 column path (config 5): resize + to_tensor [+ normalize]. */
int orc_raw_to_tensor(const uint8_t *hwc, int h, int w, int oh, int ow, const float *mean,
                      const float *std, float *out) {
  uint8_t *small = (uint8_t *)malloc((size_t)ow * oh * 3);
  int rc = orc_resize_rgb(hwc, w, h, small, ow, oh);
  if (!rc) orc_to_tensor(small, oh, ow, mean, std, out);
  free(small);
  return rc;
}

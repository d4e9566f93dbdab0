/* Offline study (not product code): how fast does a baseline-JPEG Huffman
 * decoder started at an arbitrary bit position with a guessed (b, k) state
 * resynchronise with the true decode? Input: a JPEG file (4:2:0, no DRI).
 * Prints the sync-distance distribution for several guess strategies. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int maxcode[18], valoff[18]; uint8_t vals[256]; } Tab;
static Tab dc[4], ac[4];
static int cdc[3], cac[3];
static uint8_t *bits; static long nbytes;

static void derive(Tab *t, const uint8_t *cnt, const uint8_t *v) {
  int code = 0, k = 0;
  for (int l = 1; l <= 16; l++) {
    if (cnt[l - 1]) { t->valoff[l] = k - code; code += cnt[l - 1]; k += cnt[l - 1]; t->maxcode[l] = code - 1; }
    else t->maxcode[l] = -1;
    code <<= 1;
  }
  memcpy(t->vals, v, k);
}
static inline uint32_t peek16(long p) {
  uint32_t w = 0;
  for (int i = 0; i < 4; i++) { long b = (p >> 3) + i; w = (w << 8) | (b < nbytes ? bits[b] : 0); }
  return (w << (p & 7)) >> 16;
}
static inline uint32_t getn(long p, int n) { return n ? (peek16(p) >> (16 - n)) : 0; }
static int decode(const Tab *t, long *p) {
  uint32_t w = peek16(*p);
  for (int l = 1; l <= 16; l++) { int c = w >> (16 - l); if (c <= t->maxcode[l]) { *p += l; return t->vals[(t->valoff[l] + c) & 255]; } }
  *p += 16; return 0;
}
static const int bcomp[6] = {0, 0, 0, 0, 1, 2};
/* one symbol step; state (b,k) */
static void step(long *p, int *b, int *k) {
  int c = bcomp[*b];
  if (*k == 0) { int s = decode(&dc[cdc[c]], p); *p += s; *k = 1; }
  else {
    int rs = decode(&ac[cac[c]], p); int r = rs >> 4, s = rs & 15;
    if (s) { *k += r + 1; *p += s; } else *k = (r == 15) ? *k + 16 : 64;
    if (*k >= 64) { *k = 0; *b = (*b + 1) % 6; }
  }
}
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); long L = ftell(f); fseek(f, 0, SEEK_SET);
  uint8_t *d = malloc(L); fread(d, 1, L, f); fclose(f);
  long i = 2, scan = 0;
  while (i < L) {
    int m = d[i + 1], len = (d[i + 2] << 8) | d[i + 3];
    if (m == 0xC4) { long s = i + 4, e = i + 2 + len; while (s < e) { int tc = d[s] >> 4, th = d[s] & 15; int n = 0; for (int q = 0; q < 16; q++) n += d[s + 1 + q]; derive(tc ? &ac[th] : &dc[th], d + s + 1, d + s + 17); s += 17 + n; } }
    if (m == 0xDA) { int ns = d[i + 4]; for (int q = 0; q < ns; q++) { int sel = d[i + 6 + 2 * q]; cdc[q] = sel >> 4; cac[q] = sel & 15; } scan = i + 2 + len; break; }
    i += 2 + len;
  }
  bits = malloc(L); nbytes = 0;
  for (long q = scan; q < L - 1; q++) { if (d[q] == 0xFF) { if (d[q + 1] == 0) { bits[nbytes++] = 0xFF; q++; continue; } break; } bits[nbytes++] = d[q]; }
  long nb = nbytes * 8;
  /* true decode: record state at every symbol boundary */
  int *tb = malloc(sizeof(int) * (nb + 64)); memset(tb, -1, sizeof(int) * (nb + 64));
  long p = 0; int b = 0, k = 0;
  while (p < nb - 32) { tb[p] = (b << 8) | k; step(&p, &b, &k); }
  const int guesses[][2] = {{0, 0}, {0, 1}, {0, 5}, {4, 1}, {1, 0}};
  const char *gn[] = {"b0k0", "b0k1", "b0k5", "b4k1", "b1k0"};
  srand(1);
  for (int g = 0; g < 5; g++) {
    long hist[12] = {0}; long total = 0; double sum = 0;
    for (int t = 0; t < 4000; t++) {
      long p0 = (long)((double)rand() / RAND_MAX * (nb - 200000 > 1000 ? nb - 200000 : nb / 2));
      long q = p0; int bb = guesses[g][0], kk = guesses[g][1];
      long dist = -1;
      while (q < nb - 64) {
        if (tb[q] == ((bb << 8) | kk)) { dist = q - p0; break; }
        step(&q, &bb, &kk);
      }
      if (dist < 0) continue;
      total++; sum += dist;
      int bin = 0; long x = dist; while (x >= 128 && bin < 11) { x >>= 1; bin++; }
      hist[bin]++;
    }
    printf("%s mean %.0f bits: ", gn[g], sum / total);
    long acc = 0;
    for (int q = 0; q < 12; q++) { acc += hist[q]; printf("<%ld:%.3f ", 128L << q, 1.0 - (double)acc / total); }
    printf("\n");
  }
  return 0;
}

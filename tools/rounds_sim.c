/* Offline model (not product code) of k_huff_image's convergence rounds on
 * one baseline 4:2:0 JPEG without restart markers: phase 1 from the guess
 * (b = 0, k = 0) at every range start, then rounds of re-decodes from the
 * predecessor's exit that stop at the first checkpoint (S/3, 2S/3) where
 * they merge with the slot's previous trajectory, with the memo of the
 * previous trajectory (ldt_huffman.hip image_decode). SPEC=1 adds the
 * speculation studied for round 5: every needy slot's successor is also
 * decoded from the needy slot's old exit (p, k) under the other block
 * phases b', and a slot whose new entry matches one adopts that result at
 * the start of the next round.
 * Prints rounds and the critical path: the sum over rounds of the longest
 * decode (symbol steps) of the round.
 * COUNT=1: steps are count-mode steps (LUMA_PEEK: the luma AC peek bits);
 * BLOCKS=1: the lane-per-block model of round 6's k_block_decode instead.
 * usage: rounds_sim <file.jpg> <S bits (0: auto)> <spec 0/1> [max spec lanes] */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int maxcode[18], valoff[18]; uint8_t vals[256]; } Tab;
static Tab dc[4], ac[4];
static int cdc[3], cac[3];
static uint8_t *bits;
static long nbytes;

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
static int decode(const Tab *t, long *p) {
  uint32_t w = peek16(*p);
  for (int l = 1; l <= 16; l++) { int c = w >> (16 - l); if (c <= t->maxcode[l]) { *p += l; return t->vals[(t->valoff[l] + c) & 255]; } }
  *p += 16; return 0;
}
static const int bcomp[6] = {0, 0, 0, 0, 1, 2};
static const int bcount = 6;
typedef struct { long p; int b, k; } St;
static void step(St *s) {
  int c = bcomp[s->b];
  if (s->k == 0) { int t = decode(&dc[cdc[c]], &s->p); s->p += t; s->k = 1; }
  else {
    int rs = decode(&ac[cac[c]], &s->p); int r = rs >> 4, t = rs & 15;
    if (t) { s->k += r + 1; s->p += t; } else s->k = (r == 15) ? s->k + 16 : 64;
    if (s->k >= 64) { s->k = 0; s->b = (s->b + 1) % 6; }
  }
}
/* step() that also reports a symbol no valid stream holds: a code the table
 * lacks, or an AC value or ZRL past coefficient 63 */
static int bad_step(St *s) {
  int c = bcomp[s->b];
  if (s->k == 0) { long p0 = s->p; int t = decode(&dc[cdc[c]], &s->p); int bad = s->p - p0 == 16 && t == 0; s->p += t; s->k = 1; return bad || t > 11; }
  long p0 = s->p;
  int rs = decode(&ac[cac[c]], &s->p); int r = rs >> 4, t = rs & 15;
  int bad = s->p - p0 == 16 && rs == 0;
  if (t) { s->k += r + 1; bad |= s->k > 63; s->p += t; } else if (r == 15) { s->k += 16; bad |= s->k > 63; } else s->k = 64;
  if (s->k >= 64) { s->k = 0; s->b = (s->b + 1) % 6; }
  return bad;
}
/* one count-mode step (ldt_plan.cpp count-mode entries, ldt_huffman.hip
 * count_step): a DC symbol, or, while k <= 48, a run of AC symbols whose
 * codes all lie in the 11 peeked bits (advance <= 15 before the last), else
 * one AC symbol. Returns the symbols consumed. */
static int code_len(const Tab *t, long p) {
  uint32_t w = peek16(p);
  for (int l = 1; l <= 16; l++) { int c = w >> (16 - l); if (c <= t->maxcode[l]) return l; }
  return 16;
}
static int PEEK_Y = 11; /* LUMA_PEEK env: peek bits of the luma AC count-mode table (the others 11) */
static int count_step_sim(St *s) {
  if (s->k == 0 || s->k >= 49) { step(s); return 1; }
  const int W = bcomp[s->b] == 0 ? PEEK_Y : 11;
  const long p0 = s->p; int n = 0, adv = 0;
  for (;;) {
    int c = bcomp[s->b];
    St t = *s; step(&t); n++;
    int a = t.k == 0 ? 64 : t.k - s->k; /* the symbol's coefficient advance (EOB: to the block end) */
    *s = t; adv += a;
    if (s->k == 0 || adv > 15) break;
    long used = s->p - p0;
    int cl = code_len(&ac[cac[bcomp[s->b]]], s->p);
    if (used >= W || used + cl > W) break;
    (void)c;
  }
  return n;
}
static int eq(St a, St b) { return a.p == b.p && a.b == b.b && a.k == b.k; }

typedef struct { St en, ex, cp[16]; int ncp; } Traj;
static int NCP = 2; /* checkpoints per range (NCP env; the kernel keeps 2: S/3, 2S/3) */
static long S, nbitsl;
static int nslot;

/* decode slot j from state e to the first boundary >= its range end; with
 * prev: stop at the first checkpoint equal to prev's (merge). Returns steps. */
static int COUNT = 0; /* COUNT env: steps are count-mode steps (count_step_sim), not symbols */
static inline void adv1(St *s) { if (COUNT) count_step_sim(s); else step(s); }
static int run(int j, St e, const Traj *prev, Traj *out) {
  long stop = (long)(j + 1) * S; if (stop > nbitsl) stop = nbitsl;
  St s = e; int steps = 0; out->en = e; out->ncp = 0;
  long lims[16];
  for (int c = 0; c < NCP; c++) lims[c] = (long)j * S + ((c + 1) * S) / (NCP + 1);
  for (int c = 0; c < NCP; c++) {
    while (s.p < lims[c] && s.p < stop) { adv1(&s); steps++; }
    if (s.p >= stop) { out->ex = s; return steps; }
    if (prev && prev->ncp > c && eq(prev->cp[c], s)) { out->cp[c] = s; out->ncp = c + 1; out->ex = prev->ex; return steps; }
    out->cp[c] = s; out->ncp = c + 1;
  }
  while (s.p < stop) { adv1(&s); steps++; }
  out->ex = s;
  return steps;
}

int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); long L = ftell(f); fseek(f, 0, SEEK_SET);
  uint8_t *d = malloc(L); if (fread(d, 1, L, f) != (size_t)L) return 1; fclose(f);
  long i = 2, scan = 0;
  while (i < L) {
    int m = d[i + 1], len = (d[i + 2] << 8) | d[i + 3];
    if (m == 0xC4) { long s = i + 4, e = i + 2 + len; while (s < e) { int tc = d[s] >> 4, th = d[s] & 15; int n = 0; for (int q = 0; q < 16; q++) n += d[s + 1 + q]; derive(tc ? &ac[th] : &dc[th], d + s + 1, d + s + 17); s += 17 + n; } }
    if (m == 0xDA) { int ns = d[i + 4]; for (int q = 0; q < ns; q++) { int sel = d[i + 6 + 2 * q]; cdc[q] = sel >> 4; cac[q] = sel & 15; } scan = i + 2 + len; break; }
    i += 2 + len;
  }
  bits = malloc(L); nbytes = 0;
  for (long q = scan; q < L - 1; q++) { if (d[q] == 0xFF) { if (d[q + 1] == 0) { bits[nbytes++] = 0xFF; q++; continue; } break; } bits[nbytes++] = d[q]; }
  nbitsl = nbytes * 8;
  if (getenv("BLOCKS")) {
    /* lane-per-block decode model (round 6, k_block_decode): AC symbols per
     * block, and the sum over 64-block waves of the wave's largest count */
    St s = {0, 0, 0}; int nb = 0; static int cnt[1 << 16];
    while (s.p < nbitsl - 16 && nb < (1 << 16)) { int n = 0; step(&s); while (s.k != 0) { step(&s); n++; } cnt[nb++] = n; }
    long tot = 0, summax = 0;
    for (int b = 0; b < nb; b++) tot += cnt[b];
    for (int w = 0; w * 64 < nb; w++) { int mx = 0; for (int l = w * 64; l < nb && l < w * 64 + 64; l++) if (cnt[l] > mx) mx = cnt[l]; summax += mx; }
    printf("blocks %d ac_syms %ld mean %.2f waves %d mean_wave_max %.2f lane_efficiency %.3f\n", nb, tot, (double)tot / nb,
           (nb + 63) / 64, (double)summax / ((nb + 63) / 64), (double)tot / (64.0 * summax));
    return 0;
  }
  S = atol(argv[2]);
  if (getenv("NCP")) NCP = atoi(getenv("NCP"));
  if (getenv("COUNT")) COUNT = atoi(getenv("COUNT"));
  if (getenv("LUMA_PEEK")) PEEK_Y = atoi(getenv("LUMA_PEEK"));
  const int spec = atoi(argv[3]);
  const int lanes_cap = argc > 4 ? atoi(argv[4]) : 1024;
  if (S == 0) { S = 256; while ((nbitsl + S - 1) / S > 1024) S += 64; }
  nslot = (int)((nbitsl + S - 1) / S);
  Traj *cur = calloc(nslot, sizeof(Traj)), *memo = calloc(nslot, sizeof(Traj));
  int *has_memo = calloc(nslot, sizeof(int));
  /* speculation results: per slot, up to 6 (entry, traj) */
  Traj *sp = calloc((size_t)nslot * 6, sizeof(Traj)); int *nsp = calloc(nslot, sizeof(int));
  int ph1 = 0;
  /* GUESS=<bits>: the phase-1 block phase per slot from a test decode of
   * every b over the first <bits> of the range: the b with the fewest
   * impossible symbols (first such symbol latest on a tie) */
  const long glen = getenv("GUESS") ? atol(getenv("GUESS")) : 0;
  long guess_steps = 0; int guess_right = 0;
  for (int j = 0; j < nslot; j++) {
    St e = {(long)j * S, 0, 0};
    if (glen > 0 && j > 0) {
      int best_b = 0, best_bad = 1 << 30; long best_first = -1;
      for (int bb = 0; bb < bcount; bb++) {
        St t = {(long)j * S, bb, 0}; int nbad = 0; long first = -1;
        while (t.p < (long)j * S + glen && t.p < nbitsl) { if (bad_step(&t)) { nbad++; if (first < 0) first = t.p; } guess_steps++; }
        if (first < 0) first = 1L << 40;
        if (nbad < best_bad || (nbad == best_bad && first > best_first)) { best_bad = nbad; best_b = bb; best_first = first; }
      }
      e.b = best_b;
    }
    int st = run(j, e, NULL, &cur[j]); if (st > ph1) ph1 = st;
  }
  St *ph1_ex = malloc(sizeof(St) * nslot);
  for (int j = 0; j < nslot; j++) ph1_ex[j] = cur[j].ex;
  long same_pk = 0, diff_pk = 0;
  long crit = 0; int rounds = 0, spec_hits = 0, memo_hits = 0, needy_sum = 0;
  Traj *nw = calloc(nslot, sizeof(Traj)); int *needy = calloc(nslot, sizeof(int)); int *changed = calloc(nslot, sizeof(int));
  /* ANALYSE=1: every round's entries (after the adoption loop), compared
   * with the converged ones at the end */
  const int analyse = getenv("ANALYSE") != NULL;
  St *snap_en = analyse ? calloc((size_t)nslot * 64, sizeof(St)) : NULL;
  int *snap_need = analyse ? calloc((size_t)nslot * 64, sizeof(int)) : NULL;
  for (;;) {
    rounds++;
    /* adoption loop: memo and speculation hits, until none */
    for (;;) {
      int any = 0;
      for (int j = 1; j < nslot; j++) {
        St pe = cur[j - 1].ex;
        if (eq(pe, cur[j].en)) continue;
        if (has_memo[j] && eq(memo[j].en, pe)) { Traj t = cur[j]; cur[j] = memo[j]; cur[j].ncp = 0; memo[j] = t; memo_hits++; any = 1; continue; }
        if (spec) for (int a = 0; a < nsp[j]; a++) if (eq(sp[(size_t)j * 6 + a].en, pe)) {
          memo[j] = cur[j]; has_memo[j] = 1; cur[j] = sp[(size_t)j * 6 + a]; cur[j].ncp = 0; spec_hits++; any = 1; break;
        }
      }
      if (!any) break;
    }
    int tot = 0;
    for (int j = 1; j < nslot; j++) { needy[j] = !eq(cur[j - 1].ex, cur[j].en); tot += needy[j]; }
    if (analyse && rounds <= 64)
      for (int j = 0; j < nslot; j++) { snap_en[(size_t)(rounds - 1) * nslot + j] = cur[j].en; snap_need[(size_t)(rounds - 1) * nslot + j] = j ? needy[j] : 0; }
    if (!tot) break;
    needy_sum += tot;
    int mx = 0, any_changed = 0;
    if (spec == 2) {
      /* chain following: a needy slot's lane continues into its successor
       * while its exit changed and the successor is not in this round's
       * work list (that slot's own lane re-decodes it from the snapshot) */
      Traj *snap = calloc(nslot, sizeof(Traj));
      memcpy(snap, cur, sizeof(Traj) * nslot);
      for (int j = 1; j < nslot; j++) if (needy[j]) {
        int st = run(j, snap[j - 1].ex, &cur[j], &nw[j]);
        int q = j;
        while (!eq(nw[q].ex, cur[q].ex) && q + 1 < nslot && !needy[q + 1]) {
          memo[q] = cur[q]; has_memo[q] = 1; cur[q] = nw[q];
          q++;
          if (eq(cur[q - 1].ex, cur[q].en)) break;
          if (has_memo[q] && eq(memo[q].en, cur[q - 1].ex)) { Traj t = cur[q]; cur[q] = memo[q]; cur[q].ncp = 0; memo[q] = t; memo_hits++; continue; }
          st += run(q, cur[q - 1].ex, &cur[q], &nw[q]);
          needy_sum++;
        }
        if (st > mx) mx = st;
        if (q != j || 1) { /* the last decoded slot is applied below with the others */ }
        needy[q] = 1;
      }
      free(snap);
    } else
    for (int j = 1; j < nslot; j++) if (needy[j]) {
      int st = run(j, cur[j - 1].ex, &cur[j], &nw[j]); if (st > mx) mx = st;
    }
    /* speculation for the successors of the first needy slots, lanes permitting */
    int nsl = 0;
    for (int j = 0; j < nslot; j++) nsp[j] = 0;
    if (spec) {
      int budget = (lanes_cap - tot) / 5;
      for (int j = 1; j + 1 < nslot && budget > 0; j++) if (needy[j]) {
        budget--;
        St o = cur[j].ex;
        for (int bb = 0; bb < 6; bb++) {
          if (bb == o.b) continue;
          St e = o; e.b = bb;
          int st = run(j + 1, e, &cur[j + 1], &sp[(size_t)(j + 1) * 6 + nsp[j + 1]]);
          nsp[j + 1]++; nsl++;
          if (st > mx) mx = st;
        }
      }
    }
    crit += mx;
    for (int j = 1; j < nslot; j++) if (needy[j]) {
      changed[j] = !eq(nw[j].ex, cur[j].ex);
      if (changed[j]) { if (nw[j].ex.p == cur[j].ex.p && nw[j].ex.k == cur[j].ex.k) same_pk++; else diff_pk++; }
      any_changed |= changed[j];
      memo[j] = cur[j]; has_memo[j] = 1; cur[j] = nw[j];
    }
    if (!any_changed) break;
  }
  {
    int right = 0, right_b = 0;
    for (int j = 0; j < nslot; j++) { right += eq(ph1_ex[j], cur[j].ex); right_b += ph1_ex[j].b == cur[j].ex.b; }
    printf("phase-1 exits already final: %d of %d (block phase right: %d)\n", right, nslot, right_b);
  }
  if (getenv("WAVES")) {
    /* write-pass balance: symbols each slot's lane decodes from its true
     * entry to its exit (stop at the range end with the block complete, as
     * write_run), summed per 64-slot wave as the wave's slowest lane, for the
     * slots in order, sorted by their symbols, and sorted by their blocks */
    int *sym = calloc(nslot, sizeof(int)), *blk = calloc(nslot, sizeof(int)), *ord = calloc(nslot, sizeof(int));
    int *cst = calloc(nslot, sizeof(int)), *psym = calloc(nslot, sizeof(int));
    long tot_sym = 0, kz_skip = 0;
    for (int j = 0; j < nslot; j++) {
      St s = cur[j].en; long stop = (long)(j + 1) * S; if (stop > nbitsl) stop = nbitsl;
      int n = 0, nb = 0;
      while (s.p < stop || s.k != 0) { if (s.k == 0) nb++; step(&s); n++; if (s.p >= nbitsl + 64) break; }
      sym[j] = n; blk[j] = nb; tot_sym += n;
      if (getenv("KZ")) { /* round-6 model: start at the first block start (k = 0) at/after the entry */
        St z = cur[j].en; int skip = 0;
        while (z.k != 0) { step(&z); skip++; if (z.p >= nbitsl + 64) break; }
        kz_skip += skip; sym[j] = n - skip;
      }
      /* count-mode steps of the slot's phase-1 trajectory (from the guess) */
      St c = {(long)j * S, 0, 0}; int ns = 0, nsym1 = 0;
      while (c.p < stop) { nsym1 += count_step_sim(&c); ns++; }
      cst[j] = ns; psym[j] = nsym1;
    }
    {
      St u = {0, 0, 0}; long uniq = 0;
      while (u.p < nbitsl && !(u.p >= nbitsl - 8 && u.k == 0)) { step(&u); uniq++; if (u.p >= nbitsl + 64) break; }
      printf("write symbols %ld (unique decode of the stream %ld), partial blocks re-decoded at range starts %ld\n",
             tot_sym, uniq, kz_skip);
    }
    for (int mode = 0; mode < 5; mode++) {
      for (int j = 0; j < nslot; j++) ord[j] = j;
      if (mode) for (int a = 0; a < nslot; a++) for (int b = a + 1; b < nslot; b++) {
        int ka = mode == 1 ? sym[ord[a]] : mode == 2 ? blk[ord[a]] : mode == 3 ? cst[ord[a]] : psym[ord[a]];
        int kb = mode == 1 ? sym[ord[b]] : mode == 2 ? blk[ord[b]] : mode == 3 ? cst[ord[b]] : psym[ord[b]];
        if (kb > ka) { int t = ord[a]; ord[a] = ord[b]; ord[b] = t; }
      }
      long summax = 0;
      for (int w = 0; w * 64 < nslot; w++) { int m = 0; for (int l = w * 64; l < nslot && l < w * 64 + 64; l++) if (sym[ord[l]] > m) m = sym[ord[l]]; summax += m; }
      printf("waves mode %s sum_of_wave_max %ld (avg-lane bound %.0f)\n", mode == 0 ? "in-order" : mode == 1 ? "by-symbols" : mode == 2 ? "by-blocks" : mode == 3 ? "by-phase1-count-steps" : "by-phase1-symbols", summax, (double)tot_sym / 64.0);
    }
  }
  if (analyse) {
    /* per round: needy slots, non-needy slots whose entry is already the
     * converged one (a write started then would stand), non-needy ones whose
     * entry still changes, and the final prefix (slots before the first needy) */
    for (int r = 0; r < rounds && r < 64; r++) {
      int nn = 0, good = 0, bad = 0, pre = nslot;
      for (int j = 0; j < nslot; j++) {
        if (snap_need[(size_t)r * nslot + j]) { nn++; if (pre == nslot) pre = j; continue; }
        if (eq(snap_en[(size_t)r * nslot + j], cur[j].en)) good++; else bad++;
      }
      printf("round %d needy %d stable %d unstable %d prefix %d\n", r + 1, nn, good, bad, pre);
    }
  }
  printf("S %ld slots %d ph1_steps %d rounds %d crit_steps %ld needy_avg %.1f memo_hits %d spec_hits %d changed_same_pk %ld diff_pk %ld\n", S, nslot,
         ph1, rounds, crit, (double)needy_sum / rounds, memo_hits, spec_hits, same_pk, diff_pk);
  return 0;
}

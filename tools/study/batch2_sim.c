/* Study (not product): the round-4 batched replay of MergingDigest's incremental merge, restated
 * on the CPU phase by phase as the GPU kernel (histo_exact.hip merge_batch2) does it, and compared
 * bit for bit with the plain per-merge replay (tdigest/merging_digest.go:121-243).
 *
 * Phases of one batch of B pure chunks, all against the means at the batch start:
 *   A  pos[j][p] = #means < v (the temp's column is pos - 1; pos 0: before main 0, "Z")
 *   B  n[i][j]   = #temps of chunk j placed before main i (= #p with pos <= i)
 *   C1 column i's list: its temps in (chunk, position) order, Z temps flagged in column 0's
 *   C2 k bounds per column from the exact integer prefixes (min/max of q over the batch)
 *   E  Welford along each list (column 0: a chunk's Z temps start a fresh centroid that main 0
 *      then joins -- the reference's first element always starts, merging_digest.go:216)
 *   F  merge-path decisions per temp against the drift bounds [lo_i, hi_i] of the column means
 *      (exact check against the mean merge j saw only for temps inside a bound), and sortedness
 *      hi_i <= lo_{i+1}, which makes the per-temp checks cover every main's decisions
 *   G  exact k tests of flagged columns, merge by merge
 *   F' (round 6) flip repair, at most REPAIR_CAP rounds per batch: the first chunk jp with a decision
 *      failure gets every boundary's exact count from the means merge jp saw, and the batch is
 *      re-run with those counts (the GPU re-does only the columns beside the changed boundaries)
 *   H  commit the merges before the first failure.  A decision failure (a flip) left after the
 *      repairs restarts the next batch at that merge; a structural failure runs it alone.
 *
 *   gcc -O2 -o /tmp/b2s tools/study/batch2_sim.c -lm && /tmp/b2s 4000000 64 0 [repair_cap]   */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define TC 42
#define MAXM 512
#define MAXB 128
static double delta = 100;
static const double kBand = 1e-9;
static double kq(double q) { return delta * (asin(2 * q - 1) / M_PI + 0.5); }
static uint64_t rs = 88172645463325252ull;
static double u01(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (rs >> 11) * (1.0 / 9007199254740992.0);
}
static double gauss(void) {
  double a = u01(), b = u01();
  return sqrt(-2 * log(a + 1e-300)) * cos(2 * M_PI * b);
}
typedef struct { double m, w; } C;
static int cmpc(const void* a, const void* b) {
  double x = ((const C*)a)->m, y = ((const C*)b)->m;
  return x < y ? -1 : x > y;
}

static void merge_ref(C* main_, int* nm, double* T0, const C* t, int np, double tempW) {
  C out[MAXM];
  int n = 0, mi = 0, ti = 0;
  double T = *T0 + tempW, mw = 0, last = 0;
  while (mi < *nm || ti < np) {
    C nt = ti < np ? t[ti] : (C){INFINITY, 0};
    C nmn = mi < *nm ? main_[mi] : (C){INFINITY, 0};
    C x;
    if (nmn.m < nt.m) { x = nmn; mi++; } else { x = nt; ti++; }
    double ni = kq((mw + x.w) / T);
    if (ni - last > 1 || n == 0) {
      out[n++] = x;
      last = kq(mw / T);
    } else {
      out[n - 1].w += x.w;
      out[n - 1].m += (x.m - out[n - 1].m) * x.w / out[n - 1].w;
    }
    mw += x.w;
  }
  memcpy(main_, out, n * sizeof(C));
  *nm = n;
  *T0 = T;
}

/* statistics */
static long st_repairs, st_repair_rounds; static int REPAIR_CAP = 0; static long st_flip, st_struct, st_flagged_cols, st_atrisk, st_unsorted, st_zmerges;

/* returns committed merges; *structural = the failure at the returned index is structural */
static int merge_batch2(C* main_, int nm, double* T0, C t[][TC], const double* tempW, int B, int* structural) {
  static uint8_t pos[MAXB][TC];
  static uint8_t n[MAXM + 1][MAXB];
  static uint16_t al[MAXB * TC];
  static double ms[MAXB * TC];
  static uint32_t msw[MAXB * TC];
  static uint32_t off[MAXM + 2], cnt[MAXM + 1];
  static double lo[MAXM], hi[MAXM], kb0[MAXM + 1], kb1[MAXM + 1], kb2[MAXM + 1], TP[MAXB][TC + 1];
  double mp[MAXM + 1], bT[MAXB], brT[MAXB];
  *structural = 0;
  if (nm < 2) return 0;
  for (int i = 0; i + 1 < nm; i++)
    if (!(main_[i].m <= main_[i + 1].m)) return 0; /* unsorted means: not batchable */
  mp[0] = 0;
  for (int i = 0; i < nm; i++) mp[i + 1] = mp[i] + main_[i].w;
  double T = *T0;
  for (int j = 0; j < B; j++) {
    T += tempW[j];
    bT[j] = T;
    brT[j] = 1.0 / T;
    TP[j][0] = 0;
    for (int p = 0; p < TC; p++) TP[j][p + 1] = TP[j][p] + t[j][p].w;
  }
  /* A */
  for (int j = 0; j < B; j++)
    for (int p = 0; p < TC; p++) {
      int l = 0, h = nm;
      while (l < h) { int md = (l + h) / 2; if (main_[md].m < t[j][p].m) l = md + 1; else h = md; }
      pos[j][p] = (uint8_t)l;
    }
  static int nfix[MAXB][MAXM + 1]; /* -1: no override of n[i][j] (stored [j][i]) */
  for (int j = 0; j < B; j++) for (int i = 0; i <= nm; i++) nfix[j][i] = -1;
  int repairs = 0;
again:;
  /* B: run fill */
  for (int j = 0; j < B; j++)
    for (int p = 0; p < TC; p++) {
      int c0 = pos[j][p], c1 = p + 1 < TC ? pos[j][p + 1] : nm + 1;
      if (p == 0) for (int i = 0; i < c0; i++) n[i][j] = 0;
      for (int i = c0; i < c1; i++) n[i][j] = (uint8_t)(p + 1);
    }
  for (int j = 0; j < B; j++) for (int i = 0; i <= nm; i++) if (nfix[j][i] >= 0) n[i][j] = (uint8_t)nfix[j][i];
  /* list offsets: off[i] = sum_j n[i][j] (column -1 = Z first: column 0's list holds them) */
  for (int i = 0; i <= nm; i++) {
    uint32_t s = 0;
    for (int j = 0; j < B; j++) s += n[i][j];
    off[i] = s;
  }
  /* C1: column i (0..nm-1) list = entries p in [n[i][j], n[i+1][j]) for each j; column 0 also
   * [0, n[0][j]) first (Z, flagged 0x8000) -- column 0's list starts at 0 */
  for (int i = 0; i < nm; i++) {
    uint32_t k = i == 0 ? 0 : off[i];
    for (int j = 0; j < B; j++) {
      int a = i == 0 ? 0 : n[i][j], e = n[i + 1][j];
      for (int p = a; p < e; p++) al[k++] = (uint16_t)((j << 6) | p | (i == 0 && p < n[0][j] ? 0x8000 : 0));
    }
    cnt[i] = k - (i == 0 ? 0 : off[i]);
  }
  /* C2: bounds */
  for (int i = 0; i < nm; i++) {
    double qbmin = 2, qbmax = -1, qemin = 2, Cc = 0, W = main_[i].w;
    for (int j = 0; j < B; j++) {
      double s0 = TP[j][n[i][j]], s1 = TP[j][n[i + 1][j]];
      Cc += s0;
      double P = mp[i] + Cc;
      double qb = i == 0 ? 0.0 : P * brT[j], qe = (P + W) * brT[j];
      if (qb < qbmin) qbmin = qb;
      if (qb > qbmax) qbmax = qb;
      if (qe < qemin) qemin = qe;
      W += s1 - s0;
    }
    kb0[i] = kq(fmin(qemin, 1.0));
    kb1[i] = kq(fmin(qbmax, 1.0));
    kb2[i] = kq(fmin(qbmin, 1.0));
  }
  { /* the end "column" nm: qb of main nm = the total */
    double qbmin = 2, qbmax = -1, Cc = 0;
    for (int j = 0; j < B; j++) {
      Cc += TP[j][n[nm][j]];
      double qb = (mp[nm] + Cc) * brT[j];
      if (qb < qbmin) qbmin = qb;
      if (qb > qbmax) qbmax = qb;
    }
    kb1[nm] = kq(fmin(qbmax, 1.0));
    kb2[nm] = kq(fmin(qbmin, 1.0));
  }
  /* E: Welford along the lists (column 0: Z temps start a fresh centroid, main 0 joins) */
  int zany = 0;
  for (int i = 0; i < nm; i++) {
    uint32_t o = i == 0 ? 0 : off[i];
    double mean = main_[i].m, W = main_[i].w, W0 = W;
    lo[i] = hi[i] = mean;
    double sm = 0, sw = 0;
    for (uint32_t q = 0; q < cnt[i]; q++) {
      uint16_t e = al[o + q];
      int j = (e >> 6) & 0x3f, p = e & 63, z = e >> 15;
      double v = t[j][p].m, w = t[j][p].w;
      int zstart = z && (q == 0 || !(al[o + q - 1] >> 15) || (((al[o + q - 1] >> 6) & 0x3f) != j));
      if (zstart) {
        sm = mean;
        sw = W;
        mean = v;
        W = w;
        zany = 1;
      } else {
        W += w;
        mean += (v - mean) * w / W;
      }
      int zend = z && (q + 1 == cnt[i] || !(al[o + q + 1] >> 15) || (((al[o + q + 1] >> 6) & 0x3f) != j));
      if (zend) { /* main 0 joins the centroid the Z temps started */
        W += sw;
        mean += (sm - mean) * sw / W;
      }
      ms[o + q] = mean;
      msw[o + q] = (uint32_t)(W - W0);
      if (!z || zend) {
        if (mean < lo[i]) lo[i] = mean;
        if (mean > hi[i]) hi[i] = mean;
      }
    }
  }
  if (zany) st_zmerges++;
  /* F: decisions.  jp = first merge with a decision failure */
  int jp = B;
  for (int i = 0; i + 1 < nm; i++)
    if (!(hi[i] <= lo[i + 1])) { st_unsorted++; jp = 0; } /* (then every merge: conservative) */
  /* the mean column c had before chunk j (exact) */
#define MEAN_BEFORE(c, j, out)                                                   \
  do {                                                                           \
    uint32_t o_ = (c) == 0 ? 0 : off[c], k_ = 0;                                 \
    while (k_ < cnt[c] && (int)((al[o_ + k_] >> 6) & 0x3f) < (j)) k_++;           \
    out = k_ ? ms[o_ + k_ - 1] : main_[c].m;                                     \
  } while (0)
  for (int j = 0; j < B; j++)
    for (int p = 0; p < TC; p++) {
      double v = t[j][p].m;
      int pj = pos[j][p];
      if (nfix[j][0] >= 0) { pj = 0; while (pj < nm && n[pj][j] <= p) pj++; }
      int c = pj - 1, bad = 0;
      if (c >= 0 && v <= hi[c]) {
        double mb;
        st_atrisk++;
        MEAN_BEFORE(c, j, mb);
        if (!(mb < v)) bad = 1;
      }
      if (c + 1 < nm && v > lo[c + 1]) {
        double mb;
        st_atrisk++;
        MEAN_BEFORE(c + 1, j, mb);
        if (!(v <= mb)) bad = 1;
      }
      if (bad && j < jp) jp = j;
    }
  if (jp < B && repairs < REPAIR_CAP) {
    /* repair: the exact boundaries of chunk jp from the means merge jp saw, then everything again */
    repairs++;
    st_repairs++;
    for (int i = 1; i <= nm; i++) {
      double mb;
      if (i < nm) { MEAN_BEFORE(i, jp, mb); } else mb = INFINITY;
      int c = 0;
      while (c < TC && t[jp][c].m <= mb) c++;
      /* (monotone in i only if the means merge jp saw are sorted: they are, given hi <= lo) */
      nfix[jp][i] = c;
    }
    /* n[0][j]: Z temps: v <= mean_0 */
    { double mb; MEAN_BEFORE(0, jp, mb); int c = 0; while (c < TC && t[jp][c].m <= mb) c++; nfix[jp][0] = c; }
    goto again;
  }
  /* G: flagged columns' exact tests for merges < jp; also the bound tests */
  int jsf = B;
  for (int i = 0; i < nm; i++) {
    int sure = 1;
    if (i >= 1) sure = kb0[i] - kb1[i - 1] > 1 + kBand;
    sure = sure && kb1[i + 1] - kb2[i] < 1 - kBand;
    if (sure) continue;
    st_flagged_cols++;
    double Cp = 0, Ci = 0, Cn = 0, Wi = main_[i].w;
    for (int j = 0; j < jp && j < jsf; j++) {
      double Wcur = Wi;
      if (i >= 1) Cp += TP[j][n[i - 1][j]];
      Ci += TP[j][n[i][j]];
      Cn += TP[j][n[i + 1][j]];
      double Pi = mp[i] + Ci, Pn = mp[i + 1] + Cn, Pp = i >= 1 ? mp[i - 1] + Cp : 0;
      int ok = 1;
      if (i >= 1) ok = kq((Pi + Wcur) / bT[j]) - kq((i - 1 == 0 ? 0.0 : Pp) / bT[j]) > 1;
      if (n[i + 1][j] > (i == 0 ? 0 : n[i][j])) ok = ok && kq(Pn / bT[j]) - kq(i == 0 ? 0.0 : Pi / bT[j]) <= 1;
      if (!ok) { jsf = j; break; }
      Wi += TP[j][n[i + 1][j]] - TP[j][n[i][j]];
    }
  }
  int js = jp < jsf ? jp : jsf;
  *structural = jsf <= jp && js < B;
  if (js < B) { if (*structural) st_struct++; else st_flip++; }
  /* H: commit */
  for (int i = 0; i < nm; i++) {
    uint32_t o = i == 0 ? 0 : off[i], k = 0;
    while (k < cnt[i] && (int)((al[o + k] >> 6) & 0x3f) < js) k++;
    if (k) {
      main_[i].m = ms[o + k - 1];
      main_[i].w = main_[i].w + msw[o + k - 1];
    }
  }
  if (js) *T0 = bT[js - 1];
  return js;
}

int main(int argc, char** argv) {
  long N = argc > 1 ? atol(argv[1]) : 1000000;
  int B = argc > 2 ? atoi(argv[2]) : 64;
  REPAIR_CAP = argc > 4 ? atoi(argv[4]) : 0;
  int dist = argc > 3 ? atoi(argv[3]) : 0; /* 0 lognormal+rates, 1 few distinct values, 2 uniform ints, 3 rising, 4 falling */
  long merges = N / TC;
  C (*chunks)[TC] = malloc(sizeof(C[TC]) * merges);
  double* tw = malloc(sizeof(double) * merges);
  for (long g = 0; g < merges; g++) {
    tw[g] = 0;
    for (int p = 0; p < TC; p++) {
      double u = u01();
      if (dist == 0) chunks[g][p].m = exp(log(50.0) + gauss());
      else if (dist == 1) chunks[g][p].m = (double)(int)(u01() * 7);
      else if (dist == 2) chunks[g][p].m = (double)(int)(u01() * 1000);
      else if (dist == 3) chunks[g][p].m = (double)(g * TC + p) * 0.5 - 20.0 * log(u01() + 1e-300);
      else chunks[g][p].m = 1e6 - (double)(g * TC + p) * 3.0 + 50.0 * gauss();
      chunks[g][p].w = u < 0.05 ? 10 : u < 0.1 ? 2 : 1;
      tw[g] += chunks[g][p].w;
    }
    qsort(chunks[g], TC, sizeof(C), cmpc);
  }
  C ref[MAXM], bat[MAXM];
  int nr = 0, nb = 0;
  double Tr = 0, Tb = 0;
  for (long g = 0; g < merges; g++) merge_ref(ref, &nr, &Tr, chunks[g], TC, tw[g]);
  long g = 0, batches = 0, singles = 0, committed = 0;
  while (g < merges) {
    int b = (int)(merges - g < B ? merges - g : B), c = 0, structural = 1;
    if (Tb >= 8192 && b >= 2) {
      c = merge_batch2(bat, nb, &Tb, &chunks[g], &tw[g], b, &structural);
      batches++;
      committed += c;
      g += c;
    }
    if (c < b && g < merges && (structural || c == 0)) {
      merge_ref(bat, &nb, &Tb, chunks[g], TC, tw[g]);
      singles++;
      g++;
    }
  }
  int same = nr == nb && Tr == Tb;
  for (int i = 0; same && i < nr; i++) same = ref[i].m == bat[i].m && ref[i].w == bat[i].w;
  printf("N=%ld B=%d dist=%d merges=%ld centroids=%d bit_identical=%d batches=%ld committed=%ld (%.1f per batch) "
         "singles=%ld flips=%ld structural=%ld zbatches=%ld flagged_cols=%ld atrisk=%ld unsorted=%ld\n",
         N, B, dist, merges, nr, same, batches, committed, (double)committed / (batches ? batches : 1), singles, st_flip,
         st_struct, st_zmerges, st_flagged_cols, st_atrisk, st_unsorted);
  printf("repairs %ld (%.2f per batch)\n", st_repairs, (double)st_repairs / batches);
  return !same;
}

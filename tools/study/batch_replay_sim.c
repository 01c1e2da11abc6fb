/* Study (not product): a batched exact replay of MergingDigest's incremental merge.
 *
 * The reference merges every 42 Adds (tdigest/merging_digest.go:97-205), so a hot key's window is
 * a chain of thousands of dependent mergeAllTemps.  In a hot key's steady state almost every merge
 * keeps the structure "every old main centroid starts a centroid, every temp joins the one before
 * it".  While that holds, the centroids evolve independently: centroid i's mean is a sequential
 * Welford over the temps that land between it and centroid i+1.  This program replays B merges at
 * once under that assumption -- temps placed by the means at the batch start, k tests from the
 * exact integer weight prefixes, Welford per centroid across the B merges, then every temp's and
 * main's merge-path decision re-checked against the means the merge really saw -- and commits the
 * merges before the first one whose check fails (that one runs alone).  It compares the result
 * with the plain per-merge replay bit for bit.
 *
 *   gcc -O2 -o /tmp/brs tools/study/batch_replay_sim.c -lm && /tmp/brs 1000000 16          */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define TC 42
#define MAXM 512
#define MAXB 64
static double delta = 100;
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

/* the reference's mergeAllTemps (two-pointer on the main order, Welford), sorted temps t[np] */
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

/* batched: returns the number of merges committed (0..B) */
static int merge_batch(C* main_, int nm, double* T0, C t[][TC], const double* tempW, int B) {
  static double M[MAXB + 1][MAXM], W[MAXB + 1][MAXM], P[MAXM + 1], SP[MAXB][TC + 1];
  static int n[MAXB][MAXM + 1], a[MAXB][TC];
  if (nm < 2) return 0;
  for (int i = 0; i < nm; i++) M[0][i] = main_[i].m, W[0][i] = main_[i].w;
  for (int j = 0; j < B; j++) {
    SP[j][0] = 0;
    for (int p = 0; p < TC; p++) SP[j][p + 1] = SP[j][p] + t[j][p].w;
    /* Phase 1: each temp's centroid by the batch-start means: #mains with mean < v, minus one */
    for (int p = 0; p < TC; p++) {
      int lo = 0, hi = nm;
      while (lo < hi) { int md = (lo + hi) / 2; if (M[0][md] < t[j][p].m) lo = md + 1; else hi = md; }
      a[j][p] = lo - 1;
    }
    /* n[j][i] = #temps of merge j placed before main i */
    int p = 0;
    for (int i = 0; i <= nm; i++) {
      while (p < TC && a[j][p] < i) p++;
      n[j][i] = p;
    }
  }
  /* Phase 2/3: per merge, weights and prefixes; Welford per centroid; checks.  (On the GPU the
   * centroid loop is parallel and the merge loop sequential inside each centroid's lane.) */
  double T = *T0;
  int jfail = B;
  for (int j = 0; j < B && jfail == B; j++) {
    T += tempW[j];
    /* exclusive prefix of element "main i" in merge j */
    double acc = 0;
    for (int i = 0; i <= nm; i++) {
      P[i] = acc + SP[j][n[j][i]];
      if (i < nm) acc += W[j][i];
    }
    int ok = n[j][0] == 0; /* no temp before main 0 */
    for (int i = 0; i < nm && ok; i++) {
      if (i >= 1 && !(kq((P[i] + W[j][i]) / T) - kq(P[i - 1] / T) > 1)) ok = 0;            /* main i starts */
      if (n[j][i + 1] > n[j][i] && !(kq(P[i + 1] / T) - kq(P[i] / T) <= 1)) ok = 0;     /* its temps join */
    }
    /* merge-path decisions against the means merge j really sees (M[j]) */
    for (int p = 0; p < TC && ok; p++) {
      int q = a[j][p] + 1;
      if (q < nm && !(t[j][p].m <= M[j][q])) ok = 0; /* temp p taken before main q */
    }
    for (int q = 0; q < nm && ok; q++) {
      int pq = n[j][q];
      if (pq < TC && !(M[j][q] < t[j][pq].m)) ok = 0; /* main q taken before temp pq */
    }
    if (!ok) { jfail = j; break; }
    for (int i = 0; i < nm; i++) {
      double mean = M[j][i], w = W[j][i];
      for (int p = n[j][i]; p < n[j][i + 1]; p++) {
        w += t[j][p].w;
        mean += (t[j][p].m - mean) * t[j][p].w / w;
      }
      M[j + 1][i] = mean;
      W[j + 1][i] = w;
    }
  }
  for (int i = 0; i < nm; i++) main_[i].m = M[jfail][i], main_[i].w = W[jfail][i];
  for (int j = 0; j < jfail; j++) *T0 += tempW[j];
  return jfail;
}

int main(int argc, char** argv) {
  long N = argc > 1 ? atol(argv[1]) : 1000000;
  int B = argc > 2 ? atoi(argv[2]) : 16;
  int warm = argc > 3 ? atoi(argv[3]) : 0; /* merges before batching starts */
  long merges = N / TC;
  C (*chunks)[TC] = malloc(sizeof(C[TC]) * merges);
  double* tw = malloc(sizeof(double) * merges);
  for (long g = 0; g < merges; g++) {
    tw[g] = 0;
    for (int p = 0; p < TC; p++) {
      double u = u01();
      chunks[g][p].m = exp(log(50.0) + gauss());
      chunks[g][p].w = u < 0.05 ? 10 : u < 0.1 ? 2 : 1;
      tw[g] += chunks[g][p].w;
    }
    qsort(chunks[g], TC, sizeof(C), cmpc);
  }
  C ref[MAXM], bat[MAXM];
  int nr = 0, nb = 0;
  double Tr = 0, Tb = 0;
  for (long g = 0; g < merges; g++) merge_ref(ref, &nr, &Tr, chunks[g], TC, tw[g]);
  long g = 0, batches = 0, singles = 0, committed = 0, fails0 = 0;
  int backoff = 0;
  while (g < merges) {
    int b = (int)(merges - g < B ? merges - g : B);
    int c = 0;
    if (g >= warm && backoff == 0 && b >= 2) {
      c = merge_batch(bat, nb, &Tb, &chunks[g], &tw[g], b);
      batches++;
      committed += c;
      if (c == 0) { fails0++; backoff = 4; }
      g += c;
    } else if (backoff) {
      backoff--;
    }
    if (c < b && g < merges) { /* the failing merge runs alone */
      merge_ref(bat, &nb, &Tb, chunks[g], TC, tw[g]);
      singles++;
      g++;
    }
  }
  int same = nr == nb && Tr == Tb;
  for (int i = 0; same && i < nr; i++) same = ref[i].m == bat[i].m && ref[i].w == bat[i].w;
  printf("N=%ld B=%d merges=%ld centroids=%d bit_identical=%d batches=%ld committed=%ld (%.1f per batch) "
         "singles=%ld failed_at_0=%ld\n",
         N, B, merges, nr, same, batches, committed, (double)committed / (batches ? batches : 1), singles, fails0);
  return !same;
}

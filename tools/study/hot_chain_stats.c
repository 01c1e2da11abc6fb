/* Study (not product): where a hot key's exact MergingDigest chain leaves its steady structure.
 *
 * Replays the reference's mergeAllTemps (tdigest/merging_digest.go:121-243) merge after merge on a
 * C4-shaped hot key (lognormal(ln 50, 1) values, weights 1 / 2 / 10 at 90 / 5 / 5 %) and, per
 * merge, compares with the steady prediction "every old main starts a centroid, every temp joins
 * the one before it":
 *   - violations: a main that joins (B), a temp that starts (A), temps before main 0 (Z);
 *   - the deviation region: from the first violation to the next main that starts (the chain's
 *     beforeIndex is the predicted one again from there on);
 *   - merge-path flips against stale means: the temps' positions among the means of merge j - a
 *     (a = 8 .. 256) instead of merge j's own.
 *
 *   gcc -O2 -o /tmp/hcs tools/study/hot_chain_stats.c -lm && /tmp/hcs 17000000                */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define TC 42
#define MAXM 512
#define NAGE 6
#define HIST 257
static const int ages[NAGE] = {8, 16, 32, 64, 128, 256};
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

static long vA, vB, vZ, merges_dev, region_elems, region_hist[8], nviol_hist[8];
static long cnt_change_up, cnt_change_down;

/* the reference's merge; classifies each element against the steady prediction */
static void merge_ref(C* main_, int* nm, double* T0, const C* t, int np, double tempW, int classify) {
  C out[MAXM];
  int n = 0, mi = 0, ti = 0, dev = 0, in_region = 0, nv = 0, relems = 0;
  double T = *T0 + tempW, mw = 0, last = 0;
  while (mi < *nm || ti < np) {
    C nt = ti < np ? t[ti] : (C){INFINITY, 0};
    C nmn = mi < *nm ? main_[mi] : (C){INFINITY, 0};
    C x;
    int is_main;
    if (nmn.m < nt.m) { x = nmn; mi++; is_main = 1; } else { x = nt; ti++; is_main = 0; }
    double ni = kq((mw + x.w) / T);
    int starts = ni - last > 1 || n == 0;
    if (starts) {
      out[n++] = x;
      last = kq(mw / T);
    } else {
      out[n - 1].w += x.w;
      out[n - 1].m += (x.m - out[n - 1].m) * x.w / out[n - 1].w;
    }
    mw += x.w;
    if (classify && *nm > 0) {
      int viol = 0;
      if (is_main && !starts) { vB++; viol = 1; }
      if (!is_main && starts) {
        if (mi == 0) vZ++; else vA++;
        viol = 1;
      }
      if (viol) { nv++; dev = 1; in_region = 1; }
      if (in_region) {
        relems++;
        if (is_main && starts && !viol) in_region = 0;
      }
    }
  }
  if (classify && *nm > 0) {
    if (n > *nm) cnt_change_up++;
    if (n < *nm) cnt_change_down++;
    if (dev) {
      merges_dev++;
      region_elems += relems;
      int b = relems < 2 ? 0 : relems < 4 ? 1 : relems < 8 ? 2 : relems < 16 ? 3 : relems < 32 ? 4 : 5;
      region_hist[b]++;
      nviol_hist[nv < 7 ? nv : 7]++;
    }
  }
  memcpy(main_, out, n * sizeof(C));
  *nm = n;
  *T0 = T;
}

static int pos_of(const double* m, int nm, double v) { /* #means < v */
  int lo = 0, hi = nm;
  while (lo < hi) {
    int md = (lo + hi) / 2;
    if (m[md] < v) lo = md + 1; else hi = md;
  }
  return lo;
}

int main(int argc, char** argv) {
  long N = argc > 1 ? atol(argv[1]) : 17000000;
  long merges = N / TC;
  static double hm[HIST][MAXM];
  static int hn[HIST];
  long flips[NAGE] = {0}, flip_merges[NAGE] = {0}, struct_diff[NAGE] = {0}, considered[NAGE] = {0};
  C ref[MAXM];
  int nr = 0;
  double Tr = 0;
  long steady_from = 0;
  for (long g = 0; g < merges; g++) {
    C ch[TC];
    double tw = 0;
    for (int p = 0; p < TC; p++) {
      double u = u01();
      ch[p].m = exp(log(50.0) + gauss());
      ch[p].w = u < 0.05 ? 10 : u < 0.1 ? 2 : 1;
      tw += ch[p].w;
    }
    qsort(ch, TC, sizeof(C), cmpc);
    /* flips against stale means (the current means are merge g's input) */
    int h = (int)(g % HIST);
    for (int i = 0; i < nr; i++) hm[h][i] = ref[i].m;
    hn[h] = nr;
    if (Tr >= 8192) {
      if (!steady_from) steady_from = g;
      for (int a = 0; a < NAGE; a++) {
        if (g < ages[a]) continue;
        int ho = (int)((g - ages[a]) % HIST);
        considered[a]++;
        if (hn[ho] != nr) { struct_diff[a]++; continue; }
        int f = 0;
        for (int p = 0; p < TC; p++) f += pos_of(hm[ho], nr, ch[p].m) != pos_of(hm[h], nr, ch[p].m);
        flips[a] += f;
        flip_merges[a] += f > 0;
      }
    }
    merge_ref(ref, &nr, &Tr, ch, TC, tw, Tr >= 8192);
  }
  long sm = merges - steady_from;
  printf("N=%ld merges=%ld steady_from=%ld centroids_end=%d\n", N, merges, steady_from, nr);
  printf("merges with a violation: %ld (1 in %.1f); A temp starts %ld, B main joins %ld, Z temp before main0 %ld\n",
         merges_dev, (double)sm / (merges_dev ? merges_dev : 1), vA, vB, vZ);
  printf("centroid count up %ld down %ld; region elements avg %.2f\n", cnt_change_up, cnt_change_down,
         (double)region_elems / (merges_dev ? merges_dev : 1));
  printf("region size hist [1,2-3,4-7,8-15,16-31,32+]:");
  for (int b = 0; b < 6; b++) printf(" %ld", region_hist[b]);
  printf("\nviolations per deviating merge [0..7+]:");
  for (int b = 0; b < 8; b++) printf(" %ld", nviol_hist[b]);
  printf("\n");
  for (int a = 0; a < NAGE; a++)
    printf("age %3d: merges with a flip %ld (1 in %.1f), flips %ld, structure changed %ld of %ld\n", ages[a],
           flip_merges[a], (double)considered[a] / (flip_merges[a] ? flip_merges[a] : 1), flips[a], struct_diff[a],
           considered[a]);
  return 0;
}

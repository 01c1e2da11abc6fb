/* Study (not product): how often does a window of B consecutive t-digest merges keep the
 * "old centroids start, temps join" structure, and how often does a per-centroid bound over the
 * window (k(max q_{i+1}) - k(min q_i) <= 1 - band; k(min r_i) - k(max q_{i-1}) > 1 + band)
 * prove it without per-merge k evaluations?  Restates mergeAllTemps / mergeOne
 * (tdigest/merging_digest.go:121-236) with libm asin, lognormal samples, rates 1/0.5/0.1.
 *   gcc -O2 -o /tmp/bps tools/study/batch_predict_sim.c -lm && /tmp/bps 17000000 32        */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef struct { double m, w; } C;
static double delta = 100;
static double kq(double q) { return delta * (asin(2 * q - 1) / M_PI + 0.5); }
static uint64_t rs = 88172645463325252ull;
static double u01(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (rs >> 11) * (1.0 / 9007199254740992.0); }
static double gauss(void) { double a = u01(), b = u01(); return sqrt(-2 * log(a + 1e-300)) * cos(2 * M_PI * b); }
static int cmpc(const void* a, const void* b) { double x = ((C*)a)->m, y = ((C*)b)->m; return x < y ? -1 : x > y; }
#define MAXM 512
int main(int argc, char** argv) {
  long N = argc > 1 ? atol(argv[1]) : 1000000;
  int B = argc > 2 ? atoi(argv[2]) : 32;
  const int TC = 42;
  C main_[MAXM], nm[MAXM], tmp[64];
  int m = 0;
  double T0 = 0;
  long merges = N / TC;
  /* per-window accumulators */
  static double qmin[MAXM], qmax[MAXM], rmin[MAXM], snap[MAXM];
  long pos_fail_windows = 0;
  int wposok = 1;
  int wn = 0, wok = 1, wm = -1;
  long windows = 0, win_struct = 0, win_bound = 0, struct_fail_merges = 0;
  long cent_bound_fail = 0, cent_total = 0;
  for (long g = 0; g < merges; g++) {
    double tw = 0;
    int mo0 = m;
    C pre[MAXM];
    memcpy(pre, main_, m * sizeof(C));
    for (int t = 0; t < TC; t++) {
      double u = u01();
      tmp[t].m = exp(log(50.0) + gauss());
      tmp[t].w = u < 0.05 ? 10 : u < 0.1 ? 2 : 1;
      tw += tmp[t].w;
    }
    qsort(tmp, TC, sizeof(C), cmpc);
    double T = T0 + tw, mw = 0, last = 0;
    int n = 0, mi = 0, ti = 0, pred = 1;
    double S[MAXM], R[MAXM];
    while (mi < m || ti < TC) {
      C nt = ti < TC ? tmp[ti] : (C){INFINITY, 0};
      C nmn = mi < m ? main_[mi] : (C){INFINITY, 0};
      int ismain = nmn.m < nt.m;
      C x = ismain ? nmn : nt;
      if (ismain) { S[mi] = mw; R[mi] = mw + x.w; mi++; } else ti++;
      double ni = kq((mw + x.w) / T);
      int start = ni - last > 1 || n == 0;
      if (start) { nm[n++] = x; last = kq(mw / T); } else { nm[n - 1].w += x.w; nm[n - 1].m += (x.m - nm[n - 1].m) * x.w / nm[n - 1].w; }
      if (start != ismain) pred = 0;
      mw += x.w;
    }
    int mo = m;
    memcpy(main_, nm, n * sizeof(C));
    m = n;
    T0 = T;
    if (g < 2000) continue;
    if (!pred) struct_fail_merges++;
    /* window bookkeeping (aligned windows of B merges) */
    if (wn == 0) { wposok = 1; for (int i = 0; i < mo; i++) snap[i] = pre[i].m; }
    if (wn == 0) { wok = 1; wm = mo; for (int i = 0; i <= mo; i++) { qmin[i] = 2; qmax[i] = -1; rmin[i] = 2; } }
    if (!pred || mo != wm) wok = 0;
    if (wok && wposok) {
      for (int i = 0; i < mo0; i++) {
        int a = 0, b = 0;
        for (int t = 0; t < TC; t++) { a += tmp[t].m <= snap[i]; b += tmp[t].m <= pre[i].m; }
        if (a != b) wposok = 0;
      }
    }
    if (wok) {
      for (int i = 0; i < mo; i++) {
        double q = S[i] / T, r = R[i] / T;
        if (q < qmin[i]) qmin[i] = q;
        if (q > qmax[i]) qmax[i] = q;
        if (r < rmin[i]) rmin[i] = r;
      }
      qmin[mo] = qmax[mo] = 1.0;
    }
    if (++wn == B) {
      windows++;
      if (wok && !wposok) pos_fail_windows++;
      if (wok) {
        win_struct++;
        int okb = 1;
        for (int i = 0; i < wm; i++) {
          int f = 0;
          if (kq(qmax[i + 1]) - kq(qmin[i]) > 1 - 1e-9) f = 1;
          if (i >= 1 && kq(rmin[i]) - kq(qmax[i - 1]) <= 1 + 1e-9) f = 1;
          cent_bound_fail += f;
          cent_total++;
          if (f) okb = 0;
        }
        win_bound += okb;
      }
      wn = 0;
    }
  }
  printf("N=%ld B=%d merges=%ld m=%d struct_fail_rate=%.5f windows=%ld struct_ok=%.4f bound_ok=%.4f cent_bound_fail_frac=%.5f per_window=%.3f pos_fail_windows=%.4f\n",
         N, B, merges, m, (double)struct_fail_merges / (merges - 2000), windows, (double)win_struct / windows,
         (double)win_bound / windows, (double)cent_bound_fail / (cent_total ? cent_total : 1),
         (double)cent_bound_fail / (win_struct ? win_struct : 1), (double)pos_fail_windows / windows);
  return 0;
}

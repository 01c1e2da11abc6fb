// histo_exact.hip -- bit-faithful emulation of MergingDigest's incremental merge.
//
// For every key whose window so far holds at most `exact_threshold` samples the engine
// replays tdigest/merging_digest.go exactly: samples are Add()ed (97-118) into a temp
// buffer of estimateTempBuffer(delta) = 42 entries; when a 43rd arrives the temps are
// sorted by mean and mergeAllTemps (121-205) merges them with the main list (ties take
// the temp first), feeding each element to mergeOne (210-236).  Quantile (283-313)
// merges whatever is pending first.
//
// One wave (a 64-thread block) owns one key.  A hot key replays ~800 merges back to back,
// so each merge is built for latency -- no lane-0 loops over LDS:
//   tempWeight       arrival-order fold: wave sum when every weight is an integer (exact in
//                    any order), otherwise a sequential fold through v_readlane
//   sort temps       counting rank over (mean, arrival index).  When two temps share a
//                    mean but differ in weight or sign bit the order is observable, and lane
//                    0 runs Go 1.9 sort.Sort (quickSort, restated) to reproduce its ties
//   merge positions  temp: rank + #main < mean (binary search); main: j + #temps <= mean
//   mergedWeight     wave scan (integer weights) or readlane fold (any weights)
//   k-index          indexEstimate per element, one lane per element (Go's Asin restated)
//   chain            ballot over 64 k values at a time: the next centroid starts at the
//                    first element with k(W_incl/T) - k(W_start/T) > 1
//   Welford          one lane per output centroid, in element order, as mergeOne does.
// The next chunk of samples is loaded into registers before each merge so the global
// latency hides behind it.
#include "histo.h"

namespace vn {

namespace {

constexpr uint32_t kMaxTempPerLane = 4;  // tcap <= 256 (estimateTempBuffer <= 178)

__device__ __forceinline__ bool is_int_weight(double w) { return w == __builtin_floor(w) && w <= 4503599627370496.0; }

__device__ __forceinline__ double rl_d(double v, int i) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), i);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), i);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = dadd(v, __shfl_xor(v, d, 64));
  return v;
}

// ---- Go 1.9 sort.Sort(centroidList) on lane 0 (restated from oracle/oracle.c go_sort)
struct GoSortCent {
  double* v;
  double* w;
  __device__ bool less(int i, int j) const { return v[i] < v[j]; }
  __device__ void swap(int i, int j) const {
    double a = v[i]; v[i] = v[j]; v[j] = a;
    a = w[i]; w[i] = w[j]; w[j] = a;
  }
  __device__ void insertion(int a, int b) const {
    for (int i = a + 1; i < b; i++)
      for (int j = i; j > a && less(j, j - 1); j--) swap(j, j - 1);
  }
  __device__ void sift_down(int lo, int hi, int first) const {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && less(first + child, first + child + 1)) child++;
      if (!less(first + root, first + child)) return;
      swap(first + root, first + child);
      root = child;
    }
  }
  __device__ void heap(int a, int b) const {
    int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
      swap(first, first + i);
      sift_down(lo, i, first);
    }
  }
  __device__ void median3(int m1, int m0, int m2) const {
    if (less(m1, m0)) swap(m1, m0);
    if (less(m2, m1)) {
      swap(m2, m1);
      if (less(m1, m0)) swap(m1, m0);
    }
  }
  __device__ void pivot(int lo, int hi, int& midlo, int& midhi) const {
    int m = lo + (hi - lo) / 2;
    if (hi - lo > 40) {
      int t = (hi - lo) / 8;
      median3(lo, lo + t, lo + 2 * t);
      median3(m, m - t, m + t);
      median3(hi - 1, hi - 1 - t, hi - 1 - 2 * t);
    }
    median3(lo, m, hi - 1);
    int p = lo, a = lo + 1, c = hi - 1;
    for (; a < c && less(a, p); a++) {}
    int b = a;
    for (;;) {
      for (; b < c && !less(p, b); b++) {}
      for (; b < c && less(p, c - 1); c--) {}
      if (b >= c) break;
      swap(b, c - 1);
      b++;
      c--;
    }
    bool protect = hi - c < 5;
    if (!protect && hi - c < (hi - lo) / 4) {
      int dups = 0;
      if (!less(p, hi - 1)) { swap(c, hi - 1); c++; dups++; }
      if (!less(b - 1, p)) { b--; dups++; }
      if (!less(m, p)) { swap(m, b - 1); b--; dups++; }
      protect = dups > 1;
    }
    if (protect) {
      for (;;) {
        for (; a < b && !less(b - 1, p); b--) {}
        for (; a < b && less(a, p); a++) {}
        if (a >= b) break;
        swap(a, b - 1);
        a++;
        b--;
      }
    }
    swap(p, b - 1);
    midlo = b - 1;
    midhi = c;
  }
  // quickSort with an explicit stack: the recursive calls work on disjoint ranges, so the
  // order in which they run does not change the result.
  __device__ void sort(int n) const {
    int depth = 0;
    for (int i = n; i > 0; i >>= 1) depth++;
    int sa[24], sb[24], sd[24], top = 0;  // depth <= 2*log2(n) + 1 frames
    sa[0] = 0; sb[0] = n; sd[0] = depth * 2; top = 1;
    while (top > 0) {
      top--;
      int a = sa[top], b = sb[top], d = sd[top];
      bool done = false;
      while (b - a > 12) {
        if (d == 0) { heap(a, b); done = true; break; }
        d--;
        int mlo, mhi;
        pivot(a, b, mlo, mhi);
        if (mlo - a < b - mhi) { sa[top] = a; sb[top] = mlo; sd[top] = d; top++; a = mhi; }
        else { sa[top] = mhi; sb[top] = b; sd[top] = d; top++; b = mlo; }
      }
      if (!done && b - a > 1) {
        for (int i = a + 6; i < b; i++)
          if (less(i, i - 6)) swap(i, i - 6);
        insertion(a, b);
      }
    }
  }
};

struct Lds {
  double *mm, *mw;       // main centroids [capc]
  double *tv, *tw;       // temps in Add order [TP]
  double *sv, *sw;       // Go-sorted temps (tie fallback) [TP]
  double *gm, *gw, *kin; // merged elements [capc + TP]
  uint32_t* starts;      // [capc + TP + 1]
  uint32_t* flag;        // [4]
};

// #main centroids with mean < v
__device__ __forceinline__ uint32_t main_below(const double* mm, uint32_t nm, double v) {
  uint32_t l = 0, h = nm;
  while (l < h) {
    uint32_t md = (l + h) >> 1;
    if (mm[md] < v) l = md + 1;
    else h = md;
  }
  return l;
}

// One mergeAllTemps of the np pending temps into main.
__device__ void exact_merge(const ExactCtx& x, const Lds& L, uint32_t& nm, double& mainW, uint32_t np) {
  const uint32_t lane = threadIdx.x;
  // ---- td.tempWeight (sequential sum in Add order)
  bool tint = true;
  double part = 0.0;
  for (uint32_t t = lane; t < np; t += 64) {
    double w = L.tw[t];
    tint &= is_int_weight(w);
    part = dadd(part, w);
  }
  double tempW = 0.0;
  tint = __all(tint);
  if (tint) tempW = wave_sum(part);
  if (!tint || !(tempW <= 9007199254740992.0)) {
    tempW = 0.0;
    for (uint32_t b = 0; b < np; b += 64) {
      double w = (b + lane < np) ? L.tw[b + lane] : 0.0;
      const uint32_t c = min(64u, np - b);
      for (uint32_t i = 0; i < c; i++) tempW = dadd(tempW, rl_d(w, (int)i));
    }
  }
  const double T = dadd(mainW, tempW);  // totalWeight := td.mainWeight + td.tempWeight

  // ---- temp ranks by (mean, Add index); detect observable ties
  uint32_t rank[kMaxTempPerLane];
  double tvr[kMaxTempPerLane], twr[kMaxTempPerLane];
  bool tie = false;
#pragma unroll
  for (uint32_t q = 0; q < kMaxTempPerLane; q++) {
    const uint32_t t = q * 64 + lane;
    rank[q] = 0;
    tvr[q] = 0.0;
    twr[q] = 0.0;
    if (t < np) {
      const double v = L.tv[t], w = L.tw[t];
      uint32_t r = 0;
      for (uint32_t u = 0; u < np; u++) {
        const double vu = L.tv[u];
        r += (vu < v) || (vu == v && u < t);
        if (vu == v && u != t)
          tie |= (__double_as_longlong(vu) != __double_as_longlong(v)) || (L.tw[u] != w);
      }
      rank[q] = r;
      tvr[q] = v;
      twr[q] = w;
    }
  }
  if (__any(tie)) {
    // Go's unstable quickSort decides the order of equal means: reproduce it
    for (uint32_t t = lane; t < np; t += 64) {
      L.sv[t] = L.tv[t];
      L.sw[t] = L.tw[t];
    }
    __syncthreads();
    if (lane == 0) GoSortCent{L.sv, L.sw}.sort((int)np);
    __syncthreads();
    for (uint32_t r = lane; r < np; r += 64) {
      const double v = L.sv[r];
      const uint32_t p = r + main_below(L.mm, nm, v);
      L.gm[p] = v;
      L.gw[p] = L.sw[r];
    }
  } else {
#pragma unroll
    for (uint32_t q = 0; q < kMaxTempPerLane; q++) {
      if (q * 64 + lane < np) {
        const uint32_t p = rank[q] + main_below(L.mm, nm, tvr[q]);
        L.gm[p] = tvr[q];
        L.gw[p] = twr[q];
      }
    }
  }
  for (uint32_t j = lane; j < nm; j += 64) {
    const double v = L.mm[j];
    uint32_t c = 0;
    for (uint32_t u = 0; u < np; u++) c += L.tv[u] <= v;
    L.gm[j + c] = v;
    L.gw[j + c] = L.mw[j];
  }
  __syncthreads();

  // ---- mergedWeight prefix (inclusive) -> k-index, one lane per element
  const uint32_t m = nm + np;
  bool wint = true;
  for (uint32_t j = lane; j < m; j += 64) wint &= is_int_weight(L.gw[j]);
  wint = __all(wint) && T <= 9007199254740992.0;
  double carry = 0.0;
  for (uint32_t b = 0; b < m; b += 64) {
    const uint32_t j = b + lane;
    double w = j < m ? L.gw[j] : 0.0;
    double incl;
    if (wint) {
      double v = w;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        double o = __shfl_up(v, d, 64);
        if ((int)lane >= d) v = dadd(v, o);
      }
      incl = dadd(carry, v);
    } else {
      incl = 0.0;
      double run = carry;
      const uint32_t c = min(64u, m - b);
      for (uint32_t i = 0; i < c; i++) {
        run = dadd(run, rl_d(w, (int)i));
        if (i == lane) incl = run;
      }
    }
    carry = rl_d(incl, (int)min(63u, m - b - 1));
    if (j < m) L.kin[j] = index_estimate(x.delta, ddiv(incl, T));
  }

  // ---- greedy chain (mergeOne): ballot over 64 k values at a time
  const double k0 = index_estimate(x.delta, 0.0);
  uint32_t nc = 0;
  double base = k0;
  double kprev_carry = k0;  // k of the element before the group (k(0) before element 0)
  bool overflow = false;
  for (uint32_t b = 0; b < m && !overflow; b += 64) {
    const uint32_t j = b + lane;
    const bool valid = j < m;
    const double kv = valid ? L.kin[j] : 0.0;  // written by this lane above
    double kp = __shfl_up(kv, 1, 64);
    if (lane == 0) kp = kprev_carry;
    uint32_t from = 0;
    for (;;) {
      const bool c = valid && lane >= from && (nc == 0 || dsub(kv, base) > 1.0);
      const uint64_t bal = __ballot(c);
      if (!bal) break;
      const uint32_t f = (uint32_t)__builtin_ctzll(bal);
      if (nc >= x.capc) { overflow = true; break; }
      if (lane == 0) L.starts[nc] = b + f;
      nc++;
      base = rl_d(kp, (int)f);  // k(W_start / T): the k of the element before the start
      from = f + 1;
    }
    kprev_carry = rl_d(kv, 63);
  }
  if (overflow && lane == 0) atomicOr(x.err, 1u);
  if (lane == 0) L.starts[nc] = m;
  __syncthreads();

  // ---- Welford per centroid, in element order
  for (uint32_t c = lane; c < nc; c += 64) {
    const uint32_t a = L.starts[c], e = L.starts[c + 1];
    double mean = L.gm[a], W = L.gw[a];
    for (uint32_t j = a + 1; j < e; j++) {
      const double wt = L.gw[j];
      W = dadd(W, wt);
      mean = dadd(mean, ddiv(dmul(dsub(L.gm[j], mean), wt), W));
    }
    L.mm[c] = mean;
    L.mw[c] = W;
  }
  __syncthreads();
  nm = nc;
  mainW = T;
}

__device__ __forceinline__ uint32_t round64(uint32_t v) { return (v + 63u) & ~63u; }

}  // namespace

// One 64-thread block (one wave) per key.
__global__ __launch_bounds__(64) void k_histo_exact(ExactCtx x) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t k = blockIdx.x, lane = threadIdx.x;
  if (k >= x.nkeys) return;
  const uint32_t capc = x.capc, tcap = x.tcap;
  const uint32_t TP = round64(tcap + 1);
  Lds L;
  L.mm = reinterpret_cast<double*>(smem);
  L.mw = L.mm + capc;
  L.tv = L.mw + capc;
  L.tw = L.tv + TP;
  L.sv = L.tw + TP;
  L.sw = L.sv + TP;
  L.gm = L.sw + TP;
  L.gw = L.gm + capc + TP;
  L.kin = L.gw + capc + TP;
  L.starts = reinterpret_cast<uint32_t*>(L.kin + capc + TP);
  L.flag = L.starts + capc + TP + 1;

  const uint32_t s = x.keys[k];
  const uint32_t nex = x.nex ? x.nex[k] : 0u;
  const bool final_merge = x.flush_mode || (x.hot && x.hot[k]);
  uint32_t np = x.hpend[s];
  if (nex == 0 && !(final_merge && np > 0)) return;

  const uint8_t cur = x.hcur[s];
  double* cmg = (cur ? x.cm1 : x.cm0) + (uint64_t)s * capc;
  double* cwg = (cur ? x.cw1 : x.cw0) + (uint64_t)s * capc;
  uint32_t nm = x.hncent[s];
  double* h = x.hst + (uint64_t)s * VN_HISTO_STATS;
  double mainW = h[7];
  const uint32_t lo = x.start[s];

  // first chunk of samples into registers (overlaps the state load)
  uint32_t r = 0;
  if (nex) r = min(np == tcap ? tcap : tcap - np, nex);
  double cv[kMaxTempPerLane];
  float cr[kMaxTempPerLane];
#pragma unroll
  for (uint32_t q = 0; q < kMaxTempPerLane; q++) {
    const uint32_t i = q * 64 + lane;
    if (i < r) {
      cv[q] = bitsd(x.A[lo + i]);
      cr[q] = __uint_as_float((uint32_t)x.B[lo + i]);
    }
  }
  for (uint32_t j = lane; j < nm; j += 64) {
    L.mm[j] = cmg[j];
    L.mw[j] = cwg[j];
  }
  const double* pv = x.hpv + (uint64_t)s * tcap;
  const double* pw = x.hpw + (uint64_t)s * tcap;
  for (uint32_t j = lane; j < np; j += 64) {
    L.tv[j] = pv[j];
    L.tw[j] = pw[j];
  }
  __syncthreads();

  // Histo.Sample local statistics of the replayed samples (samplers.go:346-356)
  double sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf;
  if (nex && np == tcap) {  // Add finds the temp list full: mergeAllTemps first
    exact_merge(x, L, nm, mainW, np);
    np = 0;
  }
  uint32_t pos = 0;
  while (r) {
#pragma unroll
    for (uint32_t q = 0; q < kMaxTempPerLane; q++) {
      const uint32_t i = q * 64 + lane;
      if (i < r) {
        const double v = cv[q];
        const double wt = (double)(1.0f / cr[q]);  // float64(1/sampleRate) in float32
        L.tv[np + i] = v;
        L.tw[np + i] = wt;
        sw = dadd(sw, wt);
        mn = min_go(mn, v);
        mx = max_go(mx, v);
        sxw = dadd(sxw, dmul(v, wt));
        srw = dadd(srw, dmul(ddiv(1.0, v), wt));
      }
    }
    np += r;
    pos += r;
    if (pos >= nex) break;
    // the temp list is full (np == tcap): prefetch the next chunk, then merge
    r = min(tcap, nex - pos);
#pragma unroll
    for (uint32_t q = 0; q < kMaxTempPerLane; q++) {
      const uint32_t i = q * 64 + lane;
      if (i < r) {
        cv[q] = bitsd(x.A[lo + pos + i]);
        cr[q] = __uint_as_float((uint32_t)x.B[lo + pos + i]);
      }
    }
    __syncthreads();
    exact_merge(x, L, nm, mainW, np);
    np = 0;
  }
  __syncthreads();
  if (final_merge && np > 0) {
    exact_merge(x, L, nm, mainW, np);
    np = 0;
  }
  // ---- write back the key's digest and statistics
  for (uint32_t j = lane; j < nm; j += 64) {
    cmg[j] = L.mm[j];
    cwg[j] = L.mw[j];
  }
  double* qv = x.hpv + (uint64_t)s * tcap;
  double* qw = x.hpw + (uint64_t)s * tcap;
  for (uint32_t j = lane; j < np; j += 64) {
    qv[j] = L.tv[j];
    qw[j] = L.tw[j];
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    sw = dadd(sw, __shfl_xor(sw, d, 64));
    sxw = dadd(sxw, __shfl_xor(sxw, d, 64));
    srw = dadd(srw, __shfl_xor(srw, d, 64));
    mn = min_go(mn, __shfl_xor(mn, d, 64));
    mx = max_go(mx, __shfl_xor(mx, d, 64));
  }
  if (lane == 0) {
    x.hncent[s] = nm;
    x.hpend[s] = np;
    h[7] = mainW;  // td.mainWeight (the pending temps' weight is added when they merge)
    if (nex) {
      h[0] = dadd(h[0], sw);
      h[1] = min_go(h[1], mn);
      h[2] = max_go(h[2], mx);
      h[3] = dadd(h[3], sxw);
      h[4] = dadd(h[4], srw);
      h[5] = min_go(h[5], mn);
      h[6] = max_go(h[6], mx);
    }
  }
}

size_t exact_smem_bytes(uint32_t capc, uint32_t tcap) {
  const uint32_t TP = (tcap + 1 + 63u) & ~63u;
  return sizeof(double) * (2 * capc + 4 * TP + 3 * (capc + TP)) + sizeof(uint32_t) * (capc + TP + 1 + 4);
}

void launch_histo_exact(const ExactCtx& x, hipStream_t st) {
  if (!x.nkeys) return;
  if (x.tcap > 64 * kMaxTempPerLane) throw std::runtime_error("temp buffer larger than the exact kernel supports");
  size_t sm = exact_smem_bytes(x.capc, x.tcap);
  hipLaunchKernelGGL(k_histo_exact, dim3(x.nkeys), dim3(64), sm, st, x);
}

}  // namespace vn

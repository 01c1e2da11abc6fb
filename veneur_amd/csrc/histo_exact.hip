// histo_exact.hip -- bit-faithful emulation of MergingDigest's incremental merge.
//
// For every key whose window so far holds at most `exact_threshold` samples the engine
// replays tdigest/merging_digest.go exactly: samples are Add()ed (97-118) into a temp
// buffer of estimateTempBuffer(delta) = 42 entries; when a 43rd arrives the temps are
// sorted by mean and mergeAllTemps (121-205) merges them with the main list (ties take
// the temp first), feeding each element to mergeOne (210-236).  Quantile (283-313)
// merges whatever is pending first.
//
// One wave (a 64-thread block) owns one key; lanes exchange data through LDS with
// wave_lds_sync() (no workgroup barrier, so prefetched global loads stay in flight).  A hot key replays ~800 merges back to back,
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
#include "wave_dpp.h"

namespace vn {

// indexEstimate's division form per call site (gomath.h VN_INDEX_NR; diagnostics builds only)
#ifndef VN_NR_ONE
#define VN_NR_ONE VN_INDEX_NR
#endif
#ifndef VN_NR_FOUR
#define VN_NR_FOUR VN_INDEX_NR
#endif
#ifndef VN_NR_G
#define VN_NR_G VN_INDEX_NR
#endif
#ifndef VN_EXACT_LDS_PAD
#define VN_EXACT_LDS_PAD 0  // occupancy experiments only (tools/ab_variant.sh)
#endif
// LDS bytes of the replay's layout (lds_layout), on the host and the device
__host__ __device__ inline size_t exact_smem_bytes_hd(uint32_t capc, uint32_t tcap) {
  const uint32_t TP = (tcap + 1 + 63u) & ~63u, JW = capc + TP + 1 > 320u ? capc + TP + 1 : 320u;
  uint32_t levels = 1;
  while ((1u << levels) <= capc) levels++;
  const uint32_t kin = JW <= 2 * capc ? 0 : JW;  // lds_layout: kin in the main tile when it fits
  (void)levels;
  // lds_layout: the pending temps in the chain tables' region when it holds them
  const uint32_t tables = sizeof(uint16_t) * 3 * JW, temps = 6 * JW >= 16 * TP ? 0u : 16u * TP + 8u;
  return sizeof(double) * (2 * capc + 2 * TP + 2 * JW + kin) + tables + temps + 16 + VN_EXACT_LDS_PAD;
}

#ifdef VN_ASM_MARK  // (reading the assembly: a comment at a phase boundary)
#define ASM_MARK(x) asm volatile("; MARK " x)
#else
#define ASM_MARK(x)
#endif
#ifdef VN_EXACT_PROF
// profiling build only (tools/exact_profile.py): cycles per merge phase of block 0
__device__ unsigned long long g_exact_prof[64];
__device__ __forceinline__ long long prof_stamp() {  // a scheduling fence around the stamp
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return (long long)t;
}
#ifdef VN_PROF_NOSTAMP  // (diagnosing the profiling build: counters without the clock stamps)
#define PROF_T(v) const long long v = 0
#else
#define PROF_T(v) const long long v = prof_stamp()
#endif
#ifdef VN_PROF_NOATOMIC  // (... or the stamps without the counters' atomics)
#define PROF_ADD(i, a, b) (void)((b) - (a))
#define PROF_ADDW(i, a, b) (void)((b) - (a))
#define PROF_CNT(i, pred)
#else
#define PROF_ADD(i, a, b) \
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_exact_prof[i], (unsigned long long)((b) - (a)))
// per wave (lane 0 of each wave of block 0): slot i + wave
#define PROF_ADDW(i, a, b) \
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) atomicAdd(&g_exact_prof[(i) + (threadIdx.x >> 6)], (unsigned long long)((b) - (a)))
// per wave: the number of lanes where pred holds
#define PROF_CNT(i, pred)                                                                              \
  {                                                                                                    \
    const uint64_t _m = __ballot(pred);                                                                \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) atomicAdd(&g_exact_prof[i], (unsigned long long)__popcll(_m)); \
  }
#endif
#else
#define PROF_CNT(i, pred)
#define PROF_ADDW(i, a, b)
#define PROF_T(v)
#define PROF_ADD(i, a, b)
#endif

namespace {

constexpr uint32_t kMaxTempPerLane = 4;  // tcap <= 256 (estimateTempBuffer <= 178)

// LDS pointers typed in address space 3, so every access through them is a ds_read/ds_write.
// A plain double* into LDS that reaches a function through memory (a struct passed by
// reference, a non-inlined callee) loses its address space and compiles to flat loads, which
// are slower and wait on both vmcnt and lgkmcnt.
typedef __attribute__((address_space(3))) double ldsf64;
typedef __attribute__((address_space(3))) uint32_t ldsu32;
typedef __attribute__((address_space(3))) uint16_t ldsu16;

// a merge's result (returned by value: references to the caller's locals would put them in
// scratch memory when the callee is not inlined)
struct NmW {
  uint32_t nm;
  double w;
};

__device__ __forceinline__ bool is_int_weight(double w) { return w == __builtin_floor(w) && w <= 4503599627370496.0; }
// Weights whose sums are exact in any order.  Integers below 2^52: any partial sum below 2^53
// is an integer.  Or multiples of 2^-23 up to 2^30 -- every 1/rate a float32 sample rate gives
// (float32 values >= 1 are such multiples), and sums of them, like an imported centroid's
// weight: a partial sum below 2^30 is then k * 2^-23 with k < 2^53.  The total bound that goes
// with a set of weights: exact_total_limit(all integers).
__device__ __forceinline__ bool is_exact_weight(double w) {
  const double s = w * 8388608.0;  // (a power of two: exact)
  // (and >= 1, as every weight a sampler adds: merge_fast's monotone-k argument needs it)
  return (w == __builtin_floor(w) && w <= 4503599627370496.0) || (s == __builtin_floor(s) && w >= 1.0 && w <= 1073741824.0);
}
__device__ __forceinline__ double exact_total_limit(bool all_int) { return all_int ? 9007199254740992.0 : 1073741824.0; }

__device__ __forceinline__ double rl_d(double v, int i) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), i);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), i);
  return __hiloint2double(hi, lo);
}

// Fence the next chunk's prefetch behind the current chunk's values: each listed value is
// materialised in a register here (its load waited for) and no memory access below may move
// above.  Without it the loads of chunk c + 1 issue first and the compiler's wait-count
// insertion, conservative across their exec-masked blocks, then waits for those NEW loads at the
// first use of an old value -- an L2/HBM round trip at the start of every merge.
__device__ __forceinline__ void hold2(double& a, double& b) { asm volatile("" : "+v"(a), "+v"(b)::"memory"); }
__device__ __forceinline__ void hold_stats(double& a, double& b, double& c, double& d, double& e, double& f,
                                           double& g) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g)::"memory");
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = dadd(v, __shfl_xor(v, d, 64));
  return v;
}

// ---- Go 1.9 sort.Sort(centroidList) on lane 0 (restated from oracle/oracle.c go_sort)
struct GoSortCent {
  ldsf64* v;
  ldsf64* w;
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

// what a merge needs from ExactCtx, by value (a reference to the kernel-argument struct
// would force a copy of it into scratch memory)
struct MergeParams {
  double delta;
  uint32_t capc;
  uint32_t* err;
};
// Out-of-line functions take MergeParams as three scalars: the AMDGPU calling convention passes
// at most 16 registers of aggregates directly, and MergeParams (5) + Lds (13) would put Lds on the
// private stack -- 52 B per lane written before every call and read back by the callee
#define MP_PARAMS const double mp_delta_, const uint32_t mp_capc_, uint32_t* const mp_err_
#define MP_ARGS(m) (m).delta, (m).capc, (m).err
#define MP_UNPACK(name) const MergeParams name{mp_delta_, mp_capc_, mp_err_}

struct Lds {
  ldsf64 *mm, *mw;        // main centroids [capc]
  ldsf64 *tv, *tw;        // pending temps in Add order [TP]
  ldsf64 *sv, *sw;        // sorted temps of the merge being done [TP]
  ldsf64 *gm, *gw, *kin;  // merged elements [JW]
  ldsu16* jump16;         // next-start tables next^(2^lv), two [JW] u16 in turn (entries <= JW < 65536)
  ldsu16* starts;         // [JW]
  uint32_t JW, levels;
};

// the replay's LDS layout (dynamic shared memory, exact_smem_bytes)
__device__ __forceinline__ Lds lds_layout(char* smem, uint32_t capc, uint32_t TP) {
  Lds L;
  L.JW = max(capc + TP + 1, 320u);  // >= 64 * kR: the fast merge pads its tables
  L.levels = 1;
  while ((1u << L.levels) <= capc) L.levels++;
  L.mm = (ldsf64*)smem;
  L.mw = L.mm + capc;
  L.sv = L.mw + capc;
  L.sw = L.sv + TP;
  L.gm = L.sw + TP;
  L.gw = L.gm + L.JW;
  // k of the merged elements: written after the merge has read the main centroids for the last
  // time and dead before the centroid pass writes the new ones, so it lives in the main tile
  // when it fits (delta 100: 17.3 KiB per key, 9 waves per CU instead of 8)
  const bool kin_in_main = L.JW <= 2 * capc;
  L.kin = kin_in_main ? L.mm : L.gw + L.JW;
  L.starts = (ldsu16*)(L.gw + L.JW + (kin_in_main ? 0 : L.JW));
  L.jump16 = L.starts + L.JW;
  // the pending temps (Add order) are dead during every merge -- a merge takes all of them, after
  // sort_temps has read them into sv/sw, and appends resume after it -- so they live in the chain
  // tables' region when it holds them (1 KiB less per key at delta 100)
  L.tv = 6 * L.JW >= 16 * TP ? (ldsf64*)L.starts
                             : (ldsf64*)((reinterpret_cast<uintptr_t>(L.jump16 + 2 * L.JW) + 7) & ~(uintptr_t)7);
  L.tw = L.tv + TP;
  return L;
}

// #main centroids with mean < v (main is sorted by mean)
__device__ __forceinline__ uint32_t main_below(const ldsf64* mm, uint32_t nm, double v) {
  uint32_t l = 0, h = nm;
  while (l < h) {
    uint32_t md = (l + h) >> 1;
    if (mm[md] < v) l = md + 1;
    else h = md;
  }
  return l;
}
// #sorted temps with mean <= v
__device__ __forceinline__ uint32_t temps_le(const ldsf64* sv, uint32_t np, double v) {
  uint32_t l = 0, h = np;
  while (l < h) {
    uint32_t md = (l + h) >> 1;
    if (sv[md] <= v) l = md + 1;
    else h = md;
  }
  return l;
}

// td.tempWeight of np temps in Add order: the sequential fold, computed as a wave sum when
// every weight is an integer and the total stays below 2^53 (then every order is exact).
__device__ double temp_weight(const ldsf64* tw, uint32_t np) {
  const uint32_t lane = threadIdx.x & 63;
  bool tint = true, tex = true;
  double part = 0.0;
  for (uint32_t t = lane; t < np; t += 64) {
    double w = __builtin_fabs(tw[t]);  // the chunk sorter marks imported centroids by a negative weight
    tint &= is_int_weight(w);
    tex &= is_exact_weight(w);
    part = dadd(part, w);
  }
  double tempW = 0.0;
  tint = __all(tint);
  tex = __all(tex);
  if (tex) tempW = wave_sum(part);
  if (!tex || !(tempW <= exact_total_limit(tint))) {
    tempW = 0.0;
    for (uint32_t b = 0; b < np; b += 64) {
      double w = (b + lane < np) ? tw[b + lane] : 0.0;
      const uint32_t c = min(64u, np - b);
      w = __builtin_fabs(w);
      for (uint32_t i = 0; i < c; i++) tempW = dadd(tempW, rl_d(w, (int)i));
    }
  }
  return tempW;
}

// Sort np temps (tv/tw, Add order) into sv/sw as sort.Sort(centroidList) orders them:
// counting rank over (mean, Add index); when equal means make the order observable
// (different weights or signed zeros) lane 0 runs Go's quickSort instead.  One wave.
// (ties: Go's sort.Sort itself on one lane -- rare, out of line so the chunk sorter's inlined body
// keeps a small register budget)
__device__ __noinline__ void go_sort_lane0(ldsf64* sv, ldsf64* sw, uint32_t np) { GoSortCent{sv, sw}.sort((int)np); }
__device__ __forceinline__ void sort_temps_body(const ldsf64* tv, const ldsf64* tw, ldsf64* sv, ldsf64* sw,
                                                uint32_t np) {
  const uint32_t lane = threadIdx.x & 63;
  // Temps made of at most four ascending runs with no value repeated (an imported digest's
  // centroids arrive in ascending order: a chunk of them holds one or two runs): a temp's rank
  // is its place in its run plus, per other run, the run's temps below it (a binary search).
  // Without repeats the order is the one below, repeats or more runs take the general path.
  if (np <= 64) {
    const bool in = lane < np;
    const double v = in ? tv[lane] : 0.0;
    const double vp = __shfl_up(v, 1, 64);
    const bool desc = in && lane > 0 && v < vp, eq = in && lane > 0 && v == vp;
    const uint64_t starts = __ballot(desc) | 1ull;
    if (!__any(eq) && __popcll(starts) <= 4) {
      const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
      const uint32_t mine = 63u - (uint32_t)__builtin_clzll(starts & upto);
      uint32_t rank = lane - mine;
      bool rep = false;
      uint64_t rest = starts;
      while (rest) {
        const uint32_t a = (uint32_t)__builtin_ctzll(rest);
        rest &= rest - 1;
        const uint32_t b = rest ? (uint32_t)__builtin_ctzll(rest) : np;
        if (a == mine || !in) continue;
        uint32_t l = a, h = b;  // first temp of the run not below v
        while (l < h) {
          const uint32_t md = (l + h) >> 1;
          if (tv[md] < v) l = md + 1;
          else h = md;
        }
        rep |= l < b && tv[l] == v;
        rank += l - a;
      }
      if (!__any(rep)) {
        if (in) {
          sv[rank] = v;
          sw[rank] = tw[lane];
        }
        wave_lds_sync();
        return;
      }
    }
  }
  uint32_t rank[kMaxTempPerLane];
  double vr[kMaxTempPerLane], wr[kMaxTempPerLane];
  bool tie = false;
#pragma unroll
  for (uint32_t q = 0; q < kMaxTempPerLane; q++) {
    const uint32_t t = q * 64 + lane;
    rank[q] = 0;
    vr[q] = 0.0;
    wr[q] = 0.0;
    if (t < np) {
      const double v = tv[t], w = tw[t];
      uint32_t r = 0;
      for (uint32_t u = 0; u < np; u++) {
        const double vu = tv[u];
        r += (vu < v) || (vu == v && u < t);
        if (vu == v && u != t)
          tie |= (__double_as_longlong(vu) != __double_as_longlong(v)) || (tw[u] != w);
      }
      rank[q] = r;
      vr[q] = v;
      wr[q] = w;
    }
  }
  if (__any(tie)) {
    for (uint32_t t = lane; t < np; t += 64) {
      sv[t] = tv[t];
      sw[t] = tw[t];
    }
    wave_lds_sync();
    if (lane == 0) go_sort_lane0(sv, sw, np);
  } else {
#pragma unroll
    for (uint32_t q = 0; q < kMaxTempPerLane; q++)
      if (q * 64 + lane < np) {
        sv[rank[q]] = vr[q];
        sw[rank[q]] = wr[q];
      }
  }
  wave_lds_sync();
}
// (out of line for the replays' merges; the chunk sorter inlines the body: a call there saved and
// restored its live registers through the private stack on every chunk)
__device__ __noinline__ void sort_temps(const ldsf64* tv, const ldsf64* tw, ldsf64* sv, ldsf64* sw, uint32_t np) {
  sort_temps_body(tv, tw, sv, sw, np);
}

// mergeAllTemps of the sorted temps L.sv/L.sw (np of them, Add-order weight sum tempW)
// into main L.mm/L.mw.  One wave; every step is a parallel pass of O(log) depth.
__device__ __noinline__ NmW merge_sorted(const Lds L, MP_PARAMS, const uint32_t nm, const double mainW, uint32_t np,
                                        double tempW) {
  MP_UNPACK(x);
  const uint32_t lane = threadIdx.x;
  PROF_T(p0);
  const double T = dadd(mainW, tempW);  // totalWeight := td.mainWeight + td.tempWeight
  // ---- merged order: main first only if strictly smaller (merging_digest.go:169)
  for (uint32_t t = lane; t < np; t += 64) {
    const double v = L.sv[t];
    const uint32_t p = t + main_below(L.mm, nm, v);
    L.gm[p] = v;
    L.gw[p] = L.sw[t];
  }
  for (uint32_t j = lane; j < nm; j += 64) {
    const double v = L.mm[j];
    const uint32_t p = j + temps_le(L.sv, np, v);
    L.gm[p] = v;
    L.gw[p] = L.mw[j];
  }
  wave_lds_sync();
  PROF_T(p1);
  const uint32_t m = nm + np;
  // ---- mergedWeight prefix (inclusive), then the k-index of every element
  bool wint = true, wex = true;
  for (uint32_t j = lane; j < m; j += 64) {
    wint &= is_int_weight(L.gw[j]);
    wex &= is_exact_weight(L.gw[j]);
  }
  wint = __all(wex) && T <= exact_total_limit(__all(wint));  // (sums exact in any order)
  double carry = 0.0;
  for (uint32_t b = 0; b < m; b += 64) {
    const uint32_t j = b + lane;
    const double w = j < m ? L.gw[j] : 0.0;
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
    if (j < m) L.kin[j] = incl;
  }
  for (uint32_t b = 0; b < m; b += 256) {  // independent asin evaluations, four per lane
    double q[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t j = b + 64 * u + lane;
      q[u] = j < m ? ddiv(L.kin[j], T) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t j = b + 64 * u + lane;
      if (j < m) L.kin[j] = index_estimate(x.delta, q[u]);
    }
  }
  wave_lds_sync();
  PROF_T(p2);
  // ---- greedy chain of mergeOne (210-236).  A centroid starting at element s ends before
  // next(s) = the first j > s with k_j - k_{s-1} > 1 (k_{-1} = k(0)).  next() depends on s
  // alone, so the starts 0, next(0), next(next(0)), ... follow by pointer doubling: the starts
  // t < 2^lv extend to t < 2^(lv+1) through the table of next^(2^lv), squared beside them (two
  // tables in turn).  The binary search needs k monotone; a non-monotone k (ulp-level asin
  // wiggle) takes the sequential walk instead, so the result is always the reference's.
  const double k0 = index_estimate(x.delta, 0.0);
  bool mono = true;
  // (a NaN k is not monotone either: past 2^30 with non-integer weights the in-order prefix can
  // pass T by an ulp, q > 1 and asin NaN -- Go's comparisons then merge, which the walk reproduces)
  for (uint32_t j = lane + 1; j < m; j += 64) mono &= L.kin[j] >= L.kin[j - 1];
  mono = __all(mono);
  uint32_t nc = 0;
  bool overflow = false;
  const uint32_t capc = x.capc;
  if (mono) {
    ldsu16* J0 = L.jump16;
    for (uint32_t s = lane; s <= m; s += 64) {
      uint32_t r = m;
      if (s < m) {
        const double base = s ? L.kin[s - 1] : k0;
        uint32_t l = s + 1, h = m;
        while (l < h) {
          uint32_t md = (l + h) >> 1;
          if (dsub(L.kin[md], base) > 1.0) h = md;
          else l = md + 1;
        }
        r = l;
      }
      J0[s] = (uint16_t)r;
    }
    if (lane == 0) L.starts[0] = 0;
    wave_lds_sync();
    // start t = next^t(0) for t <= capc (2^levels > capc); entries past the chain's end are m
    for (uint32_t lv = 0; lv < L.levels; lv++) {
      const uint32_t h = 1u << lv;
      const ldsu16* Jc = L.jump16 + (lv & 1u) * L.JW;
      ldsu16* Jn = L.jump16 + ((lv & 1u) ^ 1u) * L.JW;
      for (uint32_t t = h + lane; t < 2 * h && t <= capc; t += 64) L.starts[t] = Jc[L.starts[t - h]];
      if (lv + 1 < L.levels)
        for (uint32_t s = lane; s <= m; s += 64) Jn[s] = Jc[Jc[s]];
      wave_lds_sync();
    }
    for (uint32_t t = lane; t <= capc; t += 64) {
      const bool on = L.starts[t] < m;
      nc += (uint32_t)__popcll(__ballot(on));
      overflow |= on && t == capc;
    }
    overflow = __any(overflow);
    if (nc > capc) nc = capc;
  } else {
    double base = k0, kprev_carry = k0;
    for (uint32_t b = 0; b < m && !overflow; b += 64) {
      const uint32_t j = b + lane;
      const bool valid = j < m;
      const double kv = valid ? L.kin[j] : 0.0;
      double kp = __shfl_up(kv, 1, 64);
      if (lane == 0) kp = kprev_carry;
      uint32_t from = 0;
      for (;;) {
        const bool c = valid && lane >= from && (nc == 0 || dsub(kv, base) > 1.0);
        const uint64_t bal = __ballot(c);
        if (!bal) break;
        const uint32_t f = (uint32_t)__builtin_ctzll(bal);
        if (nc >= capc) { overflow = true; break; }
        if (lane == 0) L.starts[nc] = b + f;
        nc++;
        base = rl_d(kp, (int)f);
        from = f + 1;
      }
      kprev_carry = rl_d(kv, 63);
    }
  }
  if (overflow && lane == 0) atomicOr(x.err, 1u);
  if (lane == 0) L.starts[nc] = m;
  wave_lds_sync();
  PROF_T(p3);
  // ---- Welford per centroid, in element order (weight first, then mean)
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
  wave_lds_sync();
  PROF_T(p4);
  PROF_ADD(1, p0, p1);
  PROF_ADD(2, p1, p2);
  PROF_ADD(3, p2, p3);
  PROF_ADD(4, p3, p4);
  PROF_ADD(5, 0, 1);
  PROF_ADD(6, 0, (long long)m);
  PROF_ADD(7, 0, (long long)nc);
  return NmW{nc, T};
}

// a double from another lane by DPP (two dword moves); lanes without a source take ident
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_d(double v, double ident) {
  const uint64_t b = (uint64_t)__double_as_longlong(v), z = (uint64_t)__double_as_longlong(ident);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)z, (int)(uint32_t)b, CTRL, RM, 0xf, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(z >> 32), (int)(uint32_t)(b >> 32), CTRL, RM, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// inclusive sum over the wave's 64 lanes (row shifts, then the row broadcasts of lanes 15 and 31)
__device__ __forceinline__ double wave_incl_add_d(double v) {
  v = dadd(v, dpp_d<0x111, 0xf>(v, 0.0));
  v = dadd(v, dpp_d<0x112, 0xf>(v, 0.0));
  v = dadd(v, dpp_d<0x114, 0xf>(v, 0.0));
  v = dadd(v, dpp_d<0x118, 0xf>(v, 0.0));
  v = dadd(v, dpp_d<0x142, 0xa>(v, 0.0));
  return dadd(v, dpp_d<0x143, 0xc>(v, 0.0));
}
// Same merge, written branch-free for a lone wave: every per-lane loop is unrolled over kR
// rounds with fixed trip counts, clamped indices and selects, so the independent LDS loads of
// all rounds issue back to back instead of one exec-masked round at a time.
// Requires nm + np < 64 * kR <= JW (delta <= ~150) and np <= 64.
constexpr int kR = 5;     // largest instantiation: nm + np < 320
constexpr int kLogT = 7;  // steps of a search over the temps (np <= 64 < 2^7)

template <int kR>
__device__ __forceinline__ void merge_sorted_fast(const MergeParams x, const Lds L, uint32_t& nm, double& mainW, uint32_t np,
                                  double tempW) {
  // steps of a lower-bound search over at most 64 kR - 1 entries: ceil(log2(64 kR))
  constexpr int kLogR = kR <= 1 ? 6 : (kR <= 2 ? 7 : (kR <= 4 ? 8 : 9));
  constexpr int kLogMT = kLogR > kLogT ? kLogR : kLogT;  // main (nm < 64 kR) and temps (np <= 64)
  const uint32_t lane = threadIdx.x;
  PROF_T(p0);
  const double T = dadd(mainW, tempW);
  const uint32_t m = nm + np;
  // ---- merged positions: temp t after the mains strictly below it; main j after the temps <= it
  {
    const double tv = L.sv[lane < np ? lane : 0];
    double mv[kR];
    uint32_t ml[kR], mh[kR];
#pragma unroll
    for (int r = 0; r < kR; r++) {
      const uint32_t j = 64 * r + lane;
      mv[r] = L.mm[j < nm ? j : 0];
      ml[r] = 0;
      mh[r] = j < nm ? np : 0;
    }
    uint32_t tl = 0, th = lane < np ? nm : 0;
#pragma unroll
    for (int it = 0; it < kLogMT; it++) {
      const uint32_t tmd = (tl + th) >> 1;
      const double tval = L.mm[tmd < nm ? tmd : 0];
      const bool tgo = tl < th, tlt = tval < tv;
      tl = (tgo && tlt) ? tmd + 1 : tl;
      th = (tgo && !tlt) ? tmd : th;
      if (it < kLogT) {
        uint32_t mmd[kR];
        double mval[kR];
#pragma unroll
        for (int r = 0; r < kR; r++) {
          mmd[r] = (ml[r] + mh[r]) >> 1;
          mval[r] = L.sv[mmd[r] < np ? mmd[r] : 0];
        }
#pragma unroll
        for (int r = 0; r < kR; r++) {
          const bool go = ml[r] < mh[r], le = mval[r] <= mv[r];
          ml[r] = (go && le) ? mmd[r] + 1 : ml[r];
          mh[r] = (go && !le) ? mmd[r] : mh[r];
        }
      }
    }
    if (lane < np) {
      L.gm[lane + tl] = tv;
      L.gw[lane + tl] = L.sw[lane];
    }
#pragma unroll
    for (int r = 0; r < kR; r++) {
      const uint32_t j = 64 * r + lane;
      if (j < nm) {
        L.gm[j + ml[r]] = mv[r];
        L.gw[j + ml[r]] = L.mw[j];
      }
    }
  }
  wave_lds_sync();
  PROF_T(p1);
  // ---- mergedWeight prefix: per-round wave scans, then the round carries (integer weights:
  // exact in any order); otherwise the sequential fold in Go's order.  Then k per element.
  double kv[kR];
  {
    double w[kR];
    bool wint = true, wex = true;
#pragma unroll
    for (int r = 0; r < kR; r++) {
      const uint32_t j = 64 * r + lane;
      const double g = L.gw[j];
      w[r] = j < m ? g : 0.0;
      wint &= is_int_weight(w[r]);
      wex &= is_exact_weight(w[r]);
    }
    wint = __all(wex) && T <= exact_total_limit(__all(wint));  // (sums exact in any order)
    if (wint) {
      // DPP row shifts when every lane is active (see prefix_main_w0), else lane shuffles
      if (__builtin_amdgcn_read_exec() == ~0ull) {
#pragma unroll
        for (int r = 0; r < kR; r++) w[r] = wave_incl_add_d(w[r]);
      } else {
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
          for (int r = 0; r < kR; r++) {
            const double o = __shfl_up(w[r], d, 64);
            w[r] = (int)lane >= d ? dadd(w[r], o) : w[r];
          }
        }
      }
      double carry = 0.0;
#pragma unroll
      for (int r = 0; r < kR; r++) {
        const double tot = rl_d(w[r], 63);
        kv[r] = dadd(carry, w[r]);
        carry = dadd(carry, tot);
      }
    } else {
      double run = 0.0;
#pragma unroll
      for (int r = 0; r < kR; r++) {
        kv[r] = 0.0;
        const uint32_t b = 64 * r;
        const uint32_t c = b < m ? min(64u, m - b) : 0u;
        for (uint32_t i = 0; i < c; i++) {
          run = dadd(run, rl_d(w[r], (int)i));
          if (i == lane) kv[r] = run;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kR; r++) kv[r] = index_estimate<VN_NR_ONE>(x.delta, ddiv(kv[r], T));
#pragma unroll
    for (int r = 0; r < kR; r++) L.kin[64 * r + lane] = kv[r];
  }
  wave_lds_sync();
  PROF_T(p2);
  const double k0 = index_estimate(x.delta, 0.0);
  // ---- chain by pointer doubling (see merge_sorted); tables are padded to 64*kR entries
  // and every entry is <= m, so all loads below stay in range without guards
  bool mono = true;
#pragma unroll
  for (int r = 0; r < kR; r++) {
    const uint32_t j = 64 * r + lane;
    const double prev = L.kin[j ? j - 1 : 0];
    mono &= !(j >= 1 && j < m && !(kv[r] >= prev));  // (NaN: not monotone, see merge_sorted)
  }
  mono = __all(mono);
#ifdef VN_CHAIN_WALK
  mono = false;
#endif
  PROF_T(cq1);
  PROF_ADD(9, p2, cq1);
  uint32_t nc = 0;
  bool overflow = false;
  const uint32_t capc = x.capc;
  if (mono) {
    uint32_t cur[kR];  // this lane's entries of the newest jump table, kept in registers
    {
      double base[kR];
      uint32_t bl[kR], bh[kR];
#pragma unroll
      for (int r = 0; r < kR; r++) {
        const uint32_t s = 64 * r + lane;
        const double kb = L.kin[(s >= 1 ? s - 1 : 0)];
        base[r] = s >= 1 ? kb : k0;
        bl[r] = s < m ? s + 1 : m;
        bh[r] = m;
      }
#pragma unroll
      for (int it = 0; it < kLogR; it++) {
        uint32_t md[kR];
        double kval[kR];
#pragma unroll
        for (int r = 0; r < kR; r++) {
          md[r] = (bl[r] + bh[r]) >> 1;
          kval[r] = L.kin[md[r]];
        }
#pragma unroll
        for (int r = 0; r < kR; r++) {
          const bool go = bl[r] < bh[r], gt = dsub(kval[r], base[r]) > 1.0;
          bh[r] = (go && gt) ? md[r] : bh[r];
          bl[r] = (go && !gt) ? md[r] + 1 : bl[r];
        }
      }
#pragma unroll
      for (int r = 0; r < kR; r++) {
        L.jump16[64 * r + lane] = (uint16_t)bl[r];
        cur[r] = bl[r];
      }
    }
    wave_lds_sync();
    PROF_T(cq2);
    PROF_ADD(10, cq1, cq2);
    // start t = next^t(0) for this lane's t = 64 r + lane, in registers: step lv extends the
    // starts t < 2^lv to t < 2^(lv+1) through the table of next^(2^lv) (t - 2^lv: a lane of
    // round 0 below, or this lane of an earlier round), and squares that table into the other
    constexpr int kLevels = kLogR;  // 2^kLevels >= 64 kR
    uint32_t p[kR];
#pragma unroll
    for (int r = 0; r < kR; r++) p[r] = 0;
#pragma unroll
    for (int lv = 0; lv < kLevels; lv++) {
      const ldsu16* Jc = L.jump16 + (lv & 1) * L.JW;
      ldsu16* Jn = L.jump16 + ((lv & 1) ^ 1) * L.JW;
      if (lv < 6) {
        const uint32_t h = 1u << lv;
        const uint32_t src = (uint32_t)__shfl_up((int)p[0], h, 64);
        const uint32_t nx = Jc[src];
        p[0] = (lane >= h && lane < 2 * h) ? nx : p[0];
      } else {
        const int hr = 1 << (lv - 6);  // rounds hr .. 2 hr - 1 from rounds 0 .. hr - 1
#pragma unroll
        for (int r = 0; r < kR; r++)
          if (r >= hr && r < 2 * hr) p[r] = Jc[p[r >= hr ? r - hr : 0]];
      }
      if (lv + 1 < kLevels) {
        uint32_t a[kR];
#pragma unroll
        for (int r = 0; r < kR; r++) a[r] = Jc[cur[r]];
#pragma unroll
        for (int r = 0; r < kR; r++) {
          Jn[64 * r + lane] = (uint16_t)a[r];
          cur[r] = a[r];
        }
      }
      wave_lds_sync();
    }
    PROF_T(cq3);
    PROF_ADD(11, cq2, cq3);
#pragma unroll
    for (int r = 0; r < kR; r++) {
      const uint32_t t = 64 * r + lane;
      const bool on = t <= capc && p[r] < m;
      if (on && t < capc) L.starts[t] = p[r];
      nc += (uint32_t)__popcll(__ballot(on));
      overflow |= on && t == capc;
    }
    overflow = __any(overflow);
    if (nc > capc) nc = capc;
    PROF_T(c4);
    PROF_ADD(12, cq3, c4);
  } else {
    double base = k0, kprev_carry = k0;
    for (uint32_t b = 0; b < m && !overflow; b += 64) {
      const uint32_t j = b + lane;
      const bool valid = j < m;
      const double kj = valid ? L.kin[j] : 0.0;
      double kp = __shfl_up(kj, 1, 64);
      if (lane == 0) kp = kprev_carry;
      uint32_t from = 0;
      for (;;) {
        const bool c = valid && lane >= from && (nc == 0 || dsub(kj, base) > 1.0);
        const uint64_t bal = __ballot(c);
        if (!bal) break;
        const uint32_t f = (uint32_t)__builtin_ctzll(bal);
        if (nc >= capc) { overflow = true; break; }
        if (lane == 0) L.starts[nc] = b + f;
        nc++;
        base = rl_d(kp, (int)f);
        from = f + 1;
      }
      kprev_carry = rl_d(kj, 63);
    }
  }
  if (overflow && lane == 0) atomicOr(x.err, 1u);
  if (lane == 0) L.starts[nc] = m;
  wave_lds_sync();
  PROF_T(p3);
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
  wave_lds_sync();
  PROF_T(p4);
  PROF_ADD(1, p0, p1);
  PROF_ADD(2, p1, p2);
  PROF_ADD(3, p2, p3);
  PROF_ADD(4, p3, p4);
  PROF_ADD(5, 0, 1);
  PROF_ADD(6, 0, (long long)m);
  PROF_ADD(7, 0, (long long)nc);
  nm = nc;
  mainW = T;
}

__device__ __forceinline__ void merge_any(const MergeParams x, const Lds L, uint32_t& nm, double& mainW, uint32_t np,
                                          double tempW) {
  // nc <= m < 64 * R: the fast merge's start enumeration (t < 64 * R) covers every centroid
  const uint32_t m = nm + np;
  if (np > 64 || m >= 64u * kR) {
    const NmW r = merge_sorted(L, MP_ARGS(x), nm, mainW, np, tempW);
    nm = r.nm;
    mainW = r.w;
  } else if (m < 128) merge_sorted_fast<2>(x, L, nm, mainW, np, tempW);
  else if (m < 192) merge_sorted_fast<3>(x, L, nm, mainW, np, tempW);
  else if (m < 256) merge_sorted_fast<4>(x, L, nm, mainW, np, tempW);
  else merge_sorted_fast<5>(x, L, nm, mainW, np, tempW);
}

// merge_any out of line: the long replays' rare fallback, kept out of their merge loop's code
__device__ __noinline__ NmW merge_any_v(const Lds L, MP_PARAMS, uint32_t nm, double mainW, uint32_t np, double tempW) {
  MP_UNPACK(x);
  merge_any(x, L, nm, mainW, np, tempW);
  return NmW{nm, mainW};
}

// sort the pending temps in LDS and merge them
__device__ __noinline__ NmW merge_pending_v(const Lds L, MP_PARAMS, uint32_t nm, double mainW, uint32_t np) {
  MP_UNPACK(x);
  PROF_T(a0);
  const double tempW = temp_weight(L.tw, np);
  sort_temps(L.tv, L.tw, L.sv, L.sw, np);
  PROF_T(a1);
  PROF_ADD(0, a0, a1);
  merge_any(x, L, nm, mainW, np, tempW);
  return NmW{nm, mainW};
}
__device__ __forceinline__ void merge_pending(const MergeParams x, const Lds L, uint32_t& nm, double& mainW, uint32_t np) {
  const NmW r = merge_pending_v(L, MP_ARGS(x), nm, mainW, np);
  nm = r.nm;
  mainW = r.w;
}

__device__ __forceinline__ uint32_t round64(uint32_t v) { return (v + 63u) & ~63u; }

// Where a key's batch splits (shared by the chunk sorter and the replay):
//   head  [0, off0)         tops up the pending temps (merged if the list fills and more follow)
//   pure  npure chunks of tcap samples, each merged (a later sample always follows it)
//   tail  the rest          stays pending (or is merged by a final merge)
struct ExactSplit {
  uint32_t off0, npure;
};
__device__ __forceinline__ ExactSplit exact_split(uint32_t np0, uint32_t nex, uint32_t tcap) {
  const uint32_t np = (nex > 0 && np0 == tcap) ? 0u : np0;  // a full list merges before the first Add
  ExactSplit r;
  r.off0 = np == 0 ? 0u : min(tcap - np, nex);
  r.npure = nex > r.off0 ? (nex - r.off0 - 1) / tcap : 0u;
  return r;
}

__device__ __forceinline__ uint32_t last_le_u32(const uint32_t* off, uint32_t n, uint32_t o) {
  uint32_t lo = 0, hi = n;  // last k in [0, n) with off[k] <= o
  while (hi - lo > 1) {
    uint32_t m = (lo + hi) >> 1;
    if (off[m] <= o) lo = m;
    else hi = m;
  }
  return lo;
}

}  // namespace

#ifndef VN_CHUNK_XCD
#define VN_CHUNK_XCD 16  // consecutive chunks per XCD (k_exact_chunk_sort); 0: chunk g to block g
#endif
// ---- pure-chunk sorter: the contents of every full chunk are known before the replay, so
// all of them are sorted here in parallel (one wave per chunk), off the replay's critical path.
__global__ void k_exact_chunk_count(ExactCtx x) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= x.nkeys) return;
  if (x.nkeys_dev && k >= *x.nkeys_dev) {  // (past the live keys: no chunks, and keys[k] is stale)
    x.ccnt[k] = 0u;
    return;
  }
  const uint32_t nex = x.nex[k];
  x.ccnt[k] = exact_split(x.hpend[x.keys[k]], nex, x.tcap).npure;
}

// owner key of every pure chunk, so a sorting wave starts without a dependent binary search:
// the first record of pure chunk g of key k
__device__ __forceinline__ uint32_t chunk_base(const ExactCtx& x, uint32_t g, uint32_t k) {
  const uint32_t s = x.keys[k];
  const ExactSplit sp = exact_split(x.hpend[s], x.nex[k], x.tcap);
  return x.start[s] + sp.off0 + (g - x.coff[k]) * x.tcap;
}

// one thread per chunk (a thread per key would write a 17M-sample key's 400k chunks alone): its
// key and first record, so the sorter's wave starts with one load instead of a chain of five
__global__ void k_exact_chunk_owner(ExactCtx x) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= x.coff[x.nkeys]) return;
  const uint32_t k = last_le_u32(x.coff, x.nkeys, g);
  x.cown[g] = (uint64_t)k << 32 | chunk_base(x, g, k);
}

// Keys replaying at least this many samples take the batched kernel.  Its LDS is a whole CU's,
// so every batched key holds a CU for its chain: at C4 with 65536 about 250 keys per window took
// nearly every CU at once and the windows in flight waited for them.  262144 (about 60 keys; the
// rest on the four-wave kernel): C4 at N = 1 72.4 -> 61.6 / 62.2 ms per window at four engines;
// 16384 / 32768: 106 / 87 ms.  524288 (about 30 keys, each of the others under 50 ms of four-wave
// replay): the same at four engines, 55.0 / 54.7 against 56.2 / 57.8 ms at five; 2^20 at five:
// 56.5 / 55.9 / 55.9 against 54.9 / 54.8 / 55.0 (profiles/r06_batchlen/)
#ifndef VN_BATCH_MIN_LEN
#define VN_BATCH_MIN_LEN 524288u
#endif
constexpr uint32_t kBatchMinLen = VN_BATCH_MIN_LEN;

// min / max over the wave's 64 lanes (Go's math.Min / Max order: -0 below +0), complete in lane
// 63: the DPP row shifts and row broadcasts of wave_incl_add_d, every lane active
__device__ __forceinline__ double wave_min_go(double v) {
  v = min_go(v, dpp_d<0x111, 0xf>(v, kInf));
  v = min_go(v, dpp_d<0x112, 0xf>(v, kInf));
  v = min_go(v, dpp_d<0x114, 0xf>(v, kInf));
  v = min_go(v, dpp_d<0x118, 0xf>(v, kInf));
  v = min_go(v, dpp_d<0x142, 0xa>(v, kInf));
  return min_go(v, dpp_d<0x143, 0xc>(v, kInf));
}
__device__ __forceinline__ double wave_max_go(double v) {
  v = max_go(v, dpp_d<0x111, 0xf>(v, -kInf));
  v = max_go(v, dpp_d<0x112, 0xf>(v, -kInf));
  v = max_go(v, dpp_d<0x114, 0xf>(v, -kInf));
  v = max_go(v, dpp_d<0x118, 0xf>(v, -kInf));
  v = max_go(v, dpp_d<0x142, 0xa>(v, -kInf));
  return max_go(v, dpp_d<0x143, 0xc>(v, -kInf));
}

// sort pure chunk g of key k, whose first record is base (one wave)
// (pre: tcap <= 64 and the lane's record -- A, B at base + lane -- already loaded into pa / pb)
__device__ __forceinline__ void chunk_sort_one(const ExactCtx& x, const uint32_t g, const uint32_t k,
                                               const uint64_t base, char* smem, const bool pre = false,
                                               const uint64_t pa = 0, const uint64_t pb = 0) {
  const uint32_t lane = threadIdx.x;
  const uint32_t tcap = x.tcap, TP = round64(tcap + 1);
  ldsf64* tv = (ldsf64*)smem;
  ldsf64* tw = tv + TP;
  ldsf64* sv = tw + TP;
  ldsf64* sw = sv + TP;
  if (pre) {
    if (lane < tcap) {
      const uint32_t tag = (uint32_t)pb;
      const double wt = tag_weight(tag, x.impw);
      tv[lane] = bitsd(pa);
      tw[lane] = tag_is_sample(tag) ? wt : -wt;
    }
  } else {
    for (uint32_t t = lane; t < tcap; t += 64) {
      const uint32_t tag = (uint32_t)x.B[base + t];
      const double wt = tag_weight(tag, x.impw);
      tv[t] = bitsd(x.A[base + t]);
      tw[t] = tag_is_sample(tag) ? wt : -wt;  // sign: an imported centroid (no Local* statistics)
    }
  }
  wave_lds_sync();
  if (x.cstat && x.nex[k] >= kBatchMinLen) {
    // the chunk's Local* partials (Histo.Sample, samplers.go:346-356; min / max of every record for
    // the digest), for the batched keys' statistics (only they read them): read here once, with the
    // chunk; reduced over the wave by DPP (lane 63 holds the totals; sums need no fixed order: their
    // parity bound is 1e-12, weights are exact)
    double lsw = 0.0, lsxw = 0.0, lsrw = 0.0, lmn = kInf, lmx = -kInf, ldmn = kInf, ldmx = -kInf;
    for (uint32_t t = lane; t < tcap; t += 64) {
      const double v = tv[t], w = tw[t], wt = __builtin_fabs(w);
      ldmn = min_go(ldmn, v);
      ldmx = max_go(ldmx, v);
      if (w > 0.0) {
        lsw = dadd(lsw, wt);
        lmn = min_go(lmn, v);
        lmx = max_go(lmx, v);
        lsxw = dadd(lsxw, dmul(v, wt));
        lsrw = dadd(lsrw, dmul(ddiv(1.0, v), wt));
      }
    }
    lsw = wave_incl_add_d(lsw);
    lsxw = wave_incl_add_d(lsxw);
    lsrw = wave_incl_add_d(lsrw);
    lmn = wave_min_go(lmn);
    lmx = wave_max_go(lmx);
    ldmn = wave_min_go(ldmn);
    ldmx = wave_max_go(ldmx);
    if (lane == 63) {
      double* o = x.cstat + (uint64_t)g * 8;
      o[0] = lsw;
      o[1] = lsxw;
      o[2] = lsrw;
      o[3] = lmn;
      o[4] = lmx;
      o[5] = ldmn;
      o[6] = ldmx;
    }
  }
  const double tempW = temp_weight(tw, tcap);
  const bool wide = x.nex[k] >= x.long_min;  // (every record's prefix: a four-wave or batched replay)
  sort_temps_body(tv, tw, sv, sw, tcap);
  // for the long replays (replay_key_fast): the exclusive prefix of the sorted |weights| after
  // the first record, the Add-order tempW at it (negated when a weight is not an integer)
  // and for the batched replay (cpk) the same prefix as a u16 beside |w| as a u16, slot 0 carrying
  // tempW -- or 0xffffffff when some weight is not an integer or tempW >= 2^16
  bool tint = true, tex = true;
  double carry = 0.0;
  for (uint32_t b = 0; b < tcap; b += 64) {
    const uint32_t t = b + lane;
    const double w = t < tcap ? __builtin_fabs(sw[t]) : 0.0;
    tint &= is_int_weight(w);
    tex &= is_exact_weight(w);
    double v = w;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const double o = __shfl_up(v, d, 64);
      v = (int)lane >= d ? dadd(v, o) : v;
    }
    if (t < tcap) {
      const double ex = dadd(carry, dsub(v, w));
      x.csv[base + t] = sv[t];
      x.csw[base + t] = sw[t];
      if (t && wide) x.ctw[base + t] = ex;
      if (x.cpk && t && wide) x.cpk[base + t] = (ex < 65536.0 ? (uint32_t)ex << 16 : 0xffff0000u) | (w < 65536.0 ? (uint32_t)w : 0xffffu);
    }
    carry = dadd(carry, rl_d(v, 63));
  }
  tint = __all(tint);
  tex = __all(tex) && tempW <= exact_total_limit(tint);
  if (lane == 0) {
    // (the four-wave merge needs exact prefixes only; the batched one integers below 2^16)
    // (with tw_sum the one-wave replay sums an exact chunk's weights itself: the slot is read
    // only by the long replays and for a chunk whose weights have no order-free sum)
    if (wide || !tex || !x.tw_sum) x.ctw[base] = tex ? tempW : -tempW;
    // (every weight is at least 1, so tempW < 2^16 bounds each weight and prefix below 2^16 too)
    if (x.cpk) x.cpk[base] = tint && tempW < 65536.0 ? (uint32_t)tempW << 16 | (uint32_t)__builtin_fabs(sw[0]) : 0xffffffffu;
  }
}

// the first `top` keys of the longest-first order (x.order64): their chunks are sorted first, so
// their replays (the window's longest chains) start before the other keys' chunks are sorted
__device__ __forceinline__ bool is_top_key(const ExactCtx& x, uint32_t k, uint32_t top) {
  bool t = false;
  for (uint32_t y = 0; y < top; y++) t |= (uint32_t)x.order64[y] == k;
  return t;
}

// every pure chunk (one wave each), skipping the first `top` keys of x.order64 (sorted already)
// Workgroups are dealt to the 8 XCDs round-robin (block b to XCD b % 8), each XCD with its own L2.
// Adjacent chunks share the cache lines at their ends (a chunk is 42 records of 8-byte words, not
// a line multiple), so runs of kChunkRun consecutive chunks go to one XCD, the runs dealt to the
// XCDs in turn: a line is read and written through one L2 instead of two, and every XCD still
// sees the whole window's mix of chunks (one contiguous eighth each was measured slower: 7.8
// against 6.7 ms -- chunks whose ties take Go's sort on one lane cluster by key).  The grid is a
// multiple of 8 * kChunkRun (histo_exact_chunk_sort)
constexpr uint32_t kChunkRun = VN_CHUNK_XCD;
// A wave takes kChunksPerWave consecutive chunks, every one's record loads issued before it sorts
// the first.  Measured (C4, one engine, rocprofv3): 6.26 ms per window with one chunk per wave,
// 6.85 with two, 6.87 with four (66 VGPRs: seven waves per SIMD); the whole bench 54.4-54.6 against
// 55.4-55.5 ms per window with two (profiles/r06_chunkwave/)
#ifndef VN_CHUNKS_PER_WAVE
#define VN_CHUNKS_PER_WAVE 1
#endif
constexpr uint32_t kChunksPerWave = VN_CHUNKS_PER_WAVE;
__global__ __launch_bounds__(64) void k_exact_chunk_sort(ExactCtx x, uint32_t top) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t total = x.coff[x.nkeys];
#if VN_CHUNK_XCD
  const uint32_t r = blockIdx.x >> 3, q = (r / kChunkRun) * 8u + (blockIdx.x & 7u);
  const uint32_t m = q * kChunkRun + r % kChunkRun;
#else
  const uint32_t m = blockIdx.x;
#endif
  const uint32_t lane = threadIdx.x;
  const bool pre = x.tcap <= 64;
  uint32_t gk[kChunksPerWave], kk[kChunksPerWave], bk[kChunksPerWave];
  bool live[kChunksPerWave];
  uint64_t pa[kChunksPerWave], pb[kChunksPerWave];
#pragma unroll
  for (uint32_t c = 0; c < kChunksPerWave; c++) {
    const uint32_t g = m * kChunksPerWave + c;
    gk[c] = g;
    live[c] = g < total;
    kk[c] = 0u;
    bk[c] = 0u;
    pa[c] = 0ull;
    pb[c] = 0ull;
    if (!live[c]) continue;
    if (x.cown) {
      const uint64_t o = x.cown[g];
      kk[c] = (uint32_t)(o >> 32);
      bk[c] = (uint32_t)o;
    } else {
      kk[c] = last_le_u32(x.coff, x.nkeys, g);
      bk[c] = chunk_base(x, g, kk[c]);
    }
    if (top && is_top_key(x, kk[c], top)) live[c] = false;
    if (live[c] && pre && lane < x.tcap) {
      pa[c] = x.A[(uint64_t)bk[c] + lane];
      pb[c] = x.B[(uint64_t)bk[c] + lane];
    }
  }
#pragma unroll
  for (uint32_t c = 0; c < kChunksPerWave; c++) {
    if (!live[c]) continue;
    chunk_sort_one(x, gk[c], kk[c], bk[c], smem, pre, pa[c], pb[c]);
    wave_lds_sync();  // (the next chunk reuses the LDS tiles)
  }
}

// the chunks of the first `top` keys of x.order64: block (b, y) takes key y's chunks b, b + G, ...
__global__ __launch_bounds__(64) void k_exact_chunk_sort_top(ExactCtx x) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t k = (uint32_t)x.order64[blockIdx.y];
  const uint32_t a = x.coff[k], b = x.coff[k + 1];
  for (uint32_t g = a + blockIdx.x; g < b; g += gridDim.x) {
    chunk_sort_one(x, g, k, chunk_base(x, g, k), smem);
    wave_lds_sync();  // (the next chunk reuses the LDS tiles)
  }
}

// ---- the replay: one 64-thread block (one wave) per key.  TPL = temps per lane of a chunk
// (1 when estimateTempBuffer <= 64, i.e. delta <= ~150; 4 up to delta 1000).
template <int TPL>
__device__ __forceinline__ void replay_key(const ExactCtx& x, const uint32_t k) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t lane = threadIdx.x;
  const uint32_t capc = x.capc, tcap = x.tcap;
  const uint32_t TP = round64(tcap + 1);
  const Lds L = lds_layout(smem, capc, TP);

  PROF_T(k0);
  // kernel arguments into registers: nothing below may take the address of x
  const MergeParams mp{x.delta, x.capc, x.err};
  const uint64_t* const xA = x.A;
  const uint64_t* const xB = x.B;
  const double* const xcsv = x.csv;
  const double* const xcsw = x.csw;
  const double* const xctw = x.ctw;
  const double* const ximpw = x.impw;
  const uint32_t s = x.keys[k];
  const uint32_t nex = x.nex ? x.nex[k] : 0u;
  const bool final_merge = x.flush_mode || (x.hot && x.hot[k]);
  uint32_t np = x.hpend[s];
  if (x.flush_mode && x.hspn) {
    // the last replay of this key already merged its pending temps into the other buffer
    const uint32_t fn = x.hspn[s];
    if (fn) {
      if (lane == 0) {
        x.hcur[s] ^= 1;
        x.hncent[s] = fn;
        x.hst[(uint64_t)s * VN_HISTO_STATS + 7] = x.hspw[s];
        x.hpend[s] = 0;
        x.hspn[s] = 0;
      }
      return;
    }
  }
  if (nex == 0 && !(final_merge && np > 0)) return;

  const uint8_t cur = x.hcur[s];
  double* cmg = (cur ? x.cm1 : x.cm0) + (uint64_t)s * capc;
  double* cwg = (cur ? x.cw1 : x.cw0) + (uint64_t)s * capc;
  uint32_t nm = x.hncent[s];
  double* h = x.hst + (uint64_t)s * VN_HISTO_STATS;
  double mainW = h[7];
  const uint32_t lo = nex ? x.start[s] : 0u;  // start/A/B are null in flush mode (nex == 0)
  const ExactSplit sp = exact_split(np, nex, tcap);

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
  wave_lds_sync();

  // Histo.Sample local statistics of the replayed samples (samplers.go:346-356); the digest's
  // min/max (Add, merging_digest.go:106-107) also take imported centroids
  double sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf, dmn = kInf, dmx = -kInf;
  auto stat = [&](double v, double wt, bool sample) {
    dmn = min_go(dmn, v);
    dmx = max_go(dmx, v);
    if (!sample) return;
    sw = dadd(sw, wt);
    mn = min_go(mn, v);
    mx = max_go(mx, v);
    sxw = dadd(sxw, dmul(v, wt));
    srw = dadd(srw, dmul(ddiv(1.0, v), wt));
  };
  // append raw samples [a, b) of the batch to the pending temps (Add order)
  auto append = [&](uint32_t a, uint32_t b) {
    for (uint32_t i = a + lane; i < b; i += 64) {
      const double v = bitsd(xA[lo + i]);
      const uint32_t tag = (uint32_t)xB[lo + i];
      const double wt = tag_weight(tag, ximpw);
      L.tv[np + (i - a)] = v;
      L.tw[np + (i - a)] = wt;
      stat(v, wt, tag_is_sample(tag));
    }
    np += b - a;
    wave_lds_sync();
  };

  if (nex && np == tcap) {  // Add finds the temp list full: mergeAllTemps first
    merge_pending(mp, L, nm, mainW, np);
    np = 0;
  }
  // head
  if (sp.off0) {
    append(0, sp.off0);
    if (np == tcap && sp.off0 < nex) {
      merge_pending(mp, L, nm, mainW, np);
      np = 0;
    }
  }
  // pure chunks: pre-sorted by k_exact_chunk_sort; the next one is loaded before each merge.
  // With tw_sum a chunk's tempW is the wave's own sum of its weights when they have an
  // order-free sum (temp_weight's test), so no 8-byte read of a line per chunk; otherwise (and
  // without tw_sum) the chunk sorter's Add-order sum at the chunk's first record
  if (sp.npure) {
    double cv[TPL], cw[TPL], ctw = 0.0;
    const bool tw_sum = x.tw_sum != 0;
    auto load = [&](uint32_t c) {
      const uint64_t base = (uint64_t)lo + sp.off0 + (uint64_t)c * tcap;
#pragma unroll
      for (uint32_t q = 0; q < (uint32_t)TPL; q++) {
        const uint32_t t = q * 64 + lane;
        if (t < tcap) {
          cv[q] = xcsv[base + t];
          cw[q] = xcsw[base + t];
        }
      }
      if (!tw_sum) ctw = __builtin_fabs(xctw[base]);  // (negative: not all weights integers)
    };
    auto chunk_weight = [&](uint32_t c) -> double {
      if (!tw_sum) return ctw;
      bool ti = true, te = true;
      double part = 0.0;
#pragma unroll
      for (uint32_t q = 0; q < (uint32_t)TPL; q++) {
        const uint32_t t = q * 64 + lane;
        if (t < tcap) {
          const double w = __builtin_fabs(cw[q]);
          ti &= is_int_weight(w);
          te &= is_exact_weight(w);
          part = dadd(part, w);
        }
      }
      const double sum = wave_sum(part);
      if (__all(te) && sum <= exact_total_limit(__all(ti))) return sum;
      return __builtin_fabs(xctw[(uint64_t)lo + sp.off0 + (uint64_t)c * tcap]);
    };
    load(0);
    for (uint32_t c = 0; c < sp.npure; c++) {
#pragma unroll
      for (uint32_t q = 0; q < (uint32_t)TPL; q++) {
        const uint32_t t = q * 64 + lane;
        if (t < tcap) {
          L.sv[t] = cv[q];
          L.sw[t] = __builtin_fabs(cw[q]);
          stat(cv[q], __builtin_fabs(cw[q]), cw[q] > 0.0);
        }
      }
      double tempW = chunk_weight(c), tpad = 0.0;
      hold2(tempW, tpad);
      hold_stats(sw, sxw, srw, mn, mx, dmn, dmx);
      if (c + 1 < sp.npure) load(c + 1);
      wave_lds_sync();
      merge_any(mp, L, nm, mainW, tcap, tempW);
    }
  }
  // tail
  const uint32_t tail = sp.off0 + sp.npure * tcap;
  if (nex > tail) append(tail, nex);
  if (final_merge && np > 0) {
    merge_pending(mp, L, nm, mainW, np);
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
    dmn = min_go(dmn, __shfl_xor(dmn, d, 64));
    dmx = max_go(dmx, __shfl_xor(dmx, d, 64));
  }
  PROF_T(k1);
  PROF_ADD(8, k0, k1);
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
      h[5] = min_go(h[5], dmn);
      h[6] = max_go(h[6], dmx);
    }
  }
  // flush-ready digest: Quantile's mergeAllTemps (merging_digest.go:288) done now, into the
  // other buffer, while this wave still holds the key in LDS.  A later replay, a hot-path
  // merge or the window reset invalidates it; the flush then merges as usual.
  if (x.hspn) {
    uint32_t fn = 0;
    if (x.spec && !final_merge && np > 0) {
      merge_pending(mp, L, nm, mainW, np);
      double* fmg = (cur ? x.cm0 : x.cm1) + (uint64_t)s * capc;
      double* fwg = (cur ? x.cw0 : x.cw1) + (uint64_t)s * capc;
      for (uint32_t j = lane; j < nm; j += 64) {
        fmg[j] = L.mm[j];
        fwg[j] = L.mw[j];
      }
      fn = nm;
    }
    if (lane == 0) {
      x.hspn[s] = fn;
      if (fn) x.hspw[s] = mainW;
    }
  }
}

// ---- the long replays: NW waves per key, built for the latency of ONE merge (the hottest C4
// key replays ~23k merges back to back, so its merge latency is the window's critical path).
// Bit-identical to merge_sorted_fast; a different dependence structure:
//   positions     a merge-path search on each output diagonal (<= 7 steps over <= 64 temps);
//                 the element is read straight into registers
//   mergedWeight  no scan: with integer weights (every weight the key has seen, T <= 2^53) the
//                 weight before output e is mp[j] + sp[i], the exclusive prefix of the j main
//                 centroids before it (kept from the previous merge: a centroid's prefix is that
//                 of its first element) plus that of the i sorted temps (the chunk sorter's).
//                 Every partial sum is an exact integer, so it equals Go's running sum
//   chain         element s surely starts a centroid when k_s - k_{s-2} > 1 ("forced"): the
//                 centroid holding s-1 began at some c <= s-1, and with k monotone its base
//                 k_{c-1} <= k_{s-2}.  Each forced start walks the elements up to the next
//                 forced one exactly as mergeOne does (about 9 at delta 100), all in parallel
//   Welford       one thread per new centroid, its end from the start masks
// One element per thread with four waves (R = 4 / NW elements per thread in general).  A merge
// it cannot take (non-integer weights, > 64 temps, >= 256 elements) is the one-wave merge run
// by wave 0; a non-monotone k (an ulp wiggle of asin) takes the sequential walk of wave 0.
typedef __attribute__((address_space(3))) uint64_t ldsu64;

#ifndef VN_FAST_BAND
#define VN_FAST_BAND 1e-9  // (a variant build with a huge band sends every merge down the fallback)
#endif
constexpr double kBand = VN_FAST_BAND;  // certainty band of the close k's comparisons (merge_fast)

struct FastLds {
  ldsf64* mp;     // [capc + 2] exclusive prefix of the main centroids' weights; mp[nm] = mainW
  ldsf64* sp;     // [TP] exclusive prefix of the sorted temps' weights; sp[np] = tempW
  ldsf64* kk;     // [JW] k of every merged element
  ldsu64* gmask;  // [4] start mask of each 64-element group
  ldsf64* miscd;  // [2] 0: tempW broadcast
  ldsu32* flag;   // [JW] start flag of every element (written by the walkers)
  ldsu32* ism;    // [JW] 1: the element is a main centroid (0: a temp)
  ldsu32* misc;   // [8] 0: the predicted chain failed; 1: fast path ok (integer weights); 2: temps
                  //     integer; 3: a walk comparison within the band
};

__host__ __device__ inline uint32_t fast_extra_bytes(uint32_t capc, uint32_t TP, uint32_t JW) {
  return 8u * (capc + 2) + 8u * TP + 8u * JW + 8u * 4 + 8u * 2 + 4u * JW + 4u * JW + 4u * 8 + 16u;
}
__device__ __forceinline__ FastLds fast_layout_at(ldsf64* base, uint32_t capc, uint32_t TP, uint32_t JW) {
  FastLds F;
  F.mp = base;
  F.sp = F.mp + (capc + 2);
  F.kk = F.sp + TP;
  F.gmask = (ldsu64*)(F.kk + JW);
  F.miscd = (ldsf64*)(F.gmask + 4);
  F.flag = (ldsu32*)(F.miscd + 2);
  F.ism = F.flag + JW;
  F.misc = F.ism + JW;
  return F;
}
__device__ __forceinline__ FastLds fast_layout(char* p, uint32_t capc, uint32_t TP, uint32_t JW) {
  return fast_layout_at((ldsf64*)p, capc, TP, JW);
}
// FastLds again from its base and the Lds layout (capc = mw - mm, TP = tw - tv): out-of-line
// callees take the base, not the 8-register struct (see MP_PARAMS)
__device__ __forceinline__ FastLds fast_of(const Lds& L, ldsf64* base) {
  return fast_layout_at(base, (uint32_t)(L.mw - L.mm), (uint32_t)(L.tw - L.tv), L.JW);
}

template <int NW>
__device__ __forceinline__ void fast_sync() {
  if constexpr (NW == 1) wave_lds_sync();
  else lds_barrier();
}

__device__ __forceinline__ uint64_t sel4(uint32_t q, uint64_t g0, uint64_t g1, uint64_t g2, uint64_t g3) {
  return q == 0 ? g0 : (q == 1 ? g1 : (q == 2 ? g2 : g3));
}

// start flags of the m merged elements by mergeOne's sequential walk (wave 0; non-monotone k)
__device__ __noinline__ void walk_flags(const FastLds F, uint32_t m, double k0) {
  const uint32_t lane = threadIdx.x & 63;
  double base = k0, kprev_carry = k0;
  bool first = true;
  for (uint32_t b = 0; b < m; b += 64) {
    const uint32_t j = b + lane;
    const bool valid = j < m;
    const double kj = valid ? F.kk[j] : 0.0;
    double kp = __shfl_up(kj, 1, 64);
    if (lane == 0) kp = kprev_carry;
    uint32_t from = 0;
    uint64_t chosen = 0;
    for (;;) {
      const bool c = valid && lane >= from && (first || dsub(kj, base) > 1.0);
      const uint64_t bal = __ballot(c);
      if (!bal) break;
      const uint32_t f = (uint32_t)__builtin_ctzll(bal);
      chosen |= 1ull << f;
      first = false;
      base = rl_d(kp, (int)f);
      from = f + 1;
    }
    if (valid) F.flag[j] = (uint32_t)((chosen >> lane) & 1u);
    kprev_carry = rl_d(kj, 63);
  }
}

// mp[0..nm] from the main weights (wave 0); misc[1] = every weight exact (an integer, or a multiple
// of 2^-23 with a total up to 2^30) and their sum equal to mainW (then every prefix is exact);
// misc[4] = misc[1] and every weight an integer (the fast paths' totals may then reach 2^40)
__device__ __noinline__ void prefix_main_w0(const Lds L, const FastLds F, uint32_t nm, double mainW) {
  const uint32_t lane = threadIdx.x & 63;
  double carry = 0.0;
  bool ok = true, allint = true;
  for (uint32_t b = 0; b < nm; b += 64) {
    const uint32_t j = b + lane;
    const double w = j < nm ? L.mw[j] : 0.0;
    ok &= is_exact_weight(w);
    allint &= is_int_weight(w);
    // (integers: exact in any order).  DPP reads other lanes' registers, so it needs every lane
    // of the wave active: a caller that reaches here with some masked off (the compiler may
    // keep a uniform condition as a lane mask) takes the shuffle scan instead
    double v = w;
    if (__builtin_amdgcn_read_exec() == ~0ull) {
      v = wave_incl_add_d(w);
    } else {
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_up(v, d, 64);
        v = (int)lane >= d ? dadd(v, o) : v;
      }
    }
    if (j < nm) F.mp[j] = dadd(carry, dsub(v, w));
    carry = dadd(carry, rl_d(v, 63));
  }
  const bool ai = __all(allint);
  ok = __all(ok) && carry == mainW && mainW <= exact_total_limit(ai);
  if (lane == 0) {
    F.mp[nm] = mainW;
    F.misc[1] = ok ? 1u : 0u;
    F.misc[4] = ok && ai ? 1u : 0u;
  }
}

// sp[0..np] from the sorted temps' weights (wave 0, np <= 64); misc[2] = all integers
__device__ __noinline__ void prefix_temps_w0(const Lds L, const FastLds F, uint32_t np) {
  const uint32_t lane = threadIdx.x & 63;
  const double w = lane < np ? L.sw[lane] : 0.0;
  const bool allint = __all(is_int_weight(w)), ex = __all(is_exact_weight(w));
  double v = w;
  if (__builtin_amdgcn_read_exec() == ~0ull) {
    v = wave_incl_add_d(w);
  } else {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const double o = __shfl_up(v, d, 64);
      v = (int)lane >= d ? dadd(v, o) : v;
    }
  }
  const double tot = rl_d(v, 63);
  const bool ok = ex && tot <= exact_total_limit(allint);
  if (lane < np) F.sp[lane] = dsub(v, w);
  if (lane == 0) {
    F.sp[np] = tot;
    F.misc[2] = ok ? 1u : 0u;
  }
}

template <int NW>
__device__ __forceinline__ void merge_fast(const MergeParams x, const Lds L, const FastLds F, uint32_t& nm,
                                           double& mainW, const uint32_t np, const double tempW, const double k0) {
  constexpr int NT = 64 * NW, R = 4 / NW;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  PROF_T(f0);
  const double T = dadd(mainW, tempW);
  const uint32_t m = nm + np, nmc = nm ? nm - 1 : 0u;
  double xv[R], xw[R], wb[R], kv[R];
  bool ism[R];
  // ---- A: the element at each output position e: i temps and e - i mains precede it.
  // i is the number of p in [lo, hi) with P(p) = "temp p precedes main e-1-p" (true below i):
  // a four-way search, three probes per step (hi - lo <= 64 -> 16 -> 4 -> 1 -> 0: three steps
  // settle it), then one read of the element
  {
    uint32_t lo[R], hi[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint32_t e = r * NT + t;
      lo[r] = (e < m && e > nm) ? e - nm : 0u;
      hi[r] = e < m ? min(e, np) : 0u;
    }
#pragma unroll
    for (int it = 0; it < 3; it++) {
      uint32_t p1[R], p2[R], p3[R];
      double a1[R], a2[R], a3[R], b1[R], b2[R], b3[R];
#pragma unroll
      for (int r = 0; r < R; r++) {
        const uint32_t e = r * NT + t, len = hi[r] - lo[r];
        p1[r] = lo[r] + (len >> 2);
        p2[r] = lo[r] + (len >> 1);
        p3[r] = lo[r] + ((3u * len) >> 2);
        const bool go = len > 0;  // then every probe p < hi <= e, and e - 1 - p < nm
        a1[r] = L.sv[p1[r]];
        a2[r] = L.sv[p2[r]];
        a3[r] = L.sv[p3[r]];
        b1[r] = L.mm[go ? e - 1 - p1[r] : 0u];
        b2[r] = L.mm[go ? e - 1 - p2[r] : 0u];
        b3[r] = L.mm[go ? e - 1 - p3[r] : 0u];
      }
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (hi[r] > lo[r]) {  // main first only if strictly smaller: temp p precedes iff a <= b
          const bool q1 = a1[r] <= b1[r], q2 = a2[r] <= b2[r], q3 = a3[r] <= b3[r];
          const uint32_t nlo = q3 ? p3[r] + 1 : (q2 ? p2[r] + 1 : (q1 ? p1[r] + 1 : lo[r]));
          const uint32_t nhi = q3 ? hi[r] : (q2 ? p3[r] : (q1 ? p2[r] : p1[r]));
          lo[r] = nlo;
          hi[r] = nhi;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint32_t e = r * NT + t, i = lo[r], j = e < m ? e - i : 0u, jc = min(j, nmc);
      const double tv = L.sv[i], tw = L.sw[i], mv = L.mm[jc], mw = L.mw[jc];
      const bool tk = i < np && (j >= nm || tv <= mv);
      xv[r] = tk ? tv : mv;
      xw[r] = tk ? tw : mw;
      ism[r] = !tk;
      wb[r] = dadd(F.mp[min(j, nm)], F.sp[i]);
    }
  }
  PROF_T(f1);
  // ---- B: k of every element.  Only the chain's comparisons of k differences with 1 use k, so
  // a close k serves: q = mergedWeight / totalWeight exactly as Go divides, then the device
  // libm's asin (a few ulps, no divisions) in place of Go's (three divisions and a square root).
  // Every comparison below is taken only when its difference lies outside 1 +- kBand, where the
  // close and the exact k certainly agree (their k differ by < 1e-13); one inside the band sends
  // the merge to the walks and then, if still inside it there, to exact k and the sequential walk.
  // With weights >= 1 and T <= 2^40 (the fast merge's conditions) consecutive exact k
  // differ by more than 5e-11, far above asin's ulps, so exact k is increasing and the
  // forced-start argument holds.
#pragma unroll
  for (int r = 0; r < R; r++) {
    const double q = ddiv(dadd(wb[r], xw[r]), T);
    kv[r] = x.delta * (asin(dsub(dmul(2.0, q), 1.0)) * (1.0 / kPi) + 0.5);
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t e = r * NT + t;
    if (e < m) {
      L.gm[e] = xv[r];
      L.gw[e] = xw[r];
      F.kk[e] = kv[r];
      F.ism[e] = ism[r] ? 1u : 0u;
    }
  }
  if (t == 0) {
    F.misc[0] = 0u;
    F.misc[3] = 0u;
  }
  fast_sync<NW>();
  PROF_T(f2);
  // ---- C: the chain.  Predicted: every old main centroid and every forced element starts a
  // centroid, every other temp joins the one before it (in a hot key's steady state the
  // prediction is exact in ~99% of merges).  Each predicted start s verifies it in parallel:
  // with base = k_{s-1} and s' its next predicted start, k_{s'-1} - base <= 1 (every element
  // between joins, k increasing) and k_{s'} - base > 1 (s' starts).  Element 0 starts, so if
  // every check holds the predicted starts are exactly mergeOne's, by induction.  A failed or
  // in-band check sends the merge to the forced-start walks below.
  constexpr double kHi = 1.0 + kBand, kLo = 1.0 - kBand;
  bool fr[R], pr[R];
  double km1[R];
  bool bad = false;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t e = r * NT + t;
    const double a = F.kk[e >= 1 ? e - 1 : 0u], b = F.kk[e >= 2 ? e - 2 : 0u];
    km1[r] = e >= 1 ? a : k0;
    const double d = kv[r] - (e >= 2 ? b : k0);
    fr[r] = e < m && (e == 0 || d > kHi);
    bad |= e < m && e >= 1 && d >= kLo && d <= kHi;
    pr[r] = e < m && (fr[r] || ism[r]);
  }
  PROF_T(cq1);
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (pr[r]) {
      const uint32_t e = r * NT + t;
      double p2 = km1[r], p1 = kv[r];  // k_{j-2}, k_{j-1} for the forced test of element j
      uint32_t j = e + 1, sn = m;
      double ksn = 0.0, ksn1 = kv[r];    // k_{s'} and k_{s'-1}
      while (j < m && sn == m) {
        double kb[4];
        uint32_t im[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          kb[u] = F.kk[min(j + u, m - 1)];
          im[u] = F.ism[min(j + u, m - 1)];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const double k2 = u == 0 ? p2 : (u == 1 ? p1 : kb[u - 2]);
          const double d = kb[u] - k2;
          const bool look = sn == m && j + u < m;
          bad |= look && d >= kLo && d <= kHi;
          if (look && (im[u] != 0u || d > kHi)) {
            sn = j + u;
            ksn = kb[u];
            ksn1 = u == 0 ? p1 : kb[u - 1];
          }
        }
        p2 = kb[2];
        p1 = kb[3];
        j += 4;
      }
      if (sn == m) ksn1 = F.kk[m - 1];                  // the last centroid: its last element
      if (sn > e + 1) bad |= ksn1 - km1[r] > kLo;       // the last element before s' joins
      if (sn < m) bad |= !(ksn - km1[r] > kHi);         // s' starts
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint64_t bal = __ballot(pr[r]);
    if (lane == 0) F.gmask[r * NW + wv] = bal;
  }
#ifdef VN_FAST_NOPRED
  bad = true;  // (variant: every merge takes the forced-start walks)
#endif
  if (__any(bad) && lane == 0) F.misc[0] = 1u;
  fast_sync<NW>();
  PROF_T(cq2);
  if (F.misc[0]) {
    // forced-start walks: element j starts a centroid when k_j - base > 1 (base = k before the
    // current centroid's first element); a walker stops at the next forced element (k_j -
    // k_{j-2} > 1), whose own thread starts it.  Eight k per LDS round trip; the forced tests
    // of a batch do not depend on base, only the start tests chain through it.
    bool unsure = false;
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (fr[r]) {
        const uint32_t e = r * NT + t;
        F.flag[e] = 1u;
        double base = km1[r], p2 = km1[r], p1 = kv[r];  // p2 = k_{j-2}, p1 = k_{j-1}
        uint32_t j = e + 1;
        bool run = j < m;
        while (run) {
          double kb[8];
#pragma unroll
          for (int u = 0; u < 8; u++) kb[u] = F.kk[min(j + u, m - 1)];
          bool frc[8];
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const double dF = kb[u] - (u == 0 ? p2 : (u == 1 ? p1 : kb[u - 2]));
            frc[u] = j + u >= m || dF > kHi;
            unsure |= j + u < m && dF >= kLo && dF <= kHi;
          }
#pragma unroll
          for (int u = 0; u < 8; u++) {
            if (run) {
              if (frc[u]) {
                run = false;
              } else {
                const double dS = kb[u] - base;
                const bool st_ = dS > kHi;
                unsure |= dS >= kLo && dS <= kHi;
                F.flag[j] = st_ ? 1u : 0u;
                base = st_ ? (u == 0 ? p1 : kb[u - 1]) : base;
                j++;
              }
            }
          }
          p2 = kb[6];
          p1 = kb[7];
        }
      }
    }
    if (__any(unsure) && lane == 0) F.misc[3] = 1u;
    fast_sync<NW>();
    if (F.misc[3]) {  // a comparison within the band: exact k, then mergeOne's sequential walk
#pragma unroll
      for (int r = 0; r < R; r++) {
        const uint32_t e = r * NT + t;
        if (e < m) F.kk[e] = index_estimate<VN_NR_FOUR>(x.delta, ddiv(dadd(wb[r], xw[r]), T));
      }
      fast_sync<NW>();
      if (wv == 0) walk_flags(F, m, k0);
      fast_sync<NW>();
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint32_t e = r * NT + t;
      const uint64_t bal = __ballot(e < m && F.flag[e] != 0u);
      if (lane == 0) F.gmask[r * NW + wv] = bal;
    }
    fast_sync<NW>();
  }
  PROF_T(cq3);
  PROF_ADD(9, f2, cq1);
  PROF_ADD(10, cq1, cq2);
  PROF_ADD(11, cq2, cq3);
  PROF_ADD(12, 0, F.misc[0] ? 1 : 0);
  PROF_T(f3);
  // ---- D: centroid index and end of every start, Welford over its elements
  const uint64_t g0 = F.gmask[0], g1 = F.gmask[1], g2 = F.gmask[2], g3 = F.gmask[3];
  bool st[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t e = r * NT + t;
    st[r] = e < m && ((sel4((e >> 6) & 3u, g0, g1, g2, g3) >> (e & 63u)) & 1ull);
  }
  const uint32_t c0 = (uint32_t)__popcll(g0), c1 = (uint32_t)__popcll(g1), c2 = (uint32_t)__popcll(g2);
  const uint32_t nc = c0 + c1 + c2 + (uint32_t)__popcll(g3);
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (st[r]) {
      const uint32_t e = r * NT + t, q = e >> 6, ln = e & 63;
      const uint64_t gq = sel4(q, g0, g1, g2, g3);
      const uint32_t c = (q > 0 ? c0 : 0u) + (q > 1 ? c1 : 0u) + (q > 2 ? c2 : 0u) +
                         (uint32_t)__popcll(gq & ((1ull << ln) - 1ull));
      const uint64_t rest = ln == 63 ? 0ull : (gq >> (ln + 1));
      uint32_t end = m;
      if (rest) {
        end = e + 1 + (uint32_t)__builtin_ctzll(rest);
      } else {
        if (q < 3 && g3) end = 192 + (uint32_t)__builtin_ctzll(g3);
        if (q < 2 && g2) end = 128 + (uint32_t)__builtin_ctzll(g2);
        if (q < 1 && g1) end = 64 + (uint32_t)__builtin_ctzll(g1);
        end = min(end, m);
      }
      double mean = xv[r], W = xw[r];
      double gv[4], gw[4];  // the next four elements, loaded at once
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint32_t ix = min(e + 1 + u, m - 1);
        gv[u] = L.gm[ix];
        gw[u] = L.gw[ix];
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {  // (branch-free: a step past the end keeps W and mean)
        const bool in = e + 1 + u < end;
        const double W2 = dadd(W, gw[u]);
        const double mean2 = dadd(mean, ddiv(dmul(dsub(gv[u], mean), gw[u]), W2));
        W = in ? W2 : W;
        mean = in ? mean2 : mean;
      }
      for (uint32_t j = e + 5; j < end; j++) {
        const double wt = L.gw[j];
        W = dadd(W, wt);
        mean = dadd(mean, ddiv(dmul(dsub(L.gm[j], mean), wt), W));
      }
      L.mm[c] = mean;
      L.mw[c] = W;
      F.mp[c] = wb[r];
    }
  }
  if (t == 0) F.mp[nc] = T;
  fast_sync<NW>();
  PROF_T(f4);
  PROF_ADD(1, f0, f1);
  PROF_ADD(2, f1, f2);
  PROF_ADD(3, f2, f3);
  PROF_ADD(4, f3, f4);
  PROF_ADD(5, 0, 1);
  PROF_ADD(6, 0, (long long)m);
  PROF_ADD(7, 0, (long long)nc);
  nm = nc;
  mainW = T;
}

#ifndef VN_LONG_NW
#define VN_LONG_NW 4  // waves per long replay (A/B variants: 1, 2, 4)
#endif
constexpr int kMW = VN_LONG_NW;
constexpr uint32_t kMWThreads = 64 * kMW;
constexpr uint32_t kMaxLongKeys = 4096;
struct MwShared {  // one slot per purpose: a late wave may still read one while others move on
  uint32_t fb_nm;
  double fb_w;
  double red[7][kMW];
};
typedef __attribute__((address_space(3))) MwShared MwSharedL;

__host__ __device__ inline uint32_t fast_offset(uint32_t capc, uint32_t tcap) {
  return ((uint32_t)exact_smem_bytes_hd(capc, tcap) + 15u) & ~15u;
}

struct MergeState {
  uint32_t nm;
  double w;
  bool fok;   // the main weights are exact (integers, or 2^-23 multiples up to 2^30): fast merges apply
  bool fint;  // ... and all integers: the fast merges' totals may reach 2^40 (else 2^30)
};
// The largest total weight a fast merge or a batch takes: sums of 2^-23 multiples are exact in any
// order only up to 2^30 (is_exact_weight), sums of integers up to 2^40 here (the batch's ranges).
__device__ __forceinline__ double fast_total_limit(bool all_int) { return all_int ? 1099511627776.0 : 1073741824.0; }

// one mergeAllTemps of the sorted temps sv/sw (with sp when tint): the fast merge when it
// applies, else wave 0's one-wave merge (out of line) and the main prefix rebuilt after it
// tint: the temps' weights are exact (prefixes in any order); cint: ... and known to be integers
template <int NW>
__device__ __forceinline__ MergeState merge_step(const MergeParams mp, const Lds L, const FastLds F, MwSharedL& S,
                                                 MergeState st, uint32_t n_, double tempW, bool tint, bool cint,
                                                 double k0) {
  constexpr uint32_t NT = 64 * NW, R = 4 / NW;
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t m = st.nm + n_;
#ifdef VN_FAST_MERGE_OFF
  if (false) {  // A/B and debugging variant: every merge by wave 0's one-wave merge
#else
  if (st.fok && tint && n_ <= 64 && m < NT * R && m <= mp.capc &&
      dadd(st.w, tempW) <= fast_total_limit(st.fint && cint)) {
#endif
    merge_fast<NW>(mp, L, F, st.nm, st.w, n_, tempW, k0);
    st.fint = st.fint && cint;  // (a main weight that took a non-integer temp may not be one)
    return st;
  }
  if (wv == 0) {
    const NmW r = merge_any_v(L, MP_ARGS(mp), st.nm, st.w, n_, tempW);
    if (lane == 0) {
      S.fb_nm = r.nm;
      S.fb_w = r.w;
    }
  }
  fast_sync<NW>();
  st.nm = S.fb_nm;
  st.w = S.fb_w;
  if (st.fok && tint) {
    if (wv == 0) prefix_main_w0(L, F, st.nm, st.w);
    fast_sync<NW>();
    st.fok = F.misc[1] != 0u;
    st.fint = F.misc[4] != 0u;
  } else {
    st.fok = false;
    st.fint = false;
  }
  fast_sync<NW>();  // S and misc are read before anyone writes them again
  return st;
}

// ---- batched replay of consecutive pure chunks (the long replays' steady state).
//
// In a long key's steady state almost every merge keeps one structure: every old main centroid
// starts a centroid and every temp joins the one before it.  While it holds the centroid count
// stays fixed and the centroids evolve independently: centroid i's mean is a sequential Welford
// over the temps that land between it and centroid i+1, merge after merge.  merge_batch takes up
// to kBB pure chunks at once, every phase against the means at the batch start:
//   A  pos[j][p]  #means < v of every temp (all threads): the temp's column is pos - 1; pos 0
//                 ("Z") places it before main 0, where it starts the first centroid and main 0
//                 joins it (merging_digest.go:216: the first element always starts one)
//   B  n[j][i]    #temps of chunk j before main i, filled from the pos runs; the list offsets
//                 from a histogram of pos
//   C1 column i's list: its temps in (chunk, position) order -- column 0's with its chunks' Z
//                 temps, flagged -- one lane per column
//   E  Welford along each list in Go's Centroid.Add order (a chunk's Z temps start a fresh
//                 centroid that main 0 then joins), the mean after every entry recorded, and
//                 the range [lo_i, hi_i] of the column's means over the batch
//   C2 k bounds   the exact integer prefix P of main i in merge j and its weight, so q = P/T of
//                 every structure test; k is increasing, so min/max of each column's q bound
//                 all its k tests (on the waves E leaves idle, beside it)
//   F  decisions  per temp: main c before it (mean_c < v) and it before main c+1 (v <=
//                 mean_{c+1}) against the mean merge j saw -- checked exactly only for the temps
//                 inside a column's range; with hi_i <= lo_{i+1} (means sorted at every merge)
//                 these cover every main's merge-path decision
//   G  the columns whose bounds are not certain (within 1 +- kBand) tested merge by merge, one
//                 wave per column (lane = chunk, a wave scan for the prefixes)
// and commits the merges before the first failure.  Those are exactly the reference's merges
// (the checks of merge j hold given merges < j; by induction).  A decision failure (a temp the
// moving mean passed) is not a structure change: the next batch starts at that merge with its
// means fresh.  A structural failure (a centroid starts or fuses) sends that merge to
// merge_step.  tools/study/batch2_sim.c restates these phases on the CPU and compares them bit
// for bit with the per-merge replay (51.7 of 64 merges per batch on a 17M-sample key).
// The chunk sorter's means and packed weights are copied into an LDS ring (chunk c at slot
// c % kRing) by global->LDS loads that need no registers: later chunks land while a batch runs.
#ifndef VN_BATCH_MERGES
#define VN_BATCH_MERGES 64
#endif
constexpr uint32_t kBB = VN_BATCH_MERGES;  // merges per batch (list entries hold j < 64)
static_assert(kBB <= 64, "list entries and the flagged-column scan hold a chunk index below 64");
#ifndef VN_BATCH_RING
#define VN_BATCH_RING 128
#endif
constexpr uint32_t kRing = VN_BATCH_RING;  // chunk slots in LDS
constexpr uint32_t kTopExcl = 8;             // longest batched keys on CUs no other stream uses (st6)
constexpr uint32_t kTopSortBlocks = 4096;    // blocks per top key sorting its chunks first (grid-stride)
constexpr uint32_t kBM = 160;               // most centroids a batch takes (delta 100: ~135)
constexpr uint32_t kBN = kBM + 1;           // columns + the end
#ifndef VN_CHAIN_PRIO
#define VN_CHAIN_PRIO 0
#endif
constexpr uint32_t kBTmax = 42;             // largest temp buffer batched: veneur's delta 100 (samplers.go:364)
constexpr uint32_t kBMinAvail = 32;         // chunks in the ring below which a batch waits for more
#ifndef VN_BATCH_MIN_W
#define VN_BATCH_MIN_W 8192.0
#endif
constexpr double kBatchMinW = VN_BATCH_MIN_W;  // batches start once the digest holds this weight
constexpr uint32_t kBatchBackoff = 4;          // single merges after a batch that took none
#ifndef VN_BATCH_REPAIRS
#define VN_BATCH_REPAIRS 4
#endif
// flip repairs per batch (merge_batch, F'): a chunk whose temps the moving means put in another
// column than the batch-start means did is re-done for the columns it touches instead of ending
// the batch there; 0: every flip ends the batch (rounds 3-5).  Measured (4M-sample key, profiling
// build): 36.5 -> 54.3 merges committed per batch, 2590 -> 1743 batches, a repair round ~16k
// cycles; the 17M-sample key 175.9 -> 166.9 ms (profiles/r06_*)
constexpr uint32_t kRepairs = VN_BATCH_REPAIRS;
constexpr uint32_t kRepCols = 8;  // columns a batch may re-do (their per-chunk means in LDS)

typedef __attribute__((address_space(3))) uint8_t ldsu8;

constexpr uint32_t kRS = kBB + 8;  // row stride (bytes) of the n and K tables: 18 dwords, so the
                                   // rows of consecutive columns fall on different banks
constexpr uint32_t kSR = 168;      // bytes of a chunk's run-end row (columns 0..kBN, 8-byte multiple)
static_assert(kSR >= kBN + 1 && kSR % 8 == 0 && kSR / 4 <= 64, "a run-end row: a dword per lane");

struct BatchLds {
  ldsf64* rv;       // [kRing * tcap] the chunk sorter's csv: sorted temp means
  ldsu32* rp;       // [kRing * tcap] cpk: exclusive prefix of the sorted weights << 16 | |w|;
                    //                slot 0's prefix: the chunk's tempW (0xffffffff: not batchable)
  ldsf64* bT;       // [kBB] total weight after chunk j of the batch
  ldsf64* brT;      // [kBB] 1 / bT
  ldsf64* lo;       // [kBM] each column's lowest mean over the batch
  ldsf64* hi;       // [kBM] ... highest
  ldsf64* kb;       // [3][kBN] min qe, max qb, min qb per column (F takes k of them)
  ldsf64* lv;       // [kBB * tcap] the lists: each column's temps' means in (chunk, position)
                    //              order; the Welford pass overwrites each with the mean after it
  ldsu32* lw;       // [kBB * tcap] ... their weights; overwritten with the weight gained so far
  ldsu32* off;      // [kBN + 1] list start of column i (column 0 at 0, its Z temps included)
  ldsu32* ctl;      // [8] 0: first decision failure; 1: #flagged; 2: usable chunks; 3: first
                    //     structural failure; 4: no batch (means out of order, a list over 255,
                    //     a value outside the fast division's range)
  ldsu16* flagged;  // [kBM] columns whose bound tests are not certain
  ldsu8* lj;        // [kBB * tcap] each list entry's chunk, 0x80: a Z temp (column 0)
  ldsu8* pos;       // [kBB * tcap] #means < v of temp p of chunk j (j * tcap + p)
  ldsu8* nT;        // [kBN][kRS] n[j][i] -- temps of chunk j before main i -- at i * kRS + j
  ldsu8* kT;        // [kBM][kRS] K[j][i] -- column i's list entries from chunks before j
  // flip repair (F'): per boundary i (the count n[j][i] of temps <= mean i) the first chunk where
  // it is wrong (kBB: none); per column its bound tests not certain; re-done columns' per-chunk
  // mean and gain after each chunk from rfirst[slot] on, slot rslot[i] (0xff: not re-done)
  ldsu32* ffl;      // [kBN + 1]
  ldsf64* rmean;    // [kRepCols * kBB]
  ldsu32* rgain;    // [kRepCols * kBB]
  ldsu16* rlist;    // [kRepCols] the columns re-done in the current repair round
  ldsu8* fl;        // [kBM]
  ldsu8* rslot;     // [kBM]
  ldsu8* rfirst;    // [kRepCols]
  ldsu32* rctl;     // [5] a repair round's counts: 0 columns to re-do, 1 new slots, 2 boundary 0/1
                    //     wrong, 3 the list's fill, 4 the first wrong chunk of the other boundaries
};

__host__ __device__ inline uint32_t batch_bytes(uint32_t tcap) {
  const uint32_t nl = kBB * tcap;
  return 12u * kRing * tcap + 16u * kBB + 16u * kBM + 24u * kBN + 8u * (nl + 1) + 4u * (nl + 1) + 4u * (kBN + 1) + 32u +
         2u * kBM + (nl + 16u) + (nl + 16u) + 16u + kBN * kRS + kBM * kRS + 16u +
         (kRepairs ? 4u * (kBN + 1) + 12u * kRepCols * kBB + 2u * kRepCols + 2u * kBM + kRepCols + 48u : 0u);
}
__host__ __device__ inline uint32_t batch_offset(uint32_t capc, uint32_t tcap) {
  const uint32_t TP = (tcap + 1 + 63u) & ~63u, JW = capc + TP + 1 > 320u ? capc + TP + 1 : 320u;
  return (fast_offset(capc, tcap) + fast_extra_bytes(capc, TP, JW) + 15u) & ~15u;
}
__device__ __forceinline__ BatchLds batch_layout(char* p, uint32_t tcap) {
  const uint32_t nl = kBB * tcap;
  BatchLds B;
  B.rv = (ldsf64*)p;
  B.bT = B.rv + kRing * tcap;
  B.brT = B.bT + kBB;
  B.lo = B.brT + kBB;
  B.hi = B.lo + kBM;
  B.kb = B.hi + kBM;
  B.lv = B.kb + 3 * kBN;
  B.rp = (ldsu32*)(B.lv + nl + 1);  // (lv[nl], lw[nl]: where E's idle lanes store)
  B.lw = B.rp + kRing * tcap;
  B.off = B.lw + nl + 1;
  B.ctl = B.off + (kBN + 1);
  B.flagged = (ldsu16*)(B.ctl + 8);
  B.lj = (ldsu8*)(B.flagged + kBM);
  B.pos = B.lj + nl + 16;  // (lj[nl], pos[nl]: spare slots for idle lanes' stores)
  B.nT = (ldsu8*)(((uintptr_t)(B.pos + nl + 16) + 15u) & ~(uintptr_t)15u);
  B.kT = B.nT + kBN * kRS;
  B.rmean = (ldsf64*)(((uintptr_t)(B.kT + kBM * kRS) + 15u) & ~(uintptr_t)15u);
  B.rgain = (ldsu32*)(B.rmean + kRepCols * kBB);
  B.ffl = B.rgain + kRepCols * kBB;
  B.rlist = (ldsu16*)(B.ffl + kBN + 1);
  B.fl = (ldsu8*)(B.rlist + kRepCols);
  B.rslot = B.fl + kBM;
  B.rfirst = B.rslot + kBM;
  B.rctl = (ldsu32*)(((uintptr_t)(B.rfirst + kRepCols) + 3u) & ~(uintptr_t)3u);
  return B;
}

__device__ __forceinline__ void lds_min(ldsu32* p, uint32_t v) { __atomic_fetch_min(p, v, __ATOMIC_RELAXED); }
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {  // (every lane active)
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, d, 64));
  return v;
}
__device__ __forceinline__ uint32_t lds_inc(ldsu32* p) { return __atomic_fetch_add(p, 1u, __ATOMIC_RELAXED); }

// n dwords from global src into LDS dst by global->LDS dword loads: each wave instruction moves
// 64 dwords (the destination is wave-uniform, lane l its dword l).  Completion: vmcnt.
template <int NW>
__device__ __forceinline__ void dma_dwords(ldsu32* d, const uint32_t* __restrict__ s, uint32_t nd) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t q = wv; 64 * q < nd; q += NW) {
    const uint32_t k = 64 * q + lane;
    if (k < nd) __builtin_amdgcn_global_load_lds(s + k, (__attribute__((address_space(3))) void*)(d + 64 * q), 4, 0, 0);
  }
}
// chunks [x, y) (y - x <= kRing) of the chunk sorter's means and packed weights into their slots
template <int NW>
__device__ __forceinline__ void ring_fill(const BatchLds B, const double* gv, const uint32_t* gp, uint32_t x,
                                          uint32_t y, uint32_t tcap) {
  const uint32_t s0 = x % kRing, n = y - x, n1 = min(n, kRing - s0);
  const uint64_t g0 = (uint64_t)x * tcap;
  dma_dwords<NW>((ldsu32*)(B.rv + s0 * tcap), (const uint32_t*)(gv + g0), 2 * n1 * tcap);
  dma_dwords<NW>(B.rp + s0 * tcap, gp + g0, n1 * tcap);
  if (n > n1) {
    const uint64_t g1 = (uint64_t)(x + n1) * tcap;
    dma_dwords<NW>((ldsu32*)B.rv, (const uint32_t*)(gv + g1), 2 * (n - n1) * tcap);
    dma_dwords<NW>(B.rp, gp + g1, (n - n1) * tcap);
  }
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct BatchResult {
  uint32_t js;      // merges committed
  bool structural;  // merge js failed a structure test (it runs alone); else the next batch starts there
};

// inclusive sum over the 16 lanes of each DPP row (row_shr 1, 2, 4, 8; lanes without a source add 0)
__device__ __forceinline__ uint32_t row_incl_add(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  return v;
}
// a double from lane l - n of the same row (ident where there is none), as two dword moves
template <int CTRL>
__device__ __forceinline__ double row_shr_d(double v, double ident) {
  const uint64_t b = (uint64_t)__double_as_longlong(v), z = (uint64_t)__double_as_longlong(ident);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)z, (int)(uint32_t)b, CTRL, 0xf, 0xf, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(z >> 32), (int)(uint32_t)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// min / max over each row's 16 lanes, complete in lane 15 of the row
__device__ __forceinline__ double row_min_d(double v) {
  v = __builtin_fmin(v, row_shr_d<0x111>(v, 2.0));
  v = __builtin_fmin(v, row_shr_d<0x112>(v, 2.0));
  v = __builtin_fmin(v, row_shr_d<0x114>(v, 2.0));
  return __builtin_fmin(v, row_shr_d<0x118>(v, 2.0));
}
__device__ __forceinline__ double row_max_d(double v) {
  v = __builtin_fmax(v, row_shr_d<0x111>(v, -1.0));
  v = __builtin_fmax(v, row_shr_d<0x112>(v, -1.0));
  v = __builtin_fmax(v, row_shr_d<0x114>(v, -1.0));
  return __builtin_fmax(v, row_shr_d<0x118>(v, -1.0));
}

// |x| is 0 or within [2^-400, 2^400]: the Welford division of the batch then never needs
// v_div_scale's rescaling (see merge_batch, E)
__device__ __forceinline__ bool div_safe(double x) {
  const double a = __builtin_fabs(x);
  return a == 0.0 || (a >= 3.872591914849318e-121 && a <= 2.5822498780869086e120);
}

// Merges chunks c .. c+b-1 (in the ring) as far as the checks allow: L.mm/L.mw/F.mp/mainW then
// hold the digest after the committed merges.  Every phase is written for latency at one wave
// per SIMD: a thread's independent LDS loads issue together and are waited for once.
template <int NW>
__device__ __forceinline__ BatchResult merge_batch(const double delta, const double sin_hi, const double sin_lo,
                                                   const Lds L, const FastLds F, const BatchLds B,
                                                   const uint32_t nm_in, double& mainW, const uint32_t c_in,
                                                   uint32_t b, const uint32_t tcap, const bool fint) {
  // (wave-uniform values in scalar registers: every chunk address below is then scalar math)
  const uint32_t nm = __builtin_amdgcn_readfirstlane(nm_in), c = __builtin_amdgcn_readfirstlane(c_in);
  constexpr uint32_t NT = 64 * NW;
  constexpr uint32_t kA = (kBB * kBTmax + NT - 1) / NT;  // temps per thread (all threads)
  static_assert(NW == 4, "column lanes on waves 0-2, bounds on waves 2-3");
  static_assert(kBM <= 192 && kBM >= 128, "one lane of waves 0-2 per column; wave 3 takes columns 64..127");
  static_assert(kBB % 8 == 0 && kRS % 8 == 0, "rows are read and written as 8-byte words");
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t cr = c % kRing;
  auto sbase = [&](uint32_t j) {  // ring offset of the batch's chunk j
    const uint32_t s = cr + j;
    return (s >= kRing ? s - kRing : s) * tcap;
  };
  auto tw_of = [&](uint32_t j, uint32_t n) -> uint32_t {  // chunk j's sorted weight before temp n
    const uint32_t v = B.rp[sbase(j) + (n >= tcap ? 0u : n)] >> 16;
    return n == 0 ? 0u : v;  // (n = tcap: slot 0 holds tempW)
  };
  PROF_T(b0);
  // ---- totals: the usable chunks are the leading batchable ones with T <= 2^40 (every prefix
  // below is then an exact u32 / f64 integer: a chunk's tempW < 2^16, the batch's < 2^22), or
  // T <= 2^30 when some main weight is not an integer (a 2^-23 multiple: sums exact up to 2^30)
  if (wv == 0) {
    const uint32_t tw0 = B.rp[sbase(min(lane, b - 1))], tw = lane < b ? tw0 : 0xffffffffu;
    bool ok = lane < b && tw != 0xffffffffu;
    const uint32_t v = wave_incl_add_u32(ok ? tw >> 16 : 0u);  // (< 2^22: exact)
    const double T = dadd(mainW, (double)v);
    ok = ok && T <= fast_total_limit(fint);
    const uint64_t bad = __ballot(!ok);
    const uint32_t nb = min(bad ? (uint32_t)__builtin_ctzll(bad) : 64u, b);
    if (lane < b) {
      B.bT[lane] = T;
      B.brT[lane] = ddiv(1.0, T);
    }
    if (lane == 0) {
      B.ctl[0] = nb;
      B.ctl[1] = 0u;
      B.ctl[2] = nb;
      B.ctl[3] = nb;
      B.ctl[4] = 0u;
      B.ctl[5] = 0u;  // C2's next column group
      B.kb[kBN + nm] = 1.0;  // the end (q = 1)
      B.kb[2 * kBN + nm] = 1.0;
    }
  }
  // +inf past the last mean up to 192 (nm <= kBM = 160): A's searches read index min(i, 191), so
  // they need no other bound checks, and the tile needs only 192 entries (capc >= 192)
  for (uint32_t j = nm + t; j < 192u; j += NT) L.mm[j] = kInf;
  if constexpr (kRepairs > 0) {  // (F': no boundary known wrong, no column re-done, none flagged)
    for (uint32_t j = t; j <= kBN; j += NT) B.ffl[j] = kBB;
    for (uint32_t j = t; j < kBM; j += NT) {
      B.rslot[j] = 0xffu;
      B.fl[j] = 0u;
    }
    if (t < 5) B.rctl[t] = t == 4 ? kBB : 0u;
    if (t == 0) B.ctl[6] = 0u;
  }
  fast_sync<NW>();
  PROF_T(b1);
  ASM_MARK("A_BEGIN");
  b = __builtin_amdgcn_readfirstlane(B.ctl[2]);
  if (b < 2) {
    fast_sync<NW>();
    return BatchResult{0u, true};
  }
  const uint32_t nt = b * tcap;
  // ---- A: pos of every temp: lower-bound searches over the means, a thread's temps in step;
  // the first three levels from seven pivots held in registers, the rest from LDS
  uint32_t gj[kA], gp[kA], ps[kA];
  double gv[kA];
  {
    const double p0 = L.mm[127], p1 = L.mm[63], p2 = L.mm[191];
    const double p3 = L.mm[31], p4 = L.mm[95], p5 = L.mm[159], p6 = kInf;  // (223 >= nm)
    bool safe = true;
    // (chunk, position) of temp g = t + u * NT: one division, then steps of NT = qs * tcap + rs
    const uint32_t qs = NT / tcap, rs = NT - qs * tcap;
    uint32_t jg = t / tcap, pg = t - jg * tcap;
#pragma unroll
    for (uint32_t u = 0; u < kA; u++) {
      const uint32_t g = t + u * NT;
      gj[u] = jg;
      gp[u] = pg;
      pg += rs;
      jg += qs;
      const bool wrap = pg >= tcap;  // (rs < tcap: one step at most)
      pg = wrap ? pg - tcap : pg;
      jg = wrap ? jg + 1u : jg;
      const double x = B.rv[sbase(min(gj[u], kBB - 1)) + gp[u]];  // (unconditional: see D)
      gv[u] = g < nt ? x : 0.0;
      safe &= div_safe(gv[u]);
    }
#pragma unroll
    for (uint32_t u = 0; u < kA; u++) {  // (the +inf sentinels past nm bound every level)
      const double v = gv[u];
      uint32_t l = p0 < v ? 128u : 0u;
      l = (l ? p2 : p1) < v ? l + 64u : l;
      const double q = l >= 128u ? (l >= 192u ? p6 : p5) : (l >= 64u ? p4 : p3);
      l = q < v ? l + 32u : l;
      ps[u] = l;
    }
#pragma unroll
    for (uint32_t step = 16; step >= 1; step >>= 1) {
      double mv[kA];
#pragma unroll
      for (uint32_t u = 0; u < kA; u++) mv[u] = L.mm[min(ps[u] + step - 1, 191u)];
#pragma unroll
      for (uint32_t u = 0; u < kA; u++) ps[u] = mv[u] < gv[u] ? ps[u] + step : ps[u];
    }
#pragma unroll
    for (uint32_t u = 0; u < kA; u++) {  // (idle lanes store to the spare slot: no branch)
      const uint32_t g = t + u * NT;
      B.pos[g < nt ? g : kBB * tcap] = (uint8_t)ps[u];
    }
    // the run-end rows of B (kSR bytes per chunk, in the list area, which D fills later) zeroed
    ldsu64* const sr = (ldsu64*)B.lv;
    for (uint32_t q = t; q < kBB * kSR / 8; q += NT) sr[q] = 0ull;
    if (t < nm) safe &= div_safe(L.mm[t]);
    if ((t + 1 < nm && !(L.mm[t] <= L.mm[t + 1])) || !safe) B.ctl[4] = 1u;  // (t < 256: nm <= 160)
  }
  fast_sync<NW>();
  PROF_T(b2);
  if (B.ctl[4]) {  // means out of order (the pos runs would not be monotone), or a value outside
    fast_sync<NW>();  // the fast division's range: no batch
    return BatchResult{0u, true};
  }
  ASM_MARK("B_BEGIN");
  // ---- B: the n table.  n[j][i] = #temps of chunk j with pos <= i, a step function of i: the last
  // temp p of each run of equal pos c writes p + 1 at column c of chunk j's run-end row (B1); a
  // wave then takes four chunks at a time, a lane four columns, and max-scans each row over the
  // columns (within the lane's dword, then across lanes by DPP), packing the four chunks' bytes of
  // each column into one dword of the column-major table (B2)
  {
    ldsu8* const sr = (ldsu8*)B.lv;
#pragma unroll
    for (uint32_t u = 0; u < kA; u++) {
      const uint32_t g = t + u * NT;
      const uint32_t nx = B.pos[min(g + 1, nt - 1)];
      const bool end = g < nt && (gp[u] + 1 == tcap || nx != ps[u]);
      sr[end ? gj[u] * kSR + ps[u] : kBB * kSR] = (uint8_t)(gp[u] + 1);  // (else: a spare byte)
    }
  }
  fast_sync<NW>();
  {
    const ldsu32* const sr = (const ldsu32*)B.lv;
    for (uint32_t g4 = wv; 4 * g4 < b; g4 += NW) {
      uint32_t x[4];
#pragma unroll
      for (uint32_t s4 = 0; s4 < 4; s4++) {
        const uint32_t y = sr[(4 * g4 + s4) * (kSR / 4) + min(lane, kSR / 4 - 1)];
        x[s4] = lane < kSR / 4 ? y : 0u;
      }
      uint32_t out[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (uint32_t s4 = 0; s4 < 4; s4++) {
        const uint32_t b0 = x[s4] & 0xffu, m1 = max(b0, (x[s4] >> 8) & 0xffu), m2 = max(m1, (x[s4] >> 16) & 0xffu),
                       m3 = max(m2, x[s4] >> 24);
        const uint32_t carry = wave_shr1(wave_incl_max(m3));
        out[0] |= max(b0, carry) << (8 * s4);
        out[1] |= max(m1, carry) << (8 * s4);
        out[2] |= max(m2, carry) << (8 * s4);
        out[3] |= max(m3, carry) << (8 * s4);
      }
#pragma unroll
      for (uint32_t k = 0; k < 4; k++)
        if (4 * lane + k <= nm) *(ldsu32*)(B.nT + (4 * lane + k) * kRS + 4 * g4) = out[k];
    }
  }
  fast_sync<NW>();
  PROF_T(b3);
  ASM_MARK("C_BEGIN");
  // ---- C.  A column lane holds rows n[.][i] and n[.][i+1] as words (chunks j < b count):
  // the list offset off_i = sum_j n[j][i] (the temps of the columns before it, Z included;
  // column 0 at 0), the K row (a prefix over the chunks of its per-chunk counts), and the k
  // bounds (C2: waves 2 and 3, beside the others)
  constexpr uint32_t kW = kBB / 4;  // u32 words of a row
  auto load_row = [&](const ldsu8* tab, uint32_t r, uint32_t (&w)[kW]) {
    const ldsu64* const rw = (const ldsu64*)(tab + r * kRS);
#pragma unroll
    for (uint32_t q = 0; q < kW / 2; q++) {
      const uint64_t x = rw[q];
      w[2 * q] = (uint32_t)x;
      w[2 * q + 1] = (uint32_t)(x >> 32);
    }
  };
  auto wmask = [&](uint32_t q) {  // the bytes of word q that are chunks < b
    const uint32_t v = b > 4 * q ? min(b - 4 * q, 4u) : 0u;
    return v >= 4 ? 0xffffffffu : ((1u << (8 * v)) - 1u);
  };
  // C2: the q bounds of four columns at once (q = P / T from exact integer prefixes; k is
  // increasing, so F's k bounds are k of these), one DPP row per column: lane q of the row takes
  // chunks 4q .. 4q+3 (their n bytes one dword of each row), the prefixes over the chunks a row
  // scan, the min / max a row reduction.  Same integers and operations per chunk as a sequential
  // walk over the chunks, so the same bounds bit for bit
  // (two groups per queue entry, interleaved: their LDS round trips overlap)
#ifndef VN_C2_GROUPS
#define VN_C2_GROUPS 2
#endif
  constexpr uint32_t kC2H = VN_C2_GROUPS, kC2Cols = 4 * kC2H;
  const uint32_t c2q = lane & 15;
  uint32_t c2base[4];
  double c2rT[4];
  bool c2j[4];
#pragma unroll
  for (uint32_t u = 0; u < 4; u++) {  // the lane's chunks: the same in every group
    const uint32_t j = 4 * c2q + u, jc = min(j, b - 1);
    c2j[u] = j < b;
    c2base[u] = sbase(jc);
    c2rT[u] = B.brT[jc];
  }
  auto c2_group = [&](uint32_t g0) {
    ASM_MARK("C2_GROUP");
    uint32_t wa[kC2H], we[kC2H], ci[kC2H];
    bool cok[kC2H];
    double mp0[kC2H], mpw[kC2H];
#pragma unroll
    for (uint32_t h = 0; h < kC2H; h++) {
      ci[h] = g0 + 4 * h + (lane >> 4);
      cok[h] = ci[h] < nm;
      const uint32_t cc = min(ci[h], nm - 1);
      wa[h] = *(const ldsu32*)(B.nT + cc * kRS + 4 * c2q);
      we[h] = *(const ldsu32*)(B.nT + (cc + 1) * kRS + 4 * c2q);
      mp0[h] = F.mp[cc];
      mpw[h] = L.mw[cc];
    }
    uint32_t sa[kC2H][4], se[kC2H][4];
#pragma unroll
    for (uint32_t h = 0; h < kC2H; h++)
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        const uint32_t na = (wa[h] >> (8 * u)) & 0xffu, ne = (we[h] >> (8 * u)) & 0xffu;
        const uint32_t x = B.rp[c2base[u] + (na >= tcap ? 0u : na)] >> 16;
        const uint32_t y = B.rp[c2base[u] + (ne >= tcap ? 0u : ne)] >> 16;
        const bool ok = cok[h] && c2j[u];
        sa[h][u] = ok && na ? x : 0u;
        se[h][u] = ok && ne ? y : 0u;
      }
#pragma unroll
    for (uint32_t h = 0; h < kC2H; h++) {
      mpw[h] = dadd(mp0[h], mpw[h]);
      const uint32_t ta = sa[h][0] + sa[h][1] + sa[h][2] + sa[h][3], te = se[h][0] + se[h][1] + se[h][2] + se[h][3];
      uint32_t C = row_incl_add(ta) - ta, X = row_incl_add(te) - te;  // sums over the chunks before 4q
      double qemin = 2.0, qbmin = 2.0, qbmax = -1.0;
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        C += sa[h][u];
        // P = mp0 + C; qe = (P + W) / T with W = w0 + the gain before chunk j = w0 + X - (C - sa)
        const double qe = dadd(mpw[h], (double)(X + sa[h][u])) * c2rT[u];
        const double qb = dadd(mp0[h], (double)C) * c2rT[u];
        X += se[h][u];
        const bool ok = cok[h] && c2j[u];
        qemin = __builtin_fmin(qemin, ok ? qe : 2.0);
        qbmin = __builtin_fmin(qbmin, ok ? qb : 2.0);
        qbmax = __builtin_fmax(qbmax, ok ? qb : -1.0);
      }
      qemin = row_min_d(qemin);
      qbmin = row_min_d(qbmin);
      qbmax = row_max_d(qbmax);
      if (c2q == 15 && cok[h]) {
        B.kb[ci[h]] = qemin;
        B.kb[kBN + ci[h]] = ci[h] ? qbmax : 0.0;  // (column 0 starts at q = 0: with Z temps or main 0 itself)
        B.kb[2 * kBN + ci[h]] = ci[h] ? qbmin : 0.0;
      }
    }
  };
  // column groups taken from a queue by whichever wave is free (after its Welford lists); the
  // next entry is drawn before this one is worked
  auto c2_queue = [&]() {
    uint32_t g = 0;
    if (lane == 0) g = lds_inc(&B.ctl[5]);
    g = kC2Cols * __builtin_amdgcn_readfirstlane(g);
    while (g < nm) {
      uint32_t gn = 0;
      if (lane == 0) gn = lds_inc(&B.ctl[5]);
      c2_group(g);
      g = kC2Cols * __builtin_amdgcn_readfirstlane(gn);
    }
  };
  const uint32_t i = t;
  uint32_t ra[kW], re[kW];
  if (wv < 3) {
    if (i < nm) {
      load_row(B.nT, i, ra);
      load_row(B.nT, i + 1, re);
      uint32_t o = 0, carry = 0;
      uint64_t kw[kW / 2];
#pragma unroll
      for (uint32_t q = 0; q < kW; q++) {
        const uint32_t mk = wmask(q);
        const uint32_t a = i == 0 ? 0u : ra[q] & mk, e = re[q] & mk;
        uint32_t x = a;
        x = (x & 0x00ff00ffu) + ((x >> 8) & 0x00ff00ffu);
        o += (x & 0xffffu) + (x >> 16);
        // per-chunk counts e - a (bytewise, e >= a: no borrows), their bytewise prefix (x * 0x01010101
        // while sums stay below 256; the column's total is checked below)
        const uint32_t cnt = e - a, incl = cnt * 0x01010101u;
        const uint32_t ex = incl - cnt + carry * 0x01010101u;
        carry += incl >> 24;
        if (q & 1) kw[q >> 1] |= (uint64_t)ex << 32;
        else kw[q >> 1] = ex;
      }
      if (carry > 255u) B.ctl[4] = 1u;  // (a list over 255 entries: no batch)
      B.off[i] = o;
      if (i + 1 == nm) B.off[nm] = o + carry;
      ldsu64* const kr = (ldsu64*)(B.kT + i * kRS);
#pragma unroll
      for (uint32_t q = 0; q < kW / 2; q++) kr[q] = kw[q];
    }
  }
  PROF_T(cw1);
  PROF_T(cw2);
  PROF_ADDW(40, cw1, cw2);
  fast_sync<NW>();
  PROF_T(b4);
#ifdef VN_REPLAY_CHECK
  if (t == 0 && !B.ctl[4] && B.off[nm] != nt) {
    printf("VN_REPLAY_CHECK merge_batch chunk %u: lists hold %u entries, %u temps (nm %u, b %u)\n", c, B.off[nm], nt, nm, b);
    B.ctl[4] = 1u;
  }
  fast_sync<NW>();
#endif
  if (B.ctl[4]) {
    fast_sync<NW>();
    return BatchResult{0u, true};
  }
  ASM_MARK("D_BEGIN");
  // ---- D: every temp into its column's list at off_c + K[j][c] + its place in the chunk's run
  // (column 0: Z temps and main 0's own temps, p itself), with its mean and weight
  {
    // (every load unconditional, at a clamped address, and selected afterwards: a conditional load
    // compiles to a branch whose join waits for all LDS traffic in flight)
    uint32_t kk[kA], nn[kA], wq[kA], oo[kA];
#pragma unroll
    for (uint32_t u = 0; u < kA; u++) {
      const uint32_t cc = ps[u] ? min(ps[u] - 1, nm - 1) : 0u, jc = min(gj[u], kBB - 1);
      kk[u] = B.kT[cc * kRS + jc];
      const uint32_t n0 = B.nT[cc * kRS + jc];
      nn[u] = cc ? n0 : 0u;
      oo[u] = B.off[cc];
      wq[u] = B.rp[sbase(jc) + gp[u]] & 0xffffu;
    }
#pragma unroll
    for (uint32_t u = 0; u < kA; u++) {  // (idle lanes store to the spare slot: no branch)
      const uint32_t x = t + u * NT < nt ? oo[u] + kk[u] + gp[u] - nn[u] : kBB * tcap;
      B.lv[x] = gv[u];
      B.lw[x] = wq[u];
      B.lj[x] = (uint8_t)(gj[u] | (ps[u] == 0 ? 0x80u : 0u));
    }
  }
  fast_sync<NW>();
  PROF_T(b5);
  // ---- E: Welford along each list, two blocks of four entries in flight.  The division
  // ((v - mean) * w) / W is the hardware's own sequence -- v_rcp and two Newton steps on W, q0 = t *
  // y, r = fma(-W, q0, t), q = fma(r, y, q0), v_div_fixup -- without v_div_scale, which rescales
  // nothing for these operands: W is an integer in [1, 2^40], every value and mean 0 or of
  // magnitude [2^-400, 2^400] (checked in A), so t = 0 or 2^-505 <= |t| <= 2^425, far from the
  // exponents where the hardware rescales (a numerator below 1e-250 is caught and the batch
  // dropped).  The W chain and the reciprocals do not depend on the means: each block's are
  // issued ahead of its mean chain (sched_barrier), so only the seven dependent operations of
  // the mean update stay on the critical path.
  // Columns 1.. on waves 0-2 (lane = column); column 0, whose list also holds the Z temps, on
  // lane 0 of wave 3 beside them: a chunk's Z temps start a fresh centroid (main 0, the column
  // so far, waiting) and main 0 joins it after the chunk's last Z temp.
  ASM_MARK("E_BEGIN");
  PROF_T(e0);
  const uint32_t nt_all = kBB * tcap;  // the lists' spare slot
  if (wv < 3) {
    const bool col = i >= 1 && i < nm;
    const uint32_t ic = min(i, nm - 1), o0 = B.off[ic], o1 = B.off[ic + 1];
    const double mm0 = L.mm[ic], mw0 = L.mw[ic];
    const uint32_t o = col ? o0 : 0u, m = col ? o1 - o0 : 0u;
    double mean = col ? mm0 : 0.0, W = col ? mw0 : 1.0, lo = mean, hi = mean;
    uint32_t gain = 0;
    bool tiny = false;  // a numerator near the hardware's rescaling range (then no batch)
    uint32_t mmax = wave_incl_max(m);
    mmax = __builtin_amdgcn_readlane(mmax, 63);
    PROF_ADDW(56, 0, (long long)mmax);
    // (entries past a list's end are read too -- the next list's, or the layout after the
    // lists, all inside the workgroup's LDS -- and masked by q + u < m below)
    auto ld = [&](uint32_t q, double (&v)[4], uint32_t (&w)[4]) {
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        v[u] = B.lv[o + q + u];
        w[u] = B.lw[o + q + u];
      }
    };
    double v0[4], v1[4];
    uint32_t w0[4], w1[4];
    ld(0, v0, w0);
#pragma unroll 1
    for (uint32_t q = 0; q < mmax; q += 4) {
      ASM_MARK("E_BODY");
      ld(q + 4, v1, w1);
      double Wn[4], y[4], wd[4];
      bool in[4];
      uint32_t at[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {  // the W chain and the reciprocals
        in[u] = q + u < m;
        const uint32_t wz = in[u] ? w0[u] : 0u;
        wd[u] = (double)wz;
        gain += wz;
        at[u] = in[u] ? o + q + u : nt_all;  // (an idle lane's store goes to the spare slot: no branch)
        Wn[u] = dadd(u ? Wn[u - 1] : W, wd[u]);
        const double r0 = __builtin_amdgcn_rcp(Wn[u]);
        const double e0_ = __builtin_fma(-Wn[u], r0, 1.0);
        const double r1 = __builtin_fma(r0, e0_, r0);
        const double e1_ = __builtin_fma(-Wn[u], r1, 1.0);
        y[u] = __builtin_fma(r1, e1_, r1);
        B.lw[at[u]] = gain;
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {  // the mean chain
        // (an entry past the list's end: weight 0 and value 0, so the step adds a zero and no
        // select sits on the chain -- a -0 mean may become +0 there, which only the lane's
        // [lo, hi], compared with <= / >, and the spare slot see)
        const double vz = in[u] ? v0[u] : 0.0;
        const double tq = dmul(dsub(vz, mean), wd[u]);
        tiny |= tq != 0.0 && __builtin_fabs(tq) < 1e-250;
        // the correctly rounded quotient tq / W: with no operand special (A's range checks, the
        // tiny test above) v_div_fixup would return the fma's result unchanged
        const double q0 = dmul(tq, y[u]);
        const double rr = __builtin_fma(-Wn[u], q0, tq);
        const double qq = __builtin_fma(rr, y[u], q0);
        mean = dadd(mean, qq);
        B.lv[at[u]] = mean;
        // (no NaN here: the hardware min / max, without the canonicalisation fmin / fmax add)
        asm("v_min_f64 %0, %1, %2" : "=v"(lo) : "v"(lo), "v"(mean));
        asm("v_max_f64 %0, %1, %2" : "=v"(hi) : "v"(hi), "v"(mean));
      }
      __builtin_amdgcn_sched_barrier(0);
      W = Wn[3];
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        v0[u] = v1[u];
        w0[u] = w1[u];
      }
    }
    if (col) {
      B.lo[i] = lo;
      B.hi[i] = hi;
    }
    if (tiny) B.ctl[4] = 1u;
  } else if (lane == 0) {
    // column 0: the exact walk, Z temps included (its list is short: the lowest centroid's)
    const uint32_t o = 0, m = B.off[1];
    double mean = L.mm[0], W = L.mw[0], lo = mean, hi = mean, sm = 0.0, sw = 0.0;
    uint32_t gain = 0, prev = 0;
    for (uint32_t q = 0; q < m; q++) {
      const uint32_t e = B.lj[o + q], nx = q + 1 < m ? B.lj[o + q + 1] : 0u;
      const double v = B.lv[o + q], w = (double)B.lw[o + q];
      const bool z = (e & 0x80u) != 0u;
      const bool zstart = z && (q == 0 || !(prev & 0x80u) || ((prev ^ e) & 63u));
      const bool zend = z && (!(nx & 0x80u) || ((nx ^ e) & 63u));
      if (zstart) {
        sm = mean;
        sw = W;
        mean = v;
        W = w;
      } else {
        W = dadd(W, w);
        mean = dadd(mean, ddiv(dmul(dsub(v, mean), w), W));
      }
      if (zend) {
        W = dadd(W, sw);
        mean = dadd(mean, ddiv(dmul(dsub(sm, mean), sw), W));
      }
      if (!z || zend) {
        lo = __builtin_fmin(lo, mean);
        hi = __builtin_fmax(hi, mean);
      }
      gain += B.lw[o + q];
      B.lv[o + q] = mean;
      B.lw[o + q] = gain;
      prev = e;
    }
    B.lo[0] = lo;
    B.hi[0] = hi;
  }
  ASM_MARK("C2Q_BEGIN");
  PROF_T(e1);
  PROF_ADD(14, e0, e1);
  PROF_ADDW(36, e0, e1);
  c2_queue();
  PROF_T(e2);
  PROF_ADDW(44, e1, e2);
  fast_sync<NW>();
  PROF_T(b6);
  ASM_MARK("F_BEGIN");
  // ---- F: decisions per temp against the columns' mean ranges (the exact mean merge j saw
  // only for a temp inside a range); bound tests per column
  // column ci's mean and gain (weight added since the batch start) before merge j: after its last
  // list entry from a chunk < j, or (F') from its re-done means once past the chunk it was re-done from
  auto mean_before = [&](uint32_t ci, uint32_t j) -> double {
    if constexpr (kRepairs > 0) {
      const uint32_t sl = B.rslot[ci];
      if (sl != 0xffu && j > B.rfirst[sl]) return B.rmean[sl * kBB + j - 1];
    }
    const uint32_t kq = B.kT[ci * kRS + j];
    return kq ? B.lv[B.off[ci] + kq - 1] : L.mm[ci];
  };
  auto gain_before = [&](uint32_t ci, uint32_t j) -> uint32_t {
    if constexpr (kRepairs > 0) {
      const uint32_t sl = B.rslot[ci];
      if (sl != 0xffu && j > B.rfirst[sl]) return B.rgain[sl * kBB + j - 1];
    }
    const uint32_t kq = B.kT[ci * kRS + j];
    return kq ? B.lw[B.off[ci] + kq - 1] : 0u;
  };
  {
    double hl[kA], lr[kA];
#pragma unroll
    for (uint32_t u = 0; u < kA; u++) {
      hl[u] = B.hi[ps[u] >= 1 ? ps[u] - 1 : 0];
      lr[u] = B.lo[min(ps[u], nm - 1)];
    }
#pragma unroll
    for (uint32_t u = 0; u < kA; u++) {
      const bool in = t + u * NT < nt;
      const bool rl = in && ps[u] >= 1 && gv[u] <= hl[u], rr = in && ps[u] < nm && gv[u] > lr[u];
      if (rl || rr) {  // (rare) inside a column's range: the exact order against the mean merge j saw
        // (a failure is a flip: boundary ps-1 -- the count of temps up to mean ps-1 -- or boundary ps
        // is wrong in chunk j; F' records the first such chunk per boundary)
        const bool badl = rl && !(mean_before(ps[u] - 1, gj[u]) < gv[u]);  // main ps-1 before it
        const bool badr = rr && !(gv[u] <= mean_before(ps[u], gj[u]));     // it before main ps
        if (badl || badr) lds_min(&B.ctl[0], gj[u]);
        if constexpr (kRepairs > 0) {
          if (badl) lds_min(&B.ffl[ps[u] - 1], gj[u]);
          if (badr) lds_min(&B.ffl[ps[u]], gj[u]);
        }
      }
    }
  }
  // k(a) - k(b) = delta / pi * (asin xa - asin xb) with x = 2q - 1: compared with kHi / kLo
  // through D = asin xa - asin xb, sin D = xa cb - xb ca and cos D = ca cb + xa xb (c = sqrt(1 - x^2)
  // = 2 sqrt(q (1 - q))); with cos D > 0, D is in (-pi/2, pi/2) where sin is increasing, so
  // D > theta iff sin D > sin theta.  No arcsine: the band (kBand in k, about 3e-11 in sin)
  // dwarfs these few roundings, and whatever it does not decide is tested exactly in G
  auto sure_col = [&](uint32_t ic) -> bool {
    auto xc = [](double qv, double& x, double& c) {
      qv = __builtin_fmin(qv, 1.0);  // (q <= 1: the reciprocal's rounding)
      x = 2.0 * qv - 1.0;
      c = 2.0 * __builtin_sqrt(qv * (1.0 - qv));
    };
    double xa, ca, xb, cb;
    bool sure = true;
    if (ic >= 1) {  // main i starts: k(min qe_i) - k(max qb_i-1) > kHi
      xc(B.kb[ic], xa, ca);
      xc(B.kb[kBN + ic - 1], xb, cb);
      sure = ca * cb + xa * xb > 0.0 && xa * cb - xb * ca > sin_hi;
    }
    // its temps join: k(max qb_i+1) - k(min qb_i) < kLo
    xc(B.kb[kBN + ic + 1], xa, ca);
    xc(B.kb[2 * kBN + ic], xb, cb);
    return sure && ca * cb + xa * xb > 0.0 && xa * cb - xb * ca < sin_lo;
  };
  if (i < nm) {
    if (i + 1 < nm && !(B.hi[i] <= B.lo[i + 1])) B.ctl[4] = 1u;
    const bool sure = sure_col(i);
    if constexpr (kRepairs > 0) B.fl[i] = sure ? 0u : 1u;
    else if (!sure) B.flagged[lds_inc(&B.ctl[1])] = (uint16_t)i;
  }
  fast_sync<NW>();
  PROF_T(b7);
  if constexpr (kRepairs > 0) {
    // ---- F': flip repair.  The first chunk jf whose count at some boundary i (the temps up to mean
    // i in merge jf) differs from the batch-start one: every such boundary of chunk jf is set to its
    // exact count from the means merge jf saw, the two columns beside each (i - 1 and i, whose temps
    // change) are re-done from chunk jf on -- their Welford chains, their C2 bounds -- and the
    // boundaries of the re-done columns are checked again for the chunks after jf, where their means
    // now differ.  Other columns' lists, means and first wrong chunks stand: a boundary depends only
    // on its own column's mean.  Up to kRepairs rounds; a flip at boundary 0 or 1 (column 0's, with
    // its Z temps) or past kRepCols re-done columns ends the batch there as before.
    // tools/study/batch2_sim.c (repair cap) restates it on the CPU: bit-identical digests.
    PROF_T(r0);
    uint32_t nrep = 0;
    for (; nrep < kRepairs; nrep++) {
      const uint32_t jf = __builtin_amdgcn_readfirstlane(B.ctl[0]);
      if (jf >= b || B.ctl[4]) break;
      // (the slots taken so far, read before R1a's barrier: R1b's lds_inc on ctl[6] may run in a
      // faster wave while a slower one still decides `bad` below, and every wave must decide alike)
      const uint32_t nslot0 = __builtin_amdgcn_readfirstlane(B.ctl[6]);
      PROF_T(q0);
      PROF_ADD(59, 0, (long long)(b - jf));
      // R1 (a thread per column): the columns to re-do (boundary c or c + 1 fixed), counted
      const uint32_t fi = i < nm ? B.ffl[i] : kBB;
      const bool fixc = fi == jf, fixn = i < nm && B.ffl[i + 1] == jf;
      const bool need = fixc || fixn, isnew = need && B.rslot[min(i, kBM - 1)] == 0xffu;
      {
        const uint64_t bn = __ballot(need), bw = __ballot(isnew), bb = __ballot(fixc && i < 2);
        // (the first wrong chunk over the boundaries R3 does not re-check: R3 adds its own to it)
        const uint32_t mo = wave_min_u32(need ? kBB : fi);
        if (lane == 0) {
          if (bn | bb) {  // (boundaries 0 and 1: column 0 is not re-done)
            __atomic_fetch_add(&B.rctl[0], (uint32_t)__popcll(bn), __ATOMIC_RELAXED);
            __atomic_fetch_add(&B.rctl[1], (uint32_t)__popcll(bw), __ATOMIC_RELAXED);
            if (bb) B.rctl[2] = 1u;
          }
          if (mo < kBB) lds_min(&B.rctl[4], mo);
        }
      }
      fast_sync<NW>();
      const uint32_t nneed = __builtin_amdgcn_readfirstlane(B.rctl[0]);
      const bool bad = B.rctl[2] != 0u || nneed > kRepCols || nslot0 + B.rctl[1] > kRepCols;
      PROF_T(q1);
      PROF_ADD(49, q0, q1);
      if (bad) break;
      // ... their slots and list, and the exact count of every fixed boundary in chunk jf (the
      // means merge jf saw: a slot taken now has rfirst = jf, so mean_before still reads the lists)
      if (need) {
        const uint32_t at = lds_inc(&B.rctl[3]);
        if (!VN_BAD(at < kRepCols, "repair list", at, kRepCols)) B.rlist[at] = (uint16_t)i;
      }
      if (isnew) {
        const uint32_t sl = lds_inc(&B.ctl[6]);
        if (!VN_BAD(sl < kRepCols && i < kBM, "repair slot", sl, i)) {
          B.rslot[i] = (uint8_t)sl;
          B.rfirst[sl] = (uint8_t)jf;
        }
      }
      if (fixc && i >= 2) {
        const uint32_t base = sbase(jf);
        const double mb = mean_before(i, jf);
        uint32_t cn = B.nT[i * kRS + jf];
        while (cn > 0u && B.rv[base + cn - 1] > mb) cn--;
        while (cn < tcap && B.rv[base + cn] <= mb) cn++;
        B.nT[i * kRS + jf] = (uint8_t)cn;
      }
      if (t == 0) B.ctl[0] = B.rctl[4];
      fast_sync<NW>();
      const uint32_t nredo = nneed;
      if (t == 0) B.rctl[0] = B.rctl[1] = B.rctl[3] = 0u, B.rctl[4] = kBB;  // (all read before the barrier above)
      PROF_T(q1b);
      PROF_ADD(34, q1, q1b);
      // R2: each re-done column's Welford chain from chunk jf on a wave of its own (Go's sequence,
      // E's operations), and the C2 bounds of the re-done columns' groups on the other waves: item
      // k < nredo is column k's chain, item nredo + k its group's bounds, wave k % NW takes item k.
      // A chain's wave holds chunk j's first four temps of the column in lane j (one LDS round trip
      // for the whole walk); the walk reads them with v_readlane (the chunk index is uniform), so
      // only the mean's seven dependent operations per temp remain on the critical path, and each
      // lane keeps the mean and gain after its chunk (a chunk without temps keeps the last ones).
      static_assert(kBB <= 64, "a chain's wave holds one chunk per lane");
      for (uint32_t k = wv; k < 2u * nredo; k += NW) {
        if (k >= nredo) {
          c2_group(kC2Cols * (B.rlist[k - nredo] / kC2Cols));
          continue;
        }
        const uint32_t c = B.rlist[k], sl = B.rslot[c];
        if (VN_BAD(c < nm && sl < kRepCols, "repair chain column", c, sl)) continue;
        const uint32_t jl = min(lane, kBB - 1u), tl = tcap - 1u;
        const uint32_t aj = B.nT[c * kRS + jl], ej = B.nT[(c + 1) * kRS + jl], bj = sbase(min(lane, b - 1u));
        double vq[4];
        uint32_t wq[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
          vq[u] = B.rv[bj + min(aj + u, tl)];
          wq[u] = B.rp[bj + min(aj + u, tl)] & 0xffffu;
        }
        double mean = mean_before(c, jf), lo = B.lo[c], hi = B.hi[c];
        uint32_t gain = gain_before(c, jf);
        double W = dadd(L.mw[c], (double)gain);
        double rm = mean;
        uint32_t rg = gain;
        bool tiny = false;
        auto step = [&](double v, uint32_t w) {
          const double wd = (double)w;
          gain += w;
          W = dadd(W, wd);
          const double r0 = __builtin_amdgcn_rcp(W);
          const double e0_ = __builtin_fma(-W, r0, 1.0);
          const double r1 = __builtin_fma(r0, e0_, r0);
          const double e1_ = __builtin_fma(-W, r1, 1.0);
          const double y = __builtin_fma(r1, e1_, r1);
          const double tq = dmul(dsub(v, mean), wd);
          tiny |= tq != 0.0 && __builtin_fabs(tq) < 1e-250;
          const double q0 = dmul(tq, y);
          const double rr = __builtin_fma(-W, q0, tq);
          mean = dadd(mean, __builtin_fma(rr, y, q0));
          asm("v_min_f64 %0, %1, %2" : "=v"(lo) : "v"(lo), "v"(mean));
          asm("v_max_f64 %0, %1, %2" : "=v"(hi) : "v"(hi), "v"(mean));
        };
        auto rl64 = [](double x, uint32_t l) {
          const uint64_t u = (uint64_t)__double_as_longlong(x);
          const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), (int)l);
          const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, (int)l);
          return __longlong_as_double((long long)(((uint64_t)h << 32) | o));
        };
        // the chunks jf <= j < b with temps of this column, in order
        uint64_t todo = __ballot(lane >= jf && lane < b && ej > aj);
        while (todo) {
          const uint32_t jj = (uint32_t)__builtin_ctzll(todo);
          todo &= todo - 1u;
          const uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)(ej - aj), (int)jj);
#pragma unroll
          for (uint32_t u = 0; u < 4; u++)
            if (u < n) step(rl64(vq[u], jj), (uint32_t)__builtin_amdgcn_readlane((int)wq[u], (int)jj));
          if (n > 4u) {  // (rare: more than four temps of the column in one chunk)
            const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)aj, (int)jj), bs = sbase(jj);
            for (uint32_t u = 4; u < n; u++) step(B.rv[bs + a0 + u], B.rp[bs + a0 + u] & 0xffffu);
          }
          if (lane >= jj) {
            rm = mean;
            rg = gain;
          }
        }
        if (lane >= jf && lane < b) {
          B.rmean[sl * kBB + lane] = rm;
          B.rgain[sl * kBB + lane] = rg;
        }
        if (lane == 0) {
          B.lo[c] = lo;
          B.hi[c] = hi;
          if (tiny) B.ctl[4] = 1u;  // (a numerator near the rescaling range: no batch)
        }
      }
      PROF_T(q2w);
      PROF_ADDW(60, q1, q2w);
      fast_sync<NW>();
      PROF_T(q2);
      PROF_ADD(50, q1, q2);
      // R3: the re-done columns' boundaries checked again for every chunk after jf (a wave per
      // column, lane = chunk: the count of temps up to the column's mean must be the table's), the
      // means still in order, the bound tests of the columns beside them again
      for (uint32_t f = wv; f < nredo; f += NW) {
        const uint32_t c = B.rlist[f], j = lane;
        const bool in = j > jf && j < b;
        const uint32_t jj = in ? j : jf + 1u;
        const double mb = mean_before(c, min(jj, b - 1));
        const uint32_t a = B.nT[c * kRS + min(jj, kBB - 1)], base = sbase(min(jj, b - 1));
        const double vlo = B.rv[base + (a ? a - 1u : 0u)], vhi = B.rv[base + min(a, tcap - 1)];
        const bool wrong = in && ((a > 0u && vlo > mb) || (a < tcap && vhi <= mb));
        const uint64_t fail = __ballot(wrong);
        if (lane == 0) {
          B.ffl[c] = fail ? (uint32_t)__builtin_ctzll(fail) : kBB;
          if (fail) lds_min(&B.ctl[0], (uint32_t)__builtin_ctzll(fail));
          if ((c >= 1 && !(B.hi[c - 1] <= B.lo[c])) || (c + 1 < nm && !(B.hi[c] <= B.lo[c + 1]))) B.ctl[4] = 1u;
        }
        if (lane < 3) {
          const uint32_t ic = c + lane - 1u;  // columns c - 1, c, c + 1
          if (ic < nm) B.fl[ic] = sure_col(ic) ? 0u : 1u;
        }
      }
      fast_sync<NW>();
      PROF_T(q3);
      PROF_ADD(51, q2, q3);
    }
    if (i < nm && B.fl[i]) B.flagged[lds_inc(&B.ctl[1])] = (uint16_t)i;
    fast_sync<NW>();
    PROF_T(r1);
    PROF_ADD(32, 0, (long long)nrep);
    PROF_ADD(33, r0, r1);
    PROF_ADD(35, 0, (long long)B.ctl[6]);
  }
  ASM_MARK("G_BEGIN");
  // ---- G: exact tests of the flagged columns, one wave per column, lane = chunk
  const uint32_t nflag = __builtin_amdgcn_readfirstlane(B.ctl[1]);
  for (uint32_t f = wv; f < nflag; f += NW) {
    const uint32_t ic = B.flagged[f], j = lane;
    const bool in = j < b;
    const uint32_t jj = in ? j : 0u;
    const uint32_t nP = ic >= 1 ? B.nT[(ic - 1) * kRS + jj] : 0u, nI = ic >= 1 ? B.nT[ic * kRS + jj] : 0u,
                   nN = B.nT[(ic + 1) * kRS + jj];
    const uint32_t xP = in ? tw_of(jj, nP) : 0u, xI = in ? tw_of(jj, nI) : 0u, xN = in ? tw_of(jj, nN) : 0u;
    // (inclusive prefixes over the chunks: DPP wave scans, every lane of the wave active)
    const uint32_t cP = wave_incl_add_u32(xP), cI = wave_incl_add_u32(xI), cN = wave_incl_add_u32(xN);
    const double T = B.bT[jj];
    const double Pi = dadd(F.mp[ic], (double)cI), Pn = dadd(F.mp[ic + 1], (double)cN);
    const double Wi = dadd(L.mw[ic], (double)((cN - xN) - (cI - xI)));  // weight before merge j
    bool ok = true;
    if (ic >= 1) {
      const double qp = ic == 1 ? 0.0 : ddiv(dadd(F.mp[ic - 1], (double)cP), T);
      ok = dsub(index_estimate<VN_NR_G>(delta, ddiv(dadd(Pi, Wi), T)), index_estimate<VN_NR_G>(delta, qp)) > 1.0;
    }
    if (nN > nI)
      ok = ok && !(dsub(index_estimate<VN_NR_G>(delta, ddiv(Pn, T)),
                        index_estimate<VN_NR_G>(delta, ic == 0 ? 0.0 : ddiv(Pi, T))) > 1.0);
    const uint64_t fail = __ballot(in && !ok);
    if (fail && lane == 0) lds_min(&B.ctl[3], (uint32_t)__builtin_ctzll(fail));
  }
  fast_sync<NW>();
  PROF_T(b8);
  ASM_MARK("H_BEGIN");
  uint32_t jd = __builtin_amdgcn_readfirstlane(B.ctl[0]);
  const uint32_t jst = __builtin_amdgcn_readfirstlane(B.ctl[3]);
  if (B.ctl[4]) jd = 0;  // (means out of order somewhere: no batch)
  const uint32_t js = min(jd, jst);
  const bool structural = jst <= jd || js == 0;
  if (js > 0) {
    // commit merges 0..js-1: each column's mean and weight after its last entry before js
    if (i < nm) {
      const uint32_t o = B.off[i];
      const uint32_t kq = js < b ? (uint32_t)B.kT[i * kRS + js] : B.off[i + 1] - o;
      uint32_t sl = 0xffu;
      if constexpr (kRepairs > 0) sl = B.rslot[i];
      if (sl != 0xffu && js > B.rfirst[sl]) {  // (F': a re-done column)
        L.mm[i] = B.rmean[sl * kBB + js - 1];
        L.mw[i] = dadd(L.mw[i], (double)B.rgain[sl * kBB + js - 1]);
      } else if (kq) {
        L.mm[i] = B.lv[o + kq - 1];
        L.mw[i] = dadd(L.mw[i], (double)B.lw[o + kq - 1]);
      }
    }
    mainW = B.bT[js - 1];
    fast_sync<NW>();
    if (wv == 0) prefix_main_w0(L, F, nm, mainW);
  }
  fast_sync<NW>();
  PROF_T(b9);
  ASM_MARK("MB_END");
  PROF_ADD(16, b0, b1);
  PROF_ADD(17, b1, b2);
  PROF_ADD(18, b2, b3);
  PROF_ADD(19, b3, b4);
  PROF_ADD(15, b4, b5);
  PROF_ADD(20, b5, b6);
  PROF_ADD(21, b6, b7);
  PROF_ADD(48, b7, b8);
  PROF_ADD(13, b8, b9);
  PROF_ADD(23, 0, 1);
  PROF_ADD(24, 0, (long long)js);
  PROF_ADD(25, 0, (long long)nflag);
  PROF_ADD(26, 0, (long long)b);
  PROF_ADD(22, 0, (long long)(structural ? 1 : 0));
  return BatchResult{js, structural};
}

#ifdef VN_REPLAY_CHECK
// Diagnostics build (VARIANT_FLAGS=-DVN_REPLAY_CHECK): the digest's invariants after every merge of
// the long replays -- 1 <= nm <= capc, the means in order, and (exact weights) the main weights
// summing to mainW in any order.  The first violation of a key is printed with where it happened
// and the key is abandoned (its state in HBM left as it was before the call), so a broken merge
// is named instead of feeding later merges.
template <int NW>
__device__ bool replay_check(const Lds L, const FastLds F, uint32_t nm, double mainW, uint32_t capc, bool fok,
                             uint32_t s, uint32_t c, int where, uint32_t a0, uint32_t a1) {
  constexpr uint32_t NT = 64 * NW;
  const uint32_t t = threadIdx.x, wv = t >> 6, lane = t & 63;
  if (t == 0) F.misc[6] = 0u;
  fast_sync<NW>();
  const uint32_t n = min(nm, capc);
  bool bad = nm == 0 || nm > capc;
  for (uint32_t j = t; j + 1 < n; j += NT)
    if (!(L.mm[j] <= L.mm[j + 1])) bad = true;
  if (bad) __atomic_fetch_or(&F.misc[6], 1u, __ATOMIC_RELAXED);
  if (wv == 0 && fok) {
    double acc = 0.0;
    for (uint32_t b = 0; b < n; b += 64) acc = dadd(acc, wave_sum(b + lane < n ? L.mw[b + lane] : 0.0));
    if (lane == 0 && acc != mainW) __atomic_fetch_or(&F.misc[6], 2u, __ATOMIC_RELAXED);
  }
  fast_sync<NW>();
  const uint32_t r = F.misc[6];
  fast_sync<NW>();
  if (r && t == 0)
    printf("VN_REPLAY_CHECK slot %u chunk %u where %d (%u, %u): flags %u nm %u mainW %.17g mm0 %.17g mw0 %.17g\n", s, c,
           where, a0, a1, r, nm, mainW, L.mm[0], L.mw[0]);
  return r != 0u;
}
#endif

// replay of one key with NW waves (tcap <= 64, ingest only: no flush-mode adoption); BATCH:
// merge_batch where the key's state allows (the dynamic LDS then holds the batch tables)
template <int NW, bool BATCH>
__device__ void replay_key_fast(const ExactCtx& x, const uint32_t k, MwSharedL& S, const uint32_t pos = 0xffffffffu) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr uint32_t NT = 64 * NW;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t capc = x.capc, tcap = x.tcap;
  const uint32_t TP = round64(tcap + 1);
  const Lds L = lds_layout(smem, capc, TP);
  const FastLds F = fast_layout(smem + fast_offset(capc, tcap), capc, TP, L.JW);

  const MergeParams mp{x.delta, x.capc, x.err};
  const uint64_t* const xA = x.A;
  const uint64_t* const xB = x.B;
  const double* const xcsv = x.csv;
  const double* const xcsw = x.csw;
  const double* const xctw = x.ctw;
  const double* const ximpw = x.impw;
  const uint32_t s = x.keys[k];
  const uint32_t nex = x.nex ? x.nex[k] : 0u;
  const bool final_merge = x.hot && x.hot[k];
  uint32_t np = x.hpend[s];
  if (nex == 0 && !(final_merge && np > 0)) return;

  const uint8_t cur = x.hcur[s];
  double* cmg = (cur ? x.cm1 : x.cm0) + (uint64_t)s * capc;
  double* cwg = (cur ? x.cw1 : x.cw0) + (uint64_t)s * capc;
  uint32_t nm = x.hncent[s];
  double* h = x.hst + (uint64_t)s * VN_HISTO_STATS;
  double mainW = h[7];
  const uint32_t lo = x.start[s];
  const ExactSplit sp = exact_split(np, nex, tcap);
  const double k0 = index_estimate(x.delta, 0.0);
  for (uint32_t j = t; j < nm; j += NT) {
    L.mm[j] = cmg[j];
    L.mw[j] = cwg[j];
  }
  const double* pv = x.hpv + (uint64_t)s * tcap;
  const double* pw = x.hpw + (uint64_t)s * tcap;
  for (uint32_t j = t; j < np; j += NT) {
    L.tv[j] = pv[j];
    L.tw[j] = pw[j];
  }
  fast_sync<NW>();
  if (wv == 0) prefix_main_w0(L, F, nm, mainW);
  fast_sync<NW>();
  bool fok = F.misc[1] != 0u;   // the main weights are exact: the fast merges apply
  bool fint = F.misc[4] != 0u;  // ... and integers (fast_total_limit)

  double sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf, dmn = kInf, dmx = -kInf;
  auto stat = [&](double v, double wt, bool sample) {
    dmn = min_go(dmn, v);
    dmx = max_go(dmx, v);
    if (!sample) return;
    sw = dadd(sw, wt);
    mn = min_go(mn, v);
    mx = max_go(mx, v);
    sxw = dadd(sxw, dmul(v, wt));
    srw = dadd(srw, dmul(ddiv(1.0, v), wt));
  };
  auto append = [&](uint32_t a, uint32_t b) {
    for (uint32_t i = a + t; i < b; i += NT) {
      const double v = bitsd(xA[lo + i]);
      const uint32_t tag = (uint32_t)xB[lo + i];
      const double wt = tag_weight(tag, ximpw);
      L.tv[np + (i - a)] = v;
      L.tw[np + (i - a)] = wt;
      stat(v, wt, tag_is_sample(tag));
    }
    np += b - a;
    fast_sync<NW>();
  };
  // a merge of the sorted temps sv/sw (with sp when tint): the fast merge when it applies, else
  // wave 0's one-wave merge (and the main prefix rebuilt after it)
  auto merge_sorted_any = [&](uint32_t n_, double tempW, bool tint, bool cint) {
    const MergeState r = merge_step<NW>(mp, L, F, S, MergeState{nm, mainW, fok, fint}, n_, tempW, tint, cint, k0);
    nm = r.nm;
    mainW = r.w;
    fok = r.fok;
    fint = r.fint;
  };
  // the pending temps (a call's first merge of a continuing key, a final or flush-ready merge):
  // wave 0 sorts them and merges them with the one-wave merge (Go's mergeAllTemps restated), then
  // rebuilds the main prefix.  (The four-wave fast merge out of line here, merge_step_cold, gave
  // wrong digests in continuing calls in some builds -- tools/probe/repro_batch3_calls.py, DESIGN.md
  // §4 -- while the same merge inlined for every chunk stayed exact: this merge, once per key and
  // call, takes the plain path.)
  auto merge_pend = [&]() {
    if (wv == 0) {
      const double tw_ = temp_weight(L.tw, np);
      sort_temps(L.tv, L.tw, L.sv, L.sw, np);
      const NmW r = merge_any_v(L, MP_ARGS(mp), nm, mainW, np, tw_);
      prefix_main_w0(L, F, r.nm, r.w);
      if (lane == 0) {
        S.fb_nm = r.nm;
        S.fb_w = r.w;
      }
    }
    fast_sync<NW>();
    nm = S.fb_nm;
    mainW = S.fb_w;
    fok = F.misc[1] != 0u;
    fint = F.misc[4] != 0u;
    fast_sync<NW>();  // (S and misc are read before anyone writes them again)
  };

  if (nex && np == tcap) {
    merge_pend();
    np = 0;
  }
  if (sp.off0) {
    append(0, sp.off0);
    if (np == tcap && sp.off0 < nex) {
      merge_pend();
      np = 0;
    }
  }
  if (sp.npure) {
    // the chunk sorter's arrays at the chunk's records: sorted means and signed weights (an
    // imported centroid negative), and in ctw the temps' Add-order weight sum at the first
    // record (negative when a weight is not an integer), their sorted exclusive prefix after it
    double cv = 0.0, cw = 0.0, cp = 0.0, ctw = 0.0;
    uint32_t ccpk = 0xffffffffu;  // the batched replay's packing of slot 0: not all-ones = integer weights
    auto load = [&](uint32_t c) {
      const uint64_t base = (uint64_t)lo + sp.off0 + (uint64_t)c * tcap;
      if (t < tcap) {
        cv = xcsv[base + t];
        cw = xcsw[base + t];
        cp = xctw[base + t];
      }
      ctw = xctw[base];
      ccpk = x.cpk ? x.cpk[base] : 0xffffffffu;
    };
    // chunks [c0, c1) one merge at a time, the next chunk's loads in flight during each merge
    auto singles = [&](uint32_t c0, uint32_t c1) -> bool {  // (false: VN_REPLAY_CHECK abandoned the key)
      load(c0);
      for (uint32_t c = c0; c < c1; c++) {
        // 0: some weight not exact; 1: exact; 2: exact and integers
        double tempW = __builtin_fabs(ctw), tintd = ctw >= 0.0 ? (ccpk != 0xffffffffu ? 2.0 : 1.0) : 0.0;
        if (t < tcap) {
          L.sv[t] = cv;
          L.sw[t] = __builtin_fabs(cw);
          F.sp[t] = t ? cp : 0.0;
          if (!BATCH) stat(cv, __builtin_fabs(cw), cw > 0.0);  // (batched: the prologue's)
        }
        if (t == tcap) F.sp[tcap] = tempW;
        hold2(tempW, tintd);
        hold_stats(sw, sxw, srw, mn, mx, dmn, dmx);
        if (c + 1 < c1) load(c + 1);
        fast_sync<NW>();
#ifdef VN_REPLAY_CHECK
        const uint32_t nm_was = nm;
#endif
        merge_sorted_any(tcap, tempW, tintd != 0.0, tintd == 2.0);
#ifdef VN_REPLAY_CHECK
        if (replay_check<NW>(L, F, nm, mainW, capc, fok, s, c, 1, nm_was, (uint32_t)tintd)) return false;
#endif
      }
      return true;
    };
    if constexpr (!BATCH) {
      if (!singles(0, sp.npure)) return;
    } else {
    const BatchLds Bt = batch_layout(smem + batch_offset(capc, tcap), tcap);
    const uint64_t cb = (uint64_t)lo + sp.off0;
    const double* const gv = xcsv + cb;
    const double* const gw = xcsw + cb;
    const uint32_t* const gp = x.cpk + cb;
    // the pure chunks' Local* statistics first, every thread streaming its share (off the merge
    // chain: the replay below adds none); the loads of four records in flight per thread
#ifndef VN_NO_PROLOGUE
    if (x.lstat && pos < kLongStatKeys) {
      // reduced beforehand over the whole GPU (k_exact_long_stats): slice t's partials into
      // thread t's accumulators, folded with the rest below
      if (t < kLongStatSlices) {
        const double* q = x.lstat + ((uint64_t)pos * kLongStatSlices + t) * 8;
        sw = dadd(sw, q[0]);
        sxw = dadd(sxw, q[1]);
        srw = dadd(srw, q[2]);
        mn = min_go(mn, q[3]);
        mx = max_go(mx, q[4]);
        dmn = min_go(dmn, q[5]);
        dmx = max_go(dmx, q[6]);
      }
    } else if (x.cstat) {
      // past the pre-reduced keys: the chunk sorter's per-chunk partials of this key, 64 B per
      // chunk instead of 16 B per sample
      for (uint64_t g = t; g < sp.npure; g += NT) {
        const double* q = x.cstat + ((uint64_t)x.coff[k] + g) * 8;
        sw = dadd(sw, q[0]);
        sxw = dadd(sxw, q[1]);
        srw = dadd(srw, q[2]);
        mn = min_go(mn, q[3]);
        mx = max_go(mx, q[4]);
        dmn = min_go(dmn, q[5]);
        dmx = max_go(dmx, q[6]);
      }
    } else {
      const uint64_t ne = (uint64_t)sp.npure * tcap;
      uint64_t e = t;
      for (; e + 3 * NT < ne; e += 4 * NT) {
        double v[4], w[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          v[u] = gv[e + u * NT];
          w[u] = gw[e + u * NT];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) stat(v[u], __builtin_fabs(w[u]), w[u] > 0.0);
      }
      for (; e < ne; e += NT) stat(gv[e], __builtin_fabs(gw[e]), gw[e] > 0.0);
    }
#endif
    // sin(pi kHi / delta), sin(pi kLo / delta): merge_batch's certain k tests (F)
    // (a short series: theta = pi k / delta is small, and the band dwarfs its error)
    auto sin_small = [](double th) {
      const double t2 = th * th;
      return th * (1.0 - t2 / 6.0 * (1.0 - t2 / 20.0 * (1.0 - t2 / 42.0 * (1.0 - t2 / 72.0))));
    };
    const double sin_hi = sin_small(kPi * (1.0 + kBand) / mp.delta), sin_lo = sin_small(kPi * (1.0 - kBand) / mp.delta);
#if VN_CHAIN_PRIO
    // the batched keys are the window's longest chains: their waves win instruction issue over
    // other kernels' waves sharing their SIMDs (windows in flight put such waves beside them)
    __builtin_amdgcn_s_setprio(VN_CHAIN_PRIO);
#endif
    uint32_t ring_lo = 0, ring_hi = 0;  // chunks [ring_lo, ring_hi) are in the ring (or on their way)
    uint32_t c = 0;
    while (c < sp.npure) {
      const uint32_t left = sp.npure - c;
      if (!(fok && nm >= 1 && nm <= kBM && left >= 2 && mainW >= kBatchMinW && tcap <= kBTmax && 8 * tcap >= kSR &&
            capc >= 192)) {
        // not (yet) batchable: a run of single merges, then look again
        const uint32_t c1 = min(sp.npure, c + kBatchBackoff);
        PROF_T(s3);
        if (!singles(c, c1)) {
          dma_wait();
          return;
        }
        PROF_T(s4);
        PROF_ADD(30, s3, s4);
        PROF_ADD(31, 0, (long long)(c1 - c));
        c = c1;
        continue;
      }
      if (c < ring_lo || c > ring_hi) ring_lo = ring_hi = c;  // (after a run of singles)
      dma_wait();  // everything issued so far has landed (this wave's share; the barrier: all)
      if (ring_hi - c < min(left, kBMinAvail)) {  // too few chunks at hand: fill the batch now
        const uint32_t e = min(sp.npure, c + kBB);
        ring_fill<NW>(Bt, gv, gp, ring_hi, e, tcap);
        ring_hi = e;
        dma_wait();
      }
      fast_sync<NW>();
      const uint32_t b = min(min(kBB, left), ring_hi - c);
      // the chunks after it, while it runs (their slots hold chunks < c)
      const uint32_t pe = min(c + kRing, sp.npure);
      if (pe > ring_hi) {
        ring_fill<NW>(Bt, gv, gp, ring_hi, pe, tcap);
        ring_hi = pe;
      }
      ring_lo = max(c, ring_hi > kRing ? ring_hi - kRing : 0u);
      PROF_T(s0);
#ifdef VN_REPLAY_CHECK
      const uint32_t nm_was = nm;
#endif
      const BatchResult r = merge_batch<NW>(mp.delta, sin_hi, sin_lo, L, F, Bt, nm, mainW, c, b, tcap, fint);
#ifdef VN_REPLAY_CHECK
      if (r.js && replay_check<NW>(L, F, nm, mainW, capc, fok, s, c, 2, r.js, b | (nm_was << 8))) {
        dma_wait();
        return;
      }
#endif
      PROF_T(s1);
      PROF_ADD(27, s0, s1);
      const uint32_t cb_end = c + b;  // (the batch's chunks: landed in the ring)
      c += r.js;
      if (r.js < b && r.structural) {  // that merge alone (after a batch that took nothing: a run)
        const uint32_t c1 = min(sp.npure, c + (r.js == 0 ? kBatchBackoff : 1u));
        // from the ring where the chunk is there and batchable (no global round trip: under a
        // busy memory system that latency would sit on the chain), else from the sorter's arrays
        uint32_t cs = c;
        for (; cs < c1 && cs < cb_end; cs++) {
          const uint32_t sb = (cs % kRing) * tcap;
          const uint32_t p0 = Bt.rp[sb];
          if (p0 == 0xffffffffu) break;
          if (t < tcap) {
            const uint32_t pk = Bt.rp[sb + t];
            L.sv[t] = Bt.rv[sb + t];
            L.sw[t] = (double)(pk & 0xffffu);
            F.sp[t] = t ? (double)(pk >> 16) : 0.0;
          }
          if (t == tcap) F.sp[tcap] = (double)(p0 >> 16);
          fast_sync<NW>();
#ifdef VN_REPLAY_CHECK
          const uint32_t nm_was2 = nm;
#endif
          merge_sorted_any(tcap, (double)(p0 >> 16), true, true);
#ifdef VN_REPLAY_CHECK
          if (replay_check<NW>(L, F, nm, mainW, capc, fok, s, cs, 3, nm_was2, 0u)) {
            dma_wait();
            return;
          }
#endif
        }
        if (cs < c1 && !singles(cs, c1)) {
          dma_wait();
          return;
        }
        PROF_T(s2);
        PROF_ADD(28, s1, s2);
        PROF_ADD(29, 0, (long long)(c1 - c));
        c = c1;
      }
    }
    dma_wait();  // (nothing may still be landing in LDS when the block moves on)
    }
  }
  const uint32_t tail = sp.off0 + sp.npure * tcap;
  if (nex > tail) append(tail, nex);
  if (final_merge && np > 0) {
    merge_pend();
    np = 0;
  }
  for (uint32_t j = t; j < nm; j += NT) {
    cmg[j] = L.mm[j];
    cwg[j] = L.mw[j];
  }
  double* qv = x.hpv + (uint64_t)s * tcap;
  double* qw = x.hpw + (uint64_t)s * tcap;
  for (uint32_t j = t; j < np; j += NT) {
    qv[j] = L.tv[j];
    qw[j] = L.tw[j];
  }
  // the statistics: each thread's partials folded over the wave, then the waves in order
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    sw = dadd(sw, __shfl_xor(sw, d, 64));
    sxw = dadd(sxw, __shfl_xor(sxw, d, 64));
    srw = dadd(srw, __shfl_xor(srw, d, 64));
    mn = min_go(mn, __shfl_xor(mn, d, 64));
    mx = max_go(mx, __shfl_xor(mx, d, 64));
    dmn = min_go(dmn, __shfl_xor(dmn, d, 64));
    dmx = max_go(dmx, __shfl_xor(dmx, d, 64));
  }
  if (lane == 0) {
    S.red[0][wv] = sw;
    S.red[1][wv] = sxw;
    S.red[2][wv] = srw;
    S.red[3][wv] = mn;
    S.red[4][wv] = mx;
    S.red[5][wv] = dmn;
    S.red[6][wv] = dmx;
  }
  fast_sync<NW>();
  if (t == 0) {
    for (int q = 1; q < NW; q++) {
      sw = dadd(sw, S.red[0][q]);
      sxw = dadd(sxw, S.red[1][q]);
      srw = dadd(srw, S.red[2][q]);
      mn = min_go(mn, S.red[3][q]);
      mx = max_go(mx, S.red[4][q]);
      dmn = min_go(dmn, S.red[5][q]);
      dmx = max_go(dmx, S.red[6][q]);
    }
    x.hncent[s] = nm;
    x.hpend[s] = np;
    h[7] = mainW;
    if (nex) {
      h[0] = dadd(h[0], sw);
      h[1] = min_go(h[1], mn);
      h[2] = max_go(h[2], mx);
      h[3] = dadd(h[3], sxw);
      h[4] = dadd(h[4], srw);
      h[5] = min_go(h[5], dmn);
      h[6] = max_go(h[6], dmx);
    }
  }
  fast_sync<NW>();
  if (x.hspn) {
    uint32_t fn = 0;
    if (x.spec && !final_merge && np > 0) {
      merge_pend();
      double* fmg = (cur ? x.cm0 : x.cm1) + (uint64_t)s * capc;
      double* fwg = (cur ? x.cw0 : x.cw1) + (uint64_t)s * capc;
      for (uint32_t j = t; j < nm; j += NT) {
        fmg[j] = L.mm[j];
        fwg[j] = L.mw[j];
      }
      fn = nm;
    }
    if (t == 0) {
      x.hspn[s] = fn;
      if (fn) x.hspw[s] = mainW;
    }
  }
}

// One wave per key: key index blockIdx.x, or the blockIdx.x-th of x.order / x.order64 (the
// latter longest first, so the longest replays do not start last).
template <int TPL>
__global__ __launch_bounds__(64) void k_histo_exact(ExactCtx x) {
  const uint32_t i = blockIdx.x;
  if (x.mw_count && i < *x.mw_count) return;  // replayed by k_histo_exact_mw
  const uint32_t k = x.order64 ? (uint32_t)x.order64[i] : x.order ? x.order[i] : i;
  if (k < x.nkeys) replay_key<TPL>(x, k);
}

// the long keys of the order, four waves each: entries [nmw[1], nmw[0]) (k_histo_exact_mw) and,
// batched with the larger LDS, the longest [0, nmw[1]) (k_histo_exact_mwb)
template <bool BATCH>
__device__ __forceinline__ void replay_long(const ExactCtx& x, const uint32_t* __restrict__ nmw, uint32_t first = 0,
                                            uint32_t last = 0xffffffffu) {
  __shared__ MwShared S;
  const uint32_t n = min(BATCH ? nmw[1] : nmw[0], last);
  for (uint32_t i = (BATCH ? first : nmw[1]) + blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t k = x.order64 ? (uint32_t)x.order64[i] : x.order ? x.order[i] : i;
    if (k < x.nkeys) replay_key_fast<kMW, BATCH>(x, k, *(MwSharedL*)&S, BATCH ? i : 0xffffffffu);
    __syncthreads();  // the next key reuses the LDS
  }
}
__global__ __launch_bounds__(kMWThreads) void k_histo_exact_mw(ExactCtx x, const uint32_t* __restrict__ nmw) {
  replay_long<false>(x, nmw);
}
#ifndef VN_CHAIN_EXCLUSIVE
#define VN_CHAIN_EXCLUSIVE 0  // (measured worse: 83.4 against 79.9 ms per C4 window)
#endif
__global__ __launch_bounds__(kMWThreads) void k_histo_exact_mwb(ExactCtx x, const uint32_t* __restrict__ nmw,
                                                                 uint32_t first, uint32_t last) {
#if VN_CHAIN_EXCLUSIVE
  // The batched replay is issue-bound at one wave per SIMD: a wave of another
  // kernel sharing its SIMD takes issue slots from the chain.  Claiming the whole register file
  // (the last accumulation register) leaves no room for one: the CU runs this workgroup alone.
  asm volatile("" ::: "a255");
#endif
  replay_long<true>(x, nmw, first, last);
}
// The Local* statistics of the batched keys' pure chunks (Histo.Sample, samplers.go:346-356:
// weight, min, max, sum(x w), sum(w / x) of the samples; min / max of every record for the
// digest), reduced over the whole GPU before their replays: block (slice, y) takes one of
// kLongStatSlices contiguous slices of entry y's pure chunks and writes its partials.  (Reduced
// inside the replay's own workgroup, this stream of a hot key's records -- hundreds of MB --
// ran at one CU's memory-level parallelism, on the key's critical path.)  Entries [y0, y1) of
// the longest-first order that are batched (< mw_count[1]).
__device__ __forceinline__ void long_stats_entry(const ExactCtx& x, const uint32_t y, double (&red)[7][4]) {
  const uint32_t k = (uint32_t)x.order64[y];
  double sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf, dmn = kInf, dmx = -kInf;
  if (k < x.nkeys) {
    const uint32_t s = x.keys[k];
    const ExactSplit sp = exact_split(x.hpend[s], x.nex[k], x.tcap);
    if (x.cstat) {  // the chunk sorter's per-chunk partials: 64 B per chunk instead of 16 B per sample
      const uint64_t g0 = x.coff[k], ng = sp.npure;
      const uint64_t per = (ng + kLongStatSlices - 1) / kLongStatSlices;
      const uint64_t a = min(ng, per * blockIdx.x), b = min(ng, a + per);
      for (uint64_t g = a + threadIdx.x; g < b; g += 256) {
        const double* q = x.cstat + (g0 + g) * 8;
        sw = dadd(sw, q[0]);
        sxw = dadd(sxw, q[1]);
        srw = dadd(srw, q[2]);
        mn = min_go(mn, q[3]);
        mx = max_go(mx, q[4]);
        dmn = min_go(dmn, q[5]);
        dmx = max_go(dmx, q[6]);
      }
    }
    const uint64_t base = (uint64_t)x.start[s] + sp.off0, ne = x.cstat ? 0ull : (uint64_t)sp.npure * x.tcap;
    const uint64_t per = (ne + kLongStatSlices - 1) / kLongStatSlices;
    const uint64_t a = min(ne, per * blockIdx.x), b = min(ne, a + per);
    for (uint64_t e = a + threadIdx.x; e < b; e += 256) {
      const double v = x.csv[base + e], w = x.csw[base + e], wt = __builtin_fabs(w);
      dmn = min_go(dmn, v);
      dmx = max_go(dmx, v);
      if (w > 0.0) {  // (an imported centroid: negative, the digest's min / max only)
        sw = dadd(sw, wt);
        mn = min_go(mn, v);
        mx = max_go(mx, v);
        sxw = dadd(sxw, dmul(v, wt));
        srw = dadd(srw, dmul(ddiv(1.0, v), wt));
      }
    }
  }
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    sw = dadd(sw, __shfl_xor(sw, d, 64));
    sxw = dadd(sxw, __shfl_xor(sxw, d, 64));
    srw = dadd(srw, __shfl_xor(srw, d, 64));
    mn = min_go(mn, __shfl_xor(mn, d, 64));
    mx = max_go(mx, __shfl_xor(mx, d, 64));
    dmn = min_go(dmn, __shfl_xor(dmn, d, 64));
    dmx = max_go(dmx, __shfl_xor(dmx, d, 64));
  }
  if (lane == 0) {
    red[0][wv] = sw;
    red[1][wv] = sxw;
    red[2][wv] = srw;
    red[3][wv] = mn;
    red[4][wv] = mx;
    red[5][wv] = dmn;
    red[6][wv] = dmx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; q++) {
      sw = dadd(sw, red[0][q]);
      sxw = dadd(sxw, red[1][q]);
      srw = dadd(srw, red[2][q]);
      mn = min_go(mn, red[3][q]);
      mx = max_go(mx, red[4][q]);
      dmn = min_go(dmn, red[5][q]);
      dmx = max_go(dmx, red[6][q]);
    }
    double* o = x.lstat + ((uint64_t)y * kLongStatSlices + blockIdx.x) * 8;
    o[0] = sw;
    o[1] = sxw;
    o[2] = srw;
    o[3] = mn;
    o[4] = mx;
    o[5] = dmn;
    o[6] = dmx;
  }
  __syncthreads();  // (red is reused by the next entry)
}
__global__ __launch_bounds__(256) void k_exact_long_stats(ExactCtx x, uint32_t y0, uint32_t y1) {
  __shared__ double red[7][4];
  const uint32_t yn = min(y1, min(x.mw_count[1], kLongStatKeys));
  for (uint32_t y = y0 + blockIdx.y; y < yn; y += gridDim.y) long_stats_entry(x, y, red);
}

// how many entries of the longest-first order replay at least min_len samples (out[0]), and at
// least batch_len (out[1], <= out[0])
__global__ void k_exact_count_long(uint32_t n, const uint64_t* __restrict__ order64, uint32_t min_len,
                                   uint32_t batch_len, uint32_t cap, uint32_t* __restrict__ out) {
  for (int q = 0; q < 2; q++) {
    const uint32_t len = q ? max(batch_len, min_len) : min_len;
    uint32_t lo = 0, hi = n;  // first entry shorter than len
    while (lo < hi) {
      const uint32_t md = (lo + hi) >> 1;
      if (0xFFFFFFFu - (uint32_t)(order64[md] >> 32) >= len) lo = md + 1;
      else hi = md;
    }
    out[q] = min(lo, cap);
  }
}

// keys [0, *cnt) of x.keys, grid-stride: a bounded grid when only the device knows the count
template <int TPL>
__global__ __launch_bounds__(64) void k_histo_exact_list(ExactCtx x, const uint32_t* __restrict__ cnt) {
  const uint32_t n = *cnt;
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) replay_key<TPL>(x, k);
}

void histo_exact_replay_list(const ExactCtx& x, const uint32_t* dev_count, uint32_t max_keys, hipStream_t st) {
  if (!max_keys) return;
  if (x.tcap > 64 * kMaxTempPerLane) throw std::runtime_error("temp buffer larger than the exact kernel supports");
  const size_t sm = exact_smem_bytes(x.capc, x.tcap);
  if (sm > 160 * 1024) throw std::runtime_error("compression too large for the exact replay's LDS budget");
  const uint32_t grid = std::min<uint32_t>(max_keys, 4096);
  if (x.tcap <= 64) hipLaunchKernelGGL(k_histo_exact_list<1>, dim3(grid), dim3(64), sm, st, x, dev_count);
  else hipLaunchKernelGGL(k_histo_exact_list<kMaxTempPerLane>, dim3(grid), dim3(64), sm, st, x, dev_count);
}

// longest-first order of the listed keys: (0xFFFFFFF - min(nex, 0xFFFFFFF)) << 32 | key index
// (28 bits of length: a window's hot keys hold millions of samples, and the longest must start first)
__global__ void k_exact_lpt_keys(uint32_t n, const uint32_t* __restrict__ list, const uint32_t* __restrict__ nex,
                                 uint64_t* __restrict__ out, const uint32_t* __restrict__ n_dev) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (n_dev && i >= *n_dev) {  // length 0 (sorted last), no key
    out[i] = (uint64_t)0xFFFFFFFu << 32 | 0xFFFFFFFFu;
    return;
  }
  const uint32_t k = list[i], c = min(nex[k], 0xFFFFFFFu);
  out[i] = ((uint64_t)(0xFFFFFFFu - c) << 32) | k;
}

void histo_exact_order(ExactCtx& x, const uint32_t* list, uint32_t n, uint64_t* buf0, uint64_t* buf1,
                       RadixScratch& rs, hipStream_t st, const uint32_t* n_dev) {
  x.order = list;
  x.norder = n;
  if (!n) return;
  hipLaunchKernelGGL(k_exact_lpt_keys, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, list, x.nex, buf0, n_dev);
  RadixPass passes[4];
  const int np = make_passes(passes, false, 32, 28);
  x.order64 = radix_sort(buf0, nullptr, buf1, nullptr, n, passes, np, rs, st, nullptr) ? buf1 : buf0;
}

size_t exact_smem_bytes(uint32_t capc, uint32_t tcap) { return exact_smem_bytes_hd(capc, tcap); }
size_t exact_fast_smem_bytes(uint32_t capc, uint32_t tcap) {
  const uint32_t TP = (tcap + 1 + 63u) & ~63u, JW = std::max(capc + TP + 1, 320u);
  return fast_offset(capc, tcap) + fast_extra_bytes(capc, TP, JW);
}
static size_t exact_batch_smem_bytes(uint32_t capc, uint32_t tcap) {
  return batch_offset(capc, tcap) + batch_bytes(tcap);
}
#ifdef VN_EXACT_PROF
extern "C" int vn_prof_exact_read(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_exact_prof), sizeof(unsigned long long) * 64) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[64] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_exact_prof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

void histo_exact_chunk_plan(const ExactCtx& x, hipStream_t st, ScanScratch* ss, uint64_t max_chunks) {
  if (!x.nkeys || !x.nex) return;
  hipLaunchKernelGGL(k_exact_chunk_count, dim3(blocks_for(x.nkeys, 256)), dim3(256), 0, st, x);
  scan_exclusive_u32(x.ccnt, x.coff, x.nkeys, *ss, st);
  if (x.cown && max_chunks)
    hipLaunchKernelGGL(k_exact_chunk_owner, dim3(blocks_for(max_chunks, 256)), dim3(256), 0, st, x);
}

void histo_exact_chunk_sort(const ExactCtx& x, hipStream_t st, uint64_t max_chunks, uint32_t top, bool top_only) {
  if (!x.nkeys || !x.nex || !max_chunks) return;
  const size_t sm = sizeof(double) * 4 * ((x.tcap + 1 + 63u) & ~63u);
  if (top && (!x.order64 || top > x.norder || top > kTopExcl)) throw std::logic_error("chunk sort: bad top keys");
  if (top_only) {
    if (top) hipLaunchKernelGGL(k_exact_chunk_sort_top, dim3(kTopSortBlocks, top), dim3(64), sm, st, x);
    return;
  }
  const uint64_t span = VN_CHUNK_XCD ? 8ull * VN_CHUNK_XCD : 1ull;
  const uint64_t waves = (max_chunks + kChunksPerWave - 1) / kChunksPerWave;
  hipLaunchKernelGGL(k_exact_chunk_sort, dim3((uint32_t)((waves + span - 1) / span * span)), dim3(64), sm, st, x, top);
}

uint32_t histo_exact_top_keys(const ExactCtx& x) {
  const bool batch = x.cpk && x.tcap <= kBTmax && exact_batch_smem_bytes(x.capc, x.tcap) <= 160 * 1024;
  return x.mw_count && batch ? std::min<uint32_t>(kTopExcl, x.norder) : 0u;
}

void histo_exact_presort(const ExactCtx& x, hipStream_t st, ScanScratch* ss, uint64_t max_chunks) {
  // sort every pure chunk in parallel first
  histo_exact_chunk_plan(x, st, ss, max_chunks);
  histo_exact_chunk_sort(x, st, max_chunks, 0, false);
}

bool histo_exact_count_long(ExactCtx& x, uint32_t min_len, uint32_t* count, hipStream_t st) {
  x.mw_count = nullptr;
  if (!x.order64 || !x.norder || x.tcap > 64 || x.flush_mode) return false;
  if (exact_fast_smem_bytes(x.capc, x.tcap) > 160 * 1024) return false;
  // (no batching where its tables do not fit: the long keys all take k_histo_exact_mw)
  const bool batch = x.cpk && x.tcap <= kBTmax && exact_batch_smem_bytes(x.capc, x.tcap) <= 160 * 1024;
  hipLaunchKernelGGL(k_exact_count_long, dim3(1), dim3(1), 0, st, x.norder, x.order64, min_len,
                     batch ? kBatchMinLen : 0xFFFFFFFFu, std::min<uint32_t>(x.norder, kMaxLongKeys), count);
  x.mw_count = count;
  return true;
}

void histo_exact_replay_top(const ExactCtx& x, hipStream_t st_top, uint32_t top) {
  if (!top) return;
  const size_t sm = exact_batch_smem_bytes(x.capc, x.tcap);
  if (x.lstat) hipLaunchKernelGGL(k_exact_long_stats, dim3(kLongStatSlices, top), dim3(256), 0, st_top, x, 0u, top);
  hipLaunchKernelGGL(k_histo_exact_mwb, dim3(top), dim3(kMWThreads), sm, st_top, x, x.mw_count, 0u, top);
}

void histo_exact_replay_long(const ExactCtx& x, hipStream_t st, hipStream_t st_rest, hipStream_t st_top,
                             uint32_t top_done) {
  if (!x.mw_count) return;
  const uint32_t grid = std::min<uint32_t>(x.norder, kMaxLongKeys / 2);
  if (x.cpk && x.tcap <= kBTmax && exact_batch_smem_bytes(x.capc, x.tcap) <= 160 * 1024) {
    const size_t sm = exact_batch_smem_bytes(x.capc, x.tcap);
    const uint32_t top = top_done ? top_done : st_top ? std::min<uint32_t>(kTopExcl, x.norder) : 0u;
    const uint32_t nl = std::min<uint32_t>(x.norder, kLongStatKeys);
    if (top && !top_done) {
      if (x.lstat)
        hipLaunchKernelGGL(k_exact_long_stats, dim3(kLongStatSlices, top), dim3(256), 0, st_top, x, 0u, top);
      hipLaunchKernelGGL(k_histo_exact_mwb, dim3(top), dim3(kMWThreads), sm, st_top, x, x.mw_count, 0u, top);
    }
    if (x.lstat && nl > top)
      hipLaunchKernelGGL(k_exact_long_stats, dim3(kLongStatSlices, std::min<uint32_t>(nl - top, 32u)), dim3(256), 0,
                         st, x, top, nl);
    hipLaunchKernelGGL(k_histo_exact_mwb, dim3(grid), dim3(kMWThreads), sm, st, x, x.mw_count, top, 0xffffffffu);
  }
  hipLaunchKernelGGL(k_histo_exact_mw, dim3(grid), dim3(kMWThreads), exact_fast_smem_bytes(x.capc, x.tcap), st_rest, x,
                     x.mw_count);
}

void histo_exact_replay(const ExactCtx& x, hipStream_t st) {
  const uint32_t grid = (x.order || x.order64) ? x.norder : x.nkeys;
  if (!grid) return;
  if (x.tcap > 64 * kMaxTempPerLane) throw std::runtime_error("temp buffer larger than the exact kernel supports");
  size_t sm = exact_smem_bytes(x.capc, x.tcap);
  if (sm > 160 * 1024) throw std::runtime_error("compression too large for the exact replay's LDS budget");
  if (x.tcap <= 64) hipLaunchKernelGGL(k_histo_exact<1>, dim3(grid), dim3(64), sm, st, x);
  else hipLaunchKernelGGL(k_histo_exact<kMaxTempPerLane>, dim3(grid), dim3(64), sm, st, x);
}

void launch_histo_exact(const ExactCtx& x, hipStream_t st, ScanScratch* ss, uint64_t max_chunks) {
  if (!x.nkeys) return;
  if (x.tcap > 64 * kMaxTempPerLane) throw std::runtime_error("temp buffer larger than the exact kernel supports");
  histo_exact_presort(x, st, ss, max_chunks);
  histo_exact_replay(x, st);
}

}  // namespace vn

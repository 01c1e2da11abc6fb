// ingest_histo.hip -- Histo.Sample + MergingDigest for one ingest batch.
//
// Reference semantics (tdigest/merging_digest.go): samples are Add()ed to a temp list;
// mergeAllTemps (121-205) sorts the temps and two-way merges them with the main
// centroids by mean, feeding every element to mergeOne (210-236), which starts a new
// centroid when  k(W_incl/T) - k(W_start/T) > 1,  k(q) = delta*(asin(2q-1)/pi + 0.5),
// and otherwise folds the element into the last centroid with Welford's update.
//
// MI355X formulation, per batch:
//   1. records -> (ordered(value), slot<<32 | tag) pairs; the key's existing centroids are
//      appended as elements tagged with their centroid index (they are merged exactly like
//      temps are merged with main in the reference);
//   2. stable LSD radix sort by (slot, value)  -> one contiguous, value-sorted segment per key;
//   3. per 1024-element chunk: weights, local inclusive prefix, Histo local statistics;
//   4. per segment: chunk prefix (exact for veneur's integer weights), totals;
//   5. per element: k = indexEstimate(W_incl / T);
//   6. per segment: the greedy centroid chain -- each next start is the first element whose
//      k exceeds the current start's k(W_excl/T) by more than 1 (one wave walks the
//      monotone k array as it streams through LDS);
//   7. centroid sums: one-chunk segments run the reference's Welford update per centroid
//      (thread per centroid); larger segments reduce sum(x*w), sum(w) per centroid.
// The greedy boundary rule is the reference's; the batch (rather than 42-sample chunks)
// is the merge unit, which is why t-digest parity is judged by rank error.
#include "histo.h"

namespace vn {

[[maybe_unused]] constexpr uint32_t kMaxCent = 2048;  // supports compression <= ~1000

struct HistoCtx {
  uint32_t ntouched;         // grid bound on segments
  const uint32_t* count;     // device count of live segments (<= ntouched); null: all
  uint32_t capc;
  double delta;
  const uint32_t* tl;
  const uint32_t* start;
  const uint32_t* end;
  const uint32_t* chb;
  const uint64_t* A;
  const uint64_t* B;
  const double* impw;        // weights of imported centroids (kTagImport)
  double* w;
  double* wk;
  double* ch_sum;
  double* ch_pre;
  double* ch_stats;
  double* seg_T;
  uint32_t* starts;
  uint32_t* nc_new;
  double* acc_xw;
  double* acc_w;
  double* hst;
  uint32_t* hncent;
  uint8_t* hcur;
  uint32_t* hspn;  // cleared when the hot path rewrites a key (its flush-ready digest is stale)
  double* cm0;
  double* cm1;
  double* cw0;
  double* cw1;
  uint32_t* err;
};

// segment [start, end) of every slot present in a sorted (slot<<32 | x) array
// bt / touch (may be null): the key-grouping sort marks each key batch-touched and
// window-touched here, once per key, rather than once per record before the sort
// Each record's key is loaded once: the neighbours' come from the adjacent lanes (the wave's
// first and last lanes load the one key beyond the wave).
__global__ void k_seg_mark(uint64_t n, const uint64_t* __restrict__ B, uint32_t* __restrict__ start,
                           uint32_t* __restrict__ end, uint32_t* __restrict__ bt, uint32_t* __restrict__ touch) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t s = i < n ? (uint32_t)(B[i] >> 32) : 0xFFFFFFFFu;
  uint32_t prev = __shfl_up(s, 1, 64), next = __shfl_down(s, 1, 64);
  if (lane == 0 && i > 0 && i < n) prev = (uint32_t)(B[i - 1] >> 32);
  if (lane == 63 && i + 1 < n) next = (uint32_t)(B[i + 1] >> 32);
  if (i >= n) return;
  if (i == 0 || prev != s) {
    start[s] = (uint32_t)i;
    if (bt) {
      bt[s] = 1;
      touch[s] = 1;
    }
  }
  if (i == n - 1 || next != s) end[s] = (uint32_t)(i + 1);
}

#if VN_FAST_MODE  // (the opt-in fast mode's segment compression: VARIANT_FLAGS=-DVN_FAST_MODE=1)
__device__ __forceinline__ uint32_t find_seg(const uint32_t* chb, uint32_t ntouched, uint32_t c) {
  uint32_t lo = 0, hi = ntouched;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (chb[mid] <= c) lo = mid;
    else hi = mid;
  }
  return lo;
}

struct ChunkRange {
  uint32_t k, s, seg_lo, seg_hi, lo, hi, nch;
};
__device__ __forceinline__ bool chunk_range(const HistoCtx& x, ChunkRange& r, uint32_t* s_k) {
  uint32_t c = blockIdx.x;
  if (c >= x.chb[x.ntouched]) return false;
  if (threadIdx.x == 0) *s_k = find_seg(x.chb, x.ntouched, c);
  __syncthreads();
  r.k = *s_k;
  r.s = x.tl[r.k];
  r.seg_lo = x.start[r.s];
  r.seg_hi = x.end[r.s];
  r.lo = r.seg_lo + (c - x.chb[r.k]) * kHTile;
  r.hi = min(r.seg_hi, r.lo + kHTile);
  r.nch = x.chb[r.k + 1] - x.chb[r.k];
  return true;
}

// 3. weights, local inclusive prefix, local statistics of the samples
__global__ __launch_bounds__(kBlock) void k_chunk_prep(HistoCtx x) {
  __shared__ uint32_t s_k;
  __shared__ double s_tmp[4];
  ChunkRange r;
  if (!chunk_range(x, r, &s_k)) return;
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  const double* cwo = x.hcur[r.s] ? x.cw1 : x.cw0;
  double wv[kHItems];
  double run = 0.0, sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf, dmn = kInf, dmx = -kInf;
  const uint32_t base = r.lo + t * kHItems;
#pragma unroll
  for (int j = 0; j < (int)kHItems; j++) {
    uint32_t i = base + j;
    wv[j] = 0.0;
    if (i < r.hi) {
      uint64_t b = x.B[i];
      uint32_t tag = (uint32_t)b;
      double xv = from_ordered_bits(x.A[i]);
      double wt;
      if (tag & kTagCentroid) {
        wt = cwo[tag & 0x7fffffffu];
      } else {
        wt = tag_weight(tag, x.impw);
        dmn = min_go(dmn, xv);
        dmx = max_go(dmx, xv);
        if (tag_is_sample(tag)) {
          sw = dadd(sw, wt);
          mn = min_go(mn, xv);
          mx = max_go(mx, xv);
          sxw = dadd(sxw, dmul(xv, wt));
          srw = dadd(srw, dmul(ddiv(1.0, xv), wt));
        }
      }
      wv[j] = wt;
      run = dadd(run, wt);
      x.w[i] = wt;
    }
  }
  double tot;
  double acc = block_excl_scan_d(run, s_tmp, tot);
#pragma unroll
  for (int j = 0; j < (int)kHItems; j++) {
    uint32_t i = base + j;
    if (i < r.hi) {
      acc = dadd(acc, wv[j]);
      x.wk[i] = acc;
    }
  }
  sw = block_allreduce(sw, s_tmp, SumOp());
  sxw = block_allreduce(sxw, s_tmp, SumOp());
  srw = block_allreduce(srw, s_tmp, SumOp());
  mn = block_allreduce(mn, s_tmp, MinGoOp());
  mx = block_allreduce(mx, s_tmp, MaxGoOp());
  dmn = block_allreduce(dmn, s_tmp, MinGoOp());
  dmx = block_allreduce(dmx, s_tmp, MaxGoOp());
  if (t == 0) {
    x.ch_sum[c] = tot;
    double* st = x.ch_stats + (uint64_t)c * kChunkStats;
    st[0] = sw; st[1] = mn; st[2] = mx; st[3] = sxw; st[4] = srw; st[5] = dmn; st[6] = dmx;
  }
}

// 4. per segment: chunk prefix, totals, Histo local statistics into the state
__global__ __launch_bounds__(kBlock) void k_seg_scan(HistoCtx x) {
  __shared__ double s_tmp[4];
  const uint32_t k = blockIdx.x, t = threadIdx.x;
  if (x.count && k >= *x.count) return;
  const uint32_t s = x.tl[k];
  const uint32_t cb = x.chb[k], ce = x.chb[k + 1];
  double carry = 0.0, sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf, dmn = kInf, dmx = -kInf;
  for (uint32_t base = cb; base < ce; base += kBlock) {
    uint32_t c = base + t;
    double v = c < ce ? x.ch_sum[c] : 0.0;
    double tot;
    double ex = block_excl_scan_d(v, s_tmp, tot);
    if (c < ce) {
      x.ch_pre[c] = dadd(carry, ex);
      const double* st = x.ch_stats + (uint64_t)c * kChunkStats;
      sw = dadd(sw, st[0]);
      mn = min_go(mn, st[1]);
      mx = max_go(mx, st[2]);
      sxw = dadd(sxw, st[3]);
      srw = dadd(srw, st[4]);
      dmn = min_go(dmn, st[5]);
      dmx = max_go(dmx, st[6]);
    }
    carry = dadd(carry, tot);
  }
  sw = block_allreduce(sw, s_tmp, SumOp());
  sxw = block_allreduce(sxw, s_tmp, SumOp());
  srw = block_allreduce(srw, s_tmp, SumOp());
  mn = block_allreduce(mn, s_tmp, MinGoOp());
  mx = block_allreduce(mx, s_tmp, MaxGoOp());
  dmn = block_allreduce(dmn, s_tmp, MinGoOp());
  dmx = block_allreduce(dmx, s_tmp, MaxGoOp());
  if (t == 0) {
    double* h = x.hst + (uint64_t)s * VN_HISTO_STATS;
    h[0] = dadd(h[0], sw);
    h[1] = min_go(h[1], mn);
    h[2] = max_go(h[2], mx);
    h[3] = dadd(h[3], sxw);
    h[4] = dadd(h[4], srw);
    h[5] = min_go(h[5], dmn);
    h[6] = max_go(h[6], dmx);
    h[7] = carry;
    x.seg_T[k] = carry;
  }
}

// 5. k-index of every element
__global__ __launch_bounds__(kBlock) void k_chunk_kin(HistoCtx x) {
  __shared__ uint32_t s_k;
  ChunkRange r;
  if (!chunk_range(x, r, &s_k)) return;
  const uint32_t c = blockIdx.x;
  const double pre = x.ch_pre[c];
  const double T = x.seg_T[r.k];
  for (uint32_t i = r.lo + threadIdx.x; i < r.hi; i += kBlock) {
    double W = dadd(pre, x.wk[i]);
    x.wk[i] = index_estimate(x.delta, ddiv(W, T));
  }
}

// 6. Greedy centroid chain of mergeOne, one workgroup per segment.  The walk moves forward
// through the segment's k array, so the array streams through an LDS ring of windows of kCW
// elements: waves 1..3 load windows (each keeps two in flight in registers) and publish them
// into ring slots; wave 0 walks.  Each step finds the next start = the first element j > pos
// with k_j - k_{pos-1} > 1 (k monotone) by one probe of the window's 64-element group-last
// values and one probe of that group, both LDS reads; the new base k_{next-1} is a lane of the
// probed group or the previous group's (window's) last k.  Loader/walker hand-offs are LDS
// flags (workgroup scope) with bounded spins: a stalled protocol flags an error, never hangs.
constexpr uint32_t kCW = 2048;        // elements per window
constexpr uint32_t kCWL = kCW / 64;   // window elements per lane (registers) = groups per window
constexpr uint32_t kRing = 6;         // LDS ring slots (96 KiB)
constexpr uint32_t kLoaders = 7;      // one CU streams the k array: 7 loader waves x 2 windows in flight
constexpr uint32_t kChainThreads = 64 * (kLoaders + 1);
constexpr uint32_t kSpinCap = 1u << 24;

__device__ __forceinline__ double readlane_d(double v, uint32_t i) {  // i wave-uniform
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, i), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), i);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ __launch_bounds__(kChainThreads) void k_chain(HistoCtx x) {
  __shared__ double s_win[kRing][kCW];
  __shared__ double s_last[kRing][kCWL];
  __shared__ uint32_t s_st[kMaxCent + 1];
  __shared__ uint32_t s_ready[kRing];  // window id + 1 published in the slot
  __shared__ uint32_t s_done;          // windows [0, s_done) released by the walker
  __shared__ uint32_t s_nc;
  const uint32_t k = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (x.count && k >= *x.count) return;
  const uint32_t s = x.tl[k];
  const uint32_t lo = x.start[s], n = x.end[s] - lo;
  const uint32_t nch = x.chb[k + 1] - x.chb[k];
  const double* kin = x.wk + lo;
  const uint32_t capc = x.capc;
  const uint32_t nw = (n + kCW - 1) / kCW;
  if (t < kRing) s_ready[t] = 0;
  if (t == 0) s_done = 0;
  __syncthreads();

  if (wave != 0) {
    // ---- loader: windows w = wave-1, wave-1+3, ...; two in flight in registers
    double ra[kCWL], rb[kCWL];
    auto fetch = [&](double* r, uint32_t w) {
      const uint32_t b = w * kCW;
#pragma unroll
      for (uint32_t j = 0; j < kCWL; j++) {
        const uint32_t i = b + 64 * j + lane;
        r[j] = i < n ? kin[i] : kInf;
      }
    };
    auto publish = [&](const double* r, uint32_t w) -> bool {
      uint32_t spins = 0;
      while (w >= lds_ld(&s_done) + kRing) {  // slot still holds a window the walker needs
        if (++spins > kSpinCap) return false;
        __builtin_amdgcn_s_sleep(1);
      }
      double* bw = s_win[w % kRing];
#pragma unroll
      for (uint32_t j = 0; j < kCWL; j++) bw[64 * j + lane] = r[j];
      wave_lds_sync();
      if (lane < kCWL) s_last[w % kRing][lane] = bw[64 * lane + 63];
      wave_lds_sync();
      if (lane == 0) lds_st(&s_ready[w % kRing], w + 1);
      return true;
    };
    uint32_t w = wave - 1;
    if (w < nw) fetch(ra, w);
    if (w + kLoaders < nw) fetch(rb, w + kLoaders);
    for (; w < nw; w += 2 * kLoaders) {
      if (!publish(ra, w)) break;
      if (w + 2 * kLoaders < nw) fetch(ra, w + 2 * kLoaders);
      if (w + kLoaders >= nw) break;
      if (!publish(rb, w + kLoaders)) break;
      if (w + 3 * kLoaders < nw) fetch(rb, w + 3 * kLoaders);
    }
  } else {
    // ---- walker
    bool ok = true;
    auto acquire = [&](uint32_t w) {
      uint32_t spins = 0;
      while (lds_ld(&s_ready[w % kRing]) != w + 1) {
        if (++spins > kSpinCap) {
          ok = false;
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    };
    uint32_t cw = 0;          // window the walk is in
    double prev_last = 0.0;   // last k of window cw - 1
    acquire(0);
    // the window's group-last k values stay in a register (lane q < kCWL holds group q), so a
    // step costs one LDS probe (the group) plus ballots and readlanes
    double gl = s_last[0][lane < kCWL ? lane : 0];
    uint32_t nc = 0, pos = 0;
    double base = index_estimate(x.delta, 0.0);
    while (ok) {
      if (nc >= capc) {
        if (lane == 0) atomicOr(x.err, 1u);
        break;
      }
      if (lane == 0) s_st[nc] = pos;
      nc++;
      uint32_t from = pos + 1;
      if (from >= n) break;
      bool found = false;
      for (;;) {
        while (from >= (cw + 1) * kCW) {  // the start lies in a later window
          prev_last = readlane_d(gl, kCWL - 1);
          cw++;
          if (lane == 0) lds_st(&s_done, cw);  // release the window left behind
          acquire(cw);
          if (!ok) break;
          gl = s_last[cw % kRing][lane < kCWL ? lane : 0];
        }
        if (!ok) break;
        const uint32_t slot = cw % kRing;
        const uint32_t wb = cw * kCW, q0 = (from - wb) >> 6;
        const uint64_t mq = __ballot(lane >= q0 && lane < kCWL && dsub(gl, base) > 1.0);
        if (mq == 0) {
          if (wb + kCW >= n) break;  // no later element qualifies: the chain ends
          from = wb + kCW;
          continue;
        }
        const uint32_t q = (uint32_t)__ffsll((unsigned long long)mq) - 1;
        const uint32_t idx = wb + 64 * q + lane;
        const double kv = s_win[slot][64 * q + lane];
        const uint64_t m = __ballot(idx >= from && idx < n && dsub(kv, base) > 1.0);
        if (m == 0) break;  // only padding past n qualified: the chain ends
        const uint32_t f = (uint32_t)__ffsll((unsigned long long)m) - 1;
        base = f ? readlane_d(kv, f - 1) : (q ? readlane_d(gl, q - 1) : prev_last);
        pos = wb + 64 * q + f;
        found = true;
        break;
      }
      if (!found) break;
    }
    if (!ok && lane == 0) atomicOr(x.err, 4u);
    if (lane == 0) {
      s_st[nc] = n;
      s_nc = nc;
      lds_st(&s_done, nw + kRing);  // release everything: loaders still waiting finish
    }
  }
  __syncthreads();
  const uint32_t nc = s_nc;
  if (nch == 1) {
    // Welford per centroid, in element order, exactly as mergeOne does
    const uint8_t nb = x.hcur[s] ^ 1;
    double* cm = nb ? x.cm1 : x.cm0;
    double* cwn = nb ? x.cw1 : x.cw0;
    for (uint32_t ci = t; ci < nc; ci += kChainThreads) {
      uint32_t a = s_st[ci], b = s_st[ci + 1];
      double mean = from_ordered_bits(x.A[lo + a]);
      double W = x.w[lo + a];
      for (uint32_t j = a + 1; j < b; j++) {
        double xv = from_ordered_bits(x.A[lo + j]);
        double wt = x.w[lo + j];
        W = dadd(W, wt);
        mean = dadd(mean, ddiv(dmul(dsub(xv, mean), wt), W));
      }
      cm[(uint64_t)s * capc + ci] = mean;
      cwn[(uint64_t)s * capc + ci] = W;
    }
    __syncthreads();
    if (t == 0) {
      x.hncent[s] = nc;
      x.hcur[s] = nb;
      x.hspn[s] = 0;
      x.nc_new[k] = nc;
    }
    return;
  }
  for (uint32_t ci = t; ci < nc; ci += kChainThreads) {
    x.starts[(uint64_t)k * capc + ci] = s_st[ci];
    x.acc_xw[(uint64_t)k * capc + ci] = 0.0;
    x.acc_w[(uint64_t)k * capc + ci] = 0.0;
  }
  if (t == 0) x.nc_new[k] = nc;
}

// 7. centroid sums of multi-chunk segments
__global__ __launch_bounds__(kBlock) void k_chunk_cent(HistoCtx x) {
  __shared__ uint32_t s_k;
  __shared__ uint32_t s_st[kMaxCent + 1];
  __shared__ double s_xw[kMaxCent];
  __shared__ double s_w[kMaxCent];
  ChunkRange r;
  if (!chunk_range(x, r, &s_k)) return;
  if (r.nch == 1) return;
  const uint32_t t = threadIdx.x, capc = x.capc;
  const uint32_t nc = x.nc_new[r.k];
  const uint32_t n = r.seg_hi - r.seg_lo;
  for (uint32_t ci = t; ci < nc; ci += kBlock) {
    s_st[ci] = x.starts[(uint64_t)r.k * capc + ci];
    s_xw[ci] = 0.0;
    s_w[ci] = 0.0;
  }
  if (t == 0) s_st[nc] = n;
  __syncthreads();
  const uint32_t b0 = r.lo + t * kHItems;
  if (b0 < r.hi) {
    uint32_t rel = b0 - r.seg_lo;
    uint32_t l = 0, h = nc;  // last centroid with start <= rel
    while (h - l > 1) {
      uint32_t m = (l + h) >> 1;
      if (s_st[m] <= rel) l = m;
      else h = m;
    }
    uint32_t cid = l;
    double axw = 0.0, aw = 0.0;
    for (int j = 0; j < (int)kHItems; j++) {
      uint32_t i = b0 + j;
      if (i >= r.hi) break;
      rel = i - r.seg_lo;
      if (rel >= s_st[cid + 1]) {
        atomicAdd(&s_xw[cid], axw);
        atomicAdd(&s_w[cid], aw);
        axw = 0.0;
        aw = 0.0;
        while (rel >= s_st[cid + 1]) cid++;
      }
      double wt = x.w[i];
      axw = dadd(axw, dmul(from_ordered_bits(x.A[i]), wt));
      aw = dadd(aw, wt);
    }
    atomicAdd(&s_xw[cid], axw);
    atomicAdd(&s_w[cid], aw);
  }
  __syncthreads();
  for (uint32_t ci = t; ci < nc; ci += kBlock) {
    if (s_w[ci] != 0.0) {
      unsafeAtomicAdd(&x.acc_w[(uint64_t)r.k * capc + ci], s_w[ci]);
      unsafeAtomicAdd(&x.acc_xw[(uint64_t)r.k * capc + ci], s_xw[ci]);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_finalize(HistoCtx x) {
  const uint32_t k = blockIdx.x, t = threadIdx.x, capc = x.capc;
  if (x.count && k >= *x.count) return;
  if (x.chb[k + 1] - x.chb[k] == 1) return;
  const uint32_t s = x.tl[k];
  const uint32_t nc = x.nc_new[k];
  const uint8_t nb = x.hcur[s] ^ 1;
  double* cm = nb ? x.cm1 : x.cm0;
  double* cwn = nb ? x.cw1 : x.cw0;
  const uint32_t lo = x.start[s], n = x.end[s] - lo;
  for (uint32_t ci = t; ci < nc; ci += kBlock) {
    double w = x.acc_w[(uint64_t)k * capc + ci];
    // sum(x w) / sum(w) may round past the centroid's own elements when they are equal (a
    // Welford mean never does): held to [first, last] element, so the means stay in order --
    // the next merge's positions (and Go's two-way merge) take them as sorted
    const uint32_t a = x.starts[(uint64_t)k * capc + ci];
    const uint32_t b = ci + 1 < nc ? x.starts[(uint64_t)k * capc + ci + 1] : n;
    const double m = ddiv(x.acc_xw[(uint64_t)k * capc + ci], w);
    const double lo_v = from_ordered_bits(x.A[lo + a]), hi_v = from_ordered_bits(x.A[lo + b - 1]);
    cm[(uint64_t)s * capc + ci] = m < lo_v ? lo_v : (m > hi_v ? hi_v : m);
    cwn[(uint64_t)s * capc + ci] = w;
  }
  __syncthreads();
  if (t == 0) {
    x.hncent[s] = nc;
    x.hcur[s] = nb;
    x.hspn[s] = 0;
  }
}

#endif  // VN_FAST_MODE
__global__ void k_clear_flags(uint32_t n, const uint32_t* __restrict__ list, uint32_t* __restrict__ flags,
                              const uint32_t* __restrict__ n_dev = nullptr) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n && (!n_dev || k < *n_dev)) flags[list[k]] = 0;
}

// raw (arrival-order) keys: A = float64 bits, B = slot<<32 | float32 rate bits
// (rate == nullptr: imported centroids, weights in impw, tagged kTagImport | i)
__global__ void k_histo_keys_raw(uint64_t n, const uint32_t* __restrict__ slot, const double* __restrict__ val,
                                 const float* __restrict__ rate, uint64_t* __restrict__ A, uint64_t* __restrict__ B) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = slot[i];
  A[i] = dbits(val[i]);
  const uint32_t tag = rate ? __float_as_uint(rate[i]) : (kTagImport | (uint32_t)i);
  B[i] = ((uint64_t)s << 32) | (uint64_t)tag;
}

#if VN_FAST_MODE
// After the (piece, top 40 value bits) sort: each run of records with equal piece and equal top
// 40 bits (values within 2^-28 relative of each other) of at most kTieRun records is
// insertion-sorted by the full ordered 64-bit value, stably -- the record order a full 64-bit LSD
// sort produces.  One lane per run (its first record); no lane walks more than kTieRun + 1
// records.  A longer run is left as it is: long runs of one repeated value (integer-valued
// timers) are in order already; a lane that sees an adjacent pair out of full-value order inside
// one sets *resort, and the (piece, full value) sort queued behind this kernel runs (radix_sort's
// cond).  Sorting permutes records inside a run only, so every lane sees the same run bounds.
constexpr uint64_t kTieRun = 64;
#ifndef VN_TIE_RESORT
#define VN_TIE_RESORT 1  // 0: no long-run check (negative control for the near-tie test, tools/ab_variant.sh)
#endif
__device__ __forceinline__ bool same_top(const uint64_t* A, const uint64_t* B, uint64_t a, uint64_t b) {
  return (B[a] >> 32) == (B[b] >> 32) && (A[a] >> 24) == (A[b] >> 24);
}
__global__ void k_fix_ties(uint64_t* __restrict__ A, uint64_t* __restrict__ B, uint64_t n,
                           uint32_t* __restrict__ resort) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i + 1 >= n) return;
  if (!same_top(A, B, i, i + 1)) return;
  if (VN_TIE_RESORT && A[i] > A[i + 1]) {  // an inversion: does it sit in a long run?
    uint64_t lo = i, hi = i + 1;
    while (lo > 0 && i - lo < kTieRun && same_top(A, B, lo - 1, i)) lo--;
    while (hi + 1 < n && hi - lo < kTieRun && same_top(A, B, i, hi + 1)) hi++;
    if (hi - lo + 1 > kTieRun) *resort = 1u;
  }
  if (i > 0 && same_top(A, B, i - 1, i)) return;  // not the run's first record
  uint64_t j = i + 2;
  while (j < n && j - i <= kTieRun && same_top(A, B, i, j)) j++;
  if (j - i > kTieRun) return;  // long run: left to the re-sort (if out of order)
  for (uint64_t k = i + 1; k < j; k++) {  // stable insertion sort of [i, j) by A
    const uint64_t a = A[k], b = B[k];
    uint64_t m = k;
    while (m > i && A[m - 1] > a) {
      A[m] = A[m - 1];
      B[m] = B[m - 1];
      m--;
    }
    A[m] = a;
    B[m] = b;
  }
}

#endif  // VN_FAST_MODE
// Per touched key: how many of its batch samples the exact replay takes, by the key's window
// count after this batch, tot:
//   cold  tot <= E            the whole batch replays exactly (bit-exact);
//   warm  E < tot <= W*E      the first E window samples replay exactly (with the cold keys),
//                             the rest joins the geometric remainder after that replay;
//   hot   tot > W*E           not bit-exact anyway and long: only the first P (hot_prefix)
//                             window samples replay exactly, on their own stream, so the hot
//                             remainder rounds run beside the long replays of the cold keys.
// (A key past E in an earlier batch has nothing left to replay: it joins the hot rounds.)
// Warm keys keep the long exact prefix because a remainder that is small next to it changes
// the quantiles least: keys just above E showed up to 5e-3 rank error at p50 with P = 4096
// and none with P = E (tools/tdigest_study.py, 8 seeds); above W*E = 4E both stay <= 7e-4.
constexpr uint32_t kWarmFactor = 4;
__global__ void k_histo_plan(uint32_t ntouched, const uint32_t* __restrict__ tl, const uint32_t* __restrict__ start,
                             const uint32_t* __restrict__ end, uint32_t* __restrict__ hseen, uint32_t E, uint32_t P,
                             uint32_t* __restrict__ ex, uint32_t* __restrict__ remflag,
                             uint32_t* __restrict__ replayflag, uint32_t* __restrict__ hotflag,
                             uint32_t* __restrict__ warmflag, uint32_t* __restrict__ hotcnt,
                             uint32_t* __restrict__ seen0, uint32_t* __restrict__ maxex,
                             const uint32_t* __restrict__ nt_dev) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (nt_dev) {  // ntouched is an upper bound: the keys past the device's count replay nothing
    const uint32_t live = *nt_dev;
    if (k < ntouched && k >= live) {
      ex[k] = 0u;
      hotcnt[k] = 0u;
      remflag[k] = 0u;
      replayflag[k] = 0u;
      hotflag[k] = 0u;
      warmflag[k] = 0u;
      seen0[k] = 0u;
    }
    ntouched = min(ntouched, live);
  }
  // the longest exact part of a replayed (cold or warm) key: the host skips the long-key
  // launches when none reaches their length (one atomic per wave)
  uint32_t mx = 0;
  if (k < ntouched) {
    const uint32_t s = tl[k], nk = end[s] - start[s], seen = hseen[s];
    const uint64_t tot = (uint64_t)seen + nk;
    if (tot <= (uint64_t)kWarmFactor * E) mx = tot <= E ? nk : (seen < E ? E - seen : 0u);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
  if ((threadIdx.x & 63) == 0 && mx) atomicMax(maxex, mx);
  if (k >= ntouched) return;
  uint32_t s = tl[k];
  uint32_t nk = end[s] - start[s];
  uint32_t seen = hseen[s];
  const uint64_t tot = (uint64_t)seen + nk;
  const bool cold = tot <= E;
  const bool warm = !cold && seen < E && tot <= (uint64_t)kWarmFactor * E;
  const uint32_t e = cold ? nk : warm ? E - seen : (seen >= P ? 0u : min(nk, P - seen));
  ex[k] = e;
  hotcnt[k] = nk - e;
  remflag[k] = !cold;              // merge the pending temps after the exact part
  replayflag[k] = cold || warm;    // replayed on the replay stream
  hotflag[k] = !cold && !warm;     // prefix on the hot-prefix stream, rounds beside the replay
  warmflag[k] = warm;              // rounds after the replay
  seen0[k] = seen;
  hseen[s] = seen + nk;
}

// ---- geometric remainder: a hot key's samples beyond its exact prefix are merged in
// pieces cut at window positions b_0 = P, b_{i+1} = b_i + max(1, b_i * g / 100) (and at batch
// edges): each piece is one mergeAllTemps of (current centroids + the piece's samples).
// tools/tdigest_study.py measured P = 4096 with g = 10, 15, 20, 25 at <= 8e-4 rank error
// against the reference's 42-sample incremental merge for keys of 40k..3M samples, g making
// no systematic difference (one merge of the whole remainder: up to 1.9e-3); g = 25 needs
// 30 rounds for a 3M-sample key where g = 10 needs 71.
__device__ __forceinline__ uint32_t geo_upper(const uint64_t* geo, uint32_t ngeo, uint64_t p) {
  uint32_t l = 0, h = ngeo;  // first index with geo[i] > p
  while (l < h) {
    uint32_t m = (l + h) >> 1;
    if (geo[m] <= p) l = m + 1;
    else h = m;
  }
  return l;
}

// A hot key's pieces ending at boundary 1..fuse (every one fits kFuseMaxL with the centroids)
// are merged by k_rounds_fused: how many of its leading pieces that is
__device__ __forceinline__ uint32_t fused_pieces(uint32_t pi0, uint32_t npieces, uint32_t fuse) {
  if (pi0 < 1 || pi0 > fuse) return 0;
  return min(npieces, fuse + 1 - pi0);
}

// maxp[0]: most pieces of a hot key, maxp[1]: of a warm key, maxp[2]: most pieces of a hot key
// left to the round pipeline after the fused launch (fuse > 0)
__global__ void k_histo_pieces(uint32_t ntouched, const uint32_t* __restrict__ ex, const uint32_t* __restrict__ hotcnt,
                               const uint32_t* __restrict__ seen0, const uint32_t* __restrict__ warmflag,
                               const uint64_t* __restrict__ geo, uint32_t ngeo, uint32_t fuse,
                               uint32_t* __restrict__ pcnt, uint32_t* __restrict__ pi0, uint32_t* __restrict__ maxp) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ntouched) return;
  const uint32_t n = hotcnt[k];
  if (!n) {
    pcnt[k] = 0;
    return;
  }
  const uint64_t P0 = (uint64_t)seen0[k] + ex[k], P1 = P0 + n;
  const uint32_t i0 = geo_upper(geo, ngeo, P0);      // first boundary after the remainder's start
  const uint32_t i1 = geo_upper(geo, ngeo, P1 - 1);  // first boundary after its last sample
  pi0[k] = i0;
  pcnt[k] = 1 + (i1 - i0);
  atomicMax(maxp + (warmflag[k] ? 1 : 0), 1 + (i1 - i0));
  if (!warmflag[k]) atomicMax(maxp + 2, 1 + (i1 - i0) - fused_pieces(i0, 1 + (i1 - i0), fuse));
}

#if VN_FAST_MODE
// copy the hot remainder into the piece-sort input: A = ordered value bits, B = piece id << 32 |
// float32 rate bits.  Output record o belongs to the touched key k with hotoff[k] <= o < hotoff[k+1]
// (a block of 4096 outputs spans few keys, so each thread searches between the block's first
// and last key only).
__device__ __forceinline__ uint32_t last_le(const uint32_t* off, uint32_t lo, uint32_t hi, uint32_t o) {
  while (hi - lo > 1) {  // last k in [lo, hi) with off[k] <= o
    uint32_t m = (lo + hi) >> 1;
    if (off[m] <= o) lo = m;
    else hi = m;
  }
  return lo;
}
__global__ __launch_bounds__(kBlock) void k_histo_gather_hot(uint32_t ntouched, uint64_t nhotrec,
                                                             const uint32_t* __restrict__ tl,
                                                             const uint32_t* __restrict__ start,
                                                             const uint32_t* __restrict__ ex,
                                                             const uint32_t* __restrict__ hotoff,
                                                             const uint32_t* __restrict__ seen0,
                                                             const uint32_t* __restrict__ pbase,
                                                             const uint32_t* __restrict__ pi0,
                                                             const uint64_t* __restrict__ geo, uint32_t ngeo,
                                                             const uint64_t* __restrict__ A,
                                                             const uint64_t* __restrict__ B,
                                                             uint64_t* __restrict__ A2, uint64_t* __restrict__ B2) {
  __shared__ uint32_t s_k[2];
  __shared__ uint64_t s_geo[256];  // the piece boundaries (ngeo <= 255), searched once per record
  for (uint32_t g = threadIdx.x; g < ngeo; g += kBlock) s_geo[g] = geo[g];
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  if (threadIdx.x < 2) {
    uint64_t o = base + (threadIdx.x ? (uint64_t)kTile - 1 : 0);
    if (o >= nhotrec) o = nhotrec - 1;
    s_k[threadIdx.x] = last_le(hotoff, 0, ntouched, (uint32_t)o);
  }
  __syncthreads();
  const uint32_t k0 = s_k[0], k1 = s_k[1] + 1;
  for (uint32_t j = threadIdx.x; j < (uint32_t)kTile; j += kBlock) {
    const uint64_t o = base + j;
    if (o >= nhotrec) break;
    const uint32_t k = last_le(hotoff, k0, k1, (uint32_t)o);
    const uint32_t i = (uint32_t)(o - hotoff[k]);
    const uint64_t src = (uint64_t)start[tl[k]] + ex[k] + i;
    const uint64_t pos = (uint64_t)seen0[k] + ex[k] + i;  // window position of the sample
    uint32_t l = 0, h = ngeo;  // geo_upper over the LDS copy: first boundary above pos
    while (l < h) {
      const uint32_t m = (l + h) >> 1;
      if (s_geo[m] <= pos) l = m + 1;
      else h = m;
    }
    const uint32_t gid = pbase[k] + (l - pi0[k]);
    A2[o] = ordered_bits(bitsd(A[src]));
    B2[o] = ((uint64_t)gid << 32) | (B[src] & 0xffffffffull);
  }
}

// round j, planned by one workgroup: which hot keys merge a piece (pcnt > j), in hot-list
// order, and for each active key a its slot (tl2), piece (rg), current centroid count (rnc),
// merged segment [roff[a], roff[a+1]) (also start/end by slot) and chunk base chb[a];
// count = number of active keys, roff/chb[count] = totals.
__global__ __launch_bounds__(1024) void k_round_plan(uint32_t nhot, uint32_t j, const uint32_t* __restrict__ hotlist,
                                                     const uint32_t* __restrict__ tl, const uint32_t* __restrict__ pcnt,
                                                     const uint32_t* __restrict__ pbase,
                                                     const uint32_t* __restrict__ pstart,
                                                     const uint32_t* __restrict__ pend,
                                                     const uint32_t* __restrict__ hncent, uint32_t* __restrict__ tl2,
                                                     uint32_t* __restrict__ rg, uint32_t* __restrict__ rnc,
                                                     uint32_t* __restrict__ roff, uint32_t* __restrict__ chb,
                                                     uint32_t* __restrict__ start, uint32_t* __restrict__ end,
                                                     uint32_t* __restrict__ count) {
  __shared__ uint32_t s_w[3][16];
  __shared__ uint32_t s_carry[3];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t < 3) s_carry[t] = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nhot; b0 += 1024) {
    const uint32_t h = b0 + t;
    uint32_t act = 0, len = 0, nch = 0, s = 0, g = 0, nc = 0;
    if (h < nhot) {
      const uint32_t k = hotlist[h];
      if (pcnt[k] > j) {
        act = 1;
        s = tl[k];
        g = pbase[k] + j;
        nc = hncent[s];
        len = nc + (pend[g] - pstart[g]);
        nch = (len + kHTile - 1) / kHTile;
      }
    }
    uint32_t v[3] = {act, len, nch}, inc[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
      uint32_t x = v[q];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += o;
      }
      inc[q] = x;
      if (lane == 63) s_w[q][w] = x;
    }
    __syncthreads();
    uint32_t ex[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
      uint32_t base = s_carry[q];
      for (uint32_t i = 0; i < w; i++) base += s_w[q][i];
      ex[q] = base + inc[q] - v[q];
    }
    if (act) {
      const uint32_t a = ex[0];
      tl2[a] = s;
      rg[a] = g;
      rnc[a] = nc;
      roff[a] = ex[1];
      chb[a] = ex[2];
      start[s] = ex[1];
      end[s] = ex[1] + len;
    }
    __syncthreads();
    if (t < 3) {
      uint32_t tot = 0;
      for (uint32_t i = 0; i < 16; i++) tot += s_w[t][i];
      s_carry[t] += tot;
    }
    __syncthreads();
  }
  if (t == 0) {
    count[0] = s_carry[0];
    roff[s_carry[0]] = s_carry[1];
  }
  for (uint32_t i = s_carry[0] + t; i <= nhot; i += 1024) chb[i] = s_carry[2];  // chunk_range reads chb[nhot]
}

// round j: lay out (current centroids + piece j) of every active key in merged order -- a
// centroid goes before a sample only if strictly smaller (merging_digest.go:169) -- in the
// pipeline's element format (A = ordered value bits, B = slot << 32 | tag).  One thread per
// input element over all active keys (grid-stride): its output position is its own index
// plus the count of elements of the other list that precede it.
__global__ __launch_bounds__(kBlock) void k_round_merge(uint32_t capc, const uint32_t* __restrict__ count,
                                                        const uint32_t* __restrict__ tl2, const uint32_t* __restrict__ rg,
                                                        const uint32_t* __restrict__ rnc,
                                                        const uint32_t* __restrict__ roff,
                                                        const uint32_t* __restrict__ pstart,
                                                        const uint32_t* __restrict__ pend,
                                                        const uint8_t* __restrict__ hcur, const double* __restrict__ cm0,
                                                        const double* __restrict__ cm1, const uint64_t* __restrict__ A,
                                                        const uint64_t* __restrict__ B, uint64_t* __restrict__ Ao,
                                                        uint64_t* __restrict__ Bo) {
  const uint32_t nact = *count;
  const uint32_t total = roff[nact];
  for (uint32_t u = blockIdx.x * kBlock + threadIdx.x; u < total; u += gridDim.x * kBlock) {
    uint32_t a = last_le(roff, 0, nact, u);
    const uint32_t s = tl2[a], g = rg[a], nc = rnc[a], off = roff[a];
    const uint32_t ps = pstart[g], np = pend[g] - ps;
    const double* cm = (hcur[s] ? cm1 : cm0) + (uint64_t)s * capc;
    const uint32_t r = u - off;
    if (r < nc) {
      const double v = cm[r];
      uint32_t l = 0, hh = np;  // samples <= v
      while (l < hh) {
        uint32_t m = (l + hh) >> 1;
        if (from_ordered_bits(A[ps + m]) <= v) l = m + 1;
        else hh = m;
      }
      Ao[off + r + l] = ordered_bits(v);
      Bo[off + r + l] = ((uint64_t)s << 32) | 0x80000000ull | (uint64_t)(s * capc + r);
    } else {
      const uint32_t i = r - nc;
      const uint64_t av = A[ps + i];
      const double v = from_ordered_bits(av);
      uint32_t l = 0, hh = nc;  // centroids < v
      while (l < hh) {
        uint32_t m = (l + hh) >> 1;
        if (cm[m] < v) l = m + 1;
        else hh = m;
      }
      Ao[off + i + l] = av;
      Bo[off + i + l] = ((uint64_t)s << 32) | (B[ps + i] & 0xffffffffull);
    }
  }
}
// Round j of the geometric remainder merges piece j of every listed key that has one: one
// mergeAllTemps of (the key's centroids + the piece's elements).  list indexes the per-key
// arrays e->h_tl (slot), e->h_pcnt (pieces), e->h_pbase (first piece id); pieces are the
// (piece id, value)-sorted elements PA/PB with ranges e->p_start/p_end per piece id.  nrec /
// nkeys bound the merged elements (capacity check); MA/MB receive each round's merged layout.
void histo_rounds(vn_engine* e, const uint32_t* list, uint32_t nkeys, uint32_t maxp, uint64_t nrec, uint32_t nrem,
                  const uint64_t* PA, const uint64_t* PB, uint64_t* MA, uint64_t* MB, const double* impw,
                  hipStream_t st) {
  if (!nkeys || !maxp) return;
  const uint64_t maxch = (nrec + (uint64_t)nrem * e->cap_cent) / kHTile + nrem + 1;
  if (maxch > e->h_max_chunks || nrec + (uint64_t)nrem * e->cap_cent > e->h_sort_cap)
    throw std::runtime_error("histo chunk capacity exceeded");
  HistoCtx x;
  x.ntouched = nkeys;
  x.count = e->h_cnt + 5;
  x.capc = e->cap_cent;
  x.delta = e->cfg.compression;
  x.tl = e->h_tl2;
  x.start = e->h_start;
  x.end = e->h_end;
  x.chb = e->h_chb;
  x.A = MA;
  x.B = MB;
  x.impw = impw;
  x.w = e->h_w;
  x.wk = e->h_wk;
  x.ch_sum = e->ch_sum;
  x.ch_pre = e->ch_pre;
  x.ch_stats = e->ch_stats;
  x.seg_T = e->seg_T;
  x.starts = e->starts;
  x.nc_new = e->nc_new;
  x.acc_xw = e->acc_xw;
  x.acc_w = e->acc_w;
  x.hst = e->hst;
  x.hncent = e->hncent;
  x.hcur = e->hcur;
  x.hspn = e->hspn;
  x.cm0 = e->cmean[0];
  x.cm1 = e->cmean[1];
  x.cw0 = e->cw[0];
  x.cw1 = e->cw[1];
  x.err = e->h_err;
  const int merge_blocks = std::min(1024, blocks_for(nrec + (uint64_t)nrem * e->cap_cent, kBlock));
  for (uint32_t j = 0; j < maxp; j++) {
    hipLaunchKernelGGL(k_round_plan, dim3(1), dim3(1024), 0, st, nkeys, j, list, e->h_tl, e->h_pcnt, e->h_pbase,
                       e->p_start, e->p_end, e->hncent, e->h_tl2, e->r_flag, e->r_len, e->r_off, e->h_chb,
                       e->h_start, e->h_end, e->h_cnt + 5);
    hipLaunchKernelGGL(k_round_merge, dim3(merge_blocks), dim3(kBlock), 0, st, e->cap_cent, e->h_cnt + 5, e->h_tl2,
                       e->r_flag, e->r_len, e->r_off, e->p_start, e->p_end, e->hcur, e->cmean[0], e->cmean[1], PA,
                       PB, MA, MB);
    hipLaunchKernelGGL(k_chunk_prep, dim3(maxch), dim3(kBlock), 0, st, x);
    hipLaunchKernelGGL(k_seg_scan, dim3(nkeys), dim3(kBlock), 0, st, x);
    hipLaunchKernelGGL(k_chunk_kin, dim3(maxch), dim3(kBlock), 0, st, x);
    hipLaunchKernelGGL(k_chain, dim3(nkeys), dim3(kChainThreads), 0, st, x);
    hipLaunchKernelGGL(k_chunk_cent, dim3(maxch), dim3(kBlock), 0, st, x);
    hipLaunchKernelGGL(k_finalize, dim3(nkeys), dim3(kBlock), 0, st, x);
  }
}

// The rounds of a few keys with small pieces in one launch (split.hip's owner: every piece is
// the ranks' micro-centroids, <= N x 1024 of them).  One workgroup per key walks its pieces in
// order; per piece the same steps as the round pipeline above -- (centroids + piece) in merged
// order (a centroid before an element only if strictly smaller, merging_digest.go:169), the
// inclusive weight prefix, k = indexEstimate(W / T) in LDS, the greedy chain (a new centroid
// where k - k(start) > 1, mergeOne 210-236) walked by one wave, and each centroid's Welford
// update in element order (thread per centroid) -- with no host round trip and no launch per
// step.  The merged elements live in the caller's scratch (kFuseMaxL values and weights per key).
struct FusedRounds {
  const uint32_t* list;  // key indices (into tl / pcnt / pbase)
  const uint32_t* tl;
  const uint32_t* pcnt;
  const uint32_t* pbase;
  const uint32_t* pstart;
  const uint32_t* pend;
  const uint64_t* PA;    // pieces: ordered value bits, (piece << 32 | tag), sorted by (piece, value)
  const uint64_t* PB;
  const double* impw;
  uint32_t capc;
  double delta;
  double* hst;
  uint32_t* hncent;
  uint8_t* hcur;
  uint32_t* hspn;
  double *cm0, *cm1, *cw0, *cw1;
  double* val;           // [key][kFuseMaxL]
  double* w;
  double* kk;            // k of every merged element (global: the kernel needs no large LDS block)
  uint32_t* err;
  // partial mode (done != null): merge only the leading pieces that end at geometric boundary
  // 1..max_pieces (fused_pieces); done[block] = pieces merged (the round pipeline takes the rest)
  uint32_t max_pieces;
  const uint32_t* pi0;
  uint32_t* done;
};
__global__ __launch_bounds__(kBlock) void k_rounds_fused(FusedRounds x) {
  __shared__ uint32_t s_st[kMaxCent + 1];
  __shared__ double s_tmp[4];
  __shared__ uint32_t s_nc;
  const uint32_t t = threadIdx.x, lane = t & 63;
  const uint32_t key = x.list[blockIdx.x];
  const uint32_t s = x.tl[key], npieces = x.pcnt[key], capc = x.capc;
  double* val = x.val + (uint64_t)blockIdx.x * kFuseMaxL;
  double* wgt = x.w + (uint64_t)blockIdx.x * kFuseMaxL;
  double* s_k = x.kk + (uint64_t)blockIdx.x * kFuseMaxL;
  uint32_t nc = x.hncent[s];
  uint8_t cur = x.hcur[s];
  double* h = x.hst + (uint64_t)s * VN_HISTO_STATS;
  uint32_t jdone = 0;
  const uint32_t jend = x.done ? fused_pieces(x.pi0[key], npieces, x.max_pieces) : npieces;
  for (uint32_t j = 0; j < jend; j++) {
    const uint32_t g = x.pbase[key] + j;
    const uint32_t ps = x.pstart[g], np = x.pend[g] - ps;
    const double* cm = (cur ? x.cm1 : x.cm0) + (uint64_t)s * capc;
    const double* cw = (cur ? x.cw1 : x.cw0) + (uint64_t)s * capc;
    const uint32_t L = nc + np;
    if (np == 0) {  // (block-uniform) nothing to merge
      jdone = j + 1;
      continue;
    }
    if (L > kFuseMaxL) {  // the host sizes pieces (or max_pieces) below this
      if (t == 0) atomicOr(x.err, 1u);
      return;
    }
    // merged order, weights, the statistics of the piece's elements
    double sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf, dmn = kInf, dmx = -kInf;
    for (uint32_t u = t; u < L; u += kBlock) {
      if (u < nc) {
        const double v = cm[u];
        uint32_t l = 0, hh = np;  // piece elements <= v
        while (l < hh) {
          const uint32_t m = (l + hh) >> 1;
          if (from_ordered_bits(x.PA[ps + m]) <= v) l = m + 1;
          else hh = m;
        }
        val[u + l] = v;
        wgt[u + l] = cw[u];
      } else {
        const uint32_t i = u - nc;
        const double v = from_ordered_bits(x.PA[ps + i]);
        uint32_t l = 0, hh = nc;  // centroids < v
        while (l < hh) {
          const uint32_t m = (l + hh) >> 1;
          if (cm[m] < v) l = m + 1;
          else hh = m;
        }
        const uint32_t tag = (uint32_t)x.PB[ps + i];
        const double wt = tag_weight(tag, x.impw);
        dmn = min_go(dmn, v);
        dmx = max_go(dmx, v);
        if (tag_is_sample(tag)) {
          sw = dadd(sw, wt);
          mn = min_go(mn, v);
          mx = max_go(mx, v);
          sxw = dadd(sxw, dmul(v, wt));
          srw = dadd(srw, dmul(ddiv(1.0, v), wt));
        }
        val[i + l] = v;
        wgt[i + l] = wt;
      }
    }
    __syncthreads();
    // inclusive weight prefix (thread t: elements [t*q, t*q + q)), k of every element
    const uint32_t q = (L + kBlock - 1) / kBlock;
    const uint32_t i0 = min(L, t * q), i1 = min(L, i0 + q);
    double run = 0.0;
    for (uint32_t i = i0; i < i1; i++) run = dadd(run, wgt[i]);
    double T;
    double acc = block_excl_scan_d(run, s_tmp, T);
    for (uint32_t i = i0; i < i1; i++) {
      acc = dadd(acc, wgt[i]);
      s_k[i] = index_estimate(x.delta, ddiv(acc, T));
    }
    __syncthreads();
    // the chain: next start = first element after pos with k - k(before start) > 1
    if (t < 64) {
      uint32_t n2 = 0, pos = 0;
      double base = index_estimate(x.delta, 0.0);
      for (;;) {
        if (n2 >= capc) {
          if (lane == 0) atomicOr(x.err, 1u);
          break;
        }
        if (lane == 0) s_st[n2] = pos;
        n2++;
        bool found = false;
        for (uint32_t from = pos + 1; from < L; from += 64) {
          const uint32_t idx = from + lane;
          const uint64_t m = __ballot(idx < L && dsub(s_k[idx < L ? idx : 0], base) > 1.0);
          if (m) {
            pos = from + (uint32_t)__ffsll((unsigned long long)m) - 1;
            base = s_k[pos - 1];
            found = true;
            break;
          }
        }
        if (!found) break;
      }
      if (lane == 0) {
        s_st[n2] = L;
        s_nc = n2;
      }
    }
    sw = block_allreduce(sw, s_tmp, SumOp());  // (its barrier publishes the chain)
    sxw = block_allreduce(sxw, s_tmp, SumOp());
    srw = block_allreduce(srw, s_tmp, SumOp());
    mn = block_allreduce(mn, s_tmp, MinGoOp());
    mx = block_allreduce(mx, s_tmp, MaxGoOp());
    dmn = block_allreduce(dmn, s_tmp, MinGoOp());
    dmx = block_allreduce(dmx, s_tmp, MaxGoOp());
    const uint32_t ncn = s_nc;
    const uint8_t nb = cur ^ 1;
    double* cmn = (nb ? x.cm1 : x.cm0) + (uint64_t)s * capc;
    double* cwn = (nb ? x.cw1 : x.cw0) + (uint64_t)s * capc;
    for (uint32_t ci = t; ci < ncn; ci += kBlock) {
      const uint32_t a = s_st[ci], b = s_st[ci + 1];
      double mean = val[a], W = wgt[a];
      for (uint32_t i = a + 1; i < b; i++) {
        const double wt = wgt[i];
        W = dadd(W, wt);
        mean = dadd(mean, ddiv(dmul(dsub(val[i], mean), wt), W));
      }
      cmn[ci] = mean;
      cwn[ci] = W;
    }
    if (t == 0) {
      h[0] = dadd(h[0], sw);
      h[1] = min_go(h[1], mn);
      h[2] = max_go(h[2], mx);
      h[3] = dadd(h[3], sxw);
      h[4] = dadd(h[4], srw);
      h[5] = min_go(h[5], dmn);
      h[6] = max_go(h[6], dmx);
      h[7] = T;
    }
    nc = ncn;
    cur = nb;
    jdone = j + 1;
    __syncthreads();  // the new centroids are the next piece's merge input
  }
  if (t == 0 && jdone) {
    x.hncent[s] = nc;
    x.hcur[s] = cur;
    x.hspn[s] = 0;
  }
  if (t == 0 && x.done) x.done[blockIdx.x] = jdone;
}

// after a partial fused launch: the round pipeline starts at each key's first unmerged piece
__global__ void k_fuse_shift(const uint32_t* __restrict__ list, uint32_t n, const uint32_t* __restrict__ done,
                             uint32_t* __restrict__ pbase, uint32_t* __restrict__ pcnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = list[i], d = done[i];
  pbase[k] += d;
  pcnt[k] -= d;
}

void histo_rounds_fused(vn_engine* e, const uint32_t* list, uint32_t nkeys, const uint64_t* PA, const uint64_t* PB,
                        const double* impw, double* val, double* w, double* kk, hipStream_t st, uint32_t max_pieces,
                        uint32_t* done) {
  if (!nkeys) return;
  FusedRounds x;
  x.max_pieces = max_pieces;
  x.pi0 = e->h_pi0;
  x.done = done;
  x.list = list;
  x.tl = e->h_tl;
  x.pcnt = e->h_pcnt;
  x.pbase = e->h_pbase;
  x.pstart = e->p_start;
  x.pend = e->p_end;
  x.PA = PA;
  x.PB = PB;
  x.impw = impw;
  x.capc = e->cap_cent;
  x.delta = e->cfg.compression;
  x.hst = e->hst;
  x.hncent = e->hncent;
  x.hcur = e->hcur;
  x.hspn = e->hspn;
  x.cm0 = e->cmean[0];
  x.cm1 = e->cmean[1];
  x.cw0 = e->cw[0];
  x.cw1 = e->cw[1];
  x.val = val;
  x.w = w;
  x.kk = kk;
  x.err = e->h_err;
  hipLaunchKernelGGL(k_rounds_fused, dim3(nkeys), dim3(kBlock), 0, st, x);
}

// chunks of each segment: nch[k] = ceil(len / kHTile) (0 for an empty segment)
__global__ void k_seg_chunks(uint32_t nseg, const uint32_t* __restrict__ start, const uint32_t* __restrict__ end,
                             uint32_t* __restrict__ nch) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nseg) nch[k] = (end[k] - start[k] + kHTile - 1) / kHTile;
}

void histo_compress_segments(const SegCompress& c, ScanScratch& ss, hipStream_t st) {
  if (!c.nseg) return;
  hipLaunchKernelGGL(k_seg_chunks, dim3(blocks_for(c.nseg, 256)), dim3(256), 0, st, c.nseg, c.start, c.end, c.nch);
  scan_exclusive_u32(c.nch, c.chb, c.nseg, ss, st);
  HistoCtx x;
  x.ntouched = c.nseg;
  x.count = nullptr;
  x.capc = c.capc;
  x.delta = c.delta;
  x.tl = c.tl;
  x.start = c.start;
  x.end = c.end;
  x.chb = c.chb;
  x.A = c.A;
  x.B = c.B;
  x.impw = nullptr;
  x.w = c.w;
  x.wk = c.wk;
  x.ch_sum = c.ch_sum;
  x.ch_pre = c.ch_pre;
  x.ch_stats = c.ch_stats;
  x.seg_T = c.seg_T;
  x.starts = c.starts;
  x.nc_new = c.nc_new;
  x.acc_xw = c.acc_xw;
  x.acc_w = c.acc_w;
  x.hst = c.hst;
  x.hncent = c.hncent;
  x.hcur = c.hcur;
  x.hspn = c.hspn;
  x.cm0 = c.cm0;
  x.cm1 = c.cm1;
  x.cw0 = c.cw0;
  x.cw1 = c.cw1;
  x.err = c.err;
  const uint64_t maxch = c.nrec / kHTile + c.nseg + 1;
  hipLaunchKernelGGL(k_chunk_prep, dim3(maxch), dim3(kBlock), 0, st, x);
  hipLaunchKernelGGL(k_seg_scan, dim3(c.nseg), dim3(kBlock), 0, st, x);
  hipLaunchKernelGGL(k_chunk_kin, dim3(maxch), dim3(kBlock), 0, st, x);
  hipLaunchKernelGGL(k_chain, dim3(c.nseg), dim3(kChainThreads), 0, st, x);
  hipLaunchKernelGGL(k_chunk_cent, dim3(maxch), dim3(kBlock), 0, st, x);
  hipLaunchKernelGGL(k_finalize, dim3(c.nseg), dim3(kBlock), 0, st, x);
}

#endif  // VN_FAST_MODE
// timing mode: sum over the replayed keys of min(replayed samples, 160) (centroids written)
__global__ void k_replay_state(uint32_t n, const uint32_t* __restrict__ ex, unsigned long long* __restrict__ out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long v = k < n ? (unsigned long long)min(ex[k], 160u) : 0ull;
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(out, v);
}

#ifndef VN_LONG_MIN_EXACT
#define VN_LONG_MIN_EXACT 65536u
#endif
constexpr uint32_t kLongMinExact = VN_LONG_MIN_EXACT;  // exact mode: keys replaying this many samples take four waves
#ifndef VN_BULK_SIDE
#define VN_BULK_SIDE 0
#endif
constexpr bool kBulkSide = VN_BULK_SIDE != 0;
#ifndef VN_INGEST_WAITS
// 1: the histogram plan's two host waits (the default); 0: the wait-free plan of histo_process,
// measured not better -- C4 at N = 1, four engines: 76.7 against 73.9 ms per window, the ingest's
// host time 9 against 53 ms but the window's latency 303 against 278 ms: the GPU, not the host, is
// what the windows in flight wait for
#define VN_INGEST_WAITS 1
#endif
HistoGroups histo_group(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val, const float* rate) {
  HistoGroups g{};
  if (!n) return g;
  hipStream_t st = e->st;
  const uint32_t caph = e->cap[VN_HISTO];
  // ---- 1. group by key, arrival order kept (stable radix by slot); nothing here waits on
  // the host, so the caller can queue other streams' work before histo_process syncs
  hipLaunchKernelGGL(k_histo_keys_raw, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, slot, val, rate, e->hA0, e->hB0);
  RadixPass spass[4];
  int nsp = 0;
  nsp = make_passes(spass, true, 32, e->slot_bits[VN_HISTO]);
  bool fl = radix_sort(e->hA0, e->hB0, e->hA1, e->hB1, n, spass, nsp, e->rs, st, e->timing ? &e->rstat_h : nullptr);
  g.As = fl ? e->hA1 : e->hA0;
  g.Bs = fl ? e->hB1 : e->hB0;
  g.Ao = fl ? e->hA0 : e->hA1;
  g.Bo = fl ? e->hB0 : e->hB1;
  hipLaunchKernelGGL(k_seg_mark, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, g.Bs, e->h_start, e->h_end, e->h_bt,
                     e->htouch);
  compact_flags(e->h_bt, e->h_pos, e->h_tl, e->h_cnt, caph, e->ss, st);
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt, e->h_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  return g;
}

// records already grouped by key in arrival order (As / Bs as histo_group leaves them, e.g. the
// import drain's payload-ordered move): the segment bounds and touched keys only
HistoGroups histo_group_sorted(vn_engine* e, uint64_t n, uint64_t* As, uint64_t* Bs, uint64_t* Ao, uint64_t* Bo,
                               bool marked) {
  HistoGroups g{As, Bs, Ao, Bo};
  if (!n) return g;
  hipStream_t st = e->st;
  if (!marked)  // (marked: the caller set start / end / bt / touch already)
    hipLaunchKernelGGL(k_seg_mark, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, g.Bs, e->h_start, e->h_end, e->h_bt,
                       e->htouch);
  compact_flags(e->h_bt, e->h_pos, e->h_tl, e->h_cnt, e->cap[VN_HISTO], e->ss, st);
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt, e->h_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  return g;
}

void ingest_histos(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val, const float* rate,
                   const double* impw) {
  const HistoGroups g = histo_group(e, n, slot, val, rate);
  histo_process(e, n, g, impw);
}

void histo_process(vn_engine* e, uint64_t n, const HistoGroups& g, const double* impw) {
  if (!n) return;
  hipStream_t st = e->st;
  uint64_t* const As = g.As;
  uint64_t* const Bs = g.Bs;
  uint64_t* const Ao = g.Ao;
  uint64_t* const Bo = g.Bo;
  // Without the fast mode every touched key replays exactly (no hot or warm keys, no remainder):
  // the host then needs no count from the device -- the launches can be sized by an upper bound
  // (the touched keys are at most min(n, capacity)) and read the device's counts, so the call
  // queues the whole path without waiting (VN_INGEST_WAITS 0; the timing mode keeps the waits,
  // its byte counts need the sizes).
  const bool async = !VN_FAST_MODE && !e->timing && !VN_INGEST_WAITS;
  if (!async) VN_HWAIT(e, 1, VN_HIP_CHECK(hipStreamSynchronize(st)));
  const uint32_t ntouched = async ? (uint32_t)std::min<uint64_t>(n, e->cap[VN_HISTO]) : e->hf_cnt[0];
  const uint32_t* const nt_dev = async ? e->h_cnt : nullptr;  // (histo_group's touched count)
  if (!ntouched) return;

  // ---- 2. plan: exact part of every key (cold / warm / hot, k_histo_plan); the remainders
  // of warm and hot keys cut into geometric pieces
  uint32_t* const remflag = e->h_hotflag;
  VN_HIP_CHECK(hipMemsetAsync(e->h_cnt + 20, 0, sizeof(uint32_t), st));
  hipLaunchKernelGGL(k_histo_plan, dim3(blocks_for(ntouched, 256)), dim3(256), 0, st, ntouched, e->h_tl, e->h_start,
                     e->h_end, e->hseen, e->exact_threshold, e->hot_prefix, e->h_ex, remflag, e->h_coldflag,
                     e->h_vhflag, e->h_warmflag, e->h_hotcnt, e->h_seen0, e->h_cnt + 20, nt_dev);
  if (async) compact_flags(e->h_coldflag, e->h_pos, e->h_coldlist, e->h_cnt + 6, ntouched, e->ss, st);
  uint32_t nhot = 0, npieces = 0, maxp_hot = 0, maxp_warm = 0, maxp_hot_left = 0, nwarm = 0;
  uint64_t nremrec = 0;
  uint32_t nreplay = ntouched, maxex = 0xFFFFFFFFu;  // (async: upper bounds; the device holds the counts)
  if (!async) {
  compact_flags(e->h_vhflag, e->h_pos, e->h_hotlist, e->h_cnt + 1, ntouched, e->ss, st);
  compact_flags(e->h_warmflag, e->h_pos, e->h_warmlist, e->h_cnt + 8, ntouched, e->ss, st);
  compact_flags(e->h_coldflag, e->h_pos, e->h_coldlist, e->h_cnt + 6, ntouched, e->ss, st);
  scan_exclusive_u32(e->h_hotcnt, e->h_hotoff, ntouched, e->ss, st);
  VN_HIP_CHECK(hipMemsetAsync(e->h_cnt + 9, 0, 3 * sizeof(uint32_t), st));
  hipLaunchKernelGGL(k_histo_pieces, dim3(blocks_for(ntouched, 256)), dim3(256), 0, st, ntouched, e->h_ex,
                     e->h_hotcnt, e->h_seen0, e->h_warmflag, e->h_geo, e->n_geo, e->fuse_pieces, e->h_pcnt, e->h_pi0,
                     e->h_cnt + 9);
  scan_exclusive_u32(e->h_pcnt, e->h_pbase, ntouched, e->ss, st);
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 1, e->h_cnt + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 2, e->h_hotoff + ntouched, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 3, e->h_pbase + ntouched, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 4, e->h_cnt + 9, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 6, e->h_cnt + 6, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 7, e->h_cnt + 8, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 11, e->h_cnt + 11, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 13, e->h_cnt + 20, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HWAIT(e, 2, VN_HIP_CHECK(hipStreamSynchronize(st)));
  nhot = e->hf_cnt[1];
  nremrec = e->hf_cnt[2];  // remainder records of warm and hot keys
  npieces = e->hf_cnt[3];
  maxp_hot = e->hf_cnt[4];
  maxp_warm = e->hf_cnt[5];
  maxp_hot_left = e->hf_cnt[11];  // after the fused launch of the leading pieces
  nreplay = e->hf_cnt[6];  // cold + warm keys
  nwarm = e->hf_cnt[7];
  maxex = e->hf_cnt[13];  // longest exact part of a cold or warm key
  }

  // ---- 3. exact replay of MergingDigest.Add (histo_exact.hip): every pure chunk pre-sorted,
  // then the cold and warm keys on the replay stream, the hot keys' prefixes on their own
  ExactCtx xc{};
  xc.nkeys = ntouched;
  xc.nkeys_dev = nt_dev;
  xc.keys = e->h_tl;
  xc.start = e->h_start;
  xc.nex = e->h_ex;
  xc.hot = remflag;
  xc.A = As;
  xc.B = Bs;
  xc.impw = impw;
  xc.delta = e->cfg.compression;
  xc.capc = e->cap_cent;
  xc.tcap = e->temp_cap;
  xc.hst = e->hst;
  xc.hncent = e->hncent;
  xc.hcur = e->hcur;
  xc.cm0 = e->cmean[0];
  xc.cm1 = e->cmean[1];
  xc.cw0 = e->cw[0];
  xc.cw1 = e->cw[1];
  xc.hpend = e->hpend;
#ifndef VN_HISTO_SPEC
#define VN_HISTO_SPEC 1
#endif
  xc.spec = VN_HISTO_SPEC;
  xc.hspn = e->hspn;
  xc.hspw = e->hspw;
  xc.hpv = e->hpv;
  xc.hpw = e->hpw;
  xc.err = e->h_err;
  xc.flush_mode = 0;
  xc.ccnt = e->h_ccnt;
  xc.coff = e->h_coff;
  xc.cown = e->h_cown;
  xc.csv = e->h_csv;
  xc.csw = e->h_csw;
  xc.ctw = e->h_tw;
#ifndef VN_TW_SUM
#define VN_TW_SUM 1
#endif
  xc.tw_sum = VN_TW_SUM;
  xc.cpk = e->h_cpk;
  xc.lstat = e->h_lstat;
#ifndef VN_NO_CSTAT
  xc.cstat = e->h_cstat;  // (A/B build VN_NO_CSTAT: k_exact_long_stats re-reads the samples)
#endif
  const uint64_t max_chunks = n / e->temp_cap + 1;
  // the four-wave replay's threshold (replay_cold below): shorter keys take the one-wave replay
  // (exact mode: 65536 -- the short keys' one-wave replays fill the GPU with small workgroups,
  // where each four-wave one holds a larger share of a CU; C4 at N = 1 62.2 / 62.6 -> 59.9 / 60.2
  // ms per window against 8192, 32768: 60.5 / 60.8, 131072: 60.2 / 60.1; profiles/r06_longreplay/)
  const uint32_t long_min =
      e->long_replay ? e->long_replay
      : e->exact_threshold == 0xFFFFFFFFu ? kLongMinExact
                                          : std::min<uint32_t>(std::max<uint32_t>(e->exact_threshold / 4, 1024u), 8192u);
  xc.long_min = long_min;
  // (exact mode, no hot key, not timing: the longest keys' chunks are sorted first and their
  // replays start while the other chunks sort, in replay_cold)
  const bool early = e->early_top && !nhot && !e->timing && e->st5 && e->st6;
  histo_exact_chunk_plan(xc, st, &e->ss, max_chunks);
  if (!early) histo_exact_chunk_sort(xc, st, max_chunks, 0, false);
  // The hot keys' prefixes run on st4 (short) while st gathers and sorts the remainders; the
  // cold and warm keys (long) on st3 after the sort, whose passes would otherwise wait for CUs
  // behind 100k+ replay workgroups -- then the held-back set merge on the side stream.  With
  // no hot key (or when timing) everything runs in order on st.
  const bool fork = nhot && !e->timing;
  // timing mode: each replay launch bracketed by events (kernel-level roofline of k_histo_exact)
  auto clocked_replay = [&](hipStream_t s) {
    hipEvent_t a = e->timing ? e->pool_rp.next() : nullptr, b = e->timing ? e->pool_rp.next() : nullptr;
    if (a && b) VN_HIP_CHECK(hipEventRecord(a, s));
    histo_exact_replay(xc, s);
    if (a && b) VN_HIP_CHECK(hipEventRecord(b, s));
    if (e->timing) e->kstat_rp.launches++;
  };
  // the longest keys (a quarter of the threshold, at most 8192 samples, and more) replay with
  // four waves each on st5 (replay_key_fast: built for one merge's latency), beside the one-wave
  // replay of the rest on the same CUs
  auto replay_cold = [&](hipStream_t s, RadixScratch& rs) {
    histo_exact_order(xc, e->h_coldlist, nreplay, e->h_lpt0, e->h_lpt1, rs, s, async ? e->h_cnt + 6 : nullptr);
    const uint32_t min_len = long_min;
    const bool longk = maxex >= min_len && histo_exact_count_long(xc, min_len, e->h_cnt + 15, s);
    const bool side5 = longk && !e->timing && e->st5;
    hipEvent_t a = e->timing ? e->pool_rp.next() : nullptr, b = e->timing ? e->pool_rp.next() : nullptr;
    if (a && b) VN_HIP_CHECK(hipEventRecord(a, s));
    if (early) {
      // the window's longest chains first: the top keys' chunks, their replays on st6, then
      // every other chunk while they run, then the other long keys (st5, s) and the rest (s)
      const uint32_t top = side5 ? histo_exact_top_keys(xc) : 0u;
      if (top) {
        histo_exact_chunk_sort(xc, s, max_chunks, top, true);
        VN_HIP_CHECK(hipEventRecord(e->ev_fork5, s));
        VN_HIP_CHECK(hipStreamWaitEvent(e->st6, e->ev_fork5, 0));
        histo_exact_replay_top(xc, e->st6, top);
        VN_HIP_CHECK(hipEventRecord(e->ev_join6, e->st6));
      }
      histo_exact_chunk_sort(xc, s, max_chunks, top, false);
      if (side5) {
        VN_HIP_CHECK(hipEventRecord(e->ev_rest5, s));
        VN_HIP_CHECK(hipStreamWaitEvent(e->st5, e->ev_rest5, 0));
        histo_exact_replay_long(xc, e->st5, s, top ? e->st6 : nullptr, top);
        VN_HIP_CHECK(hipEventRecord(e->ev_join5, e->st5));
      } else if (longk) {
        histo_exact_replay_long(xc, s, s);
      }
      histo_exact_replay(xc, s);
      if (side5) VN_HIP_CHECK(hipStreamWaitEvent(s, e->ev_join5, 0));
      if (top) VN_HIP_CHECK(hipStreamWaitEvent(s, e->ev_join6, 0));
    } else if (side5) {  // the batched longest keys on st5, the other long keys ahead of the rest on s
      VN_HIP_CHECK(hipEventRecord(e->ev_fork5, s));
      VN_HIP_CHECK(hipStreamWaitEvent(e->st5, e->ev_fork5, 0));
      if (e->st6) VN_HIP_CHECK(hipStreamWaitEvent(e->st6, e->ev_fork5, 0));
      // (VN_BULK_SIDE: the other keys' replays -- throughput work that ends long before the
      // chain -- on the low-priority side stream, so the next windows' ingest fronts on their
      // high-priority main streams do not queue behind them)
      const bool bulk = kBulkSide && e->st2 && e->ev_bulk;
      hipStream_t sb = s;
      if (bulk) {
        VN_HIP_CHECK(hipStreamWaitEvent(e->st2, e->ev_fork5, 0));
        sb = e->st2;
      }
      histo_exact_replay_long(xc, e->st5, sb, e->st6);
      VN_HIP_CHECK(hipEventRecord(e->ev_join5, e->st5));
      if (e->st6) VN_HIP_CHECK(hipEventRecord(e->ev_join6, e->st6));
      histo_exact_replay(xc, sb);
      if (bulk) {
        VN_HIP_CHECK(hipEventRecord(e->ev_bulk, e->st2));
        VN_HIP_CHECK(hipStreamWaitEvent(s, e->ev_bulk, 0));
      }
      VN_HIP_CHECK(hipStreamWaitEvent(s, e->ev_join5, 0));
      if (e->st6) VN_HIP_CHECK(hipStreamWaitEvent(s, e->ev_join6, 0));
    } else {
      if (longk) histo_exact_replay_long(xc, s, s);
      histo_exact_replay(xc, s);
    }
    if (a && b) VN_HIP_CHECK(hipEventRecord(b, s));
    if (e->timing) e->kstat_rp.launches++;
    xc.mw_count = nullptr;
  };
  if (e->timing) {
    // 16 B per replayed sample, 40 B of local statistics and 16 B per centroid
    // written per replayed key (<= 160 centroids at delta 100; a key's sample count bounds it)
    VN_HIP_CHECK(hipMemsetAsync(e->h_cnt + 12, 0, 8, st));
    hipLaunchKernelGGL(k_replay_state, dim3(blocks_for(ntouched, 256)), dim3(256), 0, st, ntouched, e->h_ex,
                       reinterpret_cast<unsigned long long*>(e->h_cnt + 12));
    uint64_t cent = 0;
    VN_HIP_CHECK(hipMemcpyAsync(&cent, e->h_cnt + 12, 8, hipMemcpyDeviceToHost, st));
    VN_HIP_CHECK(hipStreamSynchronize(st));
    e->kstat_rp.bytes += 16ull * (n - nremrec) + 40ull * (nreplay + nhot) + 16ull * cent;
  }
  if (fork) {
    ensure_aux_streams(e, true, false);
    VN_HIP_CHECK(hipEventRecord(e->ev_fork3, st));
    VN_HIP_CHECK(hipStreamWaitEvent(e->st4, e->ev_fork3, 0));
    VN_HIP_CHECK(hipStreamWaitEvent(e->st3, e->ev_fork3, 0));
    replay_cold(e->st3, e->rs3);
    VN_HIP_CHECK(hipEventRecord(e->ev_join3, e->st3));
  } else {
    replay_cold(st, e->rs);
  }
  xc.order64 = nullptr;
  xc.order = e->h_hotlist;
  xc.norder = nhot;
  clocked_replay(fork ? e->st4 : st);
  if (fork) VN_HIP_CHECK(hipEventRecord(e->ev_join4, e->st4));

  // ---- 4. remainders of warm and hot keys: geometric pieces, merged round by round (As/Bs
  // stay with the replay)
  if (nremrec == 0) {
    set_finish(e);
    hipLaunchKernelGGL(k_clear_flags, dim3(blocks_for(ntouched, 256)), dim3(256), 0, st, ntouched, e->h_tl, e->h_bt,
                       nt_dev);
    return;
  }
#if !VN_FAST_MODE
  (void)Ao, (void)Bo, (void)npieces, (void)maxp_hot, (void)maxp_warm, (void)maxp_hot_left, (void)nwarm;
  throw std::logic_error("histo remainder without the fast mode (VN_FAST_MODE) built");
#else
  // sort the remainders by (piece, value): every piece contiguous and value-sorted
  hipLaunchKernelGGL(k_histo_gather_hot, dim3(blocks_for(nremrec, kTile)), dim3(kBlock), 0, st, ntouched, nremrec,
                     e->h_tl, e->h_start, e->h_ex, e->h_hotoff, e->h_seen0, e->h_pbase, e->h_pi0, e->h_geo,
                     e->n_geo, As, Bs, Ao, Bo);
  // (the value passes take the top 40 bits of the ordered value; k_fix_ties then orders the rare
  // runs that share them by the full 64 bits -- the same stable order a 64-bit sort gives)
  RadixPass passes[16];
  int np = 0;
  np = make_passes(passes, false, 24, 40);
  int pbits = 1;
  while (pbits < 32 && (1ull << pbits) < npieces) pbits++;
  np += make_passes(passes + np, true, 32, pbits);
  const bool fl2 = radix_sort(Ao, Bo, e->hA2, e->hB2, nremrec, passes, np, e->rs, st,
                              e->timing ? &e->rstat_h : nullptr);
  uint64_t* const SA = fl2 ? e->hA2 : Ao;  // sorted pieces
  uint64_t* const SB = fl2 ? e->hB2 : Bo;
  uint64_t* MA = fl2 ? Ao : e->hA2;        // per-round merged segments
  uint64_t* MB = fl2 ? Bo : e->hB2;
  {
    // a long run out of full-value order (rare): the whole (piece, 64-bit value) sort, queued
    // behind a device flag so no host round trip decides it; an even pass count leaves the
    // result in (SA, SB) whether it runs or not (MA / MB are free until the rounds)
    uint32_t* const resort = e->h_cnt + 14;
    VN_HIP_CHECK(hipMemsetAsync(resort, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_fix_ties, dim3(blocks_for(nremrec, 256)), dim3(256), 0, st, SA, SB, nremrec, resort);
    RadixPass full[16];
    int nf = 0;
    const int npb = (pbits + 7) / 8;
    if ((8 + npb) % 2) {  // 4 passes of 6 bits over the low 24 value bits: an even total
      for (int q = 0; q < 4; q++) full[nf++] = RadixPass{false, 6 * q, 6};
      nf += make_passes(full + nf, false, 24, 40);
    } else {
      nf += make_passes(full + nf, false, 0, 64);
    }
    nf += make_passes(full + nf, true, 32, pbits);
    if (nf % 2) throw std::logic_error("conditional re-sort needs an even pass count");
    (void)radix_sort(SA, SB, MA, MB, nremrec, full, nf, e->rs, st, nullptr, resort);
  }
  const uint64_t* PA = SA;
  const uint64_t* PB = SB;
  hipLaunchKernelGGL(k_seg_mark, dim3(blocks_for(nremrec, 256)), dim3(256), 0, st, nremrec, PB, e->p_start,
                     e->p_end, nullptr, nullptr);
  if (fork) {
    ensure_aux_streams(e, true, false);
    VN_HIP_CHECK(hipEventRecord(e->ev_fork3, st));
    if (e->set_pending) {
      VN_HIP_CHECK(hipStreamWaitEvent(e->side, e->ev_fork3, 0));
      set_finish(e);
    }
    VN_HIP_CHECK(hipStreamWaitEvent(st, e->ev_join4, 0));  // the hot rounds start from the prefixes' state
  }

  const uint32_t nrem = nhot + nwarm;
  // round j merges piece j of every key of the list that has one
  auto rounds = [&](const uint32_t* list, uint32_t nkeys, uint32_t maxp) {
    histo_rounds(e, list, nkeys, maxp, nremrec, nrem, PA, PB, MA, MB, impw, st);
  };
  // the hot keys' leading (small) pieces: merged by one workgroup per key in one launch (every
  // one fits kFuseMaxL with the centroids, by the geometry); the round loop then starts at each
  // key's next piece
  uint32_t hot_rounds = maxp_hot;
  if (nhot && e->fuse_pieces) {
    hot_rounds = maxp_hot_left;
    if (e->fz_cap < nhot) {
      VN_HIP_CHECK(hipStreamSynchronize(st));
      for (void* q : {(void*)e->fz_val, (void*)e->fz_w, (void*)e->fz_k, (void*)e->fz_done})
        if (q) VN_HIP_CHECK(hipFree(q));
      const uint32_t cap = std::max<uint32_t>(nhot, 256);
      VN_HIP_CHECK(hipMalloc(&e->fz_val, (uint64_t)cap * kFuseMaxL * sizeof(double)));
      VN_HIP_CHECK(hipMalloc(&e->fz_w, (uint64_t)cap * kFuseMaxL * sizeof(double)));
      VN_HIP_CHECK(hipMalloc(&e->fz_k, (uint64_t)cap * kFuseMaxL * sizeof(double)));
      VN_HIP_CHECK(hipMalloc(&e->fz_done, (uint64_t)cap * sizeof(uint32_t)));
      e->fz_cap = cap;
    }
    histo_rounds_fused(e, e->h_hotlist, nhot, PA, PB, impw, e->fz_val, e->fz_w, e->fz_k, st, e->fuse_pieces,
                       e->fz_done);
    hipLaunchKernelGGL(k_fuse_shift, dim3(blocks_for(nhot, 256)), dim3(256), 0, st, e->h_hotlist, nhot, e->fz_done,
                       e->h_pbase, e->h_pcnt);
  }
  // the warm keys' rounds start from their exact prefixes (the replay stream), which at C4 are
  // done about when the remainder sort is: hot and warm keys then share one loop of
  // max(hot, warm) rounds instead of hot rounds followed by warm rounds (the fused launch above
  // needs only the hot prefixes: it runs beside the tail of the replay)
  if (fork) VN_HIP_CHECK(hipStreamWaitEvent(st, e->ev_join3, 0));
  if (nhot && nwarm) {
    VN_HIP_CHECK(hipMemcpyAsync(e->h_hotlist + nhot, e->h_warmlist, (uint64_t)nwarm * sizeof(uint32_t),
                                hipMemcpyDeviceToDevice, st));
    rounds(e->h_hotlist, nhot + nwarm, std::max(hot_rounds, maxp_warm));
  } else if (nhot) {
    rounds(e->h_hotlist, nhot, hot_rounds);
  } else if (nwarm) {
    rounds(e->h_warmlist, nwarm, maxp_warm);
  }
  hipLaunchKernelGGL(k_clear_flags, dim3(blocks_for(ntouched, 256)), dim3(256), 0, st, ntouched, e->h_tl, e->h_bt);
#endif  // VN_FAST_MODE
}

}  // namespace vn

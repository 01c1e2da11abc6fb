// flush.hip -- Worker.Flush (worker.go:271-298) and the per-sampler flush math.
//
//   Counter.Flush (samplers.go:137-148): float64(value)            -> int64 value out
//   Gauge.Flush   (203-214): value
//   Histo.Flush   (373-498): Local* statistics + MergingDigest.Quantile (merging_digest.go:283-313)
//   Set.Flush     (282-293): Sketch.Estimate (hyperloglog.go:203-227) with Go's math.Log / math.Pow
//                 restated bit-for-bit, including registers.sumAndZeros' ez bug (registers.go:88-104)
// Only slots touched in the window are emitted (Upsert semantics), in ascending slot order.
// Afterwards the touched slots are reset to their empty-window state (the map swap at
// worker.go:277-284).
#include "histo.h"

namespace vn {

__global__ void k_flush_counter(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ list,
                                const int64_t* __restrict__ cval, int64_t* __restrict__ out) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < cnt[0]) out[k] = cval[list[k]];
}
__global__ void k_flush_gauge(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ list,
                              const double* __restrict__ gval, double* __restrict__ out) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < cnt[0]) out[k] = gval[list[k]];
}

// MergingDigest.Quantile over the slot's centroid tile
__device__ double td_quantile(const double* m, const double* w, uint32_t nc, double main_weight, double dmin,
                              double dmax, double quantile) {
  double q = dmul(quantile, main_weight);
  double wsf = 0.0, lower = dmin;
  for (uint32_t i = 0; i < nc; i++) {
    double upper = (i != nc - 1) ? ddiv(dadd(m[i + 1], m[i]), 2.0) : dmax;
    if (q <= dadd(wsf, w[i])) {
      double prop = ddiv(dsub(q, wsf), w[i]);
      return dadd(lower, dmul(prop, dsub(upper, lower)));
    }
    wsf = dadd(wsf, w[i]);
    lower = upper;
  }
  return __builtin_nan("");
}

// MergingDigest.CDF (merging_digest.go:247-279)
__device__ double td_cdf(const double* m, const double* w, uint32_t nc, double main_weight, double dmin, double dmax,
                         double value) {
  if (nc == 0) return __builtin_nan("");
  if (value <= dmin) return 0.0;
  if (value >= dmax) return 1.0;
  double wsf = 0.0, lower = dmin;
  for (uint32_t i = 0; i < nc; i++) {
    const double upper = (i != nc - 1) ? ddiv(dadd(m[i + 1], m[i]), 2.0) : dmax;
    if (value < upper) {
      wsf = dadd(wsf, ddiv(dmul(w[i], dsub(value, lower)), dsub(upper, lower)));
      return ddiv(wsf, main_weight);
    }
    wsf = dadd(wsf, w[i]);
    lower = upper;
  }
  return __builtin_nan("");
}

// Quantile (kind 0) / CDF (kind 1) of slot[i]'s digest at arg[i] (pending temps already merged)
__global__ void k_histo_query(uint64_t n, int kind, const uint32_t* __restrict__ slot, const double* __restrict__ arg,
                              const double* __restrict__ hst, const uint32_t* __restrict__ hncent,
                              const uint8_t* __restrict__ hcur, const double* __restrict__ cm0,
                              const double* __restrict__ cm1, const double* __restrict__ cw0,
                              const double* __restrict__ cw1, uint32_t capc, double* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slot[i];
  const double* h = hst + (uint64_t)s * VN_HISTO_STATS;
  const uint8_t c = hcur[s];
  const double* m = (c ? cm1 : cm0) + (uint64_t)s * capc;
  const double* w = (c ? cw1 : cw0) + (uint64_t)s * capc;
  out[i] = kind == 0 ? td_quantile(m, w, hncent[s], h[7], h[5], h[6], arg[i])
                     : td_cdf(m, w, hncent[s], h[7], h[5], h[6], arg[i]);
}

// Keys whose last replay left a flush-ready digest adopt it (one lane per key); the others
// with pending temps are listed for a real mergeAllTemps.
__global__ void k_histo_adopt(uint32_t n, const uint32_t* __restrict__ keys, uint32_t* __restrict__ hspn,
                              const double* __restrict__ hspw, uint8_t* __restrict__ hcur,
                              uint32_t* __restrict__ hncent, double* __restrict__ hst, uint32_t* __restrict__ hpend,
                              uint32_t* __restrict__ flag) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t s = keys[k];
  const uint32_t fn = hspn[s];
  if (fn) {
    hcur[s] ^= 1;
    hncent[s] = fn;
    hst[(uint64_t)s * VN_HISTO_STATS + 7] = hspw[s];
    hpend[s] = 0;
    hspn[s] = 0;
  }
  flag[k] = !fn && hpend[s] > 0;
}
__global__ void k_gather_u32(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ idx,
                             const uint32_t* __restrict__ src, uint32_t* __restrict__ dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cnt[0]) dst[i] = src[idx[i]];
}

// mergeAllTemps of the given keys (Quantile / CDF / GobEncode merge pending temps first)
void histo_merge_pending(vn_engine* e, const uint32_t* dev_keys, uint32_t nkeys) {
  if (!nkeys) return;
  hipLaunchKernelGGL(k_histo_adopt, dim3(blocks_for(nkeys, 256)), dim3(256), 0, e->st, nkeys, dev_keys, e->hspn,
                     e->hspw, e->hcur, e->hncent, e->hst, e->hpend, e->hm_flag);
  compact_flags(e->hm_flag, e->hm_pos, e->hm_idx, e->hm_cnt, nkeys, e->ss, e->st);
  hipLaunchKernelGGL(k_gather_u32, dim3(blocks_for(nkeys, 256)), dim3(256), 0, e->st, e->hm_cnt, e->hm_idx, dev_keys,
                     e->hm_list);
  ExactCtx xc{};
  xc.nkeys = nkeys;
  xc.keys = e->hm_list;
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
  xc.hspn = e->hspn;
  xc.hspw = e->hspw;
  xc.hpv = e->hpv;
  xc.hpw = e->hpw;
  xc.err = e->h_err;
  xc.flush_mode = 1;
  histo_exact_replay_list(xc, e->hm_cnt, nkeys, e->st);
}

void histo_query(vn_engine* e, int kind, const uint32_t* dev_slot, const double* dev_arg, uint64_t n, double* dev_out) {
  hipLaunchKernelGGL(k_histo_query, dim3(blocks_for(n, 256)), dim3(256), 0, e->st, n, kind, dev_slot, dev_arg, e->hst,
                     e->hncent, e->hcur, e->cmean[0], e->cmean[1], e->cw[0], e->cw[1], e->cap_cent, dev_out);
}

// Histo.Flush statistics and Quantile per percentile (merging_digest.go:283-313): one wave
// per key.  Quantile's walk compares q against the running weight sum P_i = P_(i-1) + w_i and
// stops at the first i with q <= P_i; the engine forms the same P_i (a wave scan when every
// weight is an integer and the total stays below 2^53 -- every partial sum is then exact, so
// the association does not matter; otherwise lane 0 folds them in order), then each
// percentile's lane binary-searches P and interpolates exactly as the walk would.
constexpr uint32_t kQWaves = 4;
__global__ __launch_bounds__(64 * kQWaves) void k_flush_histo(
    const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ list, const double* __restrict__ hst,
    const uint32_t* __restrict__ hncent, const uint8_t* __restrict__ hcur, const double* __restrict__ cm0,
    const double* __restrict__ cm1, const double* __restrict__ cw0, const double* __restrict__ cw1, uint32_t capc,
    const double* __restrict__ pct, uint32_t npct, const uint8_t* __restrict__ qmask, double* __restrict__ out_stats,
    double* __restrict__ out_q) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t k = blockIdx.x * kQWaves + wv;
  if (k >= cnt[0]) return;
  double* P = reinterpret_cast<double*>(smem) + (uint64_t)wv * capc;
  const uint32_t s = list[k];
  const double* h = hst + (uint64_t)s * VN_HISTO_STATS;
  if (lane < VN_HISTO_STATS) out_stats[(uint64_t)k * VN_HISTO_STATS + lane] = h[lane];
  if (qmask && !qmask[s]) {  // percentiles=nil for this histogram (flusher.go:41-48,181-188)
    if (lane < npct) out_q[(uint64_t)k * npct + lane] = __builtin_nan("");
    return;
  }
  const uint8_t c = hcur[s];
  const double* m = (c ? cm1 : cm0) + (uint64_t)s * capc;
  const double* w = (c ? cw1 : cw0) + (uint64_t)s * capc;
  const uint32_t nc = hncent[s];
  const double mainW = h[7];
  bool wint = mainW <= 9007199254740992.0;
  for (uint32_t j = lane; j < nc; j += 64) {
    const double x = w[j];
    P[j] = x;
    wint &= x == __builtin_trunc(x);
  }
  wint = __all(wint);
  wave_lds_sync();
  if (wint) {
    double carry = 0.0;
    for (uint32_t b = 0; b < nc; b += 64) {
      double v = b + lane < nc ? P[b + lane] : 0.0;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_up(v, d, 64);
        v = (int)lane >= d ? dadd(v, o) : v;
      }
      if (b + lane < nc) P[b + lane] = dadd(carry, v);
      carry = dadd(carry, __shfl(v, 63, 64));
    }
  } else if (lane == 0) {
    double run = 0.0;
    for (uint32_t j = 0; j < nc; j++) {
      run = dadd(run, P[j]);
      P[j] = run;
    }
  }
  wave_lds_sync();
  if (lane < npct) {
    const double q = dmul(pct[lane], mainW);
    uint32_t lo = 0, hi = nc;  // first i with q <= P[i]
    while (lo < hi) {
      const uint32_t md = (lo + hi) >> 1;
      if (q <= P[md]) hi = md;
      else lo = md + 1;
    }
    double r = __builtin_nan("");
    if (lo < nc) {
      const uint32_t i = lo;
      const double wsf = i ? P[i - 1] : 0.0;
      const double lower = i ? ddiv(dadd(m[i], m[i - 1]), 2.0) : h[5];
      const double upper = (i != nc - 1) ? ddiv(dadd(m[i + 1], m[i]), 2.0) : h[6];
      const double prop = ddiv(dsub(q, wsf), w[i]);
      r = dadd(lower, dmul(prop, dsub(upper, lower)));
    }
    out_q[(uint64_t)k * npct + lane] = r;
  }
}

// Sketch.Estimate: one workgroup per touched set slot
__global__ __launch_bounds__(kBlock) void k_flush_set(const uint32_t* __restrict__ cnt,
                                                      const uint32_t* __restrict__ list,
                                                      const uint8_t* __restrict__ mode,
                                                      const uint8_t* __restrict__ base,
                                                      const uint32_t* __restrict__ lc, const uint32_t* __restrict__ tc,
                                                      const uint32_t* __restrict__ tmp,
                                                      const uint32_t* __restrict__ arena,
                                                      const uint8_t* __restrict__ emask,
                                                      uint64_t* __restrict__ out_est, uint8_t* __restrict__ out_sparse) {
  __shared__ double s_tmp[4];
  __shared__ uint32_t s_red[4];
  const uint32_t k = blockIdx.x, t = threadIdx.x;
  if (k >= cnt[0]) return;
  const uint32_t s = list[k];
  if (emask && !emask[s]) {  // a set a local veneur only forwards (flusher.go:206-211)
    if (t == 0) {
      out_est[k] = 0;
      out_sparse[k] = mode[s] == 0;
    }
    return;
  }
  const uint32_t* ar = arena + (uint64_t)s * kArenaWords;
  if (mode[s] == 0) {
    // mergeSparse then linearCount(2^25, 2^25 - count)   (hyperloglog.go:204-207, utils.go:53-56)
    const uint32_t n = lc[s], ntmp = tc[s];
    uint32_t extra = 0;
    if (t < ntmp) {
      uint32_t c = tmp[(uint64_t)s * kTmpCap + t];
      uint32_t l = 0, h = n;
      while (l < h) {
        uint32_t m = (l + h) >> 1;
        if (ar[m] < c) l = m + 1;
        else h = m;
      }
      extra = !(l < n && ar[l] == c);
    }
    extra = block_allreduce_u32_sum(extra, s_red);
    if (t == 0) {
      uint32_t count = n + extra;
      double fm = (double)kHllMP;
      double est = dmul(fm, log_go(ddiv(fm, (double)(kHllMP - count))));
      out_est[k] = f64_to_u64_go(est);
      out_sparse[k] = 1;
    }
    return;
  }
  // dense: sum = sum 2^-(b+reg) (exact in any order: all terms are multiples of 2^-(b+15)
  // and the total stays below 2^(14-b)); ez counts zero HIGH nibbles twice when b == 0.
  const uint32_t b = base[s];
  const uint8_t* regs = reinterpret_cast<const uint8_t*>(ar);
  double sum = 0.0;
  uint32_t ezh = 0;
  for (uint32_t i = t; i < kHllM; i += kBlock) {
    uint32_t v = regs[i];
    sum = dadd(sum, ldexp_go(1.0, -(int)(b + v)));
    if ((i & 1) == 0 && b + v == 0) ezh++;  // even register = high nibble of tailcut byte i/2
  }
  sum = block_allreduce(sum, s_tmp, SumOp());
  ezh = block_allreduce_u32_sum(ezh, s_red);
  if (t == 0) {
    const double m = (double)kHllM;
    const double ez = (double)(2u * ezh);
    const double alpha = ddiv(0.7213, dadd(1.0, ddiv(1.079, m)));  // alpha(m), utils.go:34-44
    double est;
    if (b == 0) {
      double zl = log_go(dadd(ez, 1.0));  // beta14, utils.go:10-20
      double beta = dmul(-0.370393911, ez);
      beta = dadd(beta, dmul(0.070471823, zl));
      beta = dadd(beta, dmul(0.17393686, powi_go(zl, 2)));
      beta = dadd(beta, dmul(0.16339839, powi_go(zl, 3)));
      beta = dadd(beta, dmul(-0.09237745, powi_go(zl, 4)));
      beta = dadd(beta, dmul(0.03738027, powi_go(zl, 5)));
      beta = dadd(beta, dmul(-0.005384159, powi_go(zl, 6)));
      beta = dadd(beta, dmul(0.00042419, powi_go(zl, 7)));
      est = dadd(ddiv(dmul(dmul(alpha, m), dsub(m, ez)), dadd(sum, beta)), 0.5);
    } else {
      est = dadd(ddiv(dmul(dmul(alpha, m), m), sum), 0.5);
    }
    out_est[k] = f64_to_u64_go(dadd(est, 0.5));
    out_sparse[k] = 0;
  }
}

// ---- reset of the touched slots (new window)
__global__ void k_reset_counter(const uint32_t* cnt, const uint32_t* list, int64_t* cval, uint32_t* touch) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt[0]) return;
  cval[list[k]] = 0;
  touch[list[k]] = 0;
}
__global__ void k_reset_gauge(const uint32_t* cnt, const uint32_t* list, uint64_t* gseq, double* gval,
                              uint32_t* touch) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt[0]) return;
  gseq[list[k]] = 0;
  gval[list[k]] = 0.0;
  touch[list[k]] = 0;
}
__device__ __forceinline__ void histo_empty(double* h) {
  h[0] = 0.0;       // LocalWeight
  h[1] = kInf;      // LocalMin  (samplers.go:365)
  h[2] = -kInf;     // LocalMax  (366)
  h[3] = 0.0;       // LocalSum
  h[4] = 0.0;       // LocalReciprocalSum
  h[5] = kInf;      // digest min (merging_digest.go:81)
  h[6] = -kInf;     // digest max (82)
  h[7] = 0.0;       // digest weight
}
__global__ void k_reset_histo(const uint32_t* cnt, const uint32_t* list, double* hst, uint32_t* hncent,
                              uint32_t* touch, uint32_t* hseen, uint32_t* hpend,
                              uint32_t* hspn) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt[0]) return;
  uint32_t s = list[k];
  histo_empty(hst + (uint64_t)s * VN_HISTO_STATS);
  hncent[s] = 0;
  touch[s] = 0;
  hseen[s] = 0;
  hpend[s] = 0;
  hspn[s] = 0;
}
__global__ void k_reset_set(const uint32_t* cnt, const uint32_t* list, uint8_t* mode, uint8_t* base, uint32_t* nz,
                            uint32_t* lc, uint32_t* lb, uint32_t* last, uint32_t* tc, uint32_t* touch) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt[0]) return;
  uint32_t s = list[k];
  mode[s] = 0;
  base[s] = 0;
  nz[s] = kHllM;
  lc[s] = 0;
  lb[s] = 0;
  last[s] = 0;
  tc[s] = 0;
  touch[s] = 0;
}
__global__ void k_init_histo(uint32_t n, double* hst) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n) histo_empty(hst + (uint64_t)s * VN_HISTO_STATS);
}
__global__ void k_init_set(uint32_t n, uint32_t* nz) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n) nz[s] = kHllM;
}

void init_state(vn_engine* e) {
  hipStream_t st = e->st;
  if (e->cap[VN_HISTO])
    hipLaunchKernelGGL(k_init_histo, dim3(blocks_for(e->cap[VN_HISTO], 256)), dim3(256), 0, st, e->cap[VN_HISTO],
                       e->hst);
  if (e->cap[VN_SET])
    hipLaunchKernelGGL(k_init_set, dim3(blocks_for(e->cap[VN_SET], 256)), dim3(256), 0, st, e->cap[VN_SET], e->snz);
}

void flush_all(vn_engine* e, vn_flush_result* out, const uint8_t* histo_qmask, const uint8_t* set_emask) {
  hipStream_t st = e->st;
  // per-slot masks of the flush (vn_flush_masked): which histograms get percentiles, which sets
  // an estimate; null = all
  const uint8_t* qmask = nullptr;
  const uint8_t* emask = nullptr;
  if (histo_qmask && e->cap[VN_HISTO]) {
    VN_HIP_CHECK(hipMemcpyAsync(e->f_hmask, histo_qmask, e->cap[VN_HISTO], hipMemcpyHostToDevice, st));
    qmask = e->f_hmask;
  }
  if (set_emask && e->cap[VN_SET]) {
    VN_HIP_CHECK(hipMemcpyAsync(e->f_smask, set_emask, e->cap[VN_SET], hipMemcpyHostToDevice, st));
    emask = e->f_smask;
  }
  uint32_t* touch[VN_NCLASS] = {e->ctouch, e->gtouch, e->htouch, e->stouch};
  for (int c = 0; c < VN_NCLASS; c++) {
    if (!e->cap[c]) {
      VN_HIP_CHECK(hipMemsetAsync(e->f_cnt + c, 0, sizeof(uint32_t), st));
      continue;
    }
    compact_flags(touch[c], e->f_pos, e->f_list[c], e->f_cnt + c, e->cap[c], e->ss, st);
  }
  const uint32_t cc = e->cap[VN_COUNTER], cg = e->cap[VN_GAUGE], ch = e->cap[VN_HISTO], cs = e->cap[VN_SET];
  if (cc)
    hipLaunchKernelGGL(k_flush_counter, dim3(blocks_for(cc, 256)), dim3(256), 0, st, e->f_cnt + 0, e->f_list[0],
                       e->cval, e->f_cval);
  if (cg)
    hipLaunchKernelGGL(k_flush_gauge, dim3(blocks_for(cg, 256)), dim3(256), 0, st, e->f_cnt + 1, e->f_list[1],
                       e->gval, e->f_gval);
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 4, e->f_cnt, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
  const uint32_t n[4] = {e->hf_cnt[4], e->hf_cnt[5], e->hf_cnt[6], e->hf_cnt[7]};
  // Results to pinned host memory.  Counter and gauge results are final after the sync: their
  // copies run on the side stream at once.  The sets' estimates run first on the main stream
  // (all CUs, ~0.15 ms), their copies then follow on the side stream while the main stream
  // flushes the histograms and copies their (larger) results.
  hipStream_t s2 = e->timing || !e->st2 ? st : e->st2;
  for (int c : {0, 1})
    if (n[c])
      VN_HIP_CHECK(hipMemcpyAsync(e->hf_list[c], e->f_list[c], n[c] * sizeof(uint32_t), hipMemcpyDeviceToHost, s2));
  if (n[0]) VN_HIP_CHECK(hipMemcpyAsync(e->hf_cval, e->f_cval, n[0] * 8, hipMemcpyDeviceToHost, s2));
  if (n[1]) VN_HIP_CHECK(hipMemcpyAsync(e->hf_gval, e->f_gval, n[1] * 8, hipMemcpyDeviceToHost, s2));
  if (cs && n[3]) {
    hipLaunchKernelGGL(k_flush_set, dim3(n[3]), dim3(kBlock), 0, st, e->f_cnt + 3, e->f_list[3], e->smode, e->sbase,
                       e->slc, e->stc, e->stmp, e->sarena, emask, e->f_sest, e->f_ssparse);
    if (s2 != st) {
      VN_HIP_CHECK(hipEventRecord(e->ev_fork, st));
      VN_HIP_CHECK(hipStreamWaitEvent(s2, e->ev_fork, 0));
    }
    VN_HIP_CHECK(hipMemcpyAsync(e->hf_list[3], e->f_list[3], n[3] * sizeof(uint32_t), hipMemcpyDeviceToHost, s2));
    VN_HIP_CHECK(hipMemcpyAsync(e->hf_sest, e->f_sest, n[3] * 8, hipMemcpyDeviceToHost, s2));
    VN_HIP_CHECK(hipMemcpyAsync(e->hf_ssparse, e->f_ssparse, n[3], hipMemcpyDeviceToHost, s2));
  }
  if (ch && n[2]) {
    // Quantile() first merges the pending temps (merging_digest.go:287)
    histo_merge_pending(e, e->f_list[2], n[2]);
    hipLaunchKernelGGL(k_flush_histo, dim3(blocks_for(n[2], kQWaves)), dim3(64 * kQWaves),
                       sizeof(double) * kQWaves * e->cap_cent, st, e->f_cnt + 2, e->f_list[2],
                       e->hst, e->hncent, e->hcur, e->cmean[0], e->cmean[1], e->cw[0], e->cw[1], e->cap_cent,
                       e->d_pct, e->cfg.n_percentiles, qmask, e->f_hstats, e->f_hq);
    VN_HIP_CHECK(hipMemcpyAsync(e->hf_list[2], e->f_list[2], n[2] * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    VN_HIP_CHECK(hipMemcpyAsync(e->hf_hstats, e->f_hstats, (size_t)n[2] * VN_HISTO_STATS * 8, hipMemcpyDeviceToHost, st));
    if (e->cfg.n_percentiles)
      VN_HIP_CHECK(
          hipMemcpyAsync(e->hf_hq, e->f_hq, (size_t)n[2] * e->cfg.n_percentiles * 8, hipMemcpyDeviceToHost, st));
  }
  if (s2 != st) {  // the resets below follow the side stream's reads
    VN_HIP_CHECK(hipEventRecord(e->ev_join, s2));
    VN_HIP_CHECK(hipStreamWaitEvent(st, e->ev_join, 0));
  }
  // new window: reset the touched slots
  if (cc)
    hipLaunchKernelGGL(k_reset_counter, dim3(blocks_for(cc, 256)), dim3(256), 0, st, e->f_cnt + 0, e->f_list[0],
                       e->cval, e->ctouch);
  if (cg)
    hipLaunchKernelGGL(k_reset_gauge, dim3(blocks_for(cg, 256)), dim3(256), 0, st, e->f_cnt + 1, e->f_list[1],
                       e->gseq, e->gval, e->gtouch);
  if (ch)
    hipLaunchKernelGGL(k_reset_histo, dim3(blocks_for(ch, 256)), dim3(256), 0, st, e->f_cnt + 2, e->f_list[2], e->hst,
                       e->hncent, e->htouch, e->hseen, e->hpend, e->hspn);
  if (cs)
    hipLaunchKernelGGL(k_reset_set, dim3(blocks_for(cs, 256)), dim3(256), 0, st, e->f_cnt + 3, e->f_list[3], e->smode,
                       e->sbase, e->snz, e->slc, e->slb, e->slast, e->stc, e->stouch);
  VN_HIP_CHECK(hipStreamSynchronize(st));
  out->n_counter = n[0];
  out->counter_slot = e->hf_list[0];
  out->counter_value = e->hf_cval;
  out->n_gauge = n[1];
  out->gauge_slot = e->hf_list[1];
  out->gauge_value = e->hf_gval;
  out->n_histo = n[2];
  out->histo_slot = e->hf_list[2];
  out->histo_stats = e->hf_hstats;
  out->histo_quantiles = e->hf_hq;
  out->n_percentiles = e->cfg.n_percentiles;
  out->n_set = n[3];
  out->set_slot = e->hf_list[3];
  out->set_estimate = e->hf_sest;
  out->set_sparse = e->hf_ssparse;
  out->samples_processed = e->processed;
  out->samples_imported = e->imported;
  e->processed = 0;
  e->imported = 0;
  e->seq_base = 0;
}

}  // namespace vn

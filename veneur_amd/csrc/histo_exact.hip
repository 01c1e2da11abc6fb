// histo_exact.hip -- bit-faithful emulation of MergingDigest's incremental merge.
//
// For every key whose window so far holds at most `exact_threshold` samples the engine
// replays tdigest/merging_digest.go exactly: samples are Add()ed (97-118) into a temp
// buffer of estimateTempBuffer(delta) = 42 entries; when a 43rd arrives the temps are
// sorted by mean and mergeAllTemps (121-205) merges them with the main list (ties take
// the temp first), feeding each element to mergeOne (210-236).  Quantile (283-313)
// merges whatever is pending first.  One wave (64 lanes) owns one key:
//   sort temps       bitonic over (mean, arrival index) in LDS
//   merge positions  binary searches (main before temp only if strictly smaller)
//   mergedWeight     sequential prefix (lane 0) -- Go's exact rounding for any weights;
//                    a wave scan when every weight is an integer (exact either way)
//   k-index          indexEstimate per element in parallel (Go's Asin restated)
//   chain            lane 0 walks the monotone k array: new centroid iff
//                    k(W_incl/T) - k(W_start/T) > 1
//   Welford          one lane per output centroid, in element order, as mergeOne does.
#include "histo.h"

namespace vn {

__device__ __forceinline__ bool is_int_weight(double w) { return w == __builtin_floor(w) && w <= 4503599627370496.0; }

// One merge of the pending temps into main (all 64 lanes of the block-wave participate).
__device__ void exact_merge(const ExactCtx& x, double* mm, double* mw, uint32_t& nm, double& mainW, double* tv,
                            double* tw, uint32_t* ti, uint32_t np, double tempW, double* gm, double* gw, double* kin,
                            uint32_t* starts, uint32_t* s_u) {
  const uint32_t lane = threadIdx.x;
  // ---- sort temps by (ordered mean, arrival index): bitonic over P = next pow2 >= np
  uint32_t P = 1;
  while (P < np) P <<= 1;
  for (uint32_t i = lane; i < P; i += 64) {
    if (i >= np) { tv[i] = kInf; tw[i] = 0.0; }
    ti[i] = i;
  }
  __syncthreads();
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = lane; i < P; i += 64) {
        uint32_t ixj = i ^ j;
        if (ixj > i) {
          uint64_t ka = ordered_bits(tv[i]), kb = ordered_bits(tv[ixj]);
          bool gt = ka > kb || (ka == kb && ti[i] > ti[ixj]);
          bool up = (i & k) == 0;
          if (gt == up) {
            double a = tv[i], b = tw[i];
            uint32_t c = ti[i];
            tv[i] = tv[ixj]; tw[i] = tw[ixj]; ti[i] = ti[ixj];
            tv[ixj] = a; tw[ixj] = b; ti[ixj] = c;
          }
        }
      }
      __syncthreads();
    }
  }
  // ---- merged positions (mergeAllTemps: main first only if strictly smaller)
  const uint32_t m = nm + np;
  for (uint32_t t = lane; t < np; t += 64) {
    double v = tv[t];
    uint32_t l = 0, h = nm;  // #main with mean < v
    while (l < h) {
      uint32_t md = (l + h) >> 1;
      if (mm[md] < v) l = md + 1;
      else h = md;
    }
    gm[t + l] = v;
    gw[t + l] = tw[t];
  }
  for (uint32_t j = lane; j < nm; j += 64) {
    double v = mm[j];
    uint32_t l = 0, h = np;  // #temps with mean <= v
    while (l < h) {
      uint32_t md = (l + h) >> 1;
      if (tv[md] <= v) l = md + 1;
      else h = md;
    }
    gm[j + l] = v;
    gw[j + l] = mw[j];
  }
  __syncthreads();
  const double T = dadd(mainW, tempW);  // totalWeight := td.mainWeight + td.tempWeight
  // ---- mergedWeight prefix
  bool all_int = true;
  for (uint32_t j = lane; j < m; j += 64) all_int &= is_int_weight(gw[j]);
  all_int = __all(all_int) && T <= 4503599627370496.0;
  if (all_int) {
    double carry = 0.0;
    for (uint32_t base = 0; base < m; base += 64) {
      uint32_t j = base + lane;
      double v = j < m ? gw[j] : 0.0;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        double o = __shfl_up(v, d, 64);
        if ((int)lane >= d) v = dadd(v, o);
      }
      if (j < m) kin[j] = dadd(carry, v);
      carry = dadd(carry, __shfl(v, 63, 64));
    }
  } else if (lane == 0) {
    double W = 0.0;
    for (uint32_t j = 0; j < m; j++) {
      W = dadd(W, gw[j]);
      kin[j] = W;
    }
  }
  __syncthreads();
  for (uint32_t j = lane; j < m; j += 64) kin[j] = index_estimate(x.delta, ddiv(kin[j], T));
  __syncthreads();
  // ---- greedy chain (mergeOne), lane 0
  if (lane == 0) {
    uint32_t nc = 0;
    double base = 0.0;
    for (uint32_t j = 0; j < m; j++) {
      if (nc == 0 || dsub(kin[j], base) > 1.0) {
        if (nc >= x.capc) { atomicOr(x.err, 1u); break; }
        starts[nc++] = j;
        base = j ? kin[j - 1] : index_estimate(x.delta, 0.0);
      }
    }
    starts[nc] = m;
    s_u[0] = nc;
  }
  __syncthreads();
  const uint32_t nc = s_u[0];
  // ---- Welford per centroid
  for (uint32_t c = lane; c < nc; c += 64) {
    uint32_t a = starts[c], b = starts[c + 1];
    double mean = gm[a], W = gw[a];
    for (uint32_t j = a + 1; j < b; j++) {
      double wt = gw[j];
      W = dadd(W, wt);
      mean = dadd(mean, ddiv(dmul(dsub(gm[j], mean), wt), W));
    }
    mm[c] = mean;
    mw[c] = W;
  }
  __syncthreads();
  nm = nc;
  mainW = T;
}

// One 64-thread block (one wave) per key.
__global__ __launch_bounds__(64) void k_histo_exact(ExactCtx x) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t k = blockIdx.x, lane = threadIdx.x;
  if (k >= x.nkeys) return;
  const uint32_t capc = x.capc, tcap = x.tcap;
  uint32_t TP = 1;
  while (TP < tcap + 1) TP <<= 1;
  double* mm = reinterpret_cast<double*>(smem);
  double* mw = mm + capc;
  double* tv = mw + capc;
  double* tw = tv + TP;
  double* gm = tw + TP;
  double* gw = gm + capc + TP;
  double* kin = gw + capc + TP;
  uint32_t* ti = reinterpret_cast<uint32_t*>(kin + capc + TP);
  uint32_t* starts = ti + TP;
  uint32_t* s_u = starts + capc + TP + 1;

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
  for (uint32_t j = lane; j < nm; j += 64) {
    mm[j] = cmg[j];
    mw[j] = cwg[j];
  }
  const double* pv = x.hpv + (uint64_t)s * tcap;
  const double* pw = x.hpw + (uint64_t)s * tcap;
  for (uint32_t j = lane; j < np; j += 64) {
    tv[j] = pv[j];
    tw[j] = pw[j];
  }
  __syncthreads();
  double tempW = 0.0;  // td.tempWeight: sequential sum in Add order
  if (lane == 0)
    for (uint32_t j = 0; j < np; j++) tempW = dadd(tempW, tw[j]);
  tempW = __shfl(tempW, 0, 64);

  // Histo.Sample local statistics of the replayed samples (samplers.go:346-356)
  double sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf;
  const uint32_t lo = x.start[s];
  uint32_t pos = 0;
  while (pos < nex) {
    if (np == tcap) {  // Add finds the temp list full: mergeAllTemps first
      exact_merge(x, mm, mw, nm, mainW, tv, tw, ti, np, tempW, gm, gw, kin, starts, s_u);
      np = 0;
      tempW = 0.0;
    }
    const uint32_t r = min(tcap - np, nex - pos);
    for (uint32_t i = lane; i < r; i += 64) {
      double v = bitsd(x.A[lo + pos + i]);
      double wt = (double)(1.0f / __uint_as_float((uint32_t)x.B[lo + pos + i]));
      tv[np + i] = v;
      tw[np + i] = wt;
      sw = dadd(sw, wt);
      mn = min_go(mn, v);
      mx = max_go(mx, v);
      sxw = dadd(sxw, dmul(v, wt));
      srw = dadd(srw, dmul(ddiv(1.0, v), wt));
    }
    __syncthreads();
    if (lane == 0)
      for (uint32_t i = 0; i < r; i++) tempW = dadd(tempW, tw[np + i]);
    tempW = __shfl(tempW, 0, 64);
    np += r;
    pos += r;
  }
  if (final_merge && np > 0) {
    exact_merge(x, mm, mw, nm, mainW, tv, tw, ti, np, tempW, gm, gw, kin, starts, s_u);
    np = 0;
  }
  // ---- write back the key's digest and statistics
  for (uint32_t j = lane; j < nm; j += 64) {
    cmg[j] = mm[j];
    cwg[j] = mw[j];
  }
  double* qv = x.hpv + (uint64_t)s * tcap;
  double* qw = x.hpw + (uint64_t)s * tcap;
  for (uint32_t j = lane; j < np; j += 64) {
    qv[j] = tv[j];
    qw[j] = tw[j];
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
  uint32_t TP = 1;
  while (TP < tcap + 1) TP <<= 1;
  return sizeof(double) * (2 * capc + 2 * TP + 3 * (capc + TP)) + sizeof(uint32_t) * (TP + capc + TP + 1 + 4);
}

void launch_histo_exact(const ExactCtx& x, hipStream_t st) {
  if (!x.nkeys) return;
  size_t sm = exact_smem_bytes(x.capc, x.tcap);
  hipLaunchKernelGGL(k_histo_exact, dim3(x.nkeys), dim3(64), sm, st, x);
}

}  // namespace vn

// split.hip -- keys too hot for one GPU, split over the ranks of the engine's group.
//
// The host deals a split key's records round-robin by the key's window arrival index: record j
// goes to rank j % N, so the i-th split record a rank holds for the key is record
// j = rank + N * i of the key's window (include/veneur_amd.h, "multi-GPU").  Ranks buffer those
// records (vn_ingest_split) and at vn_flush the partial states meet on the key's owner:
//
//   counters  Counter.Sample is an exact wrapping int64 sum: the split counters' values are
//             all-reduced (sum) and the owner keeps the total (Counter.Combine, samplers.go:171-183).
//   sets      bit-identical to one Sketch.Insert over the key's whole ordered stream
//             (hyperloglog.go:168-200): the first J records (gathered) replay on every rank
//             through k_set_segments' exact state machine -- the sparse phase and the switch to
//             dense (toNormal, 152-166) only depend on them -- and the rest runs the dense
//             insert's rebase epochs (set_dense.h) distributed: per epoch an all-reduce min of
//             each zero register's first filler (T_full), an all-reduce min of the first rebase
//             candidate after it, an all-reduce max of the registers below that candidate, then
//             the rebase itself, identically on every rank.  Without a rebase this is one
//             register max-reduction.  A key still sparse after J records with more to come
//             gathers a longer prefix (the trigger sequence is order dependent).
//   histos    Histo's Local* statistics by all-reduce (sum / min / max: float sums re-associated,
//             within 1e-12 relative).  The digest is rebuilt on the owner by the single-GPU
//             hot-key scheme over the whole window: the first histo_hot_prefix
//             records (gathered, in window order) replay MergingDigest.Add exactly, then each
//             geometric piece of the window is one mergeAllTemps -- of the micro-centroids every
//             rank made of its share of the piece (its records sorted and compressed alone at
//             split_compression, tools/split_study.py: within the single-GPU scheme's rank error)
//             -- moved rank -> owner by grouped ncclSend / ncclRecv.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <new>
#include <numeric>

#include "histo.h"

namespace vn {
namespace {

// ---------------------------------------------------------------- scratch
enum ScratchId {
  kSA0, kSB0, kSA1, kSB1, kSSt, kSEn, kSCnt, kSTot, kSStat, kSMin, kSMax, kSFlag, kSPos, kSPA, kSPB, kSPA1, kSPB1,
  kSPs, kSPe, kSIdFlag, kSIdList, kSIdCnt, kSSegS, kSSegE, kSNch, kSChb, kSW, kSWk, kSChSum, kSChPre, kSChSt,
  kSSegT, kSStarts, kSNcNew, kSAccXw, kSAccW, kSHst, kSHnc, kSHcur, kSHspn, kSCm0, kSCm1, kSCw0, kSCw1, kSElem,
  kSSend, kSRecv, kSKeyOff, kSCntMat, kSCntAll, kSOwnList, kSImpA, kSImpB, kSImpA1, kSImpB1, kSImpSlot, kSImpVal,
  kSImpW, kSMicW, kSCP, kSCM, kSPcnt, kSFF, kSW32, kSCand, kSTfull, kSP0, kSDone, kSR2, kSPre, kSDev1,
  kSLocalStats, kSCtr, kSTouch, kSIota, kSFuseV, kSFuseW, kSFuseK,
  kSCtrTouch, kSCtrOwn,  // (the counters' own: their combine runs on st_ctr beside the others)
  kSCount
};

template <class T>
T* sbuf(vn_engine* e, int id, size_t n) {
  SplitState& S = e->sp;
  if (S.scratch.size() < (size_t)kSCount) {
    S.scratch.resize(kSCount, nullptr);
    S.scratch_cap.resize(kSCount, 0);
  }
  const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  if (S.scratch_cap[id] < bytes) {
    if (S.scratch[id]) (void)hipFree(S.scratch[id]);
    S.scratch[id] = nullptr;
    S.scratch_cap[id] = 0;
    VN_HIP_CHECK(hipMalloc(&S.scratch[id], bytes));
    S.scratch_cap[id] = bytes;
  }
  return static_cast<T*>(S.scratch[id]);
}

vn_comm* group_of(vn_engine* e) {
  SplitState& S = e->sp;
  if (S.comm) return S.comm;
  if (!S.solo) {
    vn_comm* c = nullptr;
    if (vn_comm_init_local(1, e->device, &c) != VN_OK) throw std::runtime_error("cannot create a one-rank group");
    S.solo = c;
  }
  return S.solo;
}

// The split engine: a second engine on the same device holding the split histograms and sets
// while they combine (slot k = split key k).  Its own streams and scratch let the whole combine
// -- local preparation, exchange, the owner's replay and rounds -- run beside this engine's
// replay of the ordinary keys; its host waits only wait for its own stream.  The finished
// states move into this engine's slots (k_split_move_*), before this engine's flush reads them.
constexpr uint32_t kMaxSplitKeys = 256;  // per class
__global__ void k_split_errors(uint32_t* __restrict__ from, uint32_t* __restrict__ to);

vn_engine* split_engine(vn_engine* e, uint64_t records) {
  SplitState& S = e->sp;
  if (S.aux && S.aux->max_records >= records) return S.aux;
  if (S.aux) {
    // (its error flags, e.g. a tile overflow of this window's compression, carry over)
    hipLaunchKernelGGL(k_split_errors, dim3(1), dim3(64), 0, S.aux->st, S.aux->h_err, e->h_err);
    VN_HIP_CHECK(hipStreamSynchronize(S.aux->st));
    vn_engine_destroy(S.aux);
    S.aux = nullptr;
  }
  vn_config c = e->cfg;
  c.capacity[VN_COUNTER] = 0;
  c.capacity[VN_GAUGE] = 0;
  c.capacity[VN_HISTO] = kMaxSplitKeys;
  c.capacity[VN_SET] = kMaxSplitKeys;
  c.max_batch_records = std::max<uint64_t>(records, 1u << 21);
  c.max_batch_member_bytes = 0;
  vn_engine* a = nullptr;
  if (vn_engine_create(&c, &a) != VN_OK) {
    const std::string m = a ? a->err : std::string("no engine");
    if (a) vn_engine_destroy(a);
    throw std::runtime_error("cannot create the split engine: " + m);
  }
  S.aux = a;
  a->long_replay = 1024;  // the owner's gathered prefixes (4096 records) are its critical path
  {
    // a stream of its own hardware queue: the engine's high-priority streams (this engine's
    // main and hot-prefix streams) share one, and behind their event waits the combine's short
    // kernels would queue until this engine's replay ends
    hipStream_t s = nullptr;
    VN_HIP_CHECK(hipStreamSynchronize(a->st));
    VN_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    VN_HIP_CHECK(hipStreamDestroy(a->st));
    a->st = s;
  }
  radix_scratch_reserve(a->rs, std::max<uint64_t>(e->cfg.split_max_records, a->max_records));
  uint32_t* iota = sbuf<uint32_t>(e, kSIota, kMaxSplitKeys);
  std::vector<uint32_t> h(kMaxSplitKeys);
  std::iota(h.begin(), h.end(), 0u);
  VN_HIP_CHECK(hipMemcpy(iota, h.data(), kMaxSplitKeys * 4, hipMemcpyHostToDevice));
  if (!S.ev_done) VN_HIP_CHECK(hipEventCreate(&S.ev_done));
  if (!S.ev_histo) VN_HIP_CHECK(hipEventCreate(&S.ev_histo));
  if (!S.ev_set_prefix) VN_HIP_CHECK(hipEventCreate(&S.ev_set_prefix));
  return a;
}

int bits_for_n(uint64_t n) {
  int b = 1;
  while (b < 40 && (1ull << b) < n) b++;
  return b;
}

template <class T>
void to_host_at(int line, T* h, const T* d, size_t n, hipStream_t st) {
  if (!n) return;
  VN_HIP_CHECK(hipMemcpyAsync(h, d, n * sizeof(T), hipMemcpyDeviceToHost, st));
#ifdef VN_SPLIT_TRACE  // diagnostics build (make prof): host clock around every wait of the combine
  const auto a = std::chrono::steady_clock::now();
  VN_HIP_CHECK(hipStreamSynchronize(st));
  const auto b = std::chrono::steady_clock::now();
  fprintf(stderr, "split-trace line %d t %.1f wait %.1f\n", line,
          std::chrono::duration<double, std::micro>(b.time_since_epoch()).count(),
          std::chrono::duration<double, std::micro>(b - a).count());
#else
  (void)line;
  VN_HIP_CHECK(hipStreamSynchronize(st));
#endif
}
#define to_host(...) to_host_at(__LINE__, __VA_ARGS__)
template <class T>
void to_dev(T* d, const T* h, size_t n, hipStream_t st) {
  if (!n) return;
  VN_HIP_CHECK(hipMemcpyAsync(d, h, n * sizeof(T), hipMemcpyHostToDevice, st));
}

// per key: first / one-past-last record of its run in a key-sorted array (key in the high 32
// bits of B); keys without records keep start == end == 0 (memset first)
__global__ void k_key_runs(uint64_t n, const uint64_t* __restrict__ B, uint32_t* __restrict__ start,
                           uint32_t* __restrict__ end) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = (uint32_t)(B[i] >> 32);
  if (i == 0 || (uint32_t)(B[i - 1] >> 32) != k) start[k] = (uint32_t)i;
  if (i == n - 1 || (uint32_t)(B[i + 1] >> 32) != k) end[k] = (uint32_t)(i + 1);
}

// ---------------------------------------------------------------- ingest
__global__ void k_split_validate(vn_split_batch b, uint32_t nh, uint32_t ns, uint32_t* __restrict__ err) {
  const uint64_t nmax = max(b.n_histo, b.n_set);
  uint32_t f = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nmax; i += (uint64_t)gridDim.x * blockDim.x) {
    if (i < b.n_histo) {
      const double v = b.histo_value[i];
      const float r = b.histo_rate[i];
      if (b.histo_key[i] >= nh) f |= 1u;
      if (v != v || v - v != 0.0) f |= 2u;
      if (!(r > 0.0f && r <= 1.0f)) f |= 4u;
    }
    if (i < b.n_set) {
      if (b.set_key[i] >= ns) f |= 1u;
      if (!b.set_hash && b.set_member_off[i + 1] < b.set_member_off[i]) f |= 8u;
    }
  }
  for (int d = 32; d >= 1; d >>= 1) f |= __shfl_xor(f, d, 64);
  if (f && (threadIdx.x & 63) == 0) atomicOr(err, f);
}

__global__ void k_split_set_codes(uint64_t n, const uint32_t* __restrict__ key, const uint32_t* __restrict__ off,
                                  const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ hashes,
                                  uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t x = hashes ? hashes[i] : metro64(bytes + off[i], off[i + 1] - off[i], kMetroSeed);
  out[i] = ((uint64_t)key[i] << 32) | (uint64_t)encode_hash(x);
}

// the split engine's error flags join this engine's (read at its flush)
__global__ void k_split_errors(uint32_t* __restrict__ from, uint32_t* __restrict__ to) {
  if (threadIdx.x == 0 && from[0]) {
    atomicOr(to, from[0]);
    from[0] = 0;
  }
}

// ---------------------------------------------------------------- counters
__global__ void k_sc_gather(uint32_t n, const uint32_t* __restrict__ slot, const int64_t* __restrict__ cval,
                            const uint32_t* __restrict__ touch, int64_t* __restrict__ v, uint32_t* __restrict__ t) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  v[i] = cval[slot[i]];
  t[i] = touch[slot[i]] ? 1u : 0u;
}
__global__ void k_sc_scatter(uint32_t n, const uint32_t* __restrict__ slot, const uint32_t* __restrict__ owner, int me,
                             const int64_t* __restrict__ v, const uint32_t* __restrict__ t, int64_t* __restrict__ cval,
                             uint32_t* __restrict__ touch) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool own = owner[i] == (uint32_t)me;
  cval[slot[i]] = own ? v[i] : 0;
  touch[slot[i]] = own ? t[i] : 0u;
}

// the owner list is on the device since vn_split_keys (kSCtrOwn): nothing to copy or wait for at
// flush, so vn_split_combine returns once the exchange is issued
void split_counter_owners(vn_engine*, hipStream_t) {}
void split_counters(vn_engine* e, vn_comm* c, hipStream_t st) {
  SplitState& S = e->sp;
  const uint32_t H = (uint32_t)S.slot[VN_COUNTER].size();
  if (!H) return;
  int64_t* v = sbuf<int64_t>(e, kSCtr, H);
  uint32_t* t = sbuf<uint32_t>(e, kSCtrTouch, H);
  uint32_t* own = sbuf<uint32_t>(e, kSCtrOwn, H);  // (split_counter_owners)
  hipLaunchKernelGGL(k_sc_gather, dim3(blocks_for(H, 256)), dim3(256), 0, st, H, S.d_slot[VN_COUNTER], e->cval,
                     e->ctouch, v, t);
  comm_allreduce(c, v, v, H, kI64, kSum, st);
  comm_allreduce(c, t, t, H, kU32, kMax, st);
  hipLaunchKernelGGL(k_sc_scatter, dim3(blocks_for(H, 256)), dim3(256), 0, st, H, S.d_slot[VN_COUNTER], own, c->rank,
                     v, t, e->cval, e->ctouch);
}

// ---------------------------------------------------------------- histograms
__global__ void k_sh_keys(uint64_t n, const uint32_t* __restrict__ key, const double* __restrict__ val,
                          const float* __restrict__ rate, uint64_t* __restrict__ A, uint64_t* __restrict__ B) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  A[i] = dbits(val[i]);
  B[i] = ((uint64_t)key[i] << 32) | (uint64_t)__float_as_uint(rate[i]);
}

// per key, over its run of the key-sorted records: record count and Histo.Sample's Local*
// statistics (samplers.go:346-356): weight, min, max, sum(x*w), sum(w/x).  Blocks of kStatChunks
// per key (grid y = key) reduce slices of the run into partials; k_sh_stats_fold combines them.
constexpr uint32_t kStatChunks = 64;
__global__ __launch_bounds__(kBlock) void k_sh_stats(const uint32_t* __restrict__ start,
                                                     const uint32_t* __restrict__ end, const uint64_t* __restrict__ A,
                                                     const uint64_t* __restrict__ B, double* __restrict__ part) {
  __shared__ double s_tmp[4];
  const uint32_t k = blockIdx.y, c = blockIdx.x;
  const uint32_t lo = start[k], hi = end[k];
  double sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf;
  for (uint32_t i = lo + c * kBlock + threadIdx.x; i < hi; i += kStatChunks * kBlock) {
    const double x = bitsd(A[i]);
    const double w = (double)(1.0f / __uint_as_float((uint32_t)B[i]));
    sw = dadd(sw, w);
    sxw = dadd(sxw, dmul(x, w));
    srw = dadd(srw, dmul(ddiv(1.0, x), w));
    mn = min_go(mn, x);
    mx = max_go(mx, x);
  }
  sw = block_allreduce(sw, s_tmp, SumOp());
  sxw = block_allreduce(sxw, s_tmp, SumOp());
  srw = block_allreduce(srw, s_tmp, SumOp());
  mn = block_allreduce(mn, s_tmp, MinGoOp());
  mx = block_allreduce(mx, s_tmp, MaxGoOp());
  if (threadIdx.x == 0) {
    double* p = part + ((uint64_t)k * kStatChunks + c) * 5;
    p[0] = sw; p[1] = sxw; p[2] = srw; p[3] = mn; p[4] = mx;
  }
}
__global__ void k_sh_stats_fold(uint32_t H, const uint32_t* __restrict__ start, const uint32_t* __restrict__ end,
                                const double* __restrict__ part, uint64_t* __restrict__ cnt, double* __restrict__ sums,
                                double* __restrict__ mins, double* __restrict__ maxs) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H) return;
  double sw = 0.0, sxw = 0.0, srw = 0.0, mn = kInf, mx = -kInf;
  for (uint32_t c = 0; c < kStatChunks; c++) {
    const double* p = part + ((uint64_t)k * kStatChunks + c) * 5;
    sw = dadd(sw, p[0]);
    sxw = dadd(sxw, p[1]);
    srw = dadd(srw, p[2]);
    mn = min_go(mn, p[3]);
    mx = max_go(mx, p[4]);
  }
  cnt[k] = end[k] - start[k];
  sums[3 * k + 0] = sw;
  sums[3 * k + 1] = sxw;
  sums[3 * k + 2] = srw;
  mins[k] = mn;
  maxs[k] = mx;
}

// one element of a split histogram on its way to the owner
struct SplitElem {
  double x;      // sample value (prefix) or micro-centroid mean
  double w;      // Histo.Sample weight float64(float32(1)/rate), or micro-centroid weight
  uint32_t key;  // split key index
  uint32_t pos;  // prefix: window index j; micro: kMicro | piece
};
constexpr uint32_t kMicro = 0x80000000u;

__device__ __forceinline__ uint32_t geo_piece(const uint64_t* geo, uint32_t ngeo, uint64_t j) {
  uint32_t l = 0, h = ngeo;  // first index with geo[i] > j; piece = that - 1 (j >= geo[0])
  while (l < h) {
    const uint32_t m = (l + h) >> 1;
    if (geo[m] <= j) l = m + 1;
    else h = m;
  }
  return l - 1;
}

// record i of the key-sorted array: prefix flag (window index j < P)
__global__ void k_sh_prefix_flags(uint64_t n, const uint64_t* __restrict__ B, const uint32_t* __restrict__ start,
                                  int me, int N, uint32_t P, uint32_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = (uint32_t)(B[i] >> 32);
  const uint64_t j = (uint64_t)me + (uint64_t)N * (i - start[k]);
  flag[i] = j < P ? 1u : 0u;
}
// prefix records -> elements (at pos[i]), the rest -> (ordered value, piece id << 32 | rate)
__global__ void k_sh_route(uint64_t n, const uint64_t* __restrict__ A, const uint64_t* __restrict__ B,
                           const uint32_t* __restrict__ start, int me, int N, uint32_t P,
                           const uint32_t* __restrict__ pos, const uint64_t* __restrict__ geo, uint32_t ngeo,
                           uint32_t G, SplitElem* __restrict__ pre, uint64_t* __restrict__ PA,
                           uint64_t* __restrict__ PB) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = (uint32_t)(B[i] >> 32);
  const uint64_t j = (uint64_t)me + (uint64_t)N * (i - start[k]);
  const uint32_t p = pos[i];
  if (j < P) {
    SplitElem el;
    el.x = bitsd(A[i]);
    el.w = (double)(1.0f / __uint_as_float((uint32_t)B[i]));
    el.key = k;
    el.pos = (uint32_t)j;
    pre[p] = el;
  } else {
    const uint64_t o = i - p;  // index among the non-prefix records
    const uint32_t id = k * G + geo_piece(geo, ngeo, j);
    PA[o] = ordered_bits(bitsd(A[i]));
    PB[o] = ((uint64_t)id << 32) | (B[i] & 0xffffffffull);
  }
}
// (key, piece) runs of the (id, value)-sorted records -> segment list
__global__ void k_sh_id_flags(uint32_t nid, const uint32_t* __restrict__ ps, const uint32_t* __restrict__ pe,
                              uint32_t* __restrict__ flag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nid) flag[i] = pe[i] > ps[i] ? 1u : 0u;
}
__global__ void k_sh_seg_ranges(uint32_t nseg, const uint32_t* __restrict__ ids, const uint32_t* __restrict__ ps,
                                const uint32_t* __restrict__ pe, uint32_t* __restrict__ ss, uint32_t* __restrict__ se,
                                uint32_t* __restrict__ tl, uint8_t* __restrict__ hcur, double* __restrict__ hst) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nseg) return;
  ss[k] = ps[ids[k]];
  se[k] = pe[ids[k]];
  tl[k] = k;
  hcur[k] = 0;
  double* h = hst + (uint64_t)k * VN_HISTO_STATS;  // empty digest state (flush.hip histo_empty)
  h[0] = 0.0; h[1] = kInf; h[2] = -kInf; h[3] = 0.0; h[4] = 0.0; h[5] = kInf; h[6] = -kInf; h[7] = 0.0;
}
// per key: prefix and micro element counts (cP from the prefix scan, cM from the segments)
__global__ void k_sh_counts(uint32_t H, const uint32_t* __restrict__ kstart, const uint32_t* __restrict__ kend,
                            const uint32_t* __restrict__ ppos, uint64_t n, const uint32_t* __restrict__ hncent,
                            const uint32_t* __restrict__ ids, uint32_t nseg, uint32_t G, uint32_t* __restrict__ cP,
                            uint32_t* __restrict__ cM) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H) return;
  const uint32_t a = kstart[k], b = kend[k];
  cP[k] = (b > a) ? ppos[b] - ppos[a] : 0u;  // ppos = exclusive scan of the prefix flags (n + 1)
  // segments of key k: ids in [k*G, (k+1)*G), contiguous in the sorted id list
  uint32_t l = 0, h = nseg;
  while (l < h) {
    const uint32_t m = (l + h) >> 1;
    if (ids[m] < k * G) l = m + 1;
    else h = m;
  }
  uint32_t m = 0;
  for (uint32_t s = l; s < nseg && ids[s] < (k + 1) * G; s++) m += hncent[s];
  cM[k] = m;
}
// elements into the send buffer at the key's offset: its prefix elements, then its micro-centroids
__global__ void k_sh_pack_prefix(uint64_t npre, const SplitElem* __restrict__ pre, const uint32_t* __restrict__ kstart,
                                 const uint32_t* __restrict__ ppos, const uint64_t* __restrict__ koff,
                                 SplitElem* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npre) return;
  const SplitElem el = pre[i];
  const uint32_t first = ppos[kstart[el.key]];  // prefix elements of the key start here in pre
  out[koff[el.key] + (i - first)] = el;
}
__global__ void k_sh_pack_micro(uint32_t nseg, const uint32_t* __restrict__ ids, uint32_t G,
                                const uint32_t* __restrict__ hncent, const uint32_t* __restrict__ moff,
                                const uint32_t* __restrict__ cP, const uint64_t* __restrict__ koff,
                                const uint32_t* __restrict__ segbase, const double* __restrict__ cm,
                                const double* __restrict__ cw, uint32_t capc, SplitElem* __restrict__ out) {
  const uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  const uint32_t id = ids[s], k = id / G, g = id % G, nc = hncent[s];
  const uint64_t base = koff[k] + cP[k] + (moff[s] - segbase[k]);
  for (uint32_t c = threadIdx.x; c < nc; c += blockDim.x) {
    SplitElem el;
    el.x = cm[(uint64_t)s * capc + c];
    el.w = cw[(uint64_t)s * capc + c];
    el.key = k;
    el.pos = kMicro | g;
    out[base + c] = el;
  }
}
// per key: exclusive scan base of its micro elements in the segment order (first segment's moff)
__global__ void k_sh_segbase(uint32_t H, const uint32_t* __restrict__ ids, uint32_t nseg, uint32_t G,
                             const uint32_t* __restrict__ moff, uint32_t* __restrict__ segbase) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H) return;
  uint32_t l = 0, h = nseg;
  while (l < h) {
    const uint32_t m = (l + h) >> 1;
    if (ids[m] < k * G) l = m + 1;
    else h = m;
  }
  segbase[k] = l < nseg ? moff[l] : 0u;
}

// owner side: received elements -> prefix sort keys (owned key index, j) or micro sort keys
__global__ void k_sh_recv_flags(uint64_t n, const SplitElem* __restrict__ el, uint32_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flag[i] = (el[i].pos & kMicro) ? 0u : 1u;
}
__global__ void k_sh_recv_split(uint64_t n, const SplitElem* __restrict__ el, const uint32_t* __restrict__ pos,
                                const uint32_t* __restrict__ local, const uint32_t* __restrict__ pbase,
                                uint64_t* __restrict__ PreA, uint64_t* __restrict__ PreB, uint64_t* __restrict__ MicA,
                                uint64_t* __restrict__ MicB, double* __restrict__ micw) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const SplitElem e = el[i];
  const uint32_t k = local[e.key];  // owned-key index
  const uint32_t p = pos[i];
  if (!(e.pos & kMicro)) {
    PreA[p] = ((uint64_t)k << 32) | e.pos;
    PreB[p] = i;
  } else {
    const uint64_t o = i - p;
    const uint32_t pid = pbase[k] + (e.pos & ~kMicro);
    MicA[o] = ordered_bits(e.x);
    MicB[o] = ((uint64_t)pid << 32) | (uint64_t)(kTagImport | (uint32_t)o);
    micw[o] = e.w;
  }
}
__global__ void k_sh_pre_gather(uint64_t n, const uint64_t* __restrict__ PreA, const uint64_t* __restrict__ PreB,
                                const SplitElem* __restrict__ el, const uint32_t* __restrict__ oslot,
                                uint32_t* __restrict__ slot, double* __restrict__ val, double* __restrict__ w) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const SplitElem e = el[PreB[i]];
  slot[i] = oslot[(uint32_t)(PreA[i] >> 32)];  // owned-key index -> slot
  val[i] = e.x;
  w[i] = e.w;
}
// owned keys: piece count from the window total; owned key k lives in the split engine's slot k
__global__ void k_sh_owned(uint32_t K, const uint32_t* __restrict__ okeys, const uint64_t* __restrict__ tot, uint32_t P,
                           const uint64_t* __restrict__ geo, uint32_t ngeo, uint32_t* __restrict__ tl,
                           uint32_t* __restrict__ pcnt) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const uint64_t t = tot[okeys[k]];
  tl[k] = k;
  pcnt[k] = t > P ? geo_piece(geo, ngeo, t - 1) + 1 : 0u;
}

// per-slot histogram state of an engine (engine.h), for moving a digest between engines
struct HistoSlots {
  double* hst;
  uint32_t *hncent, *htouch, *hseen, *hpend, *hspn;
  uint8_t* hcur;
  double *cm0, *cm1, *cw0, *cw1, *hspw, *hpv, *hpw;
};
HistoSlots histo_slots(vn_engine* e) {
  return HistoSlots{e->hst,      e->hncent,   e->htouch,   e->hseen, e->hpend, e->hspn, e->hcur, e->cmean[0],
                    e->cmean[1], e->cw[0],    e->cw[1],    e->hspw,  e->hpv,   e->hpw};
}
// owner: the split engine's digest of owned key k moves into this engine's slot of the key, the
// Local* statistics from the all-reduced partials, the digest min/max over all samples (the
// prefix replay was import-tagged); the split engine's slot is left empty for the next window
__global__ __launch_bounds__(256) void k_split_move_histo(const uint32_t* __restrict__ okeys,
                                                          const uint32_t* __restrict__ kslot,
                                                          const uint64_t* __restrict__ tot,
                                                          const double* __restrict__ sums,
                                                          const double* __restrict__ mins,
                                                          const double* __restrict__ maxs, HistoSlots src,
                                                          HistoSlots dst, uint32_t capc, uint32_t tcap,
                                                          uint32_t* __restrict__ err) {
  const uint32_t k = blockIdx.x, h = okeys[k];
  if (tot[h]) {
    const uint32_t s = kslot[h];
    if (threadIdx.x == 0 && dst.htouch[s]) atomicOr(err, kErrSplitTouched);
    const uint64_t fo = (uint64_t)k * capc, to = (uint64_t)s * capc;
    for (uint32_t i = threadIdx.x; i < capc; i += blockDim.x) {
      dst.cm0[to + i] = src.cm0[fo + i];
      dst.cm1[to + i] = src.cm1[fo + i];
      dst.cw0[to + i] = src.cw0[fo + i];
      dst.cw1[to + i] = src.cw1[fo + i];
    }
    for (uint32_t i = threadIdx.x; i < tcap; i += blockDim.x) {
      dst.hpv[(uint64_t)s * tcap + i] = src.hpv[(uint64_t)k * tcap + i];
      dst.hpw[(uint64_t)s * tcap + i] = src.hpw[(uint64_t)k * tcap + i];
    }
    if (threadIdx.x == 0) {
      const double* a = src.hst + (uint64_t)k * VN_HISTO_STATS;
      double* d = dst.hst + (uint64_t)s * VN_HISTO_STATS;
      d[0] = dadd(a[0], sums[3 * h + 0]);
      d[1] = min_go(a[1], mins[h]);
      d[2] = max_go(a[2], maxs[h]);
      d[3] = dadd(a[3], sums[3 * h + 1]);
      d[4] = dadd(a[4], sums[3 * h + 2]);
      d[5] = min_go(a[5], mins[h]);
      d[6] = max_go(a[6], maxs[h]);
      d[7] = a[7];
      dst.hncent[s] = src.hncent[k];
      dst.hcur[s] = src.hcur[k];
      dst.hseen[s] = src.hseen[k];
      dst.hpend[s] = src.hpend[k];
      dst.hspn[s] = src.hspn[k];
      dst.hspw[s] = src.hspw[k];
      dst.htouch[s] = 1;
    }
  }
  if (threadIdx.x == 0) {  // (thread 0 alone read the scalars it clears)
    double* a = src.hst + (uint64_t)k * VN_HISTO_STATS;
    a[0] = 0.0; a[1] = kInf; a[2] = -kInf; a[3] = 0.0; a[4] = 0.0; a[5] = kInf; a[6] = -kInf; a[7] = 0.0;
    src.hncent[k] = 0;
    src.htouch[k] = 0;
    src.hseen[k] = 0;
    src.hpend[k] = 0;
    src.hspn[k] = 0;
  }
}

void split_histos(vn_engine* e, vn_comm* c) {
  vn_engine* a = e->sp.aux;
  hipStream_t st = a->st;
  SplitState& S = e->sp;
  const uint32_t H = (uint32_t)S.slot[VN_HISTO].size();
  if (!H) return;
  const int N = c->nranks, me = c->rank;
  const uint64_t n = S.nh;
  // the exact mode (the default) gathers every record of a split key to its owner, in window
  // order, and replays all of them: the owner's digest is the one a single consumer builds
  const uint32_t P = e->exact_threshold == 0xFFFFFFFFu ? 0xFFFFFFFFu : e->hot_prefix;
  const uint32_t G = e->n_geo;
  if ((uint64_t)H * G >= (1ull << 31)) throw std::invalid_argument("too many split histograms");
  const int kb = bits_for_n(H);

  // 1. own records grouped by key (stable: arrival order inside a key, i.e. window index order)
  uint64_t* A0 = sbuf<uint64_t>(e, kSA0, n);
  uint64_t* B0 = sbuf<uint64_t>(e, kSB0, n);
  uint64_t* A1 = sbuf<uint64_t>(e, kSA1, n);
  uint64_t* B1 = sbuf<uint64_t>(e, kSB1, n);
  uint32_t* kst = sbuf<uint32_t>(e, kSSt, H);
  uint32_t* ken = sbuf<uint32_t>(e, kSEn, H);
  VN_HIP_CHECK(hipMemsetAsync(kst, 0, H * sizeof(uint32_t), st));
  VN_HIP_CHECK(hipMemsetAsync(ken, 0, H * sizeof(uint32_t), st));
  const uint64_t *As = A0, *Bs = B0;
  if (n) {
    hipLaunchKernelGGL(k_sh_keys, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, S.hkey, S.hval, S.hrate, A0, B0);
    RadixPass kp[5];
    const int nkp = make_passes(kp, true, 32, kb);
    const bool fl = radix_sort(A0, B0, A1, B1, n, kp, nkp, a->rs, st, nullptr);
    As = fl ? A1 : A0;
    Bs = fl ? B1 : B0;
    hipLaunchKernelGGL(k_key_runs, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, Bs, kst, ken);
  }
  // 2. Local* statistics and counts, all-reduced
  uint64_t* tot = sbuf<uint64_t>(e, kSTot, H);
  double* sums = sbuf<double>(e, kSStat, 3 * (size_t)H);
  double* mins = sbuf<double>(e, kSMin, H);
  double* maxs = sbuf<double>(e, kSMax, H);
  double* spart = sbuf<double>(e, kSLocalStats, (size_t)H * kStatChunks * 5);
  hipLaunchKernelGGL(k_sh_stats, dim3(kStatChunks, H), dim3(kBlock), 0, st, kst, ken, As, Bs, spart);
  hipLaunchKernelGGL(k_sh_stats_fold, dim3(blocks_for(H, 64)), dim3(64), 0, st, H, kst, ken, spart, tot, sums, mins,
                     maxs);
  comm_allreduce(c, tot, tot, H, kU64, kSum, st);
  comm_allreduce(c, sums, sums, 3 * (size_t)H, kF64, kSum, st);
  comm_allreduce(c, mins, mins, H, kF64, kMin, st);
  comm_allreduce(c, maxs, maxs, H, kF64, kMax, st);

  // 3. prefix records (window index < P) as elements; the rest sorted by (key, piece, value)
  uint32_t* flag = sbuf<uint32_t>(e, kSFlag, n + 1);
  uint32_t* ppos = sbuf<uint32_t>(e, kSPos, n + 1);
  SplitElem* pre = sbuf<SplitElem>(e, kSPre, std::min<uint64_t>(n, (uint64_t)H * P) + 1);
  uint64_t* PA = sbuf<uint64_t>(e, kSPA, n);
  uint64_t* PB = sbuf<uint64_t>(e, kSPB, n);
  uint64_t* PA1 = sbuf<uint64_t>(e, kSPA1, n);
  uint64_t* PB1 = sbuf<uint64_t>(e, kSPB1, n);
  uint32_t npre = 0;
  if (n) {
    hipLaunchKernelGGL(k_sh_prefix_flags, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, Bs, kst, me, N, P, flag);
    scan_exclusive_u32(flag, ppos, n, a->ss, st);
    hipLaunchKernelGGL(k_sh_route, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, As, Bs, kst, me, N, P, ppos,
                       e->h_geo, e->n_geo, G, pre, PA, PB);
    to_host(&npre, ppos + n, 1, st);
  } else {
    VN_HIP_CHECK(hipMemsetAsync(ppos, 0, sizeof(uint32_t), st));
  }
  const uint64_t nrest = n - npre;
  const uint32_t nid = H * G;
  uint32_t* ps = sbuf<uint32_t>(e, kSPs, nid);
  uint32_t* pe = sbuf<uint32_t>(e, kSPe, nid);
  VN_HIP_CHECK(hipMemsetAsync(ps, 0, (size_t)nid * 4, st));
  VN_HIP_CHECK(hipMemsetAsync(pe, 0, (size_t)nid * 4, st));
  const uint64_t *SA = PA, *SB = PB;
  if (nrest) {
    // (piece, value) order, the value by its top 40 ordered bits: values that agree there lie
    // within 2^-28 of each other and keep their arrival order -- for a share compressed into
    // micro-centroids (an approximation already) that order is as good as the exact one, and
    // the sort takes 5 value passes instead of 8
    RadixPass pp[16];
    int np = make_passes(pp, false, 24, 40);
    np += make_passes(pp + np, true, 32, bits_for_n(nid));
    const bool fl = radix_sort(PA, PB, PA1, PB1, nrest, pp, np, a->rs, st, nullptr);
    SA = fl ? PA1 : PA;
    SB = fl ? PB1 : PB;
    hipLaunchKernelGGL(k_key_runs, dim3(blocks_for(nrest, 256)), dim3(256), 0, st, nrest, SB, ps, pe);
  }
  // 4. each (key, piece) share compressed alone into micro-centroids
  uint32_t* idflag = sbuf<uint32_t>(e, kSIdFlag, nid + 1);
  uint32_t* idpos = sbuf<uint32_t>(e, kSChb, nid + 1);
  uint32_t* ids = sbuf<uint32_t>(e, kSIdList, nid);
  uint32_t* idcnt = sbuf<uint32_t>(e, kSIdCnt, 1);
  hipLaunchKernelGGL(k_sh_id_flags, dim3(blocks_for(nid, 256)), dim3(256), 0, st, nid, ps, pe, idflag);
  compact_flags(idflag, idpos, ids, idcnt, nid, a->ss, st);
  uint32_t nseg = 0;
  to_host(&nseg, idcnt, 1, st);
  const double dhi = e->cfg.split_compression > 0 ? e->cfg.split_compression : 5.0 * e->cfg.compression;
  uint32_t capc = ((uint32_t)(2.0 * dhi) + 4 + 63) / 64 * 64;
  if (capc > 2048) throw std::invalid_argument("split_compression too large (<= 1000)");
  SegCompress sc;
  sc.nseg = nseg;
  sc.nrec = nrest;
  sc.capc = capc;
  sc.delta = dhi;
  uint32_t* tl = sbuf<uint32_t>(e, kSOwnList, nseg);
  uint32_t* ss = sbuf<uint32_t>(e, kSSegS, nseg);
  uint32_t* se = sbuf<uint32_t>(e, kSSegE, nseg);
  sc.tl = tl;
  sc.start = ss;
  sc.end = se;
  sc.nch = sbuf<uint32_t>(e, kSNch, nseg + 1);
  sc.chb = sbuf<uint32_t>(e, kSDev1, nseg + 1);
  sc.A = SA;
  sc.B = SB;
  const uint64_t maxch = nrest / kHTile + nseg + 1;
  sc.w = sbuf<double>(e, kSW, nrest);
  sc.wk = sbuf<double>(e, kSWk, nrest);
  sc.ch_sum = sbuf<double>(e, kSChSum, maxch);
  sc.ch_pre = sbuf<double>(e, kSChPre, maxch);
  sc.ch_stats = sbuf<double>(e, kSChSt, maxch * kChunkStats);
  sc.seg_T = sbuf<double>(e, kSSegT, nseg);
  sc.starts = sbuf<uint32_t>(e, kSStarts, (size_t)nseg * capc);
  sc.nc_new = sbuf<uint32_t>(e, kSNcNew, nseg + 1);
  sc.acc_xw = sbuf<double>(e, kSAccXw, (size_t)nseg * capc);
  sc.acc_w = sbuf<double>(e, kSAccW, (size_t)nseg * capc);
  sc.hst = sbuf<double>(e, kSHst, (size_t)nseg * VN_HISTO_STATS);
  uint32_t* hnc = sbuf<uint32_t>(e, kSHnc, nseg);
  sc.hncent = hnc;
  uint8_t* hcur = sbuf<uint8_t>(e, kSHcur, nseg);
  sc.hcur = hcur;
  sc.hspn = sbuf<uint32_t>(e, kSHspn, nseg);
  sc.cm0 = sbuf<double>(e, kSCm0, (size_t)nseg * capc);
  sc.cm1 = sbuf<double>(e, kSCm1, (size_t)nseg * capc);
  sc.cw0 = sbuf<double>(e, kSCw0, (size_t)nseg * capc);
  sc.cw1 = sbuf<double>(e, kSCw1, (size_t)nseg * capc);
  sc.err = a->h_err;
  if (nseg) {
#if VN_FAST_MODE
    hipLaunchKernelGGL(k_sh_seg_ranges, dim3(blocks_for(nseg, 256)), dim3(256), 0, st, nseg, ids, ps, pe, ss, se, tl,
                       hcur, sc.hst);
    histo_compress_segments(sc, a->ss, st);
#else
    throw std::logic_error("split histo pieces without the fast mode (VN_FAST_MODE) built");
#endif
  }
  // 5. per key element counts -> send layout grouped by owner
  uint32_t* cP = sbuf<uint32_t>(e, kSCP, H);
  uint32_t* cM = sbuf<uint32_t>(e, kSCM, H);
  uint32_t* moff = sbuf<uint32_t>(e, kSNcNew, nseg + 1);  // (nc_new is free again)
  uint32_t* segbase = sbuf<uint32_t>(e, kSPcnt, H);
  if (nseg) scan_exclusive_u32(hnc, moff, nseg, a->ss, st);
  else VN_HIP_CHECK(hipMemsetAsync(moff, 0, sizeof(uint32_t), st));
  hipLaunchKernelGGL(k_sh_counts, dim3(blocks_for(H, 256)), dim3(256), 0, st, H, kst, ken, ppos, n, hnc, ids, nseg, G,
                     cP, cM);
  hipLaunchKernelGGL(k_sh_segbase, dim3(blocks_for(H, 256)), dim3(256), 0, st, H, ids, nseg, G, moff, segbase);
  std::vector<uint32_t> hcP(H), hcM(H);
  to_host(hcP.data(), cP, H, st);
  to_host(hcM.data(), cM, H, st);
  const std::vector<uint32_t>& owner = S.owner[VN_HISTO];
  std::vector<uint64_t> koff(H), soff(N + 1, 0);
  {
    std::vector<uint32_t> order(H);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return owner[a] < owner[b]; });
    uint64_t o = 0;
    for (uint32_t k : order) {
      koff[k] = o;
      o += (uint64_t)hcP[k] + hcM[k];
      soff[owner[k] + 1] = o;
    }
    for (int p = 1; p <= N; p++) soff[p] = std::max(soff[p], soff[p - 1]);
  }
  const uint64_t nsend = soff[N];
  SplitElem* sendb = sbuf<SplitElem>(e, kSSend, nsend);
  uint64_t* dkoff = sbuf<uint64_t>(e, kSKeyOff, H);
  to_dev(dkoff, koff.data(), H, st);
  if (npre)
    hipLaunchKernelGGL(k_sh_pack_prefix, dim3(blocks_for(npre, 256)), dim3(256), 0, st, (uint64_t)npre, pre, kst, ppos,
                       dkoff, sendb);
  if (nseg)
    hipLaunchKernelGGL(k_sh_pack_micro, dim3(nseg), dim3(256), 0, st, nseg, ids, G, hnc, moff, cP, dkoff, segbase,
                       sc.cm1, sc.cw1, capc, sendb);
  // 6. element counts rank -> rank, then the personalised exchange (grouped send / recv)
  uint64_t* cmat = sbuf<uint64_t>(e, kSCntMat, N);
  uint64_t* call = sbuf<uint64_t>(e, kSCntAll, (size_t)N * N);
  std::vector<uint64_t> mine(N);
  for (int p = 0; p < N; p++) mine[p] = soff[p + 1] - soff[p];
  to_dev(cmat, mine.data(), N, st);
  comm_allgather(c, cmat, call, N * sizeof(uint64_t), st);
  std::vector<uint64_t> hall((size_t)N * N);
  to_host(hall.data(), call, (size_t)N * N, st);
  std::vector<uint64_t> sb(N + 1), rb(N + 1, 0);
  for (int p = 0; p <= N; p++) sb[p] = soff[p] * sizeof(SplitElem);
  for (int p = 0; p < N; p++) rb[p + 1] = rb[p] + hall[(size_t)p * N + me] * sizeof(SplitElem);
  const uint64_t nrecv = rb[N] / sizeof(SplitElem);
  SplitElem* recvb = sbuf<SplitElem>(e, kSRecv, nrecv);
  comm_alltoallv(c, sendb, sb.data(), recvb, rb.data(), st);

  // 7. owner: exact replay of the gathered prefixes, pending temps merged, then the pieces --
  // on the split engine (owned key k in its slot k), whose stream runs beside this engine's
  // replay; the finished digests move into this engine's slots (k_split_move_histo)
  std::vector<uint32_t> okeys, local(H, 0xffffffffu);
  for (uint32_t h = 0; h < H; h++)
    if (owner[h] == (uint32_t)me) {
      local[h] = (uint32_t)okeys.size();
      okeys.push_back(h);
    }
  const uint32_t K = (uint32_t)okeys.size();
  if (!K) return;
  uint32_t* dok = sbuf<uint32_t>(e, kSIdCnt, K);
  uint32_t* dlocal = sbuf<uint32_t>(e, kSSt, H);  // (key runs no longer needed)
  to_dev(dok, okeys.data(), K, st);
  to_dev(dlocal, local.data(), H, st);
  // owned keys: piece counts (from the window totals); piece ids = scan of counts
  uint32_t* otl = sbuf<uint32_t>(e, kSTouch, K);
  uint32_t* opcnt = sbuf<uint32_t>(e, kSPcnt, K + 1);
  uint32_t* opbase = sbuf<uint32_t>(e, kSCntMat, K + 1);
  hipLaunchKernelGGL(k_sh_owned, dim3(blocks_for(K, 256)), dim3(256), 0, st, K, dok, tot, P, e->h_geo, e->n_geo, otl,
                     opcnt);
  scan_exclusive_u32(opcnt, opbase, K, a->ss, st);
  uint32_t* rflag = sbuf<uint32_t>(e, kSFlag, nrecv + 1);
  uint32_t* rpos = sbuf<uint32_t>(e, kSPos, nrecv + 1);
  uint32_t nrpre = 0;
  uint64_t* PreA = sbuf<uint64_t>(e, kSImpA, nrecv);
  uint64_t* PreB = sbuf<uint64_t>(e, kSImpB, nrecv);
  uint64_t* PreA1 = sbuf<uint64_t>(e, kSImpA1, nrecv);
  uint64_t* PreB1 = sbuf<uint64_t>(e, kSImpB1, nrecv);
  uint64_t* MicA = sbuf<uint64_t>(e, kSA0, nrecv);
  uint64_t* MicB = sbuf<uint64_t>(e, kSB0, nrecv);
  uint64_t* MicA1 = sbuf<uint64_t>(e, kSA1, nrecv);
  uint64_t* MicB1 = sbuf<uint64_t>(e, kSB1, nrecv);
  double* micw = sbuf<double>(e, kSMicW, nrecv);
  if (nrecv) {
    hipLaunchKernelGGL(k_sh_recv_flags, dim3(blocks_for(nrecv, 256)), dim3(256), 0, st, nrecv, recvb, rflag);
    scan_exclusive_u32(rflag, rpos, nrecv, a->ss, st);
    hipLaunchKernelGGL(k_sh_recv_split, dim3(blocks_for(nrecv, 256)), dim3(256), 0, st, nrecv, recvb, rpos, dlocal,
                       opbase, PreA, PreB, MicA, MicB, micw);
    to_host(&nrpre, rpos + nrecv, 1, st);
  }
  const uint64_t nmic = nrecv - nrpre;
  if (std::max<uint64_t>(nrpre, nmic) > a->max_records) {  // a larger split engine (rare: grows once)
    a = split_engine(e, std::max<uint64_t>(nrpre, nmic) + std::max<uint64_t>(nrpre, nmic) / 4);
    st = a->st;
  }
  uint32_t* olist = sbuf<uint32_t>(e, kSIota, kMaxSplitKeys);  // owned key k -> split-engine slot k
  if (nrpre) {
    RadixPass rp[6];
    const int nrp = make_passes(rp, false, 0, 32 + bits_for_n(K));
    const bool fl = radix_sort(PreA, PreB, PreA1, PreB1, nrpre, rp, nrp, a->rs, st, nullptr);
    uint32_t* islot = sbuf<uint32_t>(e, kSImpSlot, nrpre);
    double* ival = sbuf<double>(e, kSImpVal, nrpre);
    double* iw = sbuf<double>(e, kSImpW, nrpre);
    hipLaunchKernelGGL(k_sh_pre_gather, dim3(blocks_for(nrpre, 256)), dim3(256), 0, st, (uint64_t)nrpre,
                       fl ? PreA1 : PreA, fl ? PreB1 : PreB, recvb, otl, islot, ival, iw);
    // MergingDigest.Add of each prefix record in window order (import-tagged: the Local*
    // statistics come from the all-reduce; the digest min/max from the samples)
    ingest_histos(a, nrpre, islot, ival, nullptr, iw);
  }
  // merge the pending temps (the single-GPU hot path does the same after the prefix)
  histo_merge_pending(a, olist, K);
  if (nmic) {
#if !VN_FAST_MODE
    (void)MicA1, (void)MicB1;
    throw std::logic_error("split histo pieces without the fast mode (VN_FAST_MODE) built");
#else
    // pieces: (piece id, mean)-sorted micro-centroids, one mergeAllTemps per piece and round
    VN_HIP_CHECK(hipMemcpyAsync(a->h_tl, otl, K * 4, hipMemcpyDeviceToDevice, st));
    VN_HIP_CHECK(hipMemcpyAsync(a->h_pcnt, opcnt, K * 4, hipMemcpyDeviceToDevice, st));
    VN_HIP_CHECK(hipMemcpyAsync(a->h_pbase, opbase, (K + 1) * 4, hipMemcpyDeviceToDevice, st));
    uint32_t npid = 0;
    to_host(&npid, opbase + K, 1, st);
    RadixPass mp[16];
    int nmp = make_passes(mp, false, 0, 64);
    nmp += make_passes(mp + nmp, true, 32, bits_for_n(npid + 1));
    const bool fl = radix_sort(MicA, MicB, MicA1, MicB1, nmic, mp, nmp, a->rs, st, nullptr);
    const uint64_t* MA_ = fl ? MicA1 : MicA;
    const uint64_t* MB_ = fl ? MicB1 : MicB;
    VN_HIP_CHECK(hipMemsetAsync(a->p_start, 0, (size_t)(npid + 1) * 4, st));
    VN_HIP_CHECK(hipMemsetAsync(a->p_end, 0, (size_t)(npid + 1) * 4, st));
    hipLaunchKernelGGL(k_key_runs, dim3(blocks_for(nmic, 256)), dim3(256), 0, st, nmic, MB_, a->p_start, a->p_end);
    if ((uint64_t)N * capc + a->cap_cent <= kFuseMaxL) {
      // every piece is at most N ranks' micro-centroids: all rounds in one launch
      double* fv = sbuf<double>(e, kSFuseV, (size_t)K * kFuseMaxL);
      double* fw = sbuf<double>(e, kSFuseW, (size_t)K * kFuseMaxL);
      double* fk = sbuf<double>(e, kSFuseK, (size_t)K * kFuseMaxL);
      histo_rounds_fused(a, olist, K, MA_, MB_, micw, fv, fw, fk, st);
    } else {
      VN_HIP_CHECK(hipMemcpyAsync(a->h_hotlist, olist, K * 4, hipMemcpyDeviceToDevice, st));
      std::vector<uint32_t> hpc(K);
      to_host(hpc.data(), opcnt, K, st);
      const uint32_t maxp = *std::max_element(hpc.begin(), hpc.end());
      histo_rounds(a, a->h_hotlist, K, maxp, nmic, K, MA_, MB_, a->hA2, a->hB2, micw, st);
    }
#endif  // VN_FAST_MODE
  }
  S.mv_histo = SplitState::HistoMove{K, dok, tot, sums, mins, maxs};  // (moved by split_flush)
}

// ---------------------------------------------------------------- sets
// gather buffer: per key the rank's first m codes (m = ceil(J / N) slots, unused = kHllNoCode)
__global__ void k_ss_prefix_send(uint32_t H, uint32_t M, const uint32_t* __restrict__ kst,
                                 const uint32_t* __restrict__ ken, const uint64_t* __restrict__ R,
                                 uint32_t* __restrict__ out) {
  const uint32_t k = blockIdx.y;
  const uint32_t lo = kst[k], n = ken[k] - lo;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < M; i += gridDim.x * blockDim.x)
    out[(uint64_t)k * M + i] = i < n ? (uint32_t)R[lo + i] : kHllNoCode;
}
// prefix stream of key k: record j = recv[j % N][k][j / N], as (slot << 32 | code) at k * J + j
__global__ void k_ss_prefix_stream(uint32_t H, uint32_t M, uint32_t N, uint32_t J, const uint64_t* __restrict__ tot,
                                   const uint32_t* __restrict__ recv, const uint32_t* __restrict__ kslot,
                                   uint64_t* __restrict__ R2, uint32_t* __restrict__ start,
                                   uint32_t* __restrict__ end) {
  const uint32_t k = blockIdx.y;
  const uint32_t L = (uint32_t)min((uint64_t)J, tot[k]);
  const uint32_t s = kslot[k];
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < L; j += gridDim.x * blockDim.x) {
    const uint32_t c = recv[((uint64_t)(j % N) * H + k) * M + j / N];
    R2[(uint64_t)k * J + j] = ((uint64_t)s << 32) | c;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    start[s] = k * J;
    end[s] = k * J + L;
  }
}
__global__ void k_ss_reset(uint32_t H, const uint32_t* __restrict__ kslot, uint8_t* mode, uint8_t* base, uint32_t* nz,
                           uint32_t* lc, uint32_t* lb, uint32_t* last, uint32_t* tc) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H) return;
  const uint32_t s = kslot[k];
  mode[s] = 0;
  base[s] = 0;
  nz[s] = kHllM;
  lc[s] = 0;
  lb[s] = 0;
  last[s] = 0;
  tc[s] = 0;
}
__global__ void k_ss_mode(uint32_t H, const uint32_t* __restrict__ kslot, const uint8_t* __restrict__ mode,
                          uint32_t* __restrict__ out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < H) out[k] = mode[kslot[k]];
}

// ---- rebase epochs (set_dense.h's exact insert, distributed).  Record i of key k's run is the
// key's record j = me + N * (i - start); only records j >= p0[k] of keys not done take part.
struct EpochCtx {
  uint32_t H;
  int me, N;
  const uint64_t* R;       // key-sorted own records: key << 32 | code
  const uint32_t* kst;
  const uint32_t* kslot;
  const uint8_t* arena8;   // registers of the key's slot (one byte each)
  const uint8_t* base;
  const uint32_t* nz;
  const uint32_t* p0;
  const uint32_t* done;
  const uint32_t* tfull;
  const uint64_t* cand;
};
__device__ __forceinline__ bool epoch_rec(const EpochCtx& x, uint64_t i, uint32_t& k, uint32_t& j, uint32_t& idx,
                                          uint32_t& r, uint32_t& code) {
  const uint64_t v = x.R[i];
  k = (uint32_t)(v >> 32);
  if (x.done[k]) return false;
  const uint64_t jj = (uint64_t)x.me + (uint64_t)x.N * (i - x.kst[k]);
  if (jj < x.p0[k]) return false;
  j = (uint32_t)jj;
  code = (uint32_t)v;
  decode_hash(code, &idx, &r);
  return true;
}
template <class T>
__device__ __forceinline__ T ld_relaxed(T* p) {  // another wave's atomic may have lowered it
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (a) first filler of every zero register: min j with r > b
__global__ void k_ep_firstfill(EpochCtx x, uint64_t n, uint32_t* ff) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t k, j, idx, r, code;
    if (!epoch_rec(x, i, k, j, idx, r, code)) continue;
    const uint32_t s = x.kslot[k];
    if (x.nz[s] == 0 || r <= x.base[s]) continue;
    uint32_t* f = &ff[(uint64_t)k * kHllM + idx];
    if (x.arena8[(uint64_t)s * (kArenaWords * 4) + idx] == 0 && j < ld_relaxed(f)) atomicMin(f, j);
  }
}
// (b) T_full per key: the last first-fill of its zero registers (none missing), or p0 - 1 when full
__global__ __launch_bounds__(kBlock) void k_ep_tfull(EpochCtx x, const uint32_t* __restrict__ ff,
                                                     uint32_t* __restrict__ tfull) {
  __shared__ uint32_t s_red[4];
  const uint32_t k = blockIdx.x;
  if (x.done[k]) return;
  const uint32_t s = x.kslot[k];
  if (x.nz[s] == 0) {
    if (threadIdx.x == 0) tfull[k] = x.p0[k] - 1;
    return;
  }
  uint32_t mx = 0, miss = 0;
  for (uint32_t i = threadIdx.x; i < kHllM; i += kBlock) {
    if (x.arena8[(uint64_t)s * (kArenaWords * 4) + i] != 0) continue;
    const uint32_t f = ff[(uint64_t)k * kHllM + i];
    if (f == 0xffffffffu) miss = 1;
    else mx = max(mx, f);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
    miss |= (uint32_t)__shfl_xor((int)miss, d, 64);
  }
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = miss ? 0xffffffffu : mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < 4; w++) t = (s_red[w] == 0xffffffffu || t == 0xffffffffu) ? 0xffffffffu : max(t, s_red[w]);
    tfull[k] = t;
  }
}
// (c) first rebase candidate strictly after T_full: uint8(r - b) >= 16 (hyperloglog.go:170).
// Once b >= 2 most records are candidates (r < b), so the minimum is taken in the wave first:
// the records are key-sorted, a wave's items nearly always share one key -- one atomic per wave
// and item, the stragglers of another key go straight to memory.
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long o = (unsigned long long)__shfl_xor((long long)v, d, 64);
    v = o < v ? o : v;
  }
  return v;
}
__global__ void k_ep_cand(EpochCtx x, uint64_t n, unsigned long long* cand) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {  // wave-uniform trip count
    const uint64_t i = i0 + threadIdx.x;
    uint32_t k = 0xffffffffu, j, idx, r, code;
    unsigned long long v = ~0ull;
    if (i < n && epoch_rec(x, i, k, j, idx, r, code)) {
      const uint32_t t = x.tfull[k];
      if (t != 0xffffffffu && j > t && ((r - x.base[x.kslot[k]]) & 0xffu) >= kHllCapacity)
        v = ((unsigned long long)j << 32) | code;
    }
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(k);
    const bool same = k == k0;
    // the minimum only falls: a candidate not below the value already there needs no atomic
    if (!same && v != ~0ull && v < ld_relaxed(&cand[k])) atomicMin(&cand[k], v);
    const unsigned long long m = wave_min_u64(same ? v : ~0ull);
    if ((threadIdx.x & 63) == 0 && m != ~0ull && k0 != 0xffffffffu && m < ld_relaxed(&cand[k0])) atomicMin(&cand[k0], m);
  }
}
// (d) registers after the plain max updates of every record before the candidate
__global__ void k_ep_regs_init(uint32_t H, const uint32_t* __restrict__ kslot, const uint8_t* __restrict__ arena8,
                               uint32_t* __restrict__ W) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)H * kHllM) return;
  const uint32_t k = (uint32_t)(i / kHllM), r = (uint32_t)(i % kHllM);
  W[i] = arena8[(uint64_t)kslot[k] * (kArenaWords * 4) + r];
}
__global__ void k_ep_apply(EpochCtx x, uint64_t n, uint32_t* __restrict__ W) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t k, j, idx, r, code;
    if (!epoch_rec(x, i, k, j, idx, r, code)) continue;
    if ((uint64_t)j >= (x.cand[k] >> 32)) continue;
    const uint32_t b = x.base[x.kslot[k]];
    if (r <= b) continue;
    const uint32_t v = min(r - b, kHllCapacity - 1);
    uint32_t* w = &W[(uint64_t)k * kHllM + idx];
    if (v > *w) atomicMax(w, v);  // registers only grow: a stale read only costs an atomic
  }
}
// (e) every rank alike: registers <- W; at the candidate the rebase (b += min, registers -= min)
// and the candidate's own insert; next epoch from the record after it
__global__ __launch_bounds__(kBlock) void k_ep_finish(uint32_t H, const uint32_t* __restrict__ kslot,
                                                      const uint32_t* __restrict__ W,
                                                      const unsigned long long* __restrict__ cand,
                                                      uint8_t* __restrict__ arena8, uint8_t* __restrict__ base,
                                                      uint32_t* __restrict__ nz, uint32_t* __restrict__ p0,
                                                      uint32_t* __restrict__ done, uint32_t* __restrict__ err) {
  __shared__ uint32_t s_red[4];
  __shared__ uint32_t s_min;
  const uint32_t k = blockIdx.x;
  if (done[k]) return;
  const uint32_t s = kslot[k];
  uint8_t* regs = arena8 + (uint64_t)s * (kArenaWords * 4);
  const uint64_t c = cand[k];
  const bool rebase = c != ~0ull;
  uint32_t mn = 0xffffffffu;
  for (uint32_t i = threadIdx.x; i < kHllM; i += kBlock) mn = min(mn, W[(uint64_t)k * kHllM + i]);
  if (threadIdx.x == 0) s_min = 0xffffffffu;
  __syncthreads();
  atomicMin(&s_min, mn);
  __syncthreads();
  const uint32_t db = rebase ? s_min : 0u;
  uint32_t z = 0;
  for (uint32_t i = threadIdx.x; i < kHllM; i += kBlock) {
    const uint32_t v = W[(uint64_t)k * kHllM + i] - db;
    regs[i] = (uint8_t)v;
    z += v == 0;
  }
  z = block_allreduce_u32_sum(z, s_red);
  if (threadIdx.x == 0) {
    if (!rebase) {
      nz[s] = z;
      done[k] = 1;
    } else {
      if (db == 0) atomicOr(err, 2u);  // the candidate follows T_full: every register is non-zero
      const uint32_t nb = base[s] + db;
      base[s] = (uint8_t)nb;
      uint32_t pi, pr;
      decode_hash((uint32_t)c, &pi, &pr);
      if (pr > nb) {
        const uint32_t v = min(pr - nb, kHllCapacity - 1);
        if (v > regs[pi]) {
          if (regs[pi] == 0) z--;
          regs[pi] = (uint8_t)v;
        }
      }
      nz[s] = z;
      p0[k] = (uint32_t)(c >> 32) + 1;
    }
  }
}
// per-slot set state of an engine (engine.h)
struct SetSlots {
  uint8_t *mode, *base;
  uint32_t *nz, *lc, *lb, *last, *tc, *touch, *tmp, *arena;
};
SetSlots set_slots(vn_engine* e) {
  return SetSlots{e->smode, e->sbase, e->snz, e->slc, e->slb, e->slast, e->stc, e->stouch, e->stmp, e->sarena};
}
// the owner's sketch moves from the split engine's slot k into this engine's slot of the key;
// every rank leaves the split engine's slot empty for the next window
__global__ __launch_bounds__(256) void k_split_move_set(const uint32_t* __restrict__ kslot,
                                                        const uint32_t* __restrict__ owner, int me,
                                                        const uint64_t* __restrict__ tot, SetSlots src,
                                                        SetSlots dst, uint32_t* __restrict__ err) {
  const uint32_t k = blockIdx.x;
  if (owner[k] == (uint32_t)me && tot[k]) {
    const uint32_t s = kslot[k];
    if (threadIdx.x == 0 && dst.touch[s]) atomicOr(err, kErrSplitTouched);
    for (uint32_t i = threadIdx.x; i < kArenaWords; i += blockDim.x)
      dst.arena[(uint64_t)s * kArenaWords + i] = src.arena[(uint64_t)k * kArenaWords + i];
    for (uint32_t i = threadIdx.x; i < kTmpCap; i += blockDim.x)
      dst.tmp[(uint64_t)s * kTmpCap + i] = src.tmp[(uint64_t)k * kTmpCap + i];
    if (threadIdx.x == 0) {
      dst.mode[s] = src.mode[k];
      dst.base[s] = src.base[k];
      dst.nz[s] = src.nz[k];
      dst.lc[s] = src.lc[k];
      dst.lb[s] = src.lb[k];
      dst.last[s] = src.last[k];
      dst.tc[s] = src.tc[k];
      dst.touch[s] = 1;
    }
  }
  if (threadIdx.x == 0) {
    src.mode[k] = 0;
    src.base[k] = 0;
    src.nz[k] = kHllM;
    src.lc[k] = 0;
    src.lb[k] = 0;
    src.last[k] = 0;
    src.tc[k] = 0;
    src.touch[k] = 0;
  }
}

void split_sets(vn_engine* e, vn_comm* c) {
  vn_engine* a = e->sp.aux;
  hipStream_t st = a->st;
  SplitState& S = e->sp;
  const uint32_t H = (uint32_t)S.slot[VN_SET].size();
  if (!H) return;
  const int N = c->nranks, me = c->rank;
  const uint64_t n = S.ns;
  // 1. own records grouped by key, arrival (= window index) order kept
  uint64_t* R0 = sbuf<uint64_t>(e, kSA0, n);
  uint64_t* R1 = sbuf<uint64_t>(e, kSA1, n);
  uint32_t* kst = sbuf<uint32_t>(e, kSSt, H);
  uint32_t* ken = sbuf<uint32_t>(e, kSEn, H);
  VN_HIP_CHECK(hipMemsetAsync(kst, 0, H * sizeof(uint32_t), st));
  VN_HIP_CHECK(hipMemsetAsync(ken, 0, H * sizeof(uint32_t), st));
  const uint64_t* R = R0;
  if (n) {
    VN_HIP_CHECK(hipMemcpyAsync(R0, S.srec, n * 8, hipMemcpyDeviceToDevice, st));
    RadixPass kp[5];
    const int nkp = make_passes(kp, false, 32, bits_for_n(H));
    R = radix_sort(R0, nullptr, R1, nullptr, n, kp, nkp, a->rs, st, nullptr) ? R1 : R0;
    hipLaunchKernelGGL(k_key_runs, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, R, kst, ken);
  }
  uint64_t* tot = sbuf<uint64_t>(e, kSTot, H);
  {
    std::vector<uint32_t> hs(H), he(H);
    to_host(hs.data(), kst, H, st);
    to_host(he.data(), ken, H, st);
    std::vector<uint64_t> cnt(H);
    for (uint32_t k = 0; k < H; k++) cnt[k] = he[k] - hs[k];
    to_dev(tot, cnt.data(), H, st);
  }
  comm_allreduce(c, tot, tot, H, kU64, kSum, st);
  std::vector<uint64_t> htot(H);
  to_host(htot.data(), tot, H, st);
  const uint64_t maxtot = *std::max_element(htot.begin(), htot.end());
  uint32_t* kslot = sbuf<uint32_t>(e, kSIota, kMaxSplitKeys);  // key k -> split-engine slot k
  uint32_t* downer = sbuf<uint32_t>(e, kSOwnList, H);
  to_dev(downer, S.owner[VN_SET].data(), H, st);

  // 2. the first J records of every key, gathered and replayed exactly (sparse phase, switch)
  // the sparse phase ends by ~8-9k distinct codes (the list passes 16 KiB); a key still sparse
  // at J with more records to come gathers 4x more (its trigger sequence goes on)
  uint64_t J = std::min<uint64_t>(12288, std::max<uint64_t>(maxtot, 1));
  for (;;) {
    const uint32_t M = (uint32_t)((J + N - 1) / N);
    uint32_t* gsend = sbuf<uint32_t>(e, kSW32, (size_t)H * M);
    uint32_t* grecv = sbuf<uint32_t>(e, kSFF, (size_t)N * H * M);
    hipLaunchKernelGGL(k_ss_prefix_send, dim3(std::min<uint32_t>(blocks_for(M, 256), 64), H), dim3(256), 0, st, H, M,
                       kst, ken, R, gsend);
    comm_allgather(c, gsend, grecv, (size_t)H * M * sizeof(uint32_t), st);
    uint64_t* R2 = sbuf<uint64_t>(e, kSR2, (size_t)H * J);
    hipLaunchKernelGGL(k_ss_reset, dim3(blocks_for(H, 256)), dim3(256), 0, st, H, kslot, a->smode, a->sbase, a->snz,
                       a->slc, a->slb, a->slast, a->stc);
    hipLaunchKernelGGL(k_ss_prefix_stream, dim3(std::min<uint64_t>(blocks_for(J, 256), 64), H), dim3(256), 0, st, H, M,
                       (uint32_t)N, (uint32_t)J, tot, grecv, kslot, R2, a->s_start, a->s_end);
    uint32_t* dH = sbuf<uint32_t>(e, kSDev1, 1);
    to_dev(dH, &H, 1, st);
    set_replay_ranges(a, R2, dH, kslot, H, st);
    uint32_t* modes = sbuf<uint32_t>(e, kSIdFlag, H);
    hipLaunchKernelGGL(k_ss_mode, dim3(blocks_for(H, 256)), dim3(256), 0, st, H, kslot, a->smode, modes);
    std::vector<uint32_t> hm(H);
    to_host(hm.data(), modes, H, st);
    bool more = false;  // a key still sparse with records beyond J: its trigger sequence goes on
    for (uint32_t k = 0; k < H; k++) more |= hm[k] == 0 && htot[k] > J;
    if (!more) break;
    if ((uint64_t)H * J * 4 > (1ull << 32)) throw std::runtime_error("split set prefix too long");
    J = std::min<uint64_t>(J * 4, maxtot);
  }

  VN_HIP_CHECK(hipEventRecord(e->sp.ev_set_prefix, st));
  // 3. the records after J: dense inserts in rebase epochs, all-reduced
  uint32_t* p0 = sbuf<uint32_t>(e, kSP0, H);
  uint32_t* done = sbuf<uint32_t>(e, kSDone, H);
  uint32_t* tfull = sbuf<uint32_t>(e, kSTfull, H);
  unsigned long long* cand = sbuf<unsigned long long>(e, kSCand, H);
  uint32_t* ff = sbuf<uint32_t>(e, kSFF, (size_t)H * kHllM);
  uint32_t* W = sbuf<uint32_t>(e, kSW32, (size_t)H * kHllM);
  {
    std::vector<uint32_t> hp0(H, (uint32_t)J), hd(H);
    for (uint32_t k = 0; k < H; k++) hd[k] = htot[k] <= J ? 1u : 0u;
    to_dev(p0, hp0.data(), H, st);
    to_dev(done, hd.data(), H, st);
  }
  EpochCtx x;
  x.H = H;
  x.me = me;
  x.N = N;
  x.R = R;
  x.kst = kst;
  x.kslot = kslot;
  x.arena8 = reinterpret_cast<const uint8_t*>(a->sarena);
  x.base = a->sbase;
  x.nz = a->snz;
  x.p0 = p0;
  x.done = done;
  x.tfull = tfull;
  x.cand = reinterpret_cast<const uint64_t*>(cand);
  const int grid = (int)std::min<uint64_t>(std::max<uint64_t>(blocks_for(n, 256), 1), 8192);
  std::vector<uint32_t> hd(H);
  for (int round = 0;; round++) {
    to_host(hd.data(), done, H, st);
    if (std::all_of(hd.begin(), hd.end(), [](uint32_t d) { return d != 0; })) break;
    if (round > 4096) throw std::runtime_error("split set rebase epochs do not converge");
    VN_HIP_CHECK(hipMemsetAsync(ff, 0xff, (size_t)H * kHllM * 4, st));
    if (n) hipLaunchKernelGGL(k_ep_firstfill, dim3(grid), dim3(256), 0, st, x, n, ff);
    comm_allreduce(c, ff, ff, (size_t)H * kHllM, kU32, kMin, st);
    hipLaunchKernelGGL(k_ep_tfull, dim3(H), dim3(kBlock), 0, st, x, ff, tfull);
    VN_HIP_CHECK(hipMemsetAsync(cand, 0xff, (size_t)H * 8, st));
    if (n) hipLaunchKernelGGL(k_ep_cand, dim3(grid), dim3(256), 0, st, x, n, cand);
    comm_allreduce(c, cand, cand, H, kU64, kMin, st);
    hipLaunchKernelGGL(k_ep_regs_init, dim3(blocks_for((uint64_t)H * kHllM, 256)), dim3(256), 0, st, H, kslot,
                       x.arena8, W);
    if (n) hipLaunchKernelGGL(k_ep_apply, dim3(grid), dim3(256), 0, st, x, n, W);
    comm_allreduce(c, W, W, (size_t)H * kHllM, kU32, kMax, st);
    hipLaunchKernelGGL(k_ep_finish, dim3(H), dim3(kBlock), 0, st, H, kslot, W, cand,
                       reinterpret_cast<uint8_t*>(a->sarena), a->sbase, a->snz, p0, done, a->h_err);
  }
  S.mv_set = SplitState::SetMove{H, downer, me, tot};  // (moved by split_flush)
}

}  // namespace

// the split engine's part of the combine: histograms, then sets, then the error flags; ev_done
// marks its end on the split engine's stream (a host thread of its own after vn_split_close)
void split_combine_aux(vn_engine* e, vn_comm* c) {
  SplitState& S = e->sp;
  split_histos(e, c);
  VN_HIP_CHECK(hipEventRecord(S.ev_histo, S.aux->st));
  VN_HIP_CHECK(hipEventRecord(S.ev_set_prefix, S.aux->st));  // (again after the set prefix, if any)
  split_sets(e, c);
  vn_engine* a = S.aux;
  hipLaunchKernelGGL(k_split_errors, dim3(1), dim3(64), 0, a->st, a->h_err, e->h_err);
  VN_HIP_CHECK(hipEventRecord(S.ev_done, a->st));
}

void split_join(vn_engine* e) {
  SplitState& S = e->sp;
  if (S.worker.joinable()) S.worker.join();
  std::exception_ptr err = S.worker_err;
  S.worker_err = nullptr;
  if (err) std::rethrow_exception(err);
}

void split_flush(vn_engine* e) {
  SplitState& S = e->sp;
  if (S.slot[VN_COUNTER].empty() && S.slot[VN_HISTO].empty() && S.slot[VN_SET].empty()) {
    S.nh = S.ns = 0;
    S.closed = false;
    return;
  }
  vn_comm* c = group_of(e);
  if (S.aux) {
    // histos and sets on the split engine's stream, beside this engine's work (already under
    // way in the worker thread after vn_split_close); this engine's stream waits for the moved
    // states, and the counters' collectives follow the split engine's (one order per group)
    if (S.closed) {
      S.closed = false;
      split_join(e);
    } else {
      split_combine_aux(e, c);
    }
    S.ran = true;
    VN_HIP_CHECK(hipStreamWaitEvent(e->st, S.ev_done, 0));
    // the finished states into this engine's slots, behind every ingest and import of the window
    // on this stream: a slot that also got records here is reported (kErrSplitTouched), not mixed
    vn_engine* a = S.aux;
    if (S.mv_histo.K)
      hipLaunchKernelGGL(k_split_move_histo, dim3(S.mv_histo.K), dim3(256), 0, e->st, S.mv_histo.okeys,
                         S.d_slot[VN_HISTO], S.mv_histo.tot, S.mv_histo.sums, S.mv_histo.mins, S.mv_histo.maxs,
                         histo_slots(a), histo_slots(e), e->cap_cent, e->temp_cap, e->h_err);
    if (S.mv_set.H)
      hipLaunchKernelGGL(k_split_move_set, dim3(S.mv_set.H), dim3(256), 0, e->st, S.d_slot[VN_SET], S.mv_set.owner,
                         S.mv_set.me, S.mv_set.tot, set_slots(a), set_slots(e), e->h_err);
    S.mv_histo = SplitState::HistoMove{};
    S.mv_set = SplitState::SetMove{};
  }
  S.closed = false;
  if (!S.slot[VN_COUNTER].empty()) {
    // on their own stream, after the window's counter aggregation (the side stream's work so
    // far), then the main stream waits for them: not behind this window's long replays
    hipStream_t src = e->timing || !e->st2 ? e->st : e->st2;
    ensure_aux_streams(e, false, true);
    split_counter_owners(e, e->st_ctr);  // (before the wait: the stream is idle)
    VN_HIP_CHECK(hipEventRecord(e->ev_ctr0, src));
    VN_HIP_CHECK(hipStreamWaitEvent(e->st_ctr, e->ev_ctr0, 0));
    split_counters(e, c, e->st_ctr);
    VN_HIP_CHECK(hipEventRecord(e->ev_ctr1, e->st_ctr));
    VN_HIP_CHECK(hipStreamWaitEvent(e->st, e->ev_ctr1, 0));
  }
  for (int k = 0; k < VN_NCLASS; k++) {
    S.slot[k].clear();
    S.owner[k].clear();
  }
  S.nh = S.ns = 0;
}

void split_destroy(vn_engine* e) {
  SplitState& S = e->sp;
  if (S.worker.joinable()) S.worker.join();
  if (S.aux) (void)hipStreamSynchronize(S.aux->st);
  for (void* p : S.scratch)
    if (p) (void)hipFree(p);
  S.scratch.clear();
  S.scratch_cap.clear();
  for (int k = 0; k < VN_NCLASS; k++)
    if (S.d_slot[k]) (void)hipFree(S.d_slot[k]);
  if (S.hkey) (void)hipFree(S.hkey);
  if (S.hval) (void)hipFree(S.hval);
  if (S.hrate) (void)hipFree(S.hrate);
  if (S.srec) (void)hipFree(S.srec);
  if (S.solo) vn_comm_destroy(S.solo);
  if (S.aux) vn_engine_destroy(S.aux);
  if (S.ev_done) (void)hipEventDestroy(S.ev_done);
  if (S.ev_histo) (void)hipEventDestroy(S.ev_histo);
  if (S.ev_set_prefix) (void)hipEventDestroy(S.ev_set_prefix);
  S.~SplitState();
  new (&S) SplitState();
}

}  // namespace vn

using namespace vn;

namespace {
int split_fail(vn_engine* e, int code, const std::string& m) {
  e->err = m;
  return code;
}
template <class F>
int split_guarded(vn_engine* e, F&& f) {
  try {
    if (e) VN_HIP_CHECK(hipSetDevice(e->device));  // as capi.hip's guarded: the engine's device
    f();
    return VN_OK;
  } catch (const HipError& h) {
    return split_fail(e, VN_EHIP, std::string(hipGetErrorString(h.err)) + " at " + h.file + ":" +
                                      std::to_string(h.line) + ": " + h.expr);
  } catch (const std::invalid_argument& x) {
    return split_fail(e, VN_EINVAL, x.what());
  } catch (const std::bad_alloc&) {
    return split_fail(e, VN_ENOMEM, "out of memory");
  } catch (const std::exception& x) {
    return split_fail(e, VN_EINVAL, x.what());
  }
}
}  // namespace

extern "C" {

int vn_engine_set_comm(vn_engine* e, vn_comm* c) {
  if (!e) return VN_EINVAL;
  if (c && c->device != e->device) return split_fail(e, VN_EINVAL, "communicator is on another device");
  e->sp.comm = c;
  return VN_OK;
}

int vn_split_keys(vn_engine* e, int cls, const uint32_t* slot, const uint32_t* owner, uint32_t n) {
  if (!e || (n && (!slot || !owner))) return VN_EINVAL;
  return split_guarded(e, [&] {
    if (cls != VN_COUNTER && cls != VN_HISTO && cls != VN_SET)
      throw std::invalid_argument("only counters, histograms and sets can be split");
    SplitState& S = e->sp;
    if (S.closed) throw std::invalid_argument("split keys change while the window's split combine runs (flush first)");
    if ((cls == VN_HISTO && S.nh) || (cls == VN_SET && S.ns))
      throw std::invalid_argument("split keys change while their records are buffered (flush first)");
    const int N = S.comm ? S.comm->nranks : 1;
    std::vector<uint32_t> seen(e->cap[cls] ? e->cap[cls] : 1, 0);
    for (uint32_t i = 0; i < n; i++) {
      if (slot[i] >= e->cap[cls]) throw std::invalid_argument("split key slot out of range");
      if (owner[i] >= (uint32_t)N) throw std::invalid_argument("split key owner out of range");
      if (seen[slot[i]]++) throw std::invalid_argument("split key slot listed twice");
    }
    if (cls != VN_COUNTER && n > kMaxSplitKeys) throw std::invalid_argument("more than 256 split keys in a class");
    if (cls != VN_COUNTER && n) split_engine(e, 0);
    S.slot[cls].assign(slot, slot + n);
    S.owner[cls].assign(owner, owner + n);
    if (n > S.d_cap[cls]) {
      if (S.d_slot[cls]) (void)hipFree(S.d_slot[cls]);
      S.d_slot[cls] = nullptr;
      S.d_cap[cls] = 0;
      VN_HIP_CHECK(hipMalloc(&S.d_slot[cls], n * sizeof(uint32_t)));
      S.d_cap[cls] = n;
    }
    // (on the engine's stream, not the null stream: see check_error_flags); the split counters'
    // owners go to the device here too, so the flush's combine issues no host copy or wait
    if (n) {
      VN_HIP_CHECK(hipMemcpyAsync(S.d_slot[cls], slot, n * sizeof(uint32_t), hipMemcpyHostToDevice, e->st));
      if (cls == VN_COUNTER)
        VN_HIP_CHECK(hipMemcpyAsync(sbuf<uint32_t>(e, kSCtrOwn, n), owner, n * sizeof(uint32_t), hipMemcpyHostToDevice,
                                    e->st));
      VN_HIP_CHECK(hipStreamSynchronize(e->st));
    }
  });
}

int vn_split_close(vn_engine* e) {
  if (!e) return VN_EINVAL;
  return split_guarded(e, [&] {
    SplitState& S = e->sp;
    if (S.closed) return;
    if (S.slot[VN_HISTO].empty() && S.slot[VN_SET].empty()) return;  // nothing for the split engine
    vn_comm* c = group_of(e);
    S.closed = true;
    const int dev = e->device;
    S.worker = std::thread([e, c, dev] {
      try {
        VN_HIP_CHECK(hipSetDevice(dev));
        split_combine_aux(e, c);
      } catch (...) {
        e->sp.worker_err = std::current_exception();
      }
    });
  });
}

int vn_split_combine(vn_engine* e) {
  if (!e) return VN_EINVAL;
  return split_guarded(e, [&] {
    // (returns once the group's exchange is issued: the engine's stream orders everything
    // after it, and vn_flush / the state reads wait for it -- not for this window's replays)
    split_flush(e);
    VN_HIP_CHECK(hipGetLastError());
  });
}

int vn_ingest_split(vn_engine* e, const vn_split_batch* b) {
  if (!e || !b) return VN_EINVAL;
  return split_guarded(e, [&] {
    SplitState& S = e->sp;
    if (S.closed) throw std::invalid_argument("split records after vn_split_close (flush first)");
    const uint32_t nh = (uint32_t)S.slot[VN_HISTO].size(), ns = (uint32_t)S.slot[VN_SET].size();
    if ((b->n_histo && !nh) || (b->n_set && !ns)) throw std::invalid_argument("records for a class with no split keys");
    if (S.nh + b->n_histo > e->cfg.split_max_records || S.ns + b->n_set > e->cfg.split_max_records)
      throw std::invalid_argument("split records exceed split_max_records");
    if ((b->n_histo && (!b->histo_key || !b->histo_value || !b->histo_rate)) ||
        (b->n_set && (!b->set_key || (!b->set_hash && (!b->set_member_off || !b->set_member_bytes)))))
      throw std::invalid_argument("split batch class with records but a null array");
    vn_engine* a = S.aux;  // exists: this class has split keys
    hipStream_t st = a->st;
    window_open(e, st);
    if (!S.cap) {
      S.cap = e->cfg.split_max_records;
      VN_HIP_CHECK(hipMalloc(&S.hkey, S.cap * 4));
      VN_HIP_CHECK(hipMalloc(&S.hval, S.cap * 8));
      VN_HIP_CHECK(hipMalloc(&S.hrate, S.cap * 4));
      VN_HIP_CHECK(hipMalloc(&S.srec, S.cap * 8));
    }
    const uint64_t nmax = std::max(b->n_histo, b->n_set);
    if (!nmax) return;
    VN_HIP_CHECK(hipMemsetAsync(a->h_err + 1, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_split_validate, dim3((int)std::min<uint64_t>(blocks_for(nmax, 256), 4096)), dim3(256), 0, st,
                       *b, nh, ns, a->h_err + 1);
    VN_HIP_CHECK(hipMemcpyAsync(a->hf_cnt + 15, a->h_err + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    VN_HIP_CHECK(hipStreamSynchronize(st));
    const uint32_t f = a->hf_cnt[15];
    if (f & 1u) throw std::invalid_argument("split key index out of range");
    if (f & 2u) throw std::invalid_argument("invalid value added");
    if (f & 4u) throw std::invalid_argument("sample rate must be >0 and <=1");
    if (f & 8u) throw std::invalid_argument("set member offsets must be non-decreasing");
    hot_sample(e, VN_HISTO, b->n_histo, b->histo_key, S.d_slot[VN_HISTO], nh, st);
    hot_sample(e, VN_SET, b->n_set, b->set_key, S.d_slot[VN_SET], ns, st);
    if (b->n_histo) {
      VN_HIP_CHECK(hipMemcpyAsync(S.hkey + S.nh, b->histo_key, b->n_histo * 4, hipMemcpyDeviceToDevice, st));
      VN_HIP_CHECK(hipMemcpyAsync(S.hval + S.nh, b->histo_value, b->n_histo * 8, hipMemcpyDeviceToDevice, st));
      VN_HIP_CHECK(hipMemcpyAsync(S.hrate + S.nh, b->histo_rate, b->n_histo * 4, hipMemcpyDeviceToDevice, st));
    }
    if (b->n_set)
      hipLaunchKernelGGL(k_split_set_codes, dim3(blocks_for(b->n_set, 256)), dim3(256), 0, st, b->n_set, b->set_key,
                         b->set_member_off, b->set_member_bytes, b->set_hash, S.srec + S.ns);
    VN_HIP_CHECK(hipGetLastError());
    S.nh += b->n_histo;
    S.ns += b->n_set;
    e->processed += b->n_histo + b->n_set;
  });
}

}  // extern "C"

// ingest_scalar.hip -- counters and gauges.
//
// Counter.Sample (samplers/samplers.go:132-134):
//     c.value += int64(sample) * int64(1/sampleRate)        // 1/sampleRate in float32
// is a wrapping int64 sum, so any grouping of the adds is bit-exact.  Gauge.Sample
// (198-200) keeps the last write in arrival order.
//
// Counters (default): a key-range partition pass writing one packed dword per record (KPackDst),
// then k_counter_runs sums each bucket run in LDS.  (k_scalar_direct, the former path: each
// block hashes a 16384-record chunk of the batch into an LDS
// table keyed by slot (wrapping i64 sums), then one device atomic per entry; a record that finds no
// free entry within 8 probes adds to its device word directly.
// Gauges (default): the same key-range partition, carrying each record's arrival index instead
// of its value (4 B read, 8 B written per record), then k_gauge_runs keeps each slot's last
// record per slice in LDS and k_gauge_resolve_direct reads the winners' values from the caller's
// array.  The former gauge path (VN_GAUGE_RUNS=0) avoids per-record device atomics too:
//   1. one stable partition pass (partition.h) by the low 8 slot bits, fused with the
//      per-record work (the counter contribution is computed while loading), so every
//      bucket's records are contiguous and still in arrival order;
//   2. k_scalar_agg: a block takes a 16384-record chunk of the partitioned batch and
//      aggregates it in an LDS hash table keyed by slot (wrapping i64 sum for counters,
//      max arrival position for gauges), then emits one device atomic per distinct slot
//      of the chunk (probe overflow falls back to a direct device atomic -- still exact);
//   3. gauges only: k_gauge_resolve stores, for every slot whose winning position lies in
//      this batch, the value found at that position of the partitioned batch.
#include "kernels.h"
#include "partition.h"

namespace vn {

namespace {

constexpr int kAggThreads = 512;
constexpr int kAggItems = 32;
constexpr int kAggChunk = kAggThreads * kAggItems;  // 16384 records per block
constexpr int kHashBits = 12;
constexpr uint32_t kHash = 1u << kHashBits;          // LDS table entries
constexpr uint32_t kEmpty = 0xffffffffu;
constexpr int kProbe = 32;
// Counters aggregate straight from the batch (k_scalar_direct): measured at C4 beside the histo
// replays, 17.5 ms of side-stream time against 48.8 ms for the partition pass + chunk aggregation
// (alone the two are 11.6 vs 10.3 ms).  Gauges keep the partition: their direct max-position
// aggregation took 28.5 ms there against ~6.5 (alone 5.8 vs 3.3 ms).
constexpr bool kScalarDirect = true;
#ifndef VN_COUNTER_RUNS
#define VN_COUNTER_RUNS 1
#endif
constexpr bool kCounterRuns = VN_COUNTER_RUNS;  // k_counter_runs below (else k_scalar_direct)
constexpr bool kGaugeDirect = false;
#ifndef VN_PART_V4
#define VN_PART_V4 1  // counters: 16-byte loads and the order-free rank in k_part_scatter
#endif
#ifndef VN_GAUGE_RUNS
#define VN_GAUGE_RUNS 1
#endif
constexpr bool kGaugeRuns = VN_GAUGE_RUNS;  // key-range partition + k_gauge_runs (else hashed k_scalar_agg)

struct CounterSrc {
  const uint32_t* slot;
  const double* val;
  const float* rate;
  using P = uint64_t;
  bool key16() const { return ((uintptr_t)slot & 15u) == 0; }
  __device__ __forceinline__ uint4 key4(uint64_t i) const { return *reinterpret_cast<const uint4*>(slot + i); }
  __device__ __forceinline__ uint32_t key(uint64_t i) const { return slot[i]; }
  __device__ __forceinline__ void load(uint64_t i, uint32_t& k, uint64_t& p) const {
    k = slot[i];
    float inv = 1.0f / rate[i];  // float32 division, as Go's 1/sampleRate on a float32
    p = (uint64_t)f64_to_i64_go(val[i]) * (uint64_t)f64_to_i64_go((double)inv);
  }
  // the sums are order-free: four adjacent records per 16-byte load when every array allows it
  bool vec16() const {
    return VN_PART_V4 && ((((uintptr_t)slot) | ((uintptr_t)val) | ((uintptr_t)rate)) & 15u) == 0;
  }
  __device__ __forceinline__ void load4(uint64_t i, uint32_t* k, uint64_t* p) const {
    const uint4 s4 = *reinterpret_cast<const uint4*>(slot + i);
    const float4 r4 = *reinterpret_cast<const float4*>(rate + i);
    const double2 v0 = *reinterpret_cast<const double2*>(val + i), v1 = *reinterpret_cast<const double2*>(val + i + 2);
    const float r[4] = {r4.x, r4.y, r4.z, r4.w};
    const double v[4] = {v0.x, v0.y, v1.x, v1.y};
    k[0] = s4.x, k[1] = s4.y, k[2] = s4.z, k[3] = s4.w;
#pragma unroll
    for (int q = 0; q < 4; q++)
      p[q] = (uint64_t)f64_to_i64_go(v[q]) * (uint64_t)f64_to_i64_go((double)(1.0f / r[q]));
  }
};

struct GaugeSrc {
  const uint32_t* slot;
  const double* val;
  using P = uint64_t;
  bool vec16() const { return false; }  // (arrival order kept within a digit)
  __device__ __forceinline__ void load4(uint64_t, uint32_t*, P*) const {}
  bool key16() const { return ((uintptr_t)slot & 15u) == 0; }
  __device__ __forceinline__ uint4 key4(uint64_t i) const { return *reinterpret_cast<const uint4*>(slot + i); }
  __device__ __forceinline__ uint32_t key(uint64_t i) const { return slot[i]; }
  __device__ __forceinline__ void load(uint64_t i, uint32_t& k, uint64_t& p) const {
    k = slot[i];
    p = (uint64_t)__double_as_longlong(val[i]);
  }
};

// Gauges by key range: the record's arrival index rides with its slot (the value stays in the
// caller's array until the winner of each slot is known).
struct GaugeIdxSrc {
  const uint32_t* slot;
  using P = uint32_t;
  bool vec16() const { return false; }  // (arrival order kept within a digit)
  __device__ __forceinline__ void load4(uint64_t, uint32_t*, P*) const {}
  bool key16() const { return ((uintptr_t)slot & 15u) == 0; }
  __device__ __forceinline__ uint4 key4(uint64_t i) const { return *reinterpret_cast<const uint4*>(slot + i); }
  __device__ __forceinline__ uint32_t key(uint64_t i) const { return slot[i]; }
  __device__ __forceinline__ void load(uint64_t i, uint32_t& k, uint32_t& p) const {
    k = slot[i];
    p = (uint32_t)i;
  }
};

// GAUGE = false: out = cval (i64 wrapping sums of pay).
// GAUGE = true : out = gseq (max of base + position + 1); pay unused.
template <bool GAUGE>
__global__ __launch_bounds__(kAggThreads) void k_scalar_agg(uint64_t n, const uint32_t* __restrict__ key,
                                                            const uint64_t* __restrict__ pay, uint64_t base,
                                                            uint64_t* __restrict__ out,
                                                            uint32_t* __restrict__ touch) {
  __shared__ uint32_t s_k[kHash];
  __shared__ unsigned long long s_v[kHash];
  for (uint32_t h = threadIdx.x; h < kHash; h += kAggThreads) {
    s_k[h] = kEmpty;
    s_v[h] = 0;
  }
  __syncthreads();
  const uint64_t c0 = (uint64_t)blockIdx.x * kAggChunk;
  for (int j = 0; j < kAggItems; j++) {
    const uint64_t i = c0 + (uint64_t)j * kAggThreads + threadIdx.x;
    if (i >= n) break;
    const uint32_t s = key[i];
    const unsigned long long v = GAUGE ? (unsigned long long)(i + 1) : (unsigned long long)pay[i];
    uint32_t h = (s * 2654435761u) >> (32 - kHashBits);
    bool done = false;
    for (int p = 0; p < kProbe; p++) {
      uint32_t k = s_k[h];
      if (k == kEmpty) k = atomicCAS(&s_k[h], kEmpty, s);
      if (k == kEmpty || k == s) {
        if (GAUGE) atomicMax(&s_v[h], v);
        else atomicAdd(&s_v[h], v);
        done = true;
        break;
      }
      h = (h + 1) & (kHash - 1);
    }
    if (!done) {
      if (GAUGE) atomicMax((unsigned long long*)&out[s], (unsigned long long)base + v);
      else atomicAdd((unsigned long long*)&out[s], v);
      touch[s] = 1;
    }
  }
  __syncthreads();
  for (uint32_t h = threadIdx.x; h < kHash; h += kAggThreads) {
    const uint32_t s = s_k[h];
    if (s == kEmpty) continue;
    if (GAUGE) atomicMax((unsigned long long*)&out[s], (unsigned long long)base + s_v[h]);
    else atomicAdd((unsigned long long*)&out[s], s_v[h]);
    touch[s] = 1;
  }
}

// The same aggregation straight from the caller's arrays (no partition pass): a block hashes a
// 16384-record chunk of the raw batch into its LDS table (at most kDirectProbe probes; a record
// that finds no entry goes to its device word directly -- the Zipf tail, mostly one record per
// key and chunk), then one device atomic per table entry.  GAUGE: max arrival position.
constexpr int kDirectProbe = 8;
template <bool GAUGE>
__global__ __launch_bounds__(kAggThreads) void k_scalar_direct(uint64_t n, const uint32_t* __restrict__ slot,
                                                               const double* __restrict__ val,
                                                               const float* __restrict__ rate, uint64_t base,
                                                               uint64_t* __restrict__ out,
                                                               uint32_t* __restrict__ touch) {
  __shared__ uint32_t s_k[kHash];
  __shared__ unsigned long long s_v[kHash];
  for (uint32_t h = threadIdx.x; h < kHash; h += kAggThreads) {
    s_k[h] = kEmpty;
    s_v[h] = 0;
  }
  __syncthreads();
  const uint64_t c0 = (uint64_t)blockIdx.x * kAggChunk;
  for (int j = 0; j < kAggItems; j++) {
    const uint64_t i = c0 + (uint64_t)j * kAggThreads + threadIdx.x;
    if (i >= n) break;
    const uint32_t s = slot[i];
    unsigned long long v;
    if (GAUGE) {
      v = (unsigned long long)(i + 1);
    } else {
      const float inv = 1.0f / rate[i];  // float32 division, as Go's 1/sampleRate on a float32
      v = (unsigned long long)((uint64_t)f64_to_i64_go(val[i]) * (uint64_t)f64_to_i64_go((double)inv));
    }
    uint32_t h = (s * 2654435761u) >> (32 - kHashBits);
    bool done = false;
    for (int p = 0; p < kDirectProbe; p++) {
      uint32_t k = s_k[h];
      if (k == kEmpty) k = atomicCAS(&s_k[h], kEmpty, s);
      if (k == kEmpty || k == s) {
        if (GAUGE) atomicMax(&s_v[h], v);
        else atomicAdd(&s_v[h], v);
        done = true;
        break;
      }
      h = (h + 1) & (kHash - 1);
    }
    if (!done) {
      if (GAUGE) atomicMax((unsigned long long*)&out[s], (unsigned long long)base + v);
      else atomicAdd((unsigned long long*)&out[s], v);
      touch[s] = 1;
    }
  }
  __syncthreads();
  for (uint32_t h = threadIdx.x; h < kHash; h += kAggThreads) {
    const uint32_t s = s_k[h];
    if (s == kEmpty) continue;
    if (GAUGE) atomicMax((unsigned long long*)&out[s], (unsigned long long)base + s_v[h]);
    else atomicAdd((unsigned long long*)&out[s], s_v[h]);
    touch[s] = 1;
  }
}

// Counters by key range (the default): one stable partition pass by the slot's high bits puts
// every record of a range of 2^shift slots in one bucket (partition.h), then each block takes a
// kRunChunk slice of the partitioned batch and sums it bucket run by bucket run into an LDS
// array indexed by the slot's low bits -- no hashing, no probing -- and adds each touched slot's
// partial to its device word once per slice.  Device atomics: at most 2^shift per slice (about
// 6M for a 400M-record C4 batch), against one per distinct slot per 16384 records (about 180M)
// for k_scalar_direct, whose requests all go to the memory side.
constexpr int kRunThreads = 512;
constexpr uint64_t kRunChunk = 131072;
constexpr uint32_t kRunMaxW = 4096;  // slots per bucket (LDS: 8 B + 1 B each)
constexpr int kRunUnroll = 4;

// The partition pass writes each counter record as ONE dword: the slot's low `shift` bits (its
// place in the bucket; the bucket is the record's run) and the record's contribution
// int64(v) * int64(float32(1/rate)) as a two's-complement field in the other 32 - shift bits.  A
// contribution outside the field (or equal to its minimum, the escape) is stored whole in the
// payload array at the same position: 4 B per record written and read back instead of 12, the
// 8-byte payload only for the rare large ones.
struct KPackDst {
  uint32_t* key;
  uint64_t* pay;
  int shift;
  static constexpr bool kPacked = true;  // (partition.h: the tile is staged as packed dwords)
  // the dword of record (k, p) bound for position pos; an escaped p is written to pay[pos] now
  __device__ __forceinline__ uint32_t pack(uint64_t pos, uint32_t k, uint64_t p) const {
    const int fb = 32 - shift;
    const int64_t v = (int64_t)p, lim = (int64_t)1 << (fb - 1);
    const uint32_t lowk = shift ? k & ((1u << shift) - 1u) : 0u;
    if (v > -lim && v < lim) return lowk | ((uint32_t)v << shift);
    pay[pos] = p;
    return lowk | ((uint32_t)lim << shift);  // (the field's minimum: escape)
  }
};

__global__ __launch_bounds__(kRunThreads) void k_counter_runs(uint64_t n, const uint32_t* __restrict__ pk,
                                                              const uint64_t* __restrict__ pp,
                                                              const uint32_t* __restrict__ offsets, uint32_t nparts,
                                                              int shift, uint64_t* __restrict__ cval,
                                                              uint32_t* __restrict__ ctouch) {
  __shared__ unsigned long long s_sum[kRunMaxW];
  __shared__ uint8_t s_hit[kRunMaxW];
  const uint32_t W = 1u << shift, t = threadIdx.x;
  const int32_t esc = (int32_t)(0u - (1u << (31 - shift)));  // KPackDst's escape field
  // one packed record (KPackDst): its slot within the bucket and its contribution
  auto unpack = [&](uint64_t r, uint32_t& k, uint64_t& p) {
    if (VN_BAD(r < n, "counter_runs record", r, n)) r = 0;
    const uint32_t x = pk[r];
    const int32_t f = (int32_t)x >> shift;
    k = x & (W - 1u);
    p = f == esc ? pp[r] : (uint64_t)(int64_t)f;
  };
  const uint64_t c0 = (uint64_t)blockIdx.x * kRunChunk, c1 = min(n, c0 + kRunChunk);
  for (uint64_t i = c0; i < c1;) {
    // the bucket of record i -- the last bucket starting at or before it -- and where its run
    // ends in this slice (every thread alike)
    uint32_t lo = 0, hi = 256;
    while (hi - lo > 1) {
      const uint32_t m = (lo + hi) >> 1;
      if ((uint64_t)offsets[(uint64_t)m * nparts] <= i) lo = m;
      else hi = m;
    }
    const uint32_t d = lo;
    const uint64_t e = min(c1, (uint64_t)offsets[(uint64_t)(d + 1) * nparts]);
    for (uint32_t j = t; j < W; j += kRunThreads) {
      s_sum[j] = 0;
      s_hit[j] = 0;
    }
    __syncthreads();
    uint64_t r = i + t;
    for (; r + (kRunUnroll - 1) * kRunThreads < e; r += kRunUnroll * kRunThreads) {
      uint32_t k[kRunUnroll];
      uint64_t p[kRunUnroll];
#pragma unroll
      for (int u = 0; u < kRunUnroll; u++) unpack(r + u * kRunThreads, k[u], p[u]);
#pragma unroll
      for (int u = 0; u < kRunUnroll; u++) {
        atomicAdd(&s_sum[k[u]], (unsigned long long)p[u]);
        s_hit[k[u]] = 1;
      }
    }
    for (; r < e; r += kRunThreads) {
      uint32_t k;
      uint64_t p;
      unpack(r, k, p);
      atomicAdd(&s_sum[k], (unsigned long long)p);
      s_hit[k] = 1;
    }
    __syncthreads();
    const uint32_t sb = d << shift;
    for (uint32_t j = t; j < W; j += kRunThreads)
      if (s_hit[j]) {
        atomicAdd((unsigned long long*)&cval[sb + j], s_sum[j]);
        ctouch[sb + j] = 1;
      }
    __syncthreads();  // the table is cleared for the next run only after every thread read it
    i = e;
  }
}

// Gauges by key range (the default): after the stable partition (GaugeIdxSrc, KV32Dst) a bucket's
// records are in arrival order, so the last record of a slot in a slice is its largest position
// there.  Each block takes a kRunChunk slice run by run, keeps 1 + the slice position of every
// slot's last record in LDS, and offers the winner's arrival index to the slot's device word
// (atomicMax of base + index + 1: across slices and batches the latest arrival wins, as
// Gauge.Sample's plain store does, samplers.go:198-200).
__global__ __launch_bounds__(kRunThreads) void k_gauge_runs(uint64_t n, const uint32_t* __restrict__ pk,
                                                            const uint32_t* __restrict__ pidx,
                                                            const uint32_t* __restrict__ offsets, uint32_t nparts,
                                                            int shift, uint64_t base, uint64_t* __restrict__ gseq,
                                                            uint32_t* __restrict__ gtouch) {
  __shared__ uint32_t s_last[kRunMaxW];
  const uint32_t W = 1u << shift, t = threadIdx.x;
  const uint64_t c0 = (uint64_t)blockIdx.x * kRunChunk, c1 = min(n, c0 + kRunChunk);
  for (uint64_t i = c0; i < c1;) {
    uint32_t lo = 0, hi = 256;
    while (hi - lo > 1) {
      const uint32_t m = (lo + hi) >> 1;
      if ((uint64_t)offsets[(uint64_t)m * nparts] <= i) lo = m;
      else hi = m;
    }
    const uint32_t d = lo;
    const uint64_t e = min(c1, (uint64_t)offsets[(uint64_t)(d + 1) * nparts]);
    for (uint32_t j = t; j < W; j += kRunThreads) s_last[j] = 0;
    __syncthreads();
    uint64_t r = i + t;
    for (; r + (kRunUnroll - 1) * kRunThreads < e; r += kRunUnroll * kRunThreads) {
      uint32_t k[kRunUnroll];
#pragma unroll
      for (int u = 0; u < kRunUnroll; u++) k[u] = pk[r + u * kRunThreads] & (W - 1u);
#pragma unroll
      for (int u = 0; u < kRunUnroll; u++) atomicMax(&s_last[k[u]], (uint32_t)(r + u * kRunThreads - c0 + 1));
    }
    for (; r < e; r += kRunThreads) atomicMax(&s_last[pk[r] & (W - 1u)], (uint32_t)(r - c0 + 1));
    __syncthreads();
    const uint32_t sb = d << shift;
    for (uint32_t j = t; j < W; j += kRunThreads) {
      const uint32_t q = s_last[j];
      if (q) {
        if (VN_BAD(c0 + q - 1 < n, "gauge_runs position", c0 + q - 1, n)) continue;
        if (VN_BAD(pidx[c0 + q - 1] < n, "gauge_runs arrival index", pidx[c0 + q - 1], n)) continue;
        atomicMax((unsigned long long*)&gseq[sb + j], (unsigned long long)(base + pidx[c0 + q - 1] + 1));
        gtouch[sb + j] = 1;
      }
    }
    __syncthreads();
    i = e;
  }
}

// gauges of the direct path: the winning position indexes the caller's value array
__global__ void k_gauge_resolve_direct(uint32_t cap, uint64_t base, uint64_t n, const uint64_t* __restrict__ gseq,
                                       const double* __restrict__ val, double* __restrict__ gval) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= cap) return;
  const uint64_t q = gseq[s];
  if (q > base && !VN_BAD(q - base - 1 < n, "gauge_resolve index", q - base - 1, n)) gval[s] = val[q - base - 1];
  (void)n;
}

__global__ void k_gauge_resolve(uint32_t cap, uint64_t base, const uint64_t* __restrict__ gseq,
                                const uint64_t* __restrict__ pay, double* __restrict__ gval) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= cap) return;
  const uint64_t q = gseq[s];
  if (q > base) gval[s] = __longlong_as_double((long long)pay[q - base - 1]);
}

__global__ void k_counter_import(uint64_t n, const uint32_t* __restrict__ slot, const int64_t* __restrict__ v,
                                 int64_t* __restrict__ cval, uint32_t* __restrict__ ctouch) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicAdd((unsigned long long*)&cval[slot[i]], (unsigned long long)v[i]);
  ctouch[slot[i]] = 1;
}

}  // namespace

void ingest_counters(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val, const float* rate) {
  if (!n) return;
  // buckets of 2^shift slots, at most 256 of them (one partition pass)
  const uint32_t cap = std::max<uint32_t>(e->cap[VN_COUNTER], 1u);
  int shift = 0;
  while (((cap - 1u) >> shift) >= 256u) shift++;
  if (kCounterRuns && (1u << shift) <= kRunMaxW) {
    RadixStats* rs = e->timing ? &e->rstat_c : nullptr;
    const uint32_t nparts =
        partition_pass(CounterSrc{slot, val, rate}, KPackDst{e->pk, e->pp, shift}, n, shift, *e->side_rs, e->side, rs,
                       16 + 4);
    hipLaunchKernelGGL(k_counter_runs, dim3((uint32_t)((n + kRunChunk - 1) / kRunChunk)), dim3(kRunThreads), 0,
                       e->side, n, e->pk, e->pp, partition_bounds(*e->side_rs, nparts), nparts, shift, (uint64_t*)e->cval,
                       e->ctouch);
    return;
  }
  if (kScalarDirect) {
    hipLaunchKernelGGL(k_scalar_direct<false>, dim3(blocks_for(n, kAggChunk)), dim3(kAggThreads), 0, e->side, n,
                       slot, val, rate, 0, (uint64_t*)e->cval, e->ctouch);
    return;
  }
  RadixStats* rs = e->timing ? &e->rstat_c : nullptr;
  partition_pass(CounterSrc{slot, val, rate}, KV64Dst{e->pk, e->pp}, n, 0, *e->side_rs, e->side, rs, 16 + 12);
  hipLaunchKernelGGL(k_scalar_agg<false>, dim3(blocks_for(n, kAggChunk)), dim3(kAggThreads), 0, e->side, n, e->pk,
                     e->pp, 0, (uint64_t*)e->cval, e->ctouch);
}

void import_counters(vn_engine* e, uint64_t n, const uint32_t* slot, const int64_t* val) {
  if (!n) return;
  hipLaunchKernelGGL(k_counter_import, dim3(blocks_for(n, 256)), dim3(256), 0, e->side, n, slot, val, e->cval,
                     e->ctouch);
}

void ingest_gauges(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val) {
  if (!n) return;
  const uint64_t base = e->seq_base;
  e->seq_base += n;
  const uint32_t cap = std::max<uint32_t>(e->cap[VN_GAUGE], 1u);
  int shift = 0;
  while (((cap - 1u) >> shift) >= 256u) shift++;
  if (kGaugeRuns && (1u << shift) <= kRunMaxW && n < (1ull << 32)) {
    RadixStats* rs = e->timing ? &e->rstat_c : nullptr;
    uint32_t* pidx = reinterpret_cast<uint32_t*>(e->pp);
    const uint32_t nparts =
        partition_pass(GaugeIdxSrc{slot}, KV32Dst{e->pk, pidx}, n, shift, *e->side_rs, e->side, rs, 4 + 8);
    hipLaunchKernelGGL(k_gauge_runs, dim3((uint32_t)((n + kRunChunk - 1) / kRunChunk)), dim3(kRunThreads), 0,
                       e->side, n, e->pk, pidx, partition_bounds(*e->side_rs, nparts), nparts, shift, base, e->gseq,
                       e->gtouch);
    hipLaunchKernelGGL(k_gauge_resolve_direct, dim3(blocks_for(cap, 256)), dim3(256), 0, e->side, cap, base, n,
                       e->gseq, val, e->gval);
    return;
  }
  if (kGaugeDirect) {
    hipLaunchKernelGGL(k_scalar_direct<true>, dim3(blocks_for(n, kAggChunk)), dim3(kAggThreads), 0, e->side, n, slot,
                       nullptr, nullptr, base, e->gseq, e->gtouch);
    hipLaunchKernelGGL(k_gauge_resolve_direct, dim3(blocks_for(e->cap[VN_GAUGE], 256)), dim3(256), 0, e->side,
                       e->cap[VN_GAUGE], base, n, e->gseq, val, e->gval);
    return;
  }
  RadixStats* rs = e->timing ? &e->rstat_c : nullptr;
  partition_pass(GaugeSrc{slot, val}, KV64Dst{e->pk, e->pp}, n, 0, *e->side_rs, e->side, rs, 12 + 12);
  hipLaunchKernelGGL(k_scalar_agg<true>, dim3(blocks_for(n, kAggChunk)), dim3(kAggThreads), 0, e->side, n, e->pk,
                     nullptr, base, e->gseq, e->gtouch);
  hipLaunchKernelGGL(k_gauge_resolve, dim3(blocks_for(e->cap[VN_GAUGE], 256)), dim3(256), 0, e->side,
                     e->cap[VN_GAUGE], base, e->gseq, e->pp, e->gval);
}

// metro64 KAT entry point
__global__ void k_metro64(const uint8_t* __restrict__ bytes, const uint32_t* __restrict__ off, uint64_t n,
                          uint64_t seed, uint64_t* __restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = metro64(bytes + off[i], off[i + 1] - off[i], seed);
}
void metro64_batch(const uint8_t* bytes, const uint32_t* off, uint64_t n, uint64_t seed, uint64_t* out,
                   hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_metro64, dim3(blocks_for(n, 256)), dim3(256), 0, st, bytes, off, n, seed, out);
}

}  // namespace vn

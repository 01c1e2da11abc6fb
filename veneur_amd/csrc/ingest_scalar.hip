// ingest_scalar.hip -- counters and gauges.
//
// Counter.Sample (samplers/samplers.go:132-134):
//     c.value += int64(sample) * int64(1/sampleRate)        // 1/sampleRate in float32
// is a wrapping int64 sum, so any grouping of the adds is bit-exact.  Gauge.Sample
// (198-200) keeps the last write in arrival order.
//
// Counters: k_scalar_direct -- each block hashes a 16384-record chunk of the batch into an LDS
// table keyed by slot (wrapping i64 sums), then one device atomic per entry; a record that finds no
// free entry within 8 probes adds to its device word directly.
// Gauges avoid per-record device atomics (a Zipf-hot key would serialise them):
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
constexpr bool kGaugeDirect = false;

struct CounterSrc {
  const uint32_t* slot;
  const double* val;
  const float* rate;
  using P = uint64_t;
  __device__ __forceinline__ uint32_t key(uint64_t i) const { return slot[i]; }
  __device__ __forceinline__ void load(uint64_t i, uint32_t& k, uint64_t& p) const {
    k = slot[i];
    float inv = 1.0f / rate[i];  // float32 division, as Go's 1/sampleRate on a float32
    p = (uint64_t)f64_to_i64_go(val[i]) * (uint64_t)f64_to_i64_go((double)inv);
  }
};

struct GaugeSrc {
  const uint32_t* slot;
  const double* val;
  using P = uint64_t;
  __device__ __forceinline__ uint32_t key(uint64_t i) const { return slot[i]; }
  __device__ __forceinline__ void load(uint64_t i, uint32_t& k, uint64_t& p) const {
    k = slot[i];
    p = (uint64_t)__double_as_longlong(val[i]);
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

// gauges of the direct path: the winning position indexes the caller's value array
__global__ void k_gauge_resolve_direct(uint32_t cap, uint64_t base, const uint64_t* __restrict__ gseq,
                                       const double* __restrict__ val, double* __restrict__ gval) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= cap) return;
  const uint64_t q = gseq[s];
  if (q > base) gval[s] = val[q - base - 1];
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
  if (kGaugeDirect) {
    hipLaunchKernelGGL(k_scalar_direct<true>, dim3(blocks_for(n, kAggChunk)), dim3(kAggThreads), 0, e->side, n, slot,
                       nullptr, nullptr, base, e->gseq, e->gtouch);
    hipLaunchKernelGGL(k_gauge_resolve_direct, dim3(blocks_for(e->cap[VN_GAUGE], 256)), dim3(256), 0, e->side,
                       e->cap[VN_GAUGE], base, e->gseq, val, e->gval);
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

// ingest_scalar.hip -- counters and gauges.
//
// Counter.Sample (samplers/samplers.go:132-134):
//     c.value += int64(sample) * int64(1/sampleRate)        // 1/sampleRate in float32
// is a wrapping int64 sum, so a device-wide atomic add per record is bit-exact in any
// order.  Gauge.Sample (198-200) keeps the last write: each record carries its arrival
// sequence number (window-global), an atomic max picks the winner per slot, and a
// second pass stores the winner's value -- bit-exact for the arrival order of the batch.
#include "kernels.h"

namespace vn {

__global__ void k_counter_ingest(uint64_t n, const uint32_t* __restrict__ slot, const double* __restrict__ val,
                                 const float* __restrict__ rate, int64_t* __restrict__ cval,
                                 uint32_t* __restrict__ ctouch) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = slot[i];
  float inv = 1.0f / rate[i];  // float32 division, as Go's 1/sampleRate on a float32
  uint64_t a = (uint64_t)f64_to_i64_go(val[i]);
  uint64_t b = (uint64_t)f64_to_i64_go((double)inv);
  atomicAdd((unsigned long long*)&cval[s], (unsigned long long)(a * b));
  ctouch[s] = 1;
}

__global__ void k_counter_import(uint64_t n, const uint32_t* __restrict__ slot, const int64_t* __restrict__ v,
                                 int64_t* __restrict__ cval, uint32_t* __restrict__ ctouch) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicAdd((unsigned long long*)&cval[slot[i]], (unsigned long long)v[i]);
  ctouch[slot[i]] = 1;
}

__global__ void k_gauge_seq(uint64_t n, const uint32_t* __restrict__ slot, uint64_t base,
                            uint64_t* __restrict__ gseq, uint32_t* __restrict__ gtouch) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = slot[i];
  atomicMax((unsigned long long*)&gseq[s], (unsigned long long)(base + i + 1));
  gtouch[s] = 1;
}

__global__ void k_gauge_resolve(uint64_t n, const uint32_t* __restrict__ slot, const double* __restrict__ val,
                                uint64_t base, const uint64_t* __restrict__ gseq, double* __restrict__ gval) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = slot[i];
  if (gseq[s] == base + i + 1) gval[s] = val[i];
}

void ingest_counters(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val, const float* rate) {
  if (!n) return;
  hipLaunchKernelGGL(k_counter_ingest, dim3(blocks_for(n, 256)), dim3(256), 0, e->st, n, slot, val, rate, e->cval,
                     e->ctouch);
}

void import_counters(vn_engine* e, uint64_t n, const uint32_t* slot, const int64_t* val) {
  if (!n) return;
  hipLaunchKernelGGL(k_counter_import, dim3(blocks_for(n, 256)), dim3(256), 0, e->st, n, slot, val, e->cval,
                     e->ctouch);
}

void ingest_gauges(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val) {
  if (!n) return;
  uint64_t base = e->seq_base;
  e->seq_base += n;
  hipLaunchKernelGGL(k_gauge_seq, dim3(blocks_for(n, 256)), dim3(256), 0, e->st, n, slot, base, e->gseq, e->gtouch);
  hipLaunchKernelGGL(k_gauge_resolve, dim3(blocks_for(n, 256)), dim3(256), 0, e->st, n, slot, val, base, e->gseq,
                     e->gval);
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

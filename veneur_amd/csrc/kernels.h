// kernels.h -- host launchers of the engine's HIP kernels (one stream per engine).
#pragma once
#include <stdexcept>
#include "engine.h"
#include "gomath.h"
#include "sketch.h"

namespace vn {

constexpr uint32_t kErrDecode = 8u;  // device error flag: malformed import payload
// device error flag: a split key's slot also received vn_ingest records or imports this window
// (its state comes whole from the split combine; the split key's records go through vn_ingest_split)
constexpr uint32_t kErrSplitTouched = 16u;

// A malformed import payload (where the reference's decoder errors or panics): VN_EDECODE.
struct DecodeError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
// after a stream sync: throws DecodeError (and clears the flag) if a decode kernel raised it
void take_decode_error(vn_engine* e);
// Worker.ImportMetric for histograms / timers: Histo.Combine of GobEncode()d digests
// (payload i = bytes[off[i], off[i+1]), device pointers)
void import_histos(vn_engine* e, uint64_t n, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes);
// merge the pending run of imported histogram centroids (before any read of or add to a histogram)
void histo_imports_drain(vn_engine* e);
// Worker.ImportMetric for sets: Set.Combine of MarshalBinary()d sketches
void import_sets(vn_engine* e, uint64_t n, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes);

// The side stream: work issued between side_begin and side_join runs on e->side, after
// everything already issued on the main stream; the main stream waits for it at the join.
void side_begin(vn_engine* e);
void ensure_aux_streams(vn_engine* e, bool fork, bool ctr);  // st3 / st4 / st_ctr at first use
void side_join(vn_engine* e);
// Counter.Sample (samplers.go:132-134) / Counter.Combine (171-183)
void ingest_counters(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val, const float* rate);
void import_counters(vn_engine* e, uint64_t n, const uint32_t* slot, const int64_t* val);
// Gauge.Sample (198-200) / Gauge.Combine (237-249): last write in arrival order wins
void ingest_gauges(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val);
// Histo.Sample (346-356) + MergingDigest.Add/mergeAllTemps (merging_digest.go:97-236)
// rate == nullptr: the records are imported centroids (Histo.Combine) with weights impw
// the histo ingest in two halves: group (sort by key, queue the segment-count read-back) and
// process (wait for the count, replay, remainder rounds); ingest_histos runs both
struct HistoGroups {
  uint64_t *As, *Bs, *Ao, *Bo;  // key-grouped records and the spare pair
};
HistoGroups histo_group(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val, const float* rate);
// records already grouped by key in As/Bs: per-key segments (k_seg_mark, unless the caller marked
// them: marked), the touched-key list
HistoGroups histo_group_sorted(vn_engine* e, uint64_t n, uint64_t* As, uint64_t* Bs, uint64_t* Ao, uint64_t* Bo,
                               bool marked = false);
void histo_process(vn_engine* e, uint64_t n, const HistoGroups& g, const double* impw = nullptr);
void ingest_histos(vn_engine* e, uint64_t n, const uint32_t* slot, const double* val, const float* rate,
                   const double* impw = nullptr);
// Set.Sample (265-267) -> Sketch.Insert (hyperloglog.go:186-200)
// queue the set segment merge held back by ingest_sets while e->set_defer is on (no-op
// otherwise); runs on e->side
void set_finish(vn_engine* e);
void ingest_sets(vn_engine* e, uint64_t n, const uint32_t* slot, const uint32_t* off, const uint8_t* bytes,
                 const uint64_t* hashes);
// k_set_segments over given record ranges (see ingest_set.hip)
void set_replay_ranges(vn_engine* e, const uint64_t* R, const uint32_t* dev_count, const uint32_t* list,
                       uint32_t grid, hipStream_t st);
// split (hot) keys at flush: combine the ranks' partial states on the owners (split.hip)
void split_flush(vn_engine* e);
// hot-key detector (hotkeys.hip): vn_hot_detect, the strided count of a class's records (map:
// split key index -> slot, or null), vn_flush's close of the window, vn_hot_keys
void hot_enable(vn_engine* e, uint32_t stride);
void hot_sample(vn_engine* e, int cls, uint64_t n, const uint32_t* key, const uint32_t* map, uint32_t nmap,
                hipStream_t st);
void hot_rotate(vn_engine* e);
uint32_t hot_collect(vn_engine* e, int cls, uint64_t min_count, uint32_t cap, uint32_t* slot, uint64_t* count);
void hot_destroy(vn_engine* e);
// first ingest call of a window: its start event (vn_timing.ms_main_ready / ms_split_ready)
void window_open(vn_engine* e, hipStream_t st);
void split_destroy(vn_engine* e);
// mergeAllTemps for the given (distinct) histo slots, device list
void histo_merge_pending(vn_engine* e, const uint32_t* dev_keys, uint32_t nkeys);
// MergingDigest.Quantile (kind 0) / CDF (kind 1) per (slot, arg); call histo_merge_pending first
void histo_query(vn_engine* e, int kind, const uint32_t* dev_slot, const double* dev_arg, uint64_t n, double* dev_out);
// exclusive scan of n u32 sizes into n+1 u64 offsets (device arrays)
void scan_sizes_u64(const uint32_t* size, uint64_t* off, uint64_t n, hipStream_t st);
// Histo.Export (GobEncode) / Set.Export (MarshalBinary) of the given slots (device list);
// histo slots must have had their pending temps merged (histo_merge_pending)
void export_histos(vn_engine* e, const uint32_t* dev_slot, uint64_t n, ExportBuffers& x);
void export_sets(vn_engine* e, const uint32_t* dev_slot, uint64_t n, ExportBuffers& x);
void ensure_export_bytes(vn_engine* e, ExportBuffers& x, uint64_t nbytes);
// Worker.Flush + Counter/Gauge/Histo/Set.Flush math; resets the window
// histo_qmask / set_emask: host arrays of cap[class] bytes (1 = percentiles / estimate), or null
void flush_all(vn_engine* e, vn_flush_result* out, const uint8_t* histo_qmask = nullptr,
               const uint8_t* set_emask = nullptr);
// initial (empty-window) state of every slot
void init_state(vn_engine* e);
// metro64 over a batch (KAT entry point)
void metro64_batch(const uint8_t* bytes, const uint32_t* off, uint64_t n, uint64_t seed, uint64_t* out,
                   hipStream_t st);

// ---------------------------------------------------------------- device helpers
// Workgroup barrier for LDS traffic only.  __syncthreads() also waits for every outstanding
// global load (s_waitcnt vmcnt(0)), which would stall register prefetches issued ahead of
// it; these kernels exchange data between threads through LDS only.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// Single-wave workgroups: LDS ordering between the lanes of the wave (DS instructions of a
// wave execute in order; the clobber stops the compiler from moving memory accesses).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

struct SumOp {
  __device__ double operator()(double a, double b) const { return dadd(a, b); }
};
struct MinGoOp {
  __device__ double operator()(double a, double b) const { return min_go(a, b); }
};
struct MaxGoOp {
  __device__ double operator()(double a, double b) const { return max_go(a, b); }
};

// exclusive prefix sum of one u32 per thread across a 256-thread block; total = block sum
__device__ __forceinline__ uint32_t block_scan_sum_u32(uint32_t v, uint32_t* s_wave, uint32_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) s_wave[w] = inc;
  __syncthreads();
  uint32_t base = 0;
  for (int i = 0; i < w; i++) base += s_wave[i];
  total = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
  __syncthreads();
  return base + inc - v;
}

// all-reduce across a 256-thread block (4 waves); s_tmp holds 4 doubles
template <class Op>
__device__ __forceinline__ double block_allreduce(double v, double* s_tmp, Op op) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = op(v, __shfl_xor(v, d, 64));
  if (lane_id() == 0) s_tmp[wave_id()] = v;
  __syncthreads();
  double r = op(op(s_tmp[0], s_tmp[1]), op(s_tmp[2], s_tmp[3]));
  __syncthreads();
  return r;
}
__device__ __forceinline__ uint32_t block_allreduce_u32_sum(uint32_t v, uint32_t* s_tmp) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  if (lane_id() == 0) s_tmp[wave_id()] = v;
  __syncthreads();
  uint32_t r = s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3];
  __syncthreads();
  return r;
}
// exclusive prefix sum (double) of one value per thread in a 256-thread block
__device__ __forceinline__ double block_excl_scan_d(double v, double* s_tmp, double& total) {
  const int lane = lane_id(), w = wave_id();
  double inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    double o = __shfl_up(inc, d, 64);
    if (lane >= d) inc = dadd(inc, o);
  }
  if (lane == 63) s_tmp[w] = inc;
  __syncthreads();
  double base = 0.0;
  for (int i = 0; i < w; i++) base = dadd(base, s_tmp[i]);
  total = dadd(dadd(dadd(s_tmp[0], s_tmp[1]), s_tmp[2]), s_tmp[3]);
  __syncthreads();
  double ex = __shfl_up(inc, 1, 64);
  if (lane == 0) ex = 0.0;
  return dadd(base, ex);
}

}  // namespace vn

/*
 * veneur_amd.h -- C-ABI of the MI355X-native per-flush sketch aggregation engine.
 *
 * This is the drop-in boundary for veneur's aggregation hot path.  Each entry point
 * replaces the body of a Go function on that path (the Go signatures stay; the cgo
 * binding a maintainer adds is in INTEGRATION.md):
 *
 *   vn_engine_create     NewWorker / NewWorkerMetrics / samplers.New*        worker.go:63-76,141-154
 *   vn_stage_acquire     (new) pinned SoA staging the Go side appends to       --
 *   vn_submit            Worker.ProcessMetric body for a staged batch          worker.go:187-227
 *                          Counter.Sample samplers.go:132-134, Gauge.Sample 198-200,
 *                          Set.Sample 265-267 (-> hyperloglog.Insert), Histo.Sample 346-356
 *                          (-> tdigest.MergingDigest.Add merging_digest.go:97-118)
 *   vn_ingest            same, batch already resident in device memory (HBM)
 *   vn_import            Worker.ImportMetric body (decoded JSONMetric values)    worker.go:230-268
 *                          Counter.Combine 171-183, Gauge.Combine 237-249
 *   vn_flush             Worker.Flush + the per-sampler flush math               worker.go:271-298
 *                          Counter.Flush 137-148, Gauge.Flush 203-214,
 *                          Histo.Flush 373-498 (-> MergingDigest.Quantile 283-313),
 *                          Set.Flush 282-293 (-> hyperloglog.Estimate 203-227)
 *   vn_read_histo/_set   state introspection (Histo.Value centroids, Set.Hll registers)
 *   vn_metro64           metro.Hash64 batch (go-metro metro64.go:7-85)
 *
 * Conventions: every function returns 0 on success or a negative VN_E* code; the
 * message is available from vn_last_error(engine).  All buffers handed out by the
 * engine are owned by the engine (the Go side never passes Go-heap pointers for C to
 * retain).  Calls on one engine are serialised by the caller (veneur's Worker mutex).
 * Slots are class-local dense indices assigned by the host's MetricKey interning
 * (one slot table per sampler map: counters, gauges, histograms+timers, sets).
 */
#ifndef VENEUR_AMD_H
#define VENEUR_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history (vn_abi_version; the binding refuses a library of another version):
 *   5  vn_config.max_batch_class_records; vn_flush no longer fails when a split key's slot also
 *      got vn_ingest records or imports -- it drops them, returns VN_OK and sets
 *      VN_WARN_SPLIT_TOUCHED in vn_flush_result.warn_flags (check it after every flush).
 *   6  counter records take any sample rate (Counter.Sample's int64(float32(1/rate)) is defined
 *      for all of them: NaN, 0 and out-of-range reciprocals give MinInt64, as Go on amd64);
 *      histogram rates must still be in (0, 1] (VN_EINVAL otherwise). */
#define VN_ABI_VERSION 6

enum {
  VN_OK = 0,
  VN_EINVAL = -1,   /* bad argument (out-of-range slot, capacity exceeded, ...) */
  VN_EHIP = -2,     /* HIP runtime error */
  VN_ENOMEM = -3,   /* device / pinned allocation failed */
  VN_EDECODE = -4,  /* malformed import payload */
};

enum { VN_COUNTER = 0, VN_GAUGE = 1, VN_HISTO = 2, VN_SET = 3, VN_NCLASS = 4 };

#define VN_MAX_PERCENTILES 16

typedef struct vn_engine vn_engine;

typedef struct {
  int32_t device;                   /* HIP device ordinal */
  uint32_t capacity[VN_NCLASS];     /* slots per class */
  double compression;               /* t-digest delta; veneur uses 100 (samplers.go:364) */
  uint32_t n_percentiles;           /* quantiles evaluated at flush, e.g. .5 .9 .99 .999 */
  double percentiles[VN_MAX_PERCENTILES];
  uint64_t max_batch_records;       /* largest batch per class passed to one ingest call */
  uint64_t max_batch_member_bytes;  /* largest set member blob per ingest call */
  /* t-digest: a key's first `histo_exact_threshold` samples of a window replay
   * MergingDigest's 42-sample incremental merge bit-for-bit (every merge of the reference,
   * in arrival order).  0 (the default) or UINT32_MAX -> every sample of every key: the
   * digests are the reference's.  A smaller value is the opt-in fast mode: samples beyond
   * it are merged in geometric pieces (rank-error parity only).  The shipped
   * library is built without it (vn_build_flags): any other value fails vn_engine_create with
   * VN_EINVAL; a variant build (-DVN_FAST_MODE=1) carries it. */
  uint32_t histo_exact_threshold;
  /* a key that passes the threshold is not bit-exact anyway: only its first
   * `histo_hot_prefix` samples are replayed exactly, the rest merge in geometric pieces
   * (see histo_piece_growth).  0 -> 4096; clamped to the threshold. */
  uint32_t histo_hot_prefix;
  /* size of each such piece, in percent of the key's window samples before it: the pieces
   * are cut at window positions b_0 = prefix, b_{i+1} = b_i + max(1, b_i * growth / 100).
   * 0 -> 25 (tools/tdigest_study.py: <= 8e-4 rank error for 10..25). */
  uint32_t histo_piece_growth;
  /* split keys: records a window may hold per class (histo, set) on this rank; 0 -> none */
  uint64_t split_max_records;
  /* compression of the micro-centroids a rank sends for its share of a split histogram's
   * piece (tools/split_study.py); 0 -> 5 * compression */
  double split_compression;
  /* CUs kept for the longest exact replays (a hot key's chain is one workgroup of four waves,
   * latency-bound for hundreds of ms): rounded up to whole groups of 8 (one CU per XCC), at
   * most a quarter of the device; every other stream of this engine (and of its split engine)
   * is masked off them.  0 (default): none -- the chains share their CUs with whatever else
   * runs.  Measured on C4 with several engines taking the windows in turn: slower at 8-32
   * CUs, kept as an option. */
  uint32_t replay_reserved_cus;
  /* per class (counter, gauge, histo, set): records of that class one ingest or import call
   * may carry, and so the size of that class's sort and partition buffers; 0 ->
   * max_batch_records.  A mixed stream's classes differ by 2-4x (C4: 425M counters, 216M
   * timers per window), and the histo buffers (9 sort arrays) dominate an engine's HBM. */
  uint64_t max_batch_class_records[VN_NCLASS];
} vn_config;

/* One ingest batch: per-class SoA streams in arrival order (the order ProcessMetric saw
 * them).  Pointers are host pointers for vn_submit / vn_ingest_host and device pointers
 * for vn_ingest.  A class with n == 0 may leave its pointers NULL.
 * Sets: either member_off (n+1 offsets into member_bytes) + member_bytes, hashed with
 * metro64(seed 1337), or set_hash (one precomputed 64-bit hash per record, the path the
 * reference's nopHash tests take). */
typedef struct {
  uint64_t n_counter;
  const uint32_t* counter_slot;
  const double* counter_value;
  const float* counter_rate;

  uint64_t n_gauge;
  const uint32_t* gauge_slot;
  const double* gauge_value;

  uint64_t n_histo;
  const uint32_t* histo_slot;
  const double* histo_value;
  const float* histo_rate;

  uint64_t n_set;
  const uint32_t* set_slot;
  const uint32_t* set_member_off;
  const uint8_t* set_member_bytes;
  const uint64_t* set_hash;
} vn_batch;

/* Counts for a batch the caller wrote into the engine's pinned stage. */
typedef struct {
  uint64_t n_counter, n_gauge, n_histo, n_set, n_set_member_bytes;
} vn_batch_counts;

/* Writable views of the engine-owned pinned staging buffers (capacity = max_batch_*). */
typedef struct {
  uint64_t capacity;
  uint64_t member_bytes_capacity;
  uint32_t* counter_slot; double* counter_value; float* counter_rate;
  uint32_t* gauge_slot; double* gauge_value;
  uint32_t* histo_slot; double* histo_value; float* histo_rate;
  uint32_t* set_slot; uint32_t* set_member_off; uint8_t* set_member_bytes;
} vn_stage;

/* Flush result: one entry per slot touched in the window (Upsert semantics), in ascending
 * slot order per class.  Engine-owned host memory, valid until the next vn_flush. */
typedef struct {
  uint64_t n_counter;
  const uint32_t* counter_slot;
  const int64_t* counter_value;        /* Counter.value (Flush emits float64(value)) */

  uint64_t n_gauge;
  const uint32_t* gauge_slot;
  const double* gauge_value;

  uint64_t n_histo;
  const uint32_t* histo_slot;
  /* per histo, VN_HISTO_STATS doubles: LocalWeight, LocalMin, LocalMax, LocalSum,
   * LocalReciprocalSum, digest min, digest max, digest count (mainWeight) */
  const double* histo_stats;
  /* per histo, n_percentiles doubles: MergingDigest.Quantile(p) (NaN when empty) */
  const double* histo_quantiles;
  uint32_t n_percentiles;

  uint64_t n_set;
  const uint32_t* set_slot;
  const uint64_t* set_estimate;        /* Sketch.Estimate() */
  const uint8_t* set_sparse;           /* 1 = sparse representation at flush */

  uint64_t samples_processed;          /* records ingested this window (worker.processed) */
  uint64_t samples_imported;           /* imported values this window (worker.imported) */
  /* The caller's misuse seen this window; the flush itself completed (VN_OK) and every output
   * above is valid.  VN_WARN_SPLIT_TOUCHED: a split key's slot also received vn_ingest records
   * or imports (its records belong to vn_ingest_split); the split combine's state was kept and
   * those records were dropped. */
  uint64_t warn_flags;
} vn_flush_result;
#define VN_WARN_SPLIT_TOUCHED 16u
#define VN_HISTO_STATS 8

/* Sparse / dense sketch state of one set slot (axiomhq Sketch fields). */
typedef struct {
  uint8_t touched, sparse, b, pad;
  uint32_t nz;            /* registers.nz (dense) */
  uint32_t list_count;    /* compressedList.count (sparse) */
  uint32_t list_bytes;    /* len(compressedList.b) (sparse) */
  uint32_t list_last;     /* compressedList.last */
  uint32_t tmp_count;     /* len(tmpSet) */
} vn_set_state;

int vn_engine_create(const vn_config* cfg, vn_engine** out);
void vn_engine_destroy(vn_engine* eng);
const char* vn_last_error(const vn_engine* eng);
int vn_abi_version(void);
/* Compile-time options of this library: VN_BUILD_FAST_MODE when the t-digest fast mode
 * (histo_exact_threshold > 0) is built in -- never in the shipped library. */
enum { VN_BUILD_FAST_MODE = 1 };
int vn_build_flags(void);
/* sizeof the library's structs, so a binding built against another header revision fails at
 * load time instead of passing a short vn_config or receiving a long vn_timing.  Returns 0
 * for an unknown id. */
enum { VN_STRUCT_CONFIG = 0, VN_STRUCT_BATCH = 1, VN_STRUCT_FLUSH_RESULT = 2, VN_STRUCT_TIMING = 3,
       VN_STRUCT_SPLIT_BATCH = 4, VN_STRUCT_STAGE = 5 };
size_t vn_struct_size(int which);

int vn_stage_acquire(vn_engine* eng, vn_stage* out);
/* stage -> HBM -> ingest; returns once the stage has been copied (it may be refilled at once) */
int vn_submit(vn_engine* eng, const vn_batch_counts* counts);
int vn_ingest_host(vn_engine* eng, const vn_batch* host_batch);  /* copies through the stage */
/* Inputs already in HBM.  The batch is validated on the device before anything is applied --
 * slots within capacity, histo values finite (merging_digest.go:98-100), counter / histo rates
 * in (0, 1], set member offsets non-decreasing -- and a faulty batch fails with VN_EINVAL and
 * leaves the window unchanged (vn_ingest_host checks the same on the host). */
int vn_ingest(vn_engine* eng, const vn_batch* device_batch);

/* ImportMetric for decoded values (Counter.Combine adds int64, Gauge.Combine overwrites in
 * arrival order); they target the GlobalOnly slot tables the host chose. */
int vn_import_counters(vn_engine* eng, const uint32_t* slot, const int64_t* value, uint64_t n);
int vn_import_gauges(vn_engine* eng, const uint32_t* slot, const double* value, uint64_t n);

/* ImportMetric for histograms and timers (worker.go:253-266): Histo.Combine
 * (samplers.go:519-526) of each payload = the forwarded MergingDigest.GobEncode() bytes
 * (merging_digest.go:361-380), payload i = bytes[off[i], off[i+1]), into histo slot[i], in
 * order.  Every centroid is Add()ed to the key's digest (MergingDigest.Merge, 344-356, in the
 * stored order instead of rand.Perm); Local* statistics are untouched.  A malformed payload, or
 * a centroid Add() would panic on, fails the whole call with VN_EDECODE and applies nothing. */
int vn_import_histos(vn_engine* eng, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes, uint64_t n);

/* ImportMetric for sets (worker.go:248-252): Set.Combine (samplers.go:313-325) of each payload
 * = the forwarded Sketch.MarshalBinary() bytes (hyperloglog.go:270-315), payload i =
 * bytes[off[i], off[i+1]), into set slot[i], in order: UnmarshalBinary + Sketch.Merge
 * (hyperloglog.go:92-149), bit-exact (a sparse payload's tmpSet is merged in ascending order
 * where Go iterates a map).  A payload of another precision is skipped, as Merge's error is
 * only logged; a truncated payload fails the whole call with VN_EDECODE and applies nothing. */
int vn_import_sets(vn_engine* eng, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes, uint64_t n);

/* The same two imports with slot/off/bytes already in device memory (HBM), e.g. payloads
 * another GPU's export sent by an RCCL all-gather (veneur_amd/dist.py hot-key exchange).
 * The call returns once the work is queued on the engine's streams, and the histo import's
 * centroid emits read the payload buffers on a stream of their own after it returns: the caller
 * keeps slot/off/bytes allocated and unmodified until the engine's next synchronizing call
 * (vn_flush / vn_flush_masked, vn_sync, a host-array import or query) has returned. */
int vn_import_histos_device(vn_engine* eng, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes,
                            uint64_t n);
int vn_import_sets_device(vn_engine* eng, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes, uint64_t n);

/* MergingDigest.Quantile (kind 0, merging_digest.go:283-313) or CDF (kind 1, 247-279) of
 * histo slot[i]'s digest in the current window at arg[i], into out[i] (host arrays).  As in
 * the reference the pending temps are merged first (mergeAllTemps mutates the digest).
 * Quantile arguments outside [0, 1] are rejected (the reference panics). */
int vn_histo_query(vn_engine* eng, int kind, const uint32_t* slot, const double* arg, uint64_t n, double* out);

/* Forward encoders (flushForward, flusher.go:264-353): one payload per requested slot, in
 * request order, as the JSONMetric.Value a local veneur POSTs to its global.
 *   vn_export_histos  Histo.Export (samplers.go:501-514) = MergingDigest.GobEncode
 *                     (merging_digest.go:361-380); merges the key's pending temps first, as
 *                     GobEncode does
 *   vn_export_sets    Set.Export (samplers.go:296-310) = Sketch.MarshalBinary
 *                     (hyperloglog.go:270-315), tmpSet in ascending order (Go: map order)
 * The result (host and device views) is engine-owned and valid until the next export call;
 * the device view feeds a GPU-to-GPU exchange (RCCL all-gather) of hot keys directly. */
typedef struct {
  uint64_t n;
  const uint64_t* off;        /* n + 1 offsets into bytes (pinned host memory) */
  const uint8_t* bytes;
  const uint64_t* dev_off;    /* the same in device memory */
  const uint8_t* dev_bytes;
} vn_export;
int vn_export_histos(vn_engine* eng, const uint32_t* slot, uint64_t n, vn_export* out);
int vn_export_sets(vn_engine* eng, const uint32_t* slot, uint64_t n, vn_export* out);

/* Hot-key detector: the split list of the next window (vn_split_keys), chosen by the engine
 * from the window it has seen.  The reference routes every record of a key to one worker
 * (server.go:655); the split is this build's addition, so it brings its own detector.
 * vn_hot_detect: from now on count every stride-th record of each vn_ingest / vn_ingest_host
 * call and of the split records of vn_ingest_split (counters, histos, sets), per slot; 0 turns
 * it off, 1 counts exactly.  vn_hot_keys: after vn_flush, the slots of class cls (VN_COUNTER,
 * VN_HISTO or VN_SET) of the flushed window whose estimated count (sampled count x stride) is
 * at least min_count, hottest first (ties: ascending slot), at most cap of them, with their
 * estimated counts (count may be NULL); *n = how many were written. */
int vn_hot_detect(vn_engine* eng, uint32_t stride);
int vn_hot_keys(vn_engine* eng, int cls, uint64_t min_count, uint32_t cap, uint32_t* slot, uint64_t* count,
                uint32_t* n);
int vn_flush(vn_engine* eng, vn_flush_result* out);
/* vn_flush for a local veneur (flusher.go:41-48,168-230): the percentiles of a histogram are
 * evaluated only where histo_quantile_mask[slot] != 0 (the others come back NaN: Server.Flush
 * passes percentiles=nil for mixed-scope histograms and timers, whose digests are forwarded
 * instead), and a set is estimated only where set_estimate_mask[slot] != 0 (mixed-scope sets
 * are forwarded, not flushed; their estimate comes back 0).  Either mask may be NULL (= all);
 * otherwise it holds capacity[VN_HISTO] / capacity[VN_SET] bytes. */
int vn_flush_masked(vn_engine* eng, const uint8_t* histo_quantile_mask, const uint8_t* set_estimate_mask,
                    vn_flush_result* out);
int vn_sync(vn_engine* eng);

/* Introspection of the current (unflushed) window. */
int vn_read_histo(vn_engine* eng, uint32_t slot, double* means, double* weights, uint32_t cap,
                  uint32_t* n_centroids, double* stats /* VN_HISTO_STATS */);
int vn_read_set(vn_engine* eng, uint32_t slot, vn_set_state* st, uint32_t* list_codes,
                uint32_t list_cap, uint32_t* tmp_codes, uint32_t tmp_cap, uint8_t* registers /* 16384 */);

/* Kernel-level entry points (known-answer checks of the HIP primitives). */
int vn_metro64(int device, const uint8_t* bytes, const uint32_t* off, uint64_t n, uint64_t seed,
               uint64_t* out);

/* Device memory helpers for callers without another HIP binding (bench / tests). */
int vn_device_alloc(int device, uint64_t bytes, void** out);
int vn_device_free(void* p);
int vn_copy_to_device(int device, void* dst, const void* src, uint64_t bytes);
int vn_device_copy(int device, void* dst, const void* src, uint64_t bytes);  /* device to device */
int vn_copy_to_host(int device, void* dst, const void* src, uint64_t bytes);
int vn_device_count(int* n);
int vn_device_synchronize(int device);

/* Timing of the last ingest+flush's kernels on the engine's stream (HIP events):
 * milliseconds of the histo sort passes, of everything, and per-phase counters. */
typedef struct {
  float ms_ingest_counter, ms_ingest_gauge, ms_ingest_histo, ms_ingest_set, ms_flush;
  float ms_sort_histo, ms_sort_set;
  uint64_t sort_passes_histo, sort_passes_set;
  float ms_radix_scatter_total;   /* sum over k_radix_scatter launches */
  uint64_t radix_scatter_launches;
  uint64_t radix_scatter_bytes;   /* algorithmic bytes moved by those launches */
  /* the exact t-digest replay (k_histo_exact): launches, time, algorithmic bytes = 16 B per
   * replayed sample + per replayed key 40 B of local statistics and 16 B per centroid written
   * (min(samples, 160) at delta 100) -- SURVEY.md §8(d) */
  float ms_histo_replay;
  uint64_t histo_replay_launches;
  uint64_t histo_replay_bytes;
  /* the HLL state machine (k_set_segments): 8 B per grouped record it reads (its per-key
   * state traffic is left out: a lower bound) */
  float ms_set_segments;
  uint64_t set_segment_launches;
  uint64_t set_segment_bytes;
  /* host wall clock of the last vn_flush (filled with timing on or off): the whole call, and
   * the split combine inside it (its waits are for the split engine's stream only) */
  float ms_flush_host;
  float ms_split_host;
  /* device clock from the window's first ingest call to: this engine's ingest work done (all
   * of it queued before vn_flush), and the split combine done (0 without split keys) */
  float ms_main_ready;
  float ms_split_ready;
  /* inside the split combine: histograms done, sets' gathered prefix replayed */
  float ms_split_histo_ready;
  float ms_split_set_prefix_ready;
  /* counter / gauge partition scatter (k_part_scatter): 16 + 12 B (counter) or 12 + 12 B (gauge)
   * per record read and written; the radix figures above cover k_radix_scatter only */
  float ms_part_scatter;
  uint64_t part_scatter_launches;
  uint64_t part_scatter_bytes;
  /* imports (vn_import_histos*): the digest decode's kernels (count and emit passes), and the
   * drains of the imported centroids through the exact replay (grouping sort, chunk sort, replay) */
  float ms_import_decode;
  float ms_import_drain;
} vn_timing;
int vn_timing_enable(vn_engine* eng, int enable);
/* The import contributions decoded while timing is on (SURVEY.md §8(d)'s C5 bytes: 16 B per
 * centroid, 8192 B per dense sketch, 4 B per sparse code): out5 = {histo payloads, their
 * centroids, set payloads, dense set payloads, sparse set codes}, summed since the last reset;
 * reset != 0 zeroes them after the read. */
int vn_import_counts(vn_engine* eng, uint64_t* out5, int reset);
int vn_get_timing(vn_engine* eng, vn_timing* out);

/* ---------------------------------------------------------------- multi-GPU
 * One engine per GPU (one process per GPU); keys are sharded the way veneur routes them to
 * workers, Digest % N (server.go:655, samplers/parser.go:213-304), so ordinary keys need no
 * exchange.  A key too hot for one GPU is *split*: the host deals its records round-robin over
 * the ranks by the key's window arrival index (record j of the key goes to rank j % N, so the
 * i-th split record a rank holds is the key's record j = rank + N*i), and at vn_flush the
 * partial states meet on the key's owner rank (Digest % N) -- the reference's local -> global
 * combine (flusher.go:264-353 -> handlers_global.go:53-63 -> worker.go:230-268) done over xGMI:
 *   counters  ncclAllReduce(sum, int64): exact (Counter.Combine)
 *   sets      the exact HLL state of the whole ordered stream (bit-identical to one Sketch
 *             that saw every record): the sparse phase from the gathered first records, then
 *             rebase epochs by ncclAllReduce min (first-fill positions, rebase candidates) and
 *             max (registers, uint8) -- the all-reduce-max fast path whenever no rebase occurs
 *   histos    Local* statistics by all-reduce (sum/min/max); the digest on the owner: the first
 *             histo_hot_prefix records replayed exactly (gathered), then one mergeAllTemps per
 *             geometric piece of the window over every rank's share of that piece, each share
 *             sorted and compressed on its own rank into micro-centroids (compression
 *             split_compression) and sent to the owner (grouped ncclSend/ncclRecv)
 * Gauges are never split (last write wins needs the arrival order; their ingest is cheap).
 * The communicator is RCCL (vn_comm_init, ids from vn_comm_unique_id on rank 0 passed over the
 * host's control plane), or an in-process group of engines on one device (vn_comm_init_local:
 * each rank's vn_flush runs in its own host thread; tests on one GPU).  Without a communicator
 * an engine is a group of one. */
typedef struct vn_comm vn_comm;
#define VN_COMM_ID_BYTES 128
enum { VN_DT_U8 = 0, VN_DT_U32 = 1, VN_DT_U64 = 2, VN_DT_I64 = 3, VN_DT_F64 = 4 };
enum { VN_OP_SUM = 0, VN_OP_MAX = 1, VN_OP_MIN = 2 };
int vn_comm_unique_id(uint8_t* id /* VN_COMM_ID_BYTES */);                       /* ncclGetUniqueId */
int vn_comm_init(const uint8_t* id, int nranks, int rank, int device, vn_comm** out);  /* ncclCommInitRank */
int vn_comm_init_local(int nranks, int device, vn_comm** out /* nranks handles */);
void vn_comm_destroy(vn_comm* comm);
const char* vn_comm_last_error(const vn_comm* comm);
int vn_comm_rank(const vn_comm* comm);
int vn_comm_nranks(const vn_comm* comm);
/* control-plane all-reduce of a device buffer (synchronous) */
int vn_comm_allreduce(vn_comm* comm, const void* send, void* recv, uint64_t count, int dtype, int op);
/* the engine exchanges its split keys over comm at vn_flush (comm outlives the engine's use) */
int vn_engine_set_comm(vn_engine* eng, vn_comm* comm);

/* The split keys of the current window, per class (counter, histo, set; gauges cannot be
 * split): the same list in the same order on every rank, slot[i] = this rank's slot of key i,
 * owner[i] = the rank that flushes it (Digest % N).  Host arrays.  Set before the window's
 * first ingest; cleared by vn_flush. */
int vn_split_keys(vn_engine* eng, int cls, const uint32_t* slot, const uint32_t* owner, uint32_t n);
/* Records of split histos / sets (device arrays), in this rank's arrival order; key = index into
 * the class's split list.  Split counters go through vn_ingest like any counter. */
typedef struct {
  uint64_t n_histo;
  const uint32_t* histo_key;
  const double* histo_value;
  const float* histo_rate;
  uint64_t n_set;
  const uint32_t* set_key;
  const uint32_t* set_member_off;
  const uint8_t* set_member_bytes;
  const uint64_t* set_hash;
} vn_split_batch;
int vn_ingest_split(vn_engine* eng, const vn_split_batch* device_batch);
/* No more split records this window: the split histos / sets start combining now, in a host
 * thread of the engine's own (their collectives are issued there), while the caller goes on
 * with vn_ingest; vn_flush / vn_split_combine join it.  Until then vn_split_keys and
 * vn_ingest_split fail, and the group must not change.  Optional: without it the combine runs
 * inside vn_flush. */
int vn_split_close(vn_engine* eng);
/* Combine the split keys now (collective over the group; vn_flush does it when they are still
 * pending): afterwards the owners hold each split key's state in its slot, the other ranks
 * have cleared theirs, and the split lists are empty.  Returns once the exchange is issued
 * (every later operation of the engine is ordered after it); it does not wait for the
 * window's own replays, so engines taking windows in turn can enter their combines in window
 * order without one window's replays holding up the next.  (With an RCCL group; the in-process
 * group of vn_comm_init_local, a test device, copies between its ranks' buffers and waits for
 * the counters' stream, which holds only the counter aggregation and the combine itself.) */
int vn_split_combine(vn_engine* eng);

/* DogStatsD metric lines (host code, no GPU): samplers/parser.go:186-307 ParseMetric over a
 * datagram split on '\n' (server.go:706-714), empty packets skipped (server.go:612-616).
 * Returns the number of non-empty lines written to out (<0 on error); joined sorted tags go to
 * tags_out. Replaces the Go parse in front of vn_stage_acquire/vn_submit. */
enum {
  VN_PARSE_OK = 0, VN_PARSE_NO_COLON, VN_PARSE_EMPTY_NAME, VN_PARSE_NO_PIPE, VN_PARSE_NO_TYPE,
  VN_PARSE_BAD_TYPE, VN_PARSE_BAD_VALUE, VN_PARSE_EMPTY_SECTION, VN_PARSE_MULTI_RATE,
  VN_PARSE_BAD_RATE, VN_PARSE_RATE_RANGE, VN_PARSE_MULTI_TAGS, VN_PARSE_UNKNOWN_SECTION,
  VN_PARSE_NOT_METRIC, VN_PARSE_TAGS_FULL
};
typedef struct {
  uint64_t line_off, name_off, value_off, tags_off; /* name/value into buf, tags into tags_out */
  double value;                                     /* non-set types */
  uint32_t line_len, name_len, value_len, tags_len, n_tags, digest;
  float rate;
  int32_t status;                                   /* VN_PARSE_* */
  uint8_t type, scope, has_tags, pad;               /* type: counter gauge histogram timer set */
} vn_parsed_line;
int64_t vn_parse_dogstatsd(const char* buf, uint64_t len, vn_parsed_line* out, uint64_t max_lines,
                           char* tags_out, uint64_t tags_cap);

/* The same parse on the GPU (csrc/parse_device.hip): buf, out and tags_out are device memory and
 * the result is identical to vn_parse_dogstatsd's, line for line and byte for byte in tags_out.
 * A parser owns its stream and scratch for buffers of up to max_bytes (< 4 GiB) bytes holding up
 * to max_lines lines.  tags_cap must be at least len (joined tags never outgrow their lines, so
 * VN_PARSE_TAGS_FULL cannot occur); *n_lines gets the number of non-empty lines.  More than
 * max_lines lines: VN_EINVAL, nothing written to out. */
typedef struct vn_parser vn_parser;
int vn_parser_create(int device, uint64_t max_bytes, uint64_t max_lines, vn_parser** out);
void vn_parser_destroy(vn_parser* p);
const char* vn_parser_last_error(const vn_parser* p);
int vn_parse_dogstatsd_device(vn_parser* p, const char* buf, uint64_t len, vn_parsed_line* out, uint64_t max_lines,
                              char* tags_out, uint64_t tags_cap, uint64_t* n_lines);
/* Device intake: the ProcessMetric path for DogStatsD text (csrc/intake.hip).  For a buffer of
 * datagram lines in HBM: the device parse above, then Worker.ProcessMetric (worker.go:187-227) for
 * every line that parses -- Upsert (worker.go:81-138) of its MetricKey into the window's key table
 * on the device (ten maps by type x scope; a new key takes the next slot of its class, in line
 * order, as the host Worker's interning does), then one vn_ingest of the staged records.  Counter
 * and histogram/timer lines with a NaN sample rate are dropped and counted (the parser accepts
 * NaN, the engine rejects it).  A buffer whose new keys pass a class's capacity fails with
 * VN_EINVAL and leaves the table and the window unchanged.  vn_intake_upsert interns keys the
 * host hands in (ImportMetric's Upsert, worker.go:230-268: map id 0..9 = counters,
 * global_counters, gauges, global_gauges, histograms, local_histograms, timers, local_timers, sets,
 * local_sets; digest = FNV-1a of name, type name and joined tags) into the same table; slot_out
 * gets each key's slot.  vn_intake_read_keys returns the window's keys (creation order) for
 * Worker.Flush's samplers; vn_intake_reset starts a new window (after vn_flush). */
typedef struct vn_intake vn_intake;
typedef struct {
  uint64_t lines;         /* non-empty lines */
  uint64_t processed;     /* ProcessMetric calls (records ingested) */
  uint64_t parse_errors;  /* lines ParseMetric rejects (logged and skipped, server.go:700-704) */
  uint64_t dropped;       /* NaN sample rates */
  uint64_t new_keys;      /* keys first seen in this buffer */
} vn_intake_stats;
typedef struct {
  uint64_t n_keys, arena_bytes;
  uint32_t next_slot[VN_NCLASS];
} vn_intake_info;
int vn_intake_create(vn_engine* eng, uint64_t max_bytes, uint64_t max_lines, vn_intake** out);
void vn_intake_destroy(vn_intake* in);
const char* vn_intake_last_error(const vn_intake* in);
int vn_intake_process(vn_intake* in, const char* buf, uint64_t len, vn_intake_stats* stats);
int vn_intake_upsert(vn_intake* in, uint64_t n, const uint8_t* map, const uint32_t* n_tags, const uint32_t* digest,
                     const uint32_t* name_off, const uint32_t* name_len, const uint32_t* tags_off,
                     const uint32_t* tags_len, const uint8_t* bytes, uint64_t nbytes, uint32_t* slot_out);
int vn_intake_keys_info(vn_intake* in, vn_intake_info* info);
/* host arrays of info.n_keys entries (arena: info.arena_bytes; a key's joined tags follow its name) */
int vn_intake_read_keys(vn_intake* in, uint8_t* map, uint32_t* slot, uint32_t* n_tags, uint64_t* name_off,
                        uint32_t* name_len, uint32_t* tags_len, uint8_t* arena);
int vn_intake_reset(vn_intake* in);

/* ---------------------------------------------------------------- flush egress (host code)
 * vn_datadog_flush: Server.Flush's metric output for the Datadog sink, natively from a flush result
 * (csrc/sink.cpp): generateInterMetrics (flusher.go:168-230) with the is_local rules, the samplers'
 * Flush (samplers.go:136-498: names, aggregates, "%s.%dpercentile"), finalizeMetrics
 * (sinks/datadog/datadog.go:160-213: routing, counters as rates, sink tags, host:/device: tags),
 * Flush's chunking (77-106) and each chunk's body as PostHelper encodes it before compression
 * (http/http.go:116-135: json.NewEncoder.Encode({"series": chunk}), Go 1.9 encoding/json).  Keys:
 * the window's MetricKeys as vn_intake_read_keys returns them (map id, slot, tag count, name and
 * joined tags).  A chunk holding NaN or Inf cannot be encoded (UnsupportedValueError): its status
 * is VN_EINVAL and its body empty, as Go posts nothing for it.  Output owned by the sink, valid
 * until its next call. */
typedef struct {
  uint64_t n_keys;
  const uint8_t* map;        /* 0..9: counters, global_counters, gauges, global_gauges, histograms,
                                local_histograms, timers, local_timers, sets, local_sets */
  const uint32_t* slot;
  const uint32_t* n_tags;
  const uint64_t* name_off;  /* into arena; the joined tags follow the name */
  const uint32_t* name_len;
  const uint32_t* tags_len;
  const uint8_t* arena;
} vn_keys;
typedef struct {
  double interval;                          /* flush interval in seconds (dd.interval) */
  int64_t timestamp;                        /* InterMetric.Timestamp (Unix seconds) */
  int32_t is_local;
  uint32_t aggregates;                      /* HistogramAggregates.Value (samplers.go:60-68 bits) */
  uint32_t n_percentiles;                   /* Server.HistogramPercentiles */
  double percentiles[VN_MAX_PERCENTILES];
  const double* engine_percentiles;         /* the flush result's quantile columns (vn_config order) */
  const char* hostname;                     /* dd.hostname */
  const char* sink_tags;                    /* dd.tags joined by ',' */
  uint32_t n_sink_tags;
  uint32_t flush_max_per_body;              /* dd.flushMaxPerBody */
} vn_dd_config;
typedef struct {
  uint64_t n_intermetrics;   /* generateInterMetrics output */
  uint64_t n_metrics;        /* DDMetrics after finalizeMetrics */
  uint32_t n_bodies;
  const uint64_t* body_off;  /* n_bodies + 1 offsets into bytes */
  const int32_t* body_status;
  const uint8_t* bytes;
} vn_dd_payload;
typedef struct vn_sink vn_sink;
int vn_sink_create(vn_sink** out);
void vn_sink_destroy(vn_sink* s);
const char* vn_sink_last_error(const vn_sink* s);
int vn_datadog_flush(vn_sink* s, const vn_flush_result* f, const vn_keys* keys, const vn_dd_config* cfg,
                     vn_dd_payload* out);

/* Diagnostic (tests): indexEstimate(compression, q[i]) (merging_digest.go:240-243) as the replays
 * evaluate it (divisions without the hardware's rescaling and fix-up steps) against the full
 * correctly rounded division sequence, on the GPU; *mismatches = values whose bits differ. */
int vn_diag_index_estimate(int device, double compression, const double* q, uint64_t n, uint64_t* mismatches,
                           double* out /* optional: 2n values, the replays' and the full division's, or null */);

/* strconv.ParseFloat(s, bits) of Go 1.9 (bits 64 or 32) as the device parser computes it, run on
 * the host: 0 ok, 1 syntax error, 2 out of range (ErrRange); *out the value (float32 widened). */
int vn_go_parse_float(const char* s, uint64_t n, int bits, double* out);

#ifdef __cplusplus
}
#endif
#endif

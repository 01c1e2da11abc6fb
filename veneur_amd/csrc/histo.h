// histo.h -- shared declarations of the t-digest (Histo) kernels.
#pragma once
// The opt-in fast mode (histo_exact_threshold > 0: past the threshold a key's window is merged
// in geometric pieces, not replayed -- DESIGN.md §4) is not in the shipped library: it cannot meet
// north_star's 1e-3 rank bound.  A variant build with VARIANT_FLAGS=-DVN_FAST_MODE=1 carries it.
#ifndef VN_FAST_MODE
#define VN_FAST_MODE 0
#endif
#include <stdexcept>

#include "kernels.h"

namespace vn {

// chunk geometry of the hot-key batch-merge kernels (ingest_histo.hip): small chunks spread a
// hot key's segment over many workgroups, since only a few hundred keys take that path
constexpr uint32_t kHItems = 4;
constexpr uint32_t kHTile = kBlock * kHItems;  // 1024 elements per chunk
constexpr uint32_t kChunkStats = 7;  // per chunk: Local weight/min/max/sum/rsum, digest min/max

// Tags in the low 32 bits of a histo element (B word):
//   sample            float32 bits of its sample rate: weight float64(float32(1) / rate)
//                     (samplers.go:347); Histo's Local* statistics count it
//   kTagImport | i    a centroid of an imported digest (Histo.Combine): weight impw[i]; it
//                     counts for the digest (Add updates min/max) but not for Local*
//   kTagCentroid | i  an existing centroid of the key (hot-key batch merge), weight from the
//                     centroid tile
constexpr uint32_t kTagCentroid = 0x80000000u;
constexpr uint32_t kTagImport = 0x40000000u;
constexpr uint32_t kTagIndex = 0x3fffffffu;
__device__ __forceinline__ bool tag_is_sample(uint32_t tag) { return (tag & (kTagCentroid | kTagImport)) == 0; }
__device__ __forceinline__ double tag_weight(uint32_t tag, const double* impw) {
  return (tag & kTagImport) ? impw[tag & kTagIndex] : (double)(1.0f / __uint_as_float(tag));
}

struct ExactCtx {
  uint32_t nkeys;
  const uint32_t* nkeys_dev;  // (null: nkeys) the live keys' count on the device when nkeys is only an upper
                              // bound (an ingest that does not wait for the count): keys past it are absent
  uint32_t long_min;  // chunk sorter: every record's ctw / cpk only for keys of at least this many exact records
                      // (the four-wave and batched replays read them; the one-wave replay only a chunk's
                      // first); 0: for every key
  const uint32_t* keys;      // slot of each processed key
  const uint32_t* order;     // replay only: key indices of this launch (nullptr: 0..nkeys-1)
  uint32_t norder;           // replay grid when order is set
  double* cstat;             // per pure chunk: its Local* partials (8 doubles, as lstat), written by the chunk
                             // sorter, summed by k_exact_long_stats; null: the latter reads the samples
  const uint32_t* mw_count;  // replay: the first *mw_count entries of order64 are replayed by the four-wave kernel,
                             // the first mw_count[1] of them batched (k_histo_exact_mwb)
  const uint64_t* order64;   // replay only: key index in the low 32 bits, longest first (norder)
  const uint32_t* start;     // per slot: first record of its segment (arrival order)
  const uint32_t* nex;       // per processed key: records to replay exactly (nullptr: none)
  const uint32_t* hot;       // per processed key: 1 -> merge pending temps after the exact part
  const uint64_t* A;         // raw float64 bits of the value
  const uint64_t* B;         // slot<<32 | tag (see above)
  const double* impw;        // weights of imported centroids (kTagImport)
  double delta;
  uint32_t capc, tcap;
  double* hst;
  uint32_t* hncent;
  uint8_t* hcur;
  double* cm0;
  double* cm1;
  double* cw0;
  double* cw1;
  uint32_t* hpend;
  double* hpv;
  double* hpw;
  uint32_t* err;
  int flush_mode;            // 1: only merge pending temps (Quantile's mergeAllTemps)
  // flush-ready digest: with spec set, a replay that leaves temps pending also merges them
  // into the other centroid buffer (hspn/hspw); the flush adopts it unless the key changed
  int spec;
  uint32_t* hspn;
  double* hspw;
  // pure-chunk pre-sort (ingest only): per key chunk count and scan, sorted chunk
  // means/weights at the chunk's record positions, Add-order weight sum at its first record
  uint32_t* ccnt;
  uint32_t* coff;
  double* csv;
  double* csw;
  double* ctw;
  int tw_sum;  // 1: the one-wave replay sums a chunk's weights itself when they have an order-free sum, and
               // the chunk sorter writes ctw's first-record slot only for the long keys and the other chunks
  // the batched replay's packed weights (null: no batched replay): per record the exclusive prefix
  // of the chunk's sorted weights (u16) << 16 | |w| (u16); a chunk's first record carries its
  // tempW as the prefix, or 0xffffffff when the chunk cannot be batched (a weight that is not an
  // integer, or a tempW of 65536 or more)
  uint32_t* cpk;
  uint64_t* cown;  // [chunks] key index << 32 | first record of every pure chunk (null: searched in coff)
  // the batched keys' pure-chunk Local* statistics, reduced in parallel before their replays
  // (k_exact_long_stats): [kLongStatKeys][kLongStatSlices][8] partials (null: the replay's own)
  double* lstat;
};
constexpr uint32_t kLongStatSlices = 64;
constexpr uint32_t kLongStatKeys = 1024;  // entries of the longest-first order with partials (the rest: in-replay)

size_t exact_smem_bytes(uint32_t capc, uint32_t tcap);
size_t exact_fast_smem_bytes(uint32_t capc, uint32_t tcap);  // the long replays' (k_histo_exact_mw)
// max_chunks: upper bound on the pure chunks of the batch (grid of the chunk sorter)
void launch_histo_exact(const ExactCtx& x, hipStream_t st, ScanScratch* ss, uint64_t max_chunks);
// the pure-chunk pre-sort alone, and the replay alone (over x.order when set)
void histo_exact_presort(const ExactCtx& x, hipStream_t st, ScanScratch* ss, uint64_t max_chunks);
// histo_exact_presort in parts: the chunk counts and owners, then the sorts -- the first `top`
// keys of x.order64 alone (top_only), or every other chunk (top keys skipped)
void histo_exact_chunk_plan(const ExactCtx& x, hipStream_t st, ScanScratch* ss, uint64_t max_chunks);
void histo_exact_chunk_sort(const ExactCtx& x, hipStream_t st, uint64_t max_chunks, uint32_t top, bool top_only);
void histo_exact_replay(const ExactCtx& x, hipStream_t st);
// The longest keys of x.order64 (>= min_len samples to replay, at most 4096) replay with four
// waves each: histo_exact_count_long counts them into count[0] (and those of at least
// kBatchMinLen samples, batched, into count[1]) on st and sets x.mw_count, so
// histo_exact_replay skips them; histo_exact_replay_long replays them (any stream after st).
bool histo_exact_count_long(ExactCtx& x, uint32_t min_len, uint32_t* count, hipStream_t st);
// the batched kernel (the longest keys) on st, the rest of the long keys on st_rest
// st_top (or null): the kTopExcl longest batched keys there, the other batched ones on st
void histo_exact_replay_long(const ExactCtx& x, hipStream_t st, hipStream_t st_rest, hipStream_t st_top = nullptr,
                             uint32_t top_done = 0);
// The longest keys first: the number of leading keys of the order (x.order64, after
// histo_exact_count_long) whose batched replays histo_exact_replay_top launches on their own
// stream (0: none); histo_exact_replay_long then skips them (top_done).
uint32_t histo_exact_top_keys(const ExactCtx& x);
void histo_exact_replay_top(const ExactCtx& x, hipStream_t st_top, uint32_t top);
// the replay over x.keys[0, *dev_count) (count known on the device only; <= max_keys)
void histo_exact_replay_list(const ExactCtx& x, const uint32_t* dev_count, uint32_t max_keys, hipStream_t st);
// replay list[0..n) longest first: sorts the order into buf0/buf1 (n each) on st and sets x
// up for histo_exact_replay
// (n_dev: the device's count of list entries when n is only an upper bound; the order then ends in
// length-0 entries of key index 0xffffffff, which every replay kernel skips)
void histo_exact_order(ExactCtx& x, const uint32_t* list, uint32_t n, uint64_t* buf0, uint64_t* buf1,
                       RadixScratch& rs, hipStream_t st, const uint32_t* n_dev = nullptr);
// the geometric remainder's rounds (ingest_histo.hip): see the definition
void histo_rounds(vn_engine* e, const uint32_t* list, uint32_t nkeys, uint32_t maxp, uint64_t nrec, uint32_t nrem,
                  const uint64_t* PA, const uint64_t* PB, uint64_t* MA, uint64_t* MB, const double* impw,
                  hipStream_t st);
// All rounds of the listed keys in one launch, one workgroup per key (pieces of <= kFuseMaxL
// elements with the key's centroids); val / w / kk: nkeys * kFuseMaxL doubles each of scratch
constexpr uint32_t kFuseMaxL = 12288;
void histo_rounds_fused(vn_engine* e, const uint32_t* list, uint32_t nkeys, const uint64_t* PA, const uint64_t* PB,
                        const double* impw, double* val, double* w, double* kk, hipStream_t st,
                        uint32_t max_pieces = ~0u, uint32_t* done = nullptr);
// One mergeAllTemps of each segment [start[k], end[k]) of (A = ordered value bits, B = tag) alone,
// at compression delta, into the pseudo-slot tiles k = tl[k] of the given arrays (the split-key
// micro-centroids, split.hip).  Per segment a capc-wide tile; w/wk sized nrec; chunk arrays sized
// nrec / kHTile + nseg + 1; nch/chb nseg + 1.
struct SegCompress {
  uint32_t nseg = 0;
  uint64_t nrec = 0;
  uint32_t capc = 0;
  double delta = 0;
  const uint32_t* tl = nullptr;
  const uint32_t* start = nullptr;
  const uint32_t* end = nullptr;
  uint32_t* nch = nullptr;
  uint32_t* chb = nullptr;
  const uint64_t* A = nullptr;
  const uint64_t* B = nullptr;
  double *w = nullptr, *wk = nullptr, *ch_sum = nullptr, *ch_pre = nullptr, *ch_stats = nullptr, *seg_T = nullptr;
  uint32_t *starts = nullptr, *nc_new = nullptr;
  double *acc_xw = nullptr, *acc_w = nullptr, *hst = nullptr;
  uint32_t *hncent = nullptr;
  uint8_t* hcur = nullptr;
  uint32_t* hspn = nullptr;
  double *cm0 = nullptr, *cm1 = nullptr, *cw0 = nullptr, *cw1 = nullptr;
  uint32_t* err = nullptr;
};
void histo_compress_segments(const SegCompress& c, ScanScratch& ss, hipStream_t st);
// estimateTempBuffer (merging_digest.go:87-93)
inline uint32_t temp_buffer_cap(double compression) {
  double c = compression < 20 ? 20 : (compression > 925 ? 925 : compression);
  return (uint32_t)(int)(7.5 + 0.37 * c - 2e-4 * c * c);
}

}  // namespace vn

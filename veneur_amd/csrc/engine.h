// engine.h -- device state of one engine (one GPU, one veneur worker group).
//
// HBM layout (per class, indexed by the class-local slot the host interned):
//   counters  cval[i64], ctouch[u32]
//   gauges    gseq[u64] (arrival seq+1 of the winning write, 0 = untouched), gval[f64], gtouch
//   histos    hst[8 x f64] = LocalWeight, LocalMin, LocalMax, LocalSum, LocalReciprocalSum,
//             digest min, digest max, digest total weight; centroid tiles cmean/cw[2][slot][cap_cent]
//             (double-buffered: an ingest writes the other buffer and flips hcur)
//   sets      header SoA (mode, b, nz, list count/bytes/last, tmp count), tmpSet codes [slot][164],
//             arena [slot][16640 u32]: the sorted unique sparse codes, or 16384 one-byte registers
#pragma once
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "../../include/veneur_amd.h"
#include "comm.h"
#include "primitives.h"

namespace vn {

constexpr uint32_t kArenaWords = 16640;  // == kHllListCap
constexpr uint32_t kTmpCap = 164;
constexpr uint32_t kImportCuts = 1024;  // slices of one histo import call found per device pass

// Import staging (vn_import_histos / vn_import_sets): payloads as received, per-payload
// parse results, and the decoded centroids.  Grown on demand.
struct ImportScratch {
  uint64_t cap_n = 0, cap_bytes = 0, cap_cent = 0;
  uint32_t* in_slot = nullptr;    // [cap_n]
  uint64_t* in_off = nullptr;     // [cap_n + 1]
  uint8_t* in_bytes = nullptr;    // [cap_bytes]
  uint32_t* cnt = nullptr;        // [cap_n + 1] per payload: centroids
  uint32_t* coff = nullptr;       // [cap_n + 1] scan of cnt
  uint32_t* cpos = nullptr;       // [cap_n] per payload: where its centroids start when all are in the
                                  // one-window layout (k_gob_emit_seg), else ~0
  uint16_t* ckpt = nullptr;       // [cap_n * 16] per payload: the byte of every 16th centroid (k_gob_emit_seg)
  void* parts = nullptr;          // [cap_n] parsed HLL payload headers (import_set.hip)
  uint32_t* cslot = nullptr;      // [cap_cent] decoded centroids: slot, mean, weight
  double* cmean = nullptr;
  double* cw = nullptr;
  double* cw_alt = nullptr;       // the other weights buffer: a drain's replay reads one while the
                                  // next slice's emit fills the other
  uint64_t acc = 0;               // imported histo centroids appended, not yet merged (import_histo.hip)
  // the run's payloads in arrival order (the drain groups them by key, not their centroids)
  uint64_t cap_pay = 0, npay = 0;
  uint32_t* pslot = nullptr;      // [cap_pay] slot
  uint32_t* pbeg = nullptr;       // [cap_pay + 1] first centroid in the run (pbeg[npay] = acc at the drain)
  uint64_t* pkey = nullptr;       // [2 cap_pay] (slot << 32 | payload) sort keys, two buffers
  uint32_t* pcnt = nullptr;       // [cap_pay + 1] centroids per payload in key order
  uint32_t* pdst = nullptr;       // [cap_pay + 1] their exclusive scan: each payload's place
  uint32_t* cuts = nullptr;       // [2 (kImportCuts + 1) + 2] a call's slices: first payloads, their
                                  // first centroids, then the count and an oversize flag
  uint32_t* hcuts = nullptr;      // pinned host copy of cuts
};

// Export results (vn_export_histos / vn_export_sets): engine-owned, valid until the next export.
struct ExportBuffers {
  uint64_t cap_n = 0, cap_bytes = 0;
  uint32_t* d_slot = nullptr;     // [cap_n] requested slots
  uint32_t* d_keys = nullptr;     // [cap_n] distinct slots (pending-temp merge)
  uint32_t* d_size = nullptr;     // [cap_n]
  uint64_t* d_off = nullptr;      // [cap_n + 1]
  uint64_t* h_off = nullptr;      // pinned copy
  uint8_t* d_bytes = nullptr;     // [cap_bytes]
  uint8_t* h_bytes = nullptr;     // pinned copy
};

struct DeviceBatch {  // device-resident staging for one ingest call
  uint32_t *c_slot, *g_slot, *h_slot, *s_slot, *s_off;
  double *c_val, *g_val, *h_val;
  float *c_rate, *h_rate;
  uint8_t* s_bytes;
};

// Split (hot) keys of the window and the records they received (split.hip).
struct SplitState {
  vn_comm* comm = nullptr;          // the engine's group (vn_engine_set_comm); null: a group of one
  vn_comm* solo = nullptr;          // that group of one, created on first use
  std::vector<uint32_t> slot[VN_NCLASS], owner[VN_NCLASS];
  uint32_t* d_slot[VN_NCLASS] = {nullptr, nullptr, nullptr, nullptr};
  uint32_t d_cap[VN_NCLASS] = {0, 0, 0, 0};
  uint64_t cap = 0;                 // records per class and window (vn_config.split_max_records)
  uint64_t nh = 0, ns = 0;          // records buffered this window
  uint32_t* hkey = nullptr;         // histo records: split key index, value, rate (arrival order)
  double* hval = nullptr;
  float* hrate = nullptr;
  uint64_t* srec = nullptr;         // set records: key << 32 | sparse code (arrival order)
  uint32_t* s_scratch_bt = nullptr; // set ingest: touched flags of the metro64 pass (unused slots)
  vn_engine* aux = nullptr;         // the split engine (split.hip): split histos / sets combine there
  hipEvent_t ev_done = nullptr;     // its combine done (this engine's stream waits on it)
  hipEvent_t ev_histo = nullptr, ev_set_prefix = nullptr;  // milestones inside it (vn_timing)
  bool ran = false;                 // ev_done recorded by this window's flush
  // the finished states' moves into this engine's slots, launched by vn_flush on this engine's
  // stream (after every ingest and import of the window), not by the combine beside it
  struct HistoMove {
    uint32_t K = 0;
    const uint32_t* okeys = nullptr;
    const uint64_t* tot = nullptr;
    const double *sums = nullptr, *mins = nullptr, *maxs = nullptr;
  } mv_histo;
  struct SetMove {
    uint32_t H = 0;
    const uint32_t* owner = nullptr;
    int me = 0;
    const uint64_t* tot = nullptr;
  } mv_set;
  // vn_split_close: the split engine's combine runs in this host thread while the caller goes
  // on ingesting; vn_flush joins it
  std::thread worker;
  bool closed = false;
  std::exception_ptr worker_err;
  std::vector<void*> scratch;       // flush scratch (freed at destroy)
  std::vector<size_t> scratch_cap;
};

}  // namespace vn

// diagnostics build (VARIANT_FLAGS=-DVN_HOST_PROF): host time of vn_ingest's waits, printed per call
#ifdef VN_HOST_PROF
#include <chrono>
#define VN_HWAIT(e, i, stmt)                                                                                   \
  do {                                                                                                         \
    const auto _t0 = std::chrono::steady_clock::now();                                                         \
    stmt;                                                                                                      \
    (e)->host_wait_ms[i] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - _t0).count(); \
  } while (0)
#else
#define VN_HWAIT(e, i, stmt) stmt
#endif
struct vn_engine {
  double host_wait_ms[4] = {0.0, 0.0, 0.0, 0.0};  // (VN_HOST_PROF) validation, grouping, plan waits
  vn_config cfg{};
  int device = 0;
  hipStream_t st = nullptr;       // main stream (histos, flush, staging copies)
  hipStream_t st2 = nullptr;      // side stream: counters, gauges and sets overlap the histo path
  hipStream_t st_imp = nullptr;   // histo import emits: the next slice beside the previous drain's replay
  hipEvent_t ev_imp_free = nullptr, ev_imp_emit = nullptr;  // the run read by its drain / its emits done
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_h2d = nullptr;    // recorded after a host batch's copies into HBM (vn_submit waits on it)
  // window milestones (vn_timing.ms_main_ready / ms_split_ready): first ingest call of the
  // window, this engine's queued ingest work done (recorded as vn_flush starts)
  hipEvent_t ev_w0 = nullptr, ev_wmain = nullptr;
  bool w_open = false;
  // replay stream: the exact replay of the keys under the threshold runs here while the hot
  // keys' short prefix and remainder rounds run on st (st itself when timing is enabled)
  hipStream_t st3 = nullptr;
  hipEvent_t ev_fork3 = nullptr, ev_join3 = nullptr;
  // hot-prefix stream: the hot keys' short replays run here while st gathers and sorts their
  // remainders
  hipStream_t st4 = nullptr;
  // the split counters' combine: after the window's counter aggregation (on the side stream),
  // not behind the main stream's replays, so vn_split_combine returns without waiting for them
  hipStream_t st_ctr = nullptr;
  hipEvent_t ev_ctr0 = nullptr, ev_ctr1 = nullptr;
  hipEvent_t ev_join4 = nullptr;
  // long-key replay stream (CU mask of st3): the longest keys' four-wave replays
  hipStream_t st5 = nullptr;
  hipEvent_t ev_fork5 = nullptr, ev_join5 = nullptr, ev_rest5 = nullptr;
  hipEvent_t ev_bulk = nullptr;  // the short keys' replays done on the side stream (VN_BULK_SIDE)
  // the few longest batched replays on CUs no other stream uses (null: st5 takes them all)
  uint32_t ev_rec = 0;           // timing: which of ev[0..4] this window recorded
  hipStream_t st6 = nullptr;     // the reserved CUs (vn_config.replay_reserved_cus), or none
  uint32_t reserved_cus = 0;
  std::vector<uint32_t> amask;   // every CU but the reserved ones
  // st3, st4 and st_ctr carry work only in the fast mode (the hot keys' fork) and in the split
  // counters' combine: they are created at first use (ensure_aux_streams), so an exact-mode
  // engine holds three streams and several engines' active streams do not share the runtime's
  // hardware queues (GPU_MAX_HW_QUEUES)
  std::vector<uint32_t> rmask;   // the replay streams' CU mask (empty: unmasked)
  int prio_hi = 0, prio_lo = 0;
  hipEvent_t ev_join6 = nullptr;
  // set segment merge held back (ingest_device): the grouped set records are merged once the
  // histo path's remainder sort is done, so the long set kernel does not crowd it out
  bool set_defer = false, set_pending = false;
  uint64_t set_pending_n = 0;
  const uint64_t* set_pending_R = nullptr;
  const uint64_t* set_pending_order = nullptr;  // LPT order of the pending set merge (or null)
  // stream + scratch the counter / gauge / set launchers use for the current call
  // (st2 normally; st when timing is enabled, so per-kernel durations are measured alone)
  hipStream_t side = nullptr;
  // hot-key detector (hotkeys.hip): every hot_stride-th record's slot counted per class, this
  // window (hk_cnt[hk_cur]) and the last flushed one (hk_cnt[hk_cur ^ 1], stride hk_prev_stride)
  uint32_t hot_stride = 0, hk_prev_stride = 0;
  int hk_cur = 0;
  uint32_t* hk_cnt[2][VN_NCLASS] = {{nullptr, nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr, nullptr}};
  uint64_t* hk_list = nullptr;
  std::string err;
  uint32_t cap[VN_NCLASS] = {0, 0, 0, 0};
  uint32_t cap_cent = 256;      // centroids per histo slot (>= 2*compression + 4)
  int slot_bits[VN_NCLASS] = {1, 1, 1, 1};
  uint64_t max_records = 0, max_member_bytes = 0;
  uint64_t max_cls[VN_NCLASS] = {};
  bool early_top = false;  // VN_EARLY_TOP A/B knob (capi.hip)  // per class: vn_config.max_batch_class_records (0 -> max_records)

  // ---- counters
  int64_t* cval = nullptr;
  uint32_t* ctouch = nullptr;
  // ---- gauges
  uint64_t* gseq = nullptr;
  double* gval = nullptr;
  uint32_t* gtouch = nullptr;
  uint64_t seq_base = 0;
  // counter / gauge partition scratch (slot, payload) [max_records]
  uint32_t* pk = nullptr;
  uint64_t* pp = nullptr;
  // ---- histos
  double* hst = nullptr;
  uint32_t* hncent = nullptr;
  uint8_t* hcur = nullptr;
  uint32_t* htouch = nullptr;
  double* cmean[2] = {nullptr, nullptr};
  double* cw[2] = {nullptr, nullptr};
  // histo ingest scratch
  uint32_t* h_bt = nullptr;      // batch-touched flags
  uint32_t* h_pos = nullptr;     // scan of flags (cap+1)
  uint32_t* h_tl = nullptr;      // touched list
  uint32_t* h_cnt = nullptr;     // device counters [16]
  uint64_t *hA0 = nullptr, *hB0 = nullptr, *hA1 = nullptr, *hB1 = nullptr;
  uint64_t h_sort_cap = 0;
  double* h_w = nullptr;         // per record weight
  double* h_wk = nullptr;        // per record local prefix weight, then k-index
  uint32_t* h_start = nullptr;   // per slot segment start / end in the sorted batch
  uint32_t* h_end = nullptr;
  uint32_t* h_nch = nullptr;     // per touched segment: chunks
  uint32_t* h_chb = nullptr;     // chunk base (cap+1)
  uint64_t h_max_chunks = 0;
  double* ch_sum = nullptr;
  double* ch_pre = nullptr;
  double* ch_stats = nullptr;    // [chunk][5]
  double* seg_T = nullptr;       // per touched seg
  uint32_t* starts = nullptr;    // [touched][cap_cent]
  uint32_t* nc_new = nullptr;
  double* acc_xw = nullptr;      // [touched][cap_cent]
  double* acc_w = nullptr;
  uint32_t* h_err = nullptr;     // device error flags
  // exact (Go-incremental) replay state and batch split
  uint32_t exact_threshold = 32768;
  uint32_t hot_prefix = 4096;    // a key past the threshold replays this many samples exactly
  uint32_t long_replay = 0;      // replays of at least this many samples take four waves (0: threshold / 4)
  uint32_t piece_growth = 25;    // remainder piece size, percent of the window samples before it
  uint32_t temp_cap = 42;        // estimateTempBuffer(compression)
  uint32_t* hseen = nullptr;     // samples seen this window per slot
  uint32_t* hpend = nullptr;     // pending temps per slot
  uint32_t* hspn = nullptr;      // centroids of the flush-ready digest in the other buffer (0: none)
  double* hspw = nullptr;        // its mainWeight
  uint32_t* hm_flag = nullptr;   // merge-pending scratch: keys still needing a final merge
  uint32_t* hm_pos = nullptr;
  uint32_t* hm_idx = nullptr;
  uint32_t* hm_list = nullptr;
  uint32_t* hm_cnt = nullptr;
  double* hpv = nullptr;         // [slot][temp_cap] pending temp means
  double* hpw = nullptr;         // [slot][temp_cap] pending temp weights
  uint32_t* h_ex = nullptr;      // per touched key: samples replayed exactly
  uint32_t* h_hotflag = nullptr;
  uint32_t* h_hotcnt = nullptr;
  uint32_t* h_hotoff = nullptr;
  uint32_t* h_hotlist = nullptr;
  uint32_t* h_coldflag = nullptr;  // per touched key: replayed on the replay stream (cold / warm)
  uint32_t* h_coldlist = nullptr;
  uint32_t* h_vhflag = nullptr;    // hot: short exact prefix, rounds beside the replay (-> h_hotlist)
  uint32_t* h_warmflag = nullptr;  // warm: exact prefix of E, rounds after the replay
  uint32_t* h_warmlist = nullptr;
  uint64_t* hA2 = nullptr;       // hot remainder sort ping-pong (As/Bs stay with the replay)
  uint64_t* hB2 = nullptr;
  uint64_t* h_lpt0 = nullptr;    // replay order of the keys under the threshold, longest first
  uint64_t* h_lpt1 = nullptr;
  double* h_csv = nullptr;       // pre-sorted pure chunks: means, weights (per record)
  double* h_csw = nullptr;
  uint32_t* h_cpk = nullptr;     // ... the batched replay's packed weights (ExactCtx::cpk)
  double* h_lstat = nullptr;     // ... the batched keys' Local* partials (ExactCtx::lstat)
  double* h_cstat = nullptr;     // ... every pure chunk's Local* partials (ExactCtx::cstat)
  uint32_t* h_tl2 = nullptr;     // slots of hot keys
  uint32_t* h_ccnt = nullptr;    // per touched key: pure chunks to pre-sort
  uint32_t* h_coff = nullptr;    // scan of h_ccnt (touched + 1)
  uint64_t* h_cown = nullptr;    // owner key index << 32 | first record, of every pure chunk
  double* h_tw = nullptr;        // per chunk (at its first record): Add-order weight sum
  // geometric remainder of hot keys (ingest_histo.hip)
  uint64_t* h_geo = nullptr;     // piece boundaries b_0 = hot_prefix, b_{i+1} = b_i + max(1, b_i / 10)
  uint32_t n_geo = 0;
  uint32_t fuse_pieces = 0;        // leading geometric pieces small enough for k_rounds_fused
  double *fz_val = nullptr, *fz_w = nullptr, *fz_k = nullptr;  // its scratch, fz_cap keys
  uint32_t* fz_done = nullptr;
  uint32_t fz_cap = 0;
  uint32_t* h_seen0 = nullptr;   // per touched key: window samples before this batch
  uint32_t* h_pcnt = nullptr;    // per touched key: remainder pieces in this batch
  uint32_t* h_pi0 = nullptr;     // per touched key: first boundary index after its remainder start
  uint32_t* h_pbase = nullptr;   // scan of h_pcnt: piece ids
  uint32_t* p_start = nullptr;   // per piece: range in the (piece, value)-sorted remainder
  uint32_t* p_end = nullptr;
  uint32_t *r_flag = nullptr, *r_len = nullptr, *r_off = nullptr, *r_pos = nullptr, *r_list = nullptr;

  // ---- sets
  uint8_t* smode = nullptr;      // 0 sparse, 1 dense
  uint8_t* sbase = nullptr;      // b
  uint32_t* snz = nullptr;
  uint32_t* slc = nullptr;
  uint32_t* slb = nullptr;
  uint32_t* slast = nullptr;
  uint32_t* stc = nullptr;
  uint32_t* stouch = nullptr;
  uint32_t* stmp = nullptr;      // [cap][164]
  uint32_t* sarena = nullptr;    // [cap][kArenaWords]
  // set ingest scratch
  uint64_t *sR0 = nullptr, *sR1 = nullptr;
  uint32_t* s_bt = nullptr;
  uint32_t* s_pos = nullptr;
  uint32_t* s_tl = nullptr;
  uint32_t* s_cnt = nullptr;     // [0] touched set keys, [1] merge work counter
  uint64_t* s_lpt0 = nullptr;    // set merge order, most records first
  uint64_t* s_lpt1 = nullptr;
  uint32_t* s_start = nullptr;
  uint32_t* s_end = nullptr;

  // ---- staging
  vn::DeviceBatch dstage{};
  vn::ImportScratch imp;
  vn::ExportBuffers exp;
  vn_stage pstage{};             // pinned host views
  // ---- flush outputs
  uint32_t* f_pos = nullptr;     // scan scratch (max cap + 1)
  uint32_t* f_list[VN_NCLASS] = {nullptr, nullptr, nullptr, nullptr};
  uint32_t* f_cnt = nullptr;     // [4]
  int64_t* f_cval = nullptr;
  double* f_gval = nullptr;
  double* f_hstats = nullptr;
  double* f_hq = nullptr;
  uint64_t* f_sest = nullptr;
  uint8_t* f_ssparse = nullptr;
  double* d_pct = nullptr;
  uint8_t* f_hmask = nullptr;    // flush masks (vn_flush_masked), cap[VN_HISTO] / cap[VN_SET] bytes
  uint8_t* f_smask = nullptr;
  // pinned host copies of the flush result
  uint32_t* hf_list[VN_NCLASS] = {nullptr, nullptr, nullptr, nullptr};
  int64_t* hf_cval = nullptr;
  double* hf_gval = nullptr;
  double* hf_hstats = nullptr;
  double* hf_hq = nullptr;
  uint64_t* hf_sest = nullptr;
  uint8_t* hf_ssparse = nullptr;
  uint32_t* hf_cnt = nullptr;    // pinned [8]

  uint64_t processed = 0, imported = 0;

  vn::RadixScratch rs;
  vn::ScanScratch ss;
  vn::RadixScratch rs2;           // side-stream scratch
  vn::ScanScratch ss2;
  vn::RadixScratch rs3;           // replay-stream scratch (longest-first key order)
  uint32_t side_cus = 0;          // CUs the side and replay streams may use (CU mask)
  vn::RadixScratch* side_rs = nullptr;
  vn::ScanScratch* side_ss = nullptr;

  // ---- timing
  bool timing = false;
  // decoded import contributions (SURVEY.md §8(d)'s C5 bytes), counted while timing is on:
  // histo payloads, their centroids, set payloads, dense ones, sparse codes (vn_import_counts)
  uint64_t imp_counts[5] = {0, 0, 0, 0, 0};
  unsigned long long* d_imp_counts = nullptr;  // device [2]: dense set payloads, sparse set codes
  hipEvent_t ev[16] = {};
  vn::EventPool pool;
  vn::SplitState sp;
  std::vector<hipEvent_t> pool_storage;
  vn_timing last{};
  vn::RadixStats rstat_c, rstat_h, rstat_s;
  // timed launches of the exact replay and of the set state machine (timing mode)
  vn::EventPool pool_rp, pool_ss, pool_ps;
  std::vector<hipEvent_t> pool_rp_storage, pool_ss_storage, pool_ps_storage, pool_id_storage, pool_im_storage;
  vn::EventPool pool_id, pool_im;  // timing: import decode kernels, import drains
  vn::RadixStats kstat_rp, kstat_ss;
};

// capi.hip -- engine lifetime and the C-ABI of include/veneur_amd.h.
#include <chrono>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <stdexcept>

#include "histo.h"

using namespace vn;

namespace {

template <class T>
void dalloc(T*& p, size_t count) {
  if (count == 0) count = 1;
  VN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)));
}
template <class T>
void dzero(T* p, size_t count, hipStream_t st) {
  if (count) VN_HIP_CHECK(hipMemsetAsync(p, 0, count * sizeof(T), st));
}
template <class T>
void halloc(T*& p, size_t count) {
  if (count == 0) count = 1;
  VN_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p), count * sizeof(T), hipHostMallocDefault));
}
template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}
template <class T>
void hfree(T*& p) {
  if (p) (void)hipHostFree(p);
  p = nullptr;
}

template <class T>
void h2d(T* dst, const T* src, uint64_t n, hipStream_t st) {
  if (n) VN_HIP_CHECK(hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyHostToDevice, st));
}

int bits_for(uint32_t cap) {
  int b = 1;
  while (b < 32 && (1u << b) < cap) b++;
  return b;
}

int fail(vn_engine* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  return code;
}

template <class F>
int guarded(vn_engine* e, F&& f) {
  try {
    // every entry point runs on the engine's device, whatever thread calls it (a Worker's flush
    // threads, a cgo goroutine's OS thread): allocations made inside a call land on that device
    if (e) VN_HIP_CHECK(hipSetDevice(e->device));
    f();
    return VN_OK;
  } catch (const HipError& h) {
    return fail(e, VN_EHIP, std::string(hipGetErrorString(h.err)) + " at " + h.file + ":" + std::to_string(h.line) +
                                ": " + h.expr);
  } catch (const DecodeError& x) {
    return fail(e, VN_EDECODE, x.what());
  } catch (const std::invalid_argument& x) {
    return fail(e, VN_EINVAL, x.what());
  } catch (const std::bad_alloc&) {
    return fail(e, VN_ENOMEM, "out of memory");
  } catch (const std::exception& x) {
    return fail(e, VN_EINVAL, x.what());
  }
}

}  // namespace
namespace vn {
void window_open(vn_engine* e, hipStream_t st) {
  if (e->w_open) return;
  VN_HIP_CHECK(hipEventRecord(e->ev_w0, st));
  e->w_open = true;
}
}  // namespace vn
namespace {
void check_slots_host(const uint32_t* slot, uint64_t n, uint32_t cap, const char* what) {
  for (uint64_t i = 0; i < n; i++)
    if (slot[i] >= cap) throw std::invalid_argument(std::string(what) + " slot out of range");
}

#ifndef VN_REPLAY_EIGHTHS
#define VN_REPLAY_EIGHTHS 6
#endif
void create_impl(vn_engine* e) {
  VN_HIP_CHECK(hipSetDevice(e->device));
  // the fast mode's remainder buffers (sort ping-pong, piece ranges, segment compression): none
  // in the exact-only build -- about 10 GB per engine at C4, room for more engines in turn
  constexpr bool kFm = VN_FAST_MODE != 0;
  // the histo path (main and replay streams) is the critical path: it gets the high queue
  // priority, the side stream's counters / gauges / sets fill whatever CUs it leaves
  int prio_lo = 0, prio_hi = 0;
  VN_HIP_CHECK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  VN_HIP_CHECK(hipStreamCreateWithPriority(&e->st, hipStreamNonBlocking, prio_hi));
  // Queue priority does not preempt: once the long set merge and the replay of the keys under
  // the threshold (100k+ workgroups, some running for milliseconds) fill the CUs, the
  // remainder rounds' chain workgroups (~100 KiB of LDS each) wait for a CU to drain -- and a
  // workgroup waits inside the shader engine it was dealt to.  Those two streams therefore
  // leave the last quarter of the CU mask to the main stream.  Measured on gfx950
  // (tools/probe/cumask_probe.hip): mask bit i is XCC i % 8, shader engine (i / 8) % 4, CU
  // i / 32 within it, so bits [3/4 ncu, ncu) are 2 CUs in every shader engine of every XCC.
  {
    hipDeviceProp_t prop;
    VN_HIP_CHECK(hipGetDeviceProperties(&prop, e->device));
    const uint32_t ncu = (uint32_t)prop.multiProcessorCount;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u), rmask((ncu + 31) / 32, 0u);
#ifndef VN_SIDE_ALL
#define VN_SIDE_ALL 0  // (A/B build knob: the side stream's mask over every CU)
#endif
    for (uint32_t i = 0; i < (VN_SIDE_ALL ? ncu : ncu - ncu / 4); i++) mask[i / 32] |= 1u << (i % 32);
    // the replay streams' share in eighths of the CUs (bits [0, n/8 ncu): whole shader-engine
    // columns of every XCC, as above)
    for (uint32_t i = 0; i < ncu * VN_REPLAY_EIGHTHS / 8; i++) rmask[i / 32] |= 1u << (i % 32);
    e->side_cus = ncu - ncu / 4;
#ifndef VN_NO_CU_MASK
#define VN_NO_CU_MASK 0  // (build knob: every stream unmasked -- the profiling runs of DESIGN.md §8)
#endif
    e->prio_hi = prio_hi;
    e->prio_lo = prio_lo;
    e->rmask = rmask;
// The main stream CU-masked to every CU: a CU-masked stream gets a hardware queue of its own,
// where an unmasked one shares one of the GPU_MAX_HW_QUEUES with other streams -- with several
// engines in turn an engine's ingest front then sat in one in-order queue behind another
// window's 170 ms chain.  Measured: C4 at N = 1, 74.2 -> 71.7 ms per window at
// four engines, 71.4 / 72.4 at five / six (96 / 92 before); the N = 8 owner's share 45.9 ms at
// four engines, 36.1 at six (profiles/r06_streams/).  (It gives up the high queue priority.)
#ifndef VN_ST_FULLMASK
#define VN_ST_FULLMASK 1
#endif
    if (VN_ST_FULLMASK && ncu >= 64) {
      std::vector<uint32_t> fmask((ncu + 31) / 32, 0u);
      for (uint32_t i = 0; i < ncu; i++) fmask[i / 32] |= 1u << (i % 32);
      VN_HIP_CHECK(hipStreamDestroy(e->st));
      VN_HIP_CHECK(hipExtStreamCreateWithCUMask(&e->st, (uint32_t)fmask.size(), fmask.data()));
    }
    if (VN_NO_CU_MASK || ncu < 64 || hipExtStreamCreateWithCUMask(&e->st2, (uint32_t)mask.size(), mask.data()) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&e->st5, (uint32_t)rmask.size(), rmask.data()) != hipSuccess) {
      (void)hipGetLastError();
      for (hipStream_t* p : {&e->st2, &e->st5})
        if (*p) {
          (void)hipStreamDestroy(*p);
          *p = nullptr;
        }
      VN_HIP_CHECK(hipStreamCreateWithPriority(&e->st2, hipStreamNonBlocking, prio_lo));
      VN_HIP_CHECK(hipStreamCreateWithPriority(&e->st5, hipStreamNonBlocking, prio_hi));
      e->side_cus = ncu;
      e->rmask.clear();
    }
#ifndef VN_SIDE_MAIN
#define VN_SIDE_MAIN 0  // (A/B build knob: counters, gauges and sets on the main stream, no side stream)
#endif
    if (VN_SIDE_MAIN && e->st2) {
      VN_HIP_CHECK(hipStreamDestroy(e->st2));
      e->st2 = nullptr;
    }
    VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_fork5, hipEventDisableTiming));
    VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_join5, hipEventDisableTiming));
    VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_rest5, hipEventDisableTiming));
    VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_bulk, hipEventDisableTiming));
    // vn_config.replay_reserved_cus: the longest batched replays (one workgroup each, hundreds of
    // ms, latency-bound at one wave per SIMD) on the last CUs, which every other stream of the
    // engine leaves alone -- the other windows' sorts and scatters no longer share those CUs'
    // SIMDs with them.  Whole groups of 8 CUs (one per XCC), at most a quarter of the chip (the
    // quarter the replay masks above already leave to the main stream)
    e->reserved_cus = 0;
    if (e->cfg.replay_reserved_cus && e->st2 && ncu >= 64) {
      const uint32_t r = std::min<uint32_t>((e->cfg.replay_reserved_cus + 7u) & ~7u, ncu / 4);
      std::vector<uint32_t> tmask((ncu + 31) / 32, 0u);
      e->amask.assign((ncu + 31) / 32, 0u);
      for (uint32_t i = 0; i < ncu; i++) (i >= ncu - r ? tmask : e->amask)[i / 32] |= 1u << (i % 32);
      VN_HIP_CHECK(hipStreamDestroy(e->st));
      VN_HIP_CHECK(hipExtStreamCreateWithCUMask(&e->st, (uint32_t)e->amask.size(), e->amask.data()));
      VN_HIP_CHECK(hipExtStreamCreateWithCUMask(&e->st6, (uint32_t)tmask.size(), tmask.data()));
      VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_join6, hipEventDisableTiming));
      e->reserved_cus = r;
    }
    // A/B build knob (make variant VARIANT_FLAGS=-DVN_EARLY_TOP=1): the longest batched replays on
    // a stream of their own, started once their own chunks are sorted (ingest_histo.hip).  Measured
    // on C4 with three engines in turn: 99.4 ms per window against 86.0 (one more stream per engine,
    // DESIGN.md §8), not kept.  A build flag, not the environment: production behaviour must not
    // change with a variable set in the caller's environment.
#ifndef VN_EARLY_TOP
#define VN_EARLY_TOP 0
#endif
    e->early_top = VN_EARLY_TOP != 0;
    if (!e->st6 && e->early_top) {
      if (e->side_cus != ncu) VN_HIP_CHECK(hipExtStreamCreateWithCUMask(&e->st6, (uint32_t)rmask.size(), rmask.data()));
      else VN_HIP_CHECK(hipStreamCreateWithPriority(&e->st6, hipStreamNonBlocking, prio_hi));
      VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_join6, hipEventDisableTiming));
    }
  }
  VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
  VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming));
  VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_join4, hipEventDisableTiming));
  VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_ctr0, hipEventDisableTiming));
  VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_ctr1, hipEventDisableTiming));
  VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_fork3, hipEventDisableTiming));
  VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_h2d, hipEventDisableTiming));
  VN_HIP_CHECK(hipEventCreate(&e->ev_w0));
  VN_HIP_CHECK(hipEventCreate(&e->ev_wmain));
  VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_join3, hipEventDisableTiming));
  hipStream_t st = e->st;
  // each class's buffers sized by its own record cap
  const uint64_t R = e->max_cls[VN_HISTO], Rcg = std::max(e->max_cls[VN_COUNTER], e->max_cls[VN_GAUGE]),
                 Rs = e->max_cls[VN_SET];
  const uint32_t cc = e->cap[VN_COUNTER], cg = e->cap[VN_GAUGE], ch = e->cap[VN_HISTO], cs = e->cap[VN_SET];
  const uint32_t capc = e->cap_cent;
  const uint32_t capmax = std::max(std::max(cc, cg), std::max(ch, cs));

  dalloc(e->cval, cc); dzero(e->cval, cc, st);
  dalloc(e->ctouch, cc); dzero(e->ctouch, cc, st);
  dalloc(e->gseq, cg); dzero(e->gseq, cg, st);
  dalloc(e->gval, cg); dzero(e->gval, cg, st);
  dalloc(e->gtouch, cg); dzero(e->gtouch, cg, st);
  dalloc(e->pk, (cc || cg) ? Rcg : 0);
  dalloc(e->pp, (cc || cg) ? Rcg : 0);

  dalloc(e->hst, (size_t)ch * VN_HISTO_STATS);
  dalloc(e->hncent, ch); dzero(e->hncent, ch, st);
  dalloc(e->hcur, ch); dzero(e->hcur, ch, st);
  dalloc(e->htouch, ch); dzero(e->htouch, ch, st);
  for (int b = 0; b < 2; b++) {
    dalloc(e->cmean[b], (size_t)ch * capc);
    dalloc(e->cw[b], (size_t)ch * capc);
  }
  dalloc(e->h_bt, ch); dzero(e->h_bt, ch, st);
  dalloc(e->h_pos, (size_t)ch + 1);
  dalloc(e->h_tl, ch);
  dalloc(e->h_cnt, 32);
  const uint64_t touch_max = ch ? std::min<uint64_t>(ch, R) : 0;
  e->h_sort_cap = ch ? R + touch_max * capc : 0;
  dalloc(e->hA0, e->h_sort_cap); dalloc(e->hB0, e->h_sort_cap);
  dalloc(e->hA1, e->h_sort_cap); dalloc(e->hB1, e->h_sort_cap);
  dalloc(e->h_w, kFm ? e->h_sort_cap : 0);
  dalloc(e->h_wk, kFm ? e->h_sort_cap : 0);
  dalloc(e->h_start, ch);
  dalloc(e->h_end, ch);
  dalloc(e->h_nch, (size_t)touch_max + 1);
  dalloc(e->h_chb, (size_t)touch_max + 2);
  e->h_max_chunks = ch ? e->h_sort_cap / kHTile + touch_max + 2 : 0;
  dalloc(e->ch_sum, kFm ? e->h_max_chunks : 0);
  dalloc(e->ch_pre, kFm ? e->h_max_chunks : 0);
  dalloc(e->ch_stats, kFm ? e->h_max_chunks * kChunkStats : 0);
  dalloc(e->seg_T, touch_max);
  dalloc(e->starts, kFm ? (size_t)touch_max * capc : 0);
  dalloc(e->nc_new, touch_max);
  dalloc(e->acc_xw, kFm ? (size_t)touch_max * capc : 0);
  dalloc(e->acc_w, kFm ? (size_t)touch_max * capc : 0);
  dalloc(e->h_err, 4); dzero(e->h_err, 4, st);
  dalloc(e->hseen, ch); dzero(e->hseen, ch, st);
  dalloc(e->hpend, ch); dzero(e->hpend, ch, st);
  dalloc(e->hspn, ch); dzero(e->hspn, ch, st);
  dalloc(e->hspw, ch);
  dalloc(e->hm_flag, ch); dalloc(e->hm_pos, (size_t)ch + 1); dalloc(e->hm_idx, ch); dalloc(e->hm_list, ch); dalloc(e->hm_cnt, 1);
  dalloc(e->hpv, (size_t)ch * e->temp_cap);
  dalloc(e->hpw, (size_t)ch * e->temp_cap);
  dalloc(e->h_ex, touch_max);
  dalloc(e->h_hotflag, touch_max);
  dalloc(e->h_hotcnt, touch_max);
  dalloc(e->h_hotoff, (size_t)touch_max + 1);
  dalloc(e->h_hotlist, touch_max);
  dalloc(e->h_coldflag, touch_max);
  dalloc(e->h_coldlist, touch_max);
  dalloc(e->h_vhflag, touch_max);
  dalloc(e->h_warmflag, touch_max);
  dalloc(e->h_warmlist, touch_max);
  dalloc(e->hA2, kFm ? e->h_sort_cap : 0); dalloc(e->hB2, kFm ? e->h_sort_cap : 0);
  dalloc(e->h_csv, ch ? R : 0); dalloc(e->h_csw, ch ? R : 0); dalloc(e->h_cpk, ch ? R : 0);  // (u32 per record)
  dalloc(e->h_lstat, ch ? (uint64_t)kLongStatKeys * kLongStatSlices * 8 : 0);
  dalloc(e->h_lpt0, touch_max); dalloc(e->h_lpt1, touch_max);
  dalloc(e->h_tl2, touch_max);
  dalloc(e->h_ccnt, touch_max);
  dalloc(e->h_coff, (size_t)touch_max + 1);
  dalloc(e->h_cown, ch ? e->h_sort_cap / std::max<uint32_t>(e->temp_cap, 1) + 2 : 0);
  dalloc(e->h_cstat, ch ? (e->h_sort_cap / std::max<uint32_t>(e->temp_cap, 1) + 2) * 8 : 0);
  dalloc(e->h_tw, e->h_sort_cap);
  dalloc(e->h_seen0, touch_max);
  dalloc(e->h_pcnt, touch_max);
  dalloc(e->h_pi0, touch_max);
  dalloc(e->h_pbase, (size_t)touch_max + 1);
  dalloc(e->p_start, kFm && ch ? R + 1 : 0);
  dalloc(e->p_end, kFm && ch ? R + 1 : 0);
  dalloc(e->r_flag, touch_max);
  dalloc(e->r_len, touch_max);
  dalloc(e->r_list, touch_max);
  dalloc(e->r_off, (size_t)touch_max + 1);
  dalloc(e->r_pos, (size_t)touch_max + 1);
  {
    // piece boundaries of the geometric remainder (see ingest_histo.hip)
    std::vector<uint64_t> geo;
    for (uint64_t b = e->hot_prefix; geo.size() < 255 && b < (1ull << 40);
         b += std::max<uint64_t>(1, b * e->piece_growth / 100))
      geo.push_back(b);
    e->n_geo = (uint32_t)geo.size();
    // the first pieces of a hot key are small: merged all in one launch (k_rounds_fused) while
    // piece + centroids fit its per-key scratch
    e->fuse_pieces = 0;
    while (e->fuse_pieces + 1 < geo.size() &&
           geo[e->fuse_pieces + 1] - geo[e->fuse_pieces] + e->cap_cent <= kFuseMaxL)
      e->fuse_pieces++;
    dalloc(e->h_geo, geo.size());
    VN_HIP_CHECK(hipMemcpyAsync(e->h_geo, geo.data(), geo.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    VN_HIP_CHECK(hipStreamSynchronize(st));
  }

  dalloc(e->smode, cs); dzero(e->smode, cs, st);
  dalloc(e->sbase, cs); dzero(e->sbase, cs, st);
  dalloc(e->snz, cs);
  dalloc(e->slc, cs); dzero(e->slc, cs, st);
  dalloc(e->slb, cs); dzero(e->slb, cs, st);
  dalloc(e->slast, cs); dzero(e->slast, cs, st);
  dalloc(e->stc, cs); dzero(e->stc, cs, st);
  dalloc(e->stouch, cs); dzero(e->stouch, cs, st);
  dalloc(e->stmp, (size_t)cs * kTmpCap);
  dalloc(e->sarena, (size_t)cs * kArenaWords);
  dalloc(e->sR0, cs ? Rs : 0);
  dalloc(e->sR1, cs ? Rs : 0);
  dalloc(e->s_bt, cs); dzero(e->s_bt, cs, st);
  dalloc(e->s_pos, (size_t)cs + 1);
  dalloc(e->s_tl, cs);
  dalloc(e->s_cnt, 4);
  dalloc(e->s_lpt0, cs); dalloc(e->s_lpt1, cs);
  dalloc(e->s_start, cs);
  dalloc(e->s_end, cs);

  // staging buffers are allocated on first use (ensure_device_stage / ensure_pinned_stage)

  // flush outputs
  dalloc(e->f_pos, (size_t)capmax + 1);
  for (int c = 0; c < VN_NCLASS; c++) {
    dalloc(e->f_list[c], e->cap[c]);
    halloc(e->hf_list[c], e->cap[c]);
  }
  dalloc(e->f_cnt, 4);
  dalloc(e->f_cval, cc); halloc(e->hf_cval, cc);
  dalloc(e->f_gval, cg); halloc(e->hf_gval, cg);
  dalloc(e->f_hstats, (size_t)ch * VN_HISTO_STATS); halloc(e->hf_hstats, (size_t)ch * VN_HISTO_STATS);
  dalloc(e->f_hq, (size_t)ch * std::max<uint32_t>(1, e->cfg.n_percentiles));
  halloc(e->hf_hq, (size_t)ch * std::max<uint32_t>(1, e->cfg.n_percentiles));
  dalloc(e->f_sest, cs); halloc(e->hf_sest, cs);
  dalloc(e->f_ssparse, cs); halloc(e->hf_ssparse, cs);
  dalloc(e->d_pct, VN_MAX_PERCENTILES);
  dalloc(e->f_hmask, ch);
  dalloc(e->f_smask, cs);
  VN_HIP_CHECK(hipMemcpyAsync(e->d_pct, e->cfg.percentiles, sizeof(double) * VN_MAX_PERCENTILES,
                              hipMemcpyHostToDevice, st));
  halloc(e->hf_cnt, 16);

  const uint64_t Rside = std::max(cs ? Rs : 0, (cc || cg) ? Rcg : 0);
  radix_scratch_reserve(e->rs, std::max<uint64_t>(e->h_sort_cap, Rside));
  radix_scratch_reserve(e->rs2, std::max<uint64_t>(Rside, 1));
  radix_scratch_reserve(e->rs3, std::max<uint64_t>(touch_max, 1));
  init_state(e);
  VN_HIP_CHECK(hipStreamSynchronize(st));
}

// a batch with more records of some class than that class's cap
static bool over_class_caps(const vn_engine* e, const vn_batch* b) {
  return b->n_counter > e->max_cls[VN_COUNTER] || b->n_gauge > e->max_cls[VN_GAUGE] ||
         b->n_histo > e->max_cls[VN_HISTO] || b->n_set > e->max_cls[VN_SET];
}

// device staging for host-provided batches (vn_ingest_host / vn_submit / imports)
void ensure_device_stage(vn_engine* e) {
  DeviceBatch& d = e->dstage;
  if (d.c_slot) return;
  const uint64_t* R = e->max_cls;
  dalloc(d.c_slot, R[VN_COUNTER]); dalloc(d.c_val, R[VN_COUNTER]); dalloc(d.c_rate, R[VN_COUNTER]);
  dalloc(d.g_slot, R[VN_GAUGE]); dalloc(d.g_val, R[VN_GAUGE]);
  dalloc(d.h_slot, R[VN_HISTO]); dalloc(d.h_val, R[VN_HISTO]); dalloc(d.h_rate, R[VN_HISTO]);
  dalloc(d.s_slot, R[VN_SET]); dalloc(d.s_off, R[VN_SET] + 1); dalloc(d.s_bytes, e->max_member_bytes);
}

// pinned host staging the Go side appends ProcessMetric records to (vn_stage_acquire)
void ensure_pinned_stage(vn_engine* e) {
  vn_stage& p = e->pstage;
  if (p.counter_slot) return;
  const uint64_t R = e->max_records;
  p.capacity = R;
  p.member_bytes_capacity = e->max_member_bytes;
  halloc(p.counter_slot, R); halloc(p.counter_value, R); halloc(p.counter_rate, R);
  halloc(p.gauge_slot, R); halloc(p.gauge_value, R);
  halloc(p.histo_slot, R); halloc(p.histo_value, R); halloc(p.histo_rate, R);
  halloc(p.set_slot, R); halloc(p.set_member_off, R + 1); halloc(p.set_member_bytes, e->max_member_bytes);
}

// import staging, grown to the call's payload count / byte size
void ensure_import(vn_engine* e, uint64_t n, uint64_t nbytes) {
  ImportScratch& s = e->imp;
  if (n > s.cap_n) {
    dfree(s.in_slot); dfree(s.in_off); dfree(s.cnt); dfree(s.coff); dfree(s.cpos); dfree(s.ckpt);
    if (s.parts) (void)hipFree(s.parts);
    s.cap_n = std::max<uint64_t>(n, 1024);
    dalloc(s.in_slot, s.cap_n);
    dalloc(s.in_off, s.cap_n + 1);
    dalloc(s.cnt, s.cap_n + 1);
    dalloc(s.coff, s.cap_n + 1);
    dalloc(s.cpos, s.cap_n);
    dalloc(s.ckpt, s.cap_n * 16);
    VN_HIP_CHECK(hipMalloc(&s.parts, s.cap_n * 64));
  }
  if (nbytes > s.cap_bytes) {
    dfree(s.in_bytes);
    s.cap_bytes = std::max<uint64_t>(nbytes, 1 << 16);
    dalloc(s.in_bytes, s.cap_bytes);
  }
  if (!s.cap_cent) {
    s.cap_cent = e->max_cls[VN_HISTO];  // the drains ingest them as histo records
    dalloc(s.cmean, s.cap_cent);
    dalloc(s.cw, s.cap_cent);
    dalloc(s.cw_alt, s.cap_cent);
    s.cap_pay = e->max_records;  // payloads of one import call, at most
    dalloc(s.pslot, s.cap_pay);
    dalloc(s.pbeg, s.cap_pay + 1);
    dalloc(s.pkey, 2 * s.cap_pay);
    dalloc(s.pcnt, s.cap_pay + 1);
    dalloc(s.pdst, s.cap_pay + 1);
    dalloc(s.cuts, 2 * (kImportCuts + 1) + 2);
    halloc(s.hcuts, 2 * (kImportCuts + 1) + 2);
  }
}

// stage host payloads (slot[n], off[n+1], bytes) for an import call
void stage_import(vn_engine* e, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes, uint64_t n,
                  uint32_t cap) {
  if (n > e->max_records) throw std::invalid_argument("import batch larger than max_batch_records");
  check_slots_host(slot, n, cap, "import");
  for (uint64_t i = 0; i < n; i++)
    if (off[i + 1] < off[i]) throw std::invalid_argument("import offsets must be non-decreasing");
  const uint64_t nb = off[n];
  ensure_import(e, n, nb);
  ImportScratch& s = e->imp;
  hipStream_t st = e->st;
  h2d(s.in_slot, slot, n, st);
  h2d(s.in_off, off, n + 1, st);
  h2d(s.in_bytes, bytes, nb, st);
}

void ensure_export(vn_engine* e, uint64_t n) {
  ExportBuffers& x = e->exp;
  if (n <= x.cap_n) return;
  dfree(x.d_slot); dfree(x.d_keys); dfree(x.d_size); dfree(x.d_off); hfree(x.h_off);
  x.cap_n = std::max<uint64_t>(n, 1024);
  dalloc(x.d_slot, x.cap_n);
  dalloc(x.d_keys, x.cap_n);
  dalloc(x.d_size, x.cap_n);
  dalloc(x.d_off, x.cap_n + 1);
  halloc(x.h_off, x.cap_n + 1);
}

void export_impl(vn_engine* e, int cls, const uint32_t* slot, uint64_t n, vn_export* out) {
  check_slots_host(slot, n, e->cap[cls], cls == VN_HISTO ? "histo" : "set");
  ensure_export(e, n);
  ExportBuffers& x = e->exp;
  h2d(x.d_slot, slot, n, e->st);
  if (cls == VN_HISTO) {  // GobEncode merges the pending temps first (merging_digest.go:362)
    histo_imports_drain(e);
    std::vector<uint32_t> keys(slot, slot + n);
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    h2d(x.d_keys, keys.data(), keys.size(), e->st);
    histo_merge_pending(e, x.d_keys, (uint32_t)keys.size());
    export_histos(e, x.d_slot, n, x);
  } else {
    export_sets(e, x.d_slot, n, x);
  }
  out->n = n;
  out->off = x.h_off;
  out->bytes = x.h_bytes;
  out->dev_off = x.d_off;
  out->dev_bytes = x.d_bytes;
}

void destroy_impl(vn_engine* e) {
  for (hipEvent_t* ev : {&e->ev_w0, &e->ev_wmain})
    if (*ev) {
      (void)hipEventDestroy(*ev);
      *ev = nullptr;
    }
  if (e->st) (void)hipStreamSynchronize(e->st);
  split_destroy(e);
  hot_destroy(e);
  dfree(e->cval); dfree(e->ctouch); dfree(e->gseq); dfree(e->gval); dfree(e->gtouch); dfree(e->pk); dfree(e->pp);
  dfree(e->hst); dfree(e->hncent); dfree(e->hcur); dfree(e->htouch);
  for (int b = 0; b < 2; b++) { dfree(e->cmean[b]); dfree(e->cw[b]); }
  dfree(e->h_bt); dfree(e->h_pos); dfree(e->h_tl); dfree(e->h_cnt);
  dfree(e->hA0); dfree(e->hB0); dfree(e->hA1); dfree(e->hB1); dfree(e->h_w); dfree(e->h_wk);
  dfree(e->h_start); dfree(e->h_end); dfree(e->h_nch); dfree(e->h_chb);
  dfree(e->ch_sum); dfree(e->ch_pre); dfree(e->ch_stats); dfree(e->seg_T);
  dfree(e->starts); dfree(e->nc_new); dfree(e->acc_xw); dfree(e->acc_w); dfree(e->h_err);
  dfree(e->hseen); dfree(e->hpend); dfree(e->hspn); dfree(e->hspw); dfree(e->hm_flag); dfree(e->hm_pos); dfree(e->hm_idx); dfree(e->hm_list); dfree(e->hm_cnt); dfree(e->hpv); dfree(e->hpw); dfree(e->h_ex); dfree(e->h_hotflag);
  dfree(e->h_coldflag); dfree(e->h_coldlist); dfree(e->h_vhflag); dfree(e->h_warmflag); dfree(e->h_warmlist); dfree(e->hA2); dfree(e->hB2); dfree(e->h_csv); dfree(e->h_csw); dfree(e->h_cpk); dfree(e->h_lstat); dfree(e->h_cstat);
  dfree(e->h_lpt0); dfree(e->h_lpt1); dfree(e->s_lpt0); dfree(e->s_lpt1);
  dfree(e->h_hotcnt); dfree(e->h_hotoff); dfree(e->h_hotlist); dfree(e->h_tl2); dfree(e->h_ccnt); dfree(e->h_coff); dfree(e->h_cown); dfree(e->h_tw);
  dfree(e->fz_val); dfree(e->fz_w); dfree(e->fz_k); dfree(e->fz_done);
  dfree(e->h_geo); dfree(e->h_seen0); dfree(e->h_pcnt); dfree(e->h_pi0); dfree(e->h_pbase); dfree(e->p_start);
  dfree(e->p_end); dfree(e->r_flag); dfree(e->r_len); dfree(e->r_list); dfree(e->r_off); dfree(e->r_pos);
  dfree(e->smode); dfree(e->sbase); dfree(e->snz); dfree(e->slc); dfree(e->slb); dfree(e->slast); dfree(e->stc);
  dfree(e->stouch); dfree(e->stmp); dfree(e->sarena); dfree(e->sR0); dfree(e->sR1); dfree(e->s_bt);
  dfree(e->s_pos); dfree(e->s_tl); dfree(e->s_cnt); dfree(e->s_start); dfree(e->s_end);
  ExportBuffers& xb = e->exp;
  dfree(xb.d_slot); dfree(xb.d_keys); dfree(xb.d_size); dfree(xb.d_off); hfree(xb.h_off); dfree(xb.d_bytes);
  hfree(xb.h_bytes);
  ImportScratch& is = e->imp;
  dfree(is.in_slot); dfree(is.in_off); dfree(is.in_bytes); dfree(is.cnt); dfree(is.coff); dfree(is.cpos); dfree(is.ckpt); dfree(is.cuts); hfree(is.hcuts); dfree(is.cslot);
  dfree(is.pslot); dfree(is.pbeg); dfree(is.pkey); dfree(is.pcnt); dfree(is.pdst);
  dfree(is.cmean); dfree(is.cw); dfree(is.cw_alt);
  if (is.parts) (void)hipFree(is.parts);
  DeviceBatch& d = e->dstage;
  dfree(d.c_slot); dfree(d.c_val); dfree(d.c_rate); dfree(d.g_slot); dfree(d.g_val);
  dfree(d.h_slot); dfree(d.h_val); dfree(d.h_rate); dfree(d.s_slot); dfree(d.s_off); dfree(d.s_bytes);
  vn_stage& p = e->pstage;
  hfree(p.counter_slot); hfree(p.counter_value); hfree(p.counter_rate); hfree(p.gauge_slot); hfree(p.gauge_value);
  hfree(p.histo_slot); hfree(p.histo_value); hfree(p.histo_rate); hfree(p.set_slot); hfree(p.set_member_off);
  hfree(p.set_member_bytes);
  dfree(e->f_pos);
  for (int c = 0; c < VN_NCLASS; c++) { dfree(e->f_list[c]); hfree(e->hf_list[c]); }
  dfree(e->f_cnt); dfree(e->f_cval); hfree(e->hf_cval); dfree(e->f_gval); hfree(e->hf_gval);
  dfree(e->f_hstats); hfree(e->hf_hstats); dfree(e->f_hq); hfree(e->hf_hq); dfree(e->f_sest); hfree(e->hf_sest);
  dfree(e->d_imp_counts); dfree(e->f_ssparse); hfree(e->hf_ssparse); dfree(e->d_pct); hfree(e->hf_cnt);
  dfree(e->f_hmask); dfree(e->f_smask);
  radix_scratch_free(e->rs);
  radix_scratch_free(e->rs2);
  radix_scratch_free(e->rs3);
  if (e->ss.partials) (void)hipFree(e->ss.partials);
  if (e->ss2.partials) (void)hipFree(e->ss2.partials);
  if (e->st2) (void)hipStreamSynchronize(e->st2);
  if (e->st3) (void)hipStreamSynchronize(e->st3);
  if (e->st_imp) {
    (void)hipStreamSynchronize(e->st_imp);
    (void)hipStreamDestroy(e->st_imp);
    e->st_imp = nullptr;
  }
  for (hipEvent_t* ev : {&e->ev_imp_free, &e->ev_imp_emit})
    if (*ev) {
      (void)hipEventDestroy(*ev);
      *ev = nullptr;
    }
  if (e->ev_fork3) (void)hipEventDestroy(e->ev_fork3);
  if (e->ev_join3) (void)hipEventDestroy(e->ev_join3);
  if (e->st3) (void)hipStreamDestroy(e->st3);
  if (e->st5) (void)hipStreamSynchronize(e->st5);
  if (e->st6) {
    (void)hipStreamSynchronize(e->st6);
    (void)hipStreamDestroy(e->st6);
    e->st6 = nullptr;
  }
  if (e->ev_join6) {
    (void)hipEventDestroy(e->ev_join6);
    e->ev_join6 = nullptr;
  }
  for (hipEvent_t* ev : {&e->ev_fork5, &e->ev_join5, &e->ev_rest5, &e->ev_bulk})
    if (*ev) {
      (void)hipEventDestroy(*ev);
      *ev = nullptr;
    }
  if (e->st5) {
    (void)hipStreamDestroy(e->st5);
    e->st5 = nullptr;
  }
  if (e->st4) (void)hipStreamSynchronize(e->st4);
  if (e->st_ctr) {
    (void)hipStreamSynchronize(e->st_ctr);
    (void)hipStreamDestroy(e->st_ctr);
    e->st_ctr = nullptr;
  }
  for (hipEvent_t* ev : {&e->ev_ctr0, &e->ev_ctr1})
    if (*ev) {
      (void)hipEventDestroy(*ev);
      *ev = nullptr;
    }
  if (e->ev_join4) (void)hipEventDestroy(e->ev_join4);
  if (e->st4) (void)hipStreamDestroy(e->st4);
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_h2d) (void)hipEventDestroy(e->ev_h2d);
  if (e->ev_join) (void)hipEventDestroy(e->ev_join);
  if (e->st2) (void)hipStreamDestroy(e->st2);
  for (auto ev : e->pool_storage) (void)hipEventDestroy(ev);
  for (auto ev : e->pool_rp_storage) (void)hipEventDestroy(ev);
  for (auto ev : e->pool_ss_storage) (void)hipEventDestroy(ev);
  for (auto ev : e->pool_ps_storage) (void)hipEventDestroy(ev);
  for (auto ev : e->pool_id_storage) (void)hipEventDestroy(ev);
  for (auto ev : e->pool_im_storage) (void)hipEventDestroy(ev);
  for (auto& ev : e->ev)
    if (ev) (void)hipEventDestroy(ev);
  if (e->st) (void)hipStreamDestroy(e->st);
}

// throws on the engine's invariant flags; returns the caller-error flags (cleared on the device)
// (every copy here is ordered on the engine's own stream: a plain hipMemcpy runs on the null
// stream, which waits for every blocking stream of the device -- the CU-masked ones, whatever
// engine they belong to -- and so would hold this flush behind another engine's replays)
uint32_t check_error_flags(vn_engine* e) {
  uint32_t flags = 0;
  VN_HIP_CHECK(hipMemcpyAsync(&flags, e->h_err, sizeof(uint32_t), hipMemcpyDeviceToHost, e->st));
  VN_HIP_CHECK(hipStreamSynchronize(e->st));
  if (flags & 1u) throw std::runtime_error("t-digest centroid tile overflow (compression too large for cap_cent)");
  if (flags & 2u) throw std::runtime_error("HLL rebase invariant violated");
  if (flags & 4u) throw std::runtime_error("t-digest chain window hand-off stalled");
  const uint32_t caller = flags & kErrSplitTouched;  // the caller's error, not the engine's: reported once
  if (caller) {
    flags &= ~caller;
    VN_HIP_CHECK(hipMemcpyAsync(e->h_err, &flags, sizeof(uint32_t), hipMemcpyHostToDevice, e->st));
    VN_HIP_CHECK(hipStreamSynchronize(e->st));
  }
  return caller;
}
void throw_caller_errors(uint32_t caller) {
  if (caller & kErrSplitTouched)
    throw std::invalid_argument("a split key's slot also received vn_ingest records or imports this window "
                                "(its records go through vn_ingest_split); the split combine's state was kept");
}

// Validation of a device-resident batch (vn_ingest), where the reference would panic or the
// parser would have rejected the line: slots within capacity (an interned key), histo values
// neither NaN nor +-Inf (MergingDigest.Add panics, merging_digest.go:98-100), histogram sample
// rates in (0, 1] (parser.go:262-272; see below), set member offsets non-decreasing.  Counter
// rates are not checked: Counter.Sample's int64(sample) * int64(float32(1/rate)) is defined for
// every float32 rate -- a NaN rate (which the parser lets through: both of its comparisons are
// false) or 0 gives int64(NaN / +Inf) = MinInt64 on amd64, which f64_to_i64_go reproduces.  A
// histogram's NaN rate is refused: Go's digest takes the NaN weight (Add checks weight <= 0) and
// its next mergeAllTemps over a NaN-mean centroid never terminates (NaN rates).  One pass over the batch, flags in h_err[1]; the host reads them before any
// state-mutating kernel is queued, so a rejected batch leaves the window untouched.
constexpr uint32_t kBadSlot = 1u, kBadValue = 2u, kBadRate = 4u, kBadOffsets = 8u;
__global__ void k_validate_batch(vn_batch b, uint32_t cc, uint32_t cg, uint32_t ch, uint32_t cs,
                                 uint32_t* __restrict__ err) {
  const uint64_t nmax = max(max(b.n_counter, b.n_gauge), max(b.n_histo, b.n_set));
  uint32_t f = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nmax; i += (uint64_t)gridDim.x * blockDim.x) {
    if (i < b.n_counter && b.counter_slot[i] >= cc) f |= kBadSlot;
    if (i < b.n_gauge && b.gauge_slot[i] >= cg) f |= kBadSlot;
    if (i < b.n_histo) {
      const double v = b.histo_value[i];
      const float r = b.histo_rate[i];
      if (b.histo_slot[i] >= ch) f |= kBadSlot;
      if (v != v || v - v != 0.0) f |= kBadValue;
      if (!(r > 0.0f && r <= 1.0f)) f |= kBadRate;
    }
    if (i < b.n_set) {
      if (b.set_slot[i] >= cs) f |= kBadSlot;
      if (!b.set_hash && b.set_member_off[i + 1] < b.set_member_off[i]) f |= kBadOffsets;
    }
  }
  // one atomic per wave that saw a fault
  for (int d = 32; d >= 1; d >>= 1) f |= __shfl_xor(f, d, 64);
  if (f && (threadIdx.x & 63) == 0) atomicOr(err, f);
}

// The same checks with 16-byte loads (four records per lane and array) when every array of
// the batch is 16-byte aligned; the records past the last full quad of a class take the
// scalar checks.
__device__ __forceinline__ bool bad_rate(float r) { return !(r > 0.0f && r <= 1.0f); }
__device__ __forceinline__ bool bad_value(double v) { return v != v || v - v != 0.0; }
__global__ void k_validate_batch4(vn_batch b, uint32_t cc, uint32_t cg, uint32_t ch, uint32_t cs,
                                  uint32_t* __restrict__ err) {
  const uint64_t nmax = max(max(b.n_counter, b.n_gauge), max(b.n_histo, b.n_set));
  const uint64_t qmax = (nmax + 3) / 4;
  uint32_t f = 0;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < qmax; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i0 = 4 * q;
    if (i0 + 4 <= b.n_counter) {
      const uint4 sl = reinterpret_cast<const uint4*>(b.counter_slot)[q];
      if (max(max(sl.x, sl.y), max(sl.z, sl.w)) >= cc) f |= kBadSlot;
    } else {
      for (uint64_t i = i0; i < b.n_counter && i < i0 + 4; i++)
        if (b.counter_slot[i] >= cc) f |= kBadSlot;
    }
    if (i0 + 4 <= b.n_gauge) {
      const uint4 sl = reinterpret_cast<const uint4*>(b.gauge_slot)[q];
      if (max(max(sl.x, sl.y), max(sl.z, sl.w)) >= cg) f |= kBadSlot;
    } else {
      for (uint64_t i = i0; i < b.n_gauge && i < i0 + 4; i++)
        if (b.gauge_slot[i] >= cg) f |= kBadSlot;
    }
    if (i0 + 4 <= b.n_histo) {
      const uint4 sl = reinterpret_cast<const uint4*>(b.histo_slot)[q];
      const float4 r = reinterpret_cast<const float4*>(b.histo_rate)[q];
      const double2 v0 = reinterpret_cast<const double2*>(b.histo_value)[2 * q];
      const double2 v1 = reinterpret_cast<const double2*>(b.histo_value)[2 * q + 1];
      if (max(max(sl.x, sl.y), max(sl.z, sl.w)) >= ch) f |= kBadSlot;
      if (bad_value(v0.x) || bad_value(v0.y) || bad_value(v1.x) || bad_value(v1.y)) f |= kBadValue;
      if (bad_rate(r.x) || bad_rate(r.y) || bad_rate(r.z) || bad_rate(r.w)) f |= kBadRate;
    } else {
      for (uint64_t i = i0; i < b.n_histo && i < i0 + 4; i++) {
        if (b.histo_slot[i] >= ch) f |= kBadSlot;
        if (bad_value(b.histo_value[i])) f |= kBadValue;
        if (bad_rate(b.histo_rate[i])) f |= kBadRate;
      }
    }
    if (i0 + 4 <= b.n_set) {
      const uint4 sl = reinterpret_cast<const uint4*>(b.set_slot)[q];
      if (max(max(sl.x, sl.y), max(sl.z, sl.w)) >= cs) f |= kBadSlot;
      if (!b.set_hash) {
        const uint4 o = reinterpret_cast<const uint4*>(b.set_member_off)[q];
        const uint32_t o4 = b.set_member_off[i0 + 4];
        if (o.y < o.x || o.z < o.y || o.w < o.z || o4 < o.w) f |= kBadOffsets;
      }
    } else {
      for (uint64_t i = i0; i < b.n_set && i < i0 + 4; i++) {
        if (b.set_slot[i] >= cs) f |= kBadSlot;
        if (!b.set_hash && b.set_member_off[i + 1] < b.set_member_off[i]) f |= kBadOffsets;
      }
    }
  }
  for (int d = 32; d >= 1; d >>= 1) f |= __shfl_xor(f, d, 64);
  if (f && (threadIdx.x & 63) == 0) atomicOr(err, f);
}

void validate_device_batch(vn_engine* e, const vn_batch* b) {
  const uint64_t nmax = std::max(std::max(b->n_counter, b->n_gauge), std::max(b->n_histo, b->n_set));
  if (!nmax) return;
  if ((b->n_counter && (!b->counter_slot || !b->counter_value || !b->counter_rate)) ||
      (b->n_gauge && (!b->gauge_slot || !b->gauge_value)) ||
      (b->n_histo && (!b->histo_slot || !b->histo_value || !b->histo_rate)) ||
      (b->n_set && (!b->set_slot || (!b->set_hash && (!b->set_member_off || !b->set_member_bytes)))))
    throw std::invalid_argument("batch class with records but a null array");
  hipStream_t st = e->st;
  VN_HIP_CHECK(hipMemsetAsync(e->h_err + 1, 0, sizeof(uint32_t), st));
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  const bool vec = a16(b->counter_slot) && a16(b->counter_rate) && a16(b->gauge_slot) && a16(b->histo_slot) &&
                   a16(b->histo_rate) && a16(b->histo_value) && a16(b->set_slot) &&
                   (b->set_hash || a16(b->set_member_off));
  if (vec) {
    const int grid = (int)std::min<uint64_t>(blocks_for((nmax + 3) / 4, 256), 4096);
    hipLaunchKernelGGL(k_validate_batch4, dim3(grid), dim3(256), 0, st, *b, e->cap[VN_COUNTER], e->cap[VN_GAUGE],
                       e->cap[VN_HISTO], e->cap[VN_SET], e->h_err + 1);
  } else {
    const int grid = (int)std::min<uint64_t>(blocks_for(nmax, 256), 4096);
    hipLaunchKernelGGL(k_validate_batch, dim3(grid), dim3(256), 0, st, *b, e->cap[VN_COUNTER], e->cap[VN_GAUGE],
                       e->cap[VN_HISTO], e->cap[VN_SET], e->h_err + 1);
  }
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 15, e->h_err + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HWAIT(e, 0, VN_HIP_CHECK(hipStreamSynchronize(st)));
  const uint32_t f = e->hf_cnt[15];
  if (f & kBadSlot) throw std::invalid_argument("slot out of range");
  if (f & kBadValue) throw std::invalid_argument("invalid value added");  // merging_digest.go:98-100
  if (f & kBadRate) throw std::invalid_argument("sample rate must be >0 and <=1");
  if (f & kBadOffsets) throw std::invalid_argument("set member offsets must be non-decreasing");
}

#ifndef VN_SETS_FIRST
#define VN_SETS_FIRST 0
#endif
constexpr bool kSetsFirst = VN_SETS_FIRST;  // side-stream order (compile-time A/B, tools/ab_variant.sh)

void ingest_device(vn_engine* e, const vn_batch* b) {
  histo_imports_drain(e);  // imports that came first merge first
  if (over_class_caps(e, b))
    throw std::invalid_argument("batch larger than max_batch_records");
  if ((b->n_counter && !e->cap[VN_COUNTER]) || (b->n_gauge && !e->cap[VN_GAUGE]) ||
      (b->n_histo && !e->cap[VN_HISTO]) || (b->n_set && !e->cap[VN_SET]))
    throw std::invalid_argument("records for a class with zero capacity");
  hipStream_t st = e->st;
  hot_sample(e, VN_COUNTER, b->n_counter, b->counter_slot, nullptr, 0, st);
  hot_sample(e, VN_HISTO, b->n_histo, b->histo_slot, nullptr, 0, st);
  hot_sample(e, VN_SET, b->n_set, b->set_slot, nullptr, 0, st);
  const bool tm = e->timing;
  if (tm) {
    e->pool.used = 0;
    e->pool_rp.used = 0;
    e->pool_ss.used = 0;
    e->pool_ps.used = 0;
    e->kstat_rp = RadixStats{&e->pool_rp, 0, 0};
    e->kstat_ss = RadixStats{&e->pool_ss, 0, 0};
    e->rstat_c = RadixStats{&e->pool_ps, 0, 0};
    e->rstat_h = RadixStats{&e->pool, 0, 0};
    e->rstat_s = RadixStats{&e->pool, 0, 0};
    VN_HIP_CHECK(hipEventRecord(e->ev[0], st));
    e->ev_rec |= 1u << 0;
  }
  if (tm) {
    // measured: one phase at a time on the main stream
    side_begin(e);
    ingest_counters(e, b->n_counter, b->counter_slot, b->counter_value, b->counter_rate);
    VN_HIP_CHECK(hipEventRecord(e->ev[1], st));
    e->ev_rec |= 1u << 1;
    ingest_gauges(e, b->n_gauge, b->gauge_slot, b->gauge_value);
    VN_HIP_CHECK(hipEventRecord(e->ev[2], st));
    e->ev_rec |= 1u << 2;
    ingest_sets(e, b->n_set, b->set_slot, b->set_member_off, b->set_member_bytes, b->set_hash);
    VN_HIP_CHECK(hipEventRecord(e->ev[3], st));
    e->ev_rec |= 1u << 3;
    ingest_histos(e, b->n_histo, b->histo_slot, b->histo_value, b->histo_rate);
    side_join(e);
  } else {
    // the histo grouping sort (critical path) is queued first on the main stream; then
    // counters, gauges and sets on the low-priority side stream (none of them waits on the
    // host); then the rest of the histo path, whose host round trips no longer hold back
    // the side work -- it fills the GPU while the replays and remainder rounds run
    side_begin(e);  // the side stream waits for what the main stream held before this call
    const HistoGroups g = histo_group(e, b->n_histo, b->histo_slot, b->histo_value, b->histo_rate);
    if (kSetsFirst) {  // the whole set path first: its long per-key merges overlap everything else
      ingest_sets(e, b->n_set, b->set_slot, b->set_member_off, b->set_member_bytes, b->set_hash);
      ingest_counters(e, b->n_counter, b->counter_slot, b->counter_value, b->counter_rate);
      ingest_gauges(e, b->n_gauge, b->gauge_slot, b->gauge_value);
    } else {
      ingest_counters(e, b->n_counter, b->counter_slot, b->counter_value, b->counter_rate);
      ingest_gauges(e, b->n_gauge, b->gauge_slot, b->gauge_value);
      e->set_defer = true;  // histo_process queues the set merge after the remainder sort
      ingest_sets(e, b->n_set, b->set_slot, b->set_member_off, b->set_member_bytes, b->set_hash);
      e->set_defer = false;
    }
    histo_process(e, b->n_histo, g);
    set_finish(e);
    side_join(e);
  }
  if (tm) {
    VN_HIP_CHECK(hipEventRecord(e->ev[4], st));
    e->ev_rec |= 1u << 4;
  }
  VN_HIP_CHECK(hipGetLastError());  // a launch that could not start (e.g. LDS over budget) fails loudly
  e->processed += b->n_counter + b->n_gauge + b->n_histo + b->n_set;
}


void ingest_host(vn_engine* e, const vn_batch* b) {
  histo_imports_drain(e);
  if (over_class_caps(e, b))
    throw std::invalid_argument("batch larger than max_batch_records");
  check_slots_host(b->counter_slot, b->n_counter, e->cap[VN_COUNTER], "counter");
  check_slots_host(b->gauge_slot, b->n_gauge, e->cap[VN_GAUGE], "gauge");
  check_slots_host(b->histo_slot, b->n_histo, e->cap[VN_HISTO], "histo");
  check_slots_host(b->set_slot, b->n_set, e->cap[VN_SET], "set");
  for (uint64_t i = 0; i < b->n_histo; i++) {
    double v = b->histo_value[i];
    float r = b->histo_rate[i];
    if (v != v || v - v != 0) throw std::invalid_argument("invalid value added");  // merging_digest.go:98-100
    if (!(r > 0.0f && r <= 1.0f)) throw std::invalid_argument("sample rate must be >0 and <=1");
  }
  hipStream_t st = e->st;
  ensure_device_stage(e);
  DeviceBatch& d = e->dstage;
  vn_batch db{};
  db.n_counter = b->n_counter;
  h2d(d.c_slot, b->counter_slot, b->n_counter, st);
  h2d(d.c_val, b->counter_value, b->n_counter, st);
  h2d(d.c_rate, b->counter_rate, b->n_counter, st);
  db.counter_slot = d.c_slot; db.counter_value = d.c_val; db.counter_rate = d.c_rate;
  db.n_gauge = b->n_gauge;
  h2d(d.g_slot, b->gauge_slot, b->n_gauge, st);
  h2d(d.g_val, b->gauge_value, b->n_gauge, st);
  db.gauge_slot = d.g_slot; db.gauge_value = d.g_val;
  db.n_histo = b->n_histo;
  h2d(d.h_slot, b->histo_slot, b->n_histo, st);
  h2d(d.h_val, b->histo_value, b->n_histo, st);
  h2d(d.h_rate, b->histo_rate, b->n_histo, st);
  db.histo_slot = d.h_slot; db.histo_value = d.h_val; db.histo_rate = d.h_rate;
  db.n_set = b->n_set;
  uint64_t* dhash = nullptr;
  if (b->n_set) {
    h2d(d.s_slot, b->set_slot, b->n_set, st);
    db.set_slot = d.s_slot;
    if (b->set_hash) {
      // hashes travel in the (u64-aligned) member byte staging area
      if (b->n_set * 8 > e->max_member_bytes) throw std::invalid_argument("set hash batch exceeds staging");
      dhash = reinterpret_cast<uint64_t*>(d.s_bytes);
      h2d(dhash, b->set_hash, b->n_set, st);
      db.set_hash = dhash;
    } else {
      uint64_t nb = b->set_member_off[b->n_set];
      if (nb > e->max_member_bytes) throw std::invalid_argument("member bytes exceed max_batch_member_bytes");
      h2d(d.s_off, b->set_member_off, b->n_set + 1, st);
      h2d(d.s_bytes, b->set_member_bytes, nb, st);
      db.set_member_off = d.s_off;
      db.set_member_bytes = d.s_bytes;
    }
  }
  // the pinned stage may be refilled as soon as its copies have been read (vn_submit waits)
  VN_HIP_CHECK(hipEventRecord(e->ev_h2d, st));
  ingest_device(e, &db);
}

}  // namespace

namespace vn {
void ensure_export_bytes(vn_engine* e, ExportBuffers& x, uint64_t nbytes) {
  (void)e;
  if (nbytes <= x.cap_bytes && x.d_bytes) return;
  dfree(x.d_bytes);
  hfree(x.h_bytes);
  x.cap_bytes = std::max<uint64_t>(nbytes, 1 << 16);
  dalloc(x.d_bytes, x.cap_bytes);
  halloc(x.h_bytes, x.cap_bytes);
}
void take_decode_error(vn_engine* e) {
  uint32_t flags = 0;
  VN_HIP_CHECK(hipMemcpyAsync(&flags, e->h_err, sizeof(uint32_t), hipMemcpyDeviceToHost, e->st));
  VN_HIP_CHECK(hipStreamSynchronize(e->st));
  if (flags & kErrDecode) {
    flags &= ~kErrDecode;
    VN_HIP_CHECK(hipMemcpyAsync(e->h_err, &flags, sizeof(uint32_t), hipMemcpyHostToDevice, e->st));
    VN_HIP_CHECK(hipStreamSynchronize(e->st));
    throw DecodeError("malformed import payload");
  }
}
// st3 / st4 (the fast mode's fork) and st_ctr (the split counters' combine), at first use
void ensure_aux_streams(vn_engine* e, bool fork, bool ctr) {
  auto make = [&](hipStream_t& s, bool replay_mask) {
    if (s) return;
    if (e->reserved_cus)
      VN_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)e->amask.size(), e->amask.data()));
    else if (replay_mask && !e->rmask.empty())
      VN_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)e->rmask.size(), e->rmask.data()));
    else
      VN_HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, e->prio_hi));
  };
  if (fork) {
    make(e->st3, true);
    make(e->st4, false);
  }
  if (ctr) make(e->st_ctr, false);
}

void side_begin(vn_engine* e) {
  if (e->timing || !e->st2) {  // measured kernels run alone (or VN_SIDE_MAIN: one stream)
    e->side = e->st;
    e->side_rs = &e->rs;
    e->side_ss = &e->ss;
    return;
  }
  e->side = e->st2;
  e->side_rs = &e->rs2;
  e->side_ss = &e->ss2;
  VN_HIP_CHECK(hipEventRecord(e->ev_fork, e->st));
  VN_HIP_CHECK(hipStreamWaitEvent(e->st2, e->ev_fork, 0));
}
void side_join(vn_engine* e) {
  if (e->side != e->st) {
    VN_HIP_CHECK(hipEventRecord(e->ev_join, e->st2));
    VN_HIP_CHECK(hipStreamWaitEvent(e->st, e->ev_join, 0));
  }
  e->side = e->st;
}
}  // namespace vn

extern "C" {

int vn_abi_version(void) { return VN_ABI_VERSION; }
int vn_build_flags(void) { return VN_FAST_MODE ? VN_BUILD_FAST_MODE : 0; }

namespace {
__global__ void k_diag_index_estimate(double c, const double* __restrict__ q, uint64_t n,
                                      unsigned long long* __restrict__ bad, double* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = vn::index_estimate<true>(c, q[i]), b = vn::index_estimate<false>(c, q[i]);
  if (vn::dbits(a) != vn::dbits(b)) atomicAdd(bad, 1ull);
  if (out) {
    out[2 * i] = a;
    out[2 * i + 1] = b;
  }
}
}  // namespace

int vn_diag_index_estimate(int device, double compression, const double* q, uint64_t n, uint64_t* mismatches,
                           double* out) {
  if (!mismatches || (n && !q)) return VN_EINVAL;
  *mismatches = 0;
  if (!n) return VN_OK;
  if (hipSetDevice(device) != hipSuccess) return VN_EHIP;
  double* dq = nullptr;
  double* dout = nullptr;
  unsigned long long* dbad = nullptr;
  unsigned long long hbad = 0;
  int rc = VN_OK;
  if (hipMalloc(&dq, n * sizeof(double)) != hipSuccess || hipMalloc(&dbad, sizeof(unsigned long long)) != hipSuccess ||
      hipMemcpy(dq, q, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(dbad, 0, sizeof(unsigned long long)) != hipSuccess ||
      (out && hipMalloc(&dout, 2 * n * sizeof(double)) != hipSuccess)) {
    rc = VN_EHIP;
  } else {
    hipLaunchKernelGGL(k_diag_index_estimate, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, nullptr, compression, dq,
                       n, dbad, dout);
    if (hipMemcpy(&hbad, dbad, sizeof(hbad), hipMemcpyDeviceToHost) != hipSuccess) rc = VN_EHIP;
    if (out && rc == VN_OK && hipMemcpy(out, dout, 2 * n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
      rc = VN_EHIP;
  }
  if (dq) (void)hipFree(dq);
  if (dout) (void)hipFree(dout);
  if (dbad) (void)hipFree(dbad);
  *mismatches = hbad;
  return rc;
}
static_assert(kErrSplitTouched == VN_WARN_SPLIT_TOUCHED, "the flush reports the device flag as is");

size_t vn_struct_size(int which) {
  switch (which) {
    case VN_STRUCT_CONFIG: return sizeof(vn_config);
    case VN_STRUCT_BATCH: return sizeof(vn_batch);
    case VN_STRUCT_FLUSH_RESULT: return sizeof(vn_flush_result);
    case VN_STRUCT_TIMING: return sizeof(vn_timing);
    case VN_STRUCT_SPLIT_BATCH: return sizeof(vn_split_batch);
    case VN_STRUCT_STAGE: return sizeof(vn_stage);
    default: return 0;
  }
}

int vn_engine_create(const vn_config* cfg, vn_engine** out) {
  if (!cfg || !out) return VN_EINVAL;
  *out = nullptr;
  vn_engine* e = new vn_engine();
  e->cfg = *cfg;
  e->device = cfg->device;
  for (int c = 0; c < VN_NCLASS; c++) {
    e->cap[c] = cfg->capacity[c];
    e->slot_bits[c] = bits_for(std::max<uint32_t>(1, cfg->capacity[c]));
  }
  if (e->cfg.compression <= 0) e->cfg.compression = 100.0;
  if (e->cfg.n_percentiles > VN_MAX_PERCENTILES) {
    delete e;
    return VN_EINVAL;
  }
  uint32_t need = (uint32_t)(2.0 * e->cfg.compression) + 4;
  e->cap_cent = ((need + 15) / 16) * 16;  // (delta 100: 208, whose replay tile gives 14 waves per CU)
  if (e->cap_cent < 64) e->cap_cent = 64;
  if (e->cap_cent > 2048 || (uint64_t)e->cap[VN_HISTO] * e->cap_cent >= (1ull << 31)) {
    delete e;
    return VN_EINVAL;
  }
  e->exact_threshold = cfg->histo_exact_threshold ? cfg->histo_exact_threshold : 0xFFFFFFFFu;  // exact
  if (!VN_FAST_MODE && e->exact_threshold != 0xFFFFFFFFu) {  // (the fast mode is a variant build: histo.h)
    delete e;
    return VN_EINVAL;
  }
#ifdef VN_LONG_REPLAY
  e->long_replay = VN_LONG_REPLAY;  // (A/B build knob: replays of at least this many samples take four waves)
#endif
  e->hot_prefix = std::min(e->exact_threshold, cfg->histo_hot_prefix ? cfg->histo_hot_prefix : 4096u);
  e->piece_growth = cfg->histo_piece_growth ? std::min(cfg->histo_piece_growth, 1000u) : 25u;
  e->temp_cap = temp_buffer_cap(e->cfg.compression);
  e->max_records = cfg->max_batch_records ? cfg->max_batch_records : (1u << 20);
  if (e->max_records > kTagIndex) {  // record indices ride in 30-bit tags
    delete e;
    return VN_EINVAL;
  }
  for (int c = 0; c < VN_NCLASS; c++) {
    e->max_cls[c] = cfg->max_batch_class_records[c] ? cfg->max_batch_class_records[c] : e->max_records;
    if (e->max_cls[c] > e->max_records) {  // a class cap narrows max_batch_records, never widens it
      delete e;
      return VN_EINVAL;
    }
  }
  e->max_member_bytes = cfg->max_batch_member_bytes ? cfg->max_batch_member_bytes : e->max_records * 16;
  if (e->max_member_bytes < e->max_records * 8) e->max_member_bytes = e->max_records * 8;
  int rc = guarded(e, [&] { create_impl(e); });
  if (rc != VN_OK) {
    destroy_impl(e);
    *out = e;  // caller may read vn_last_error, then destroy
    return rc;
  }
  *out = e;
  return VN_OK;
}

void vn_engine_destroy(vn_engine* e) {
  if (!e) return;
  destroy_impl(e);
  delete e;
}

const char* vn_last_error(const vn_engine* e) { return e ? e->err.c_str() : "null engine"; }

int vn_stage_acquire(vn_engine* e, vn_stage* out) {
  if (!e || !out) return VN_EINVAL;
  return guarded(e, [&] {
    ensure_pinned_stage(e);
    *out = e->pstage;
  });
}

int vn_submit(vn_engine* e, const vn_batch_counts* c) {
  if (!e || !c) return VN_EINVAL;
  const vn_stage& p = e->pstage;
  vn_batch b{};
  b.n_counter = c->n_counter; b.counter_slot = p.counter_slot; b.counter_value = p.counter_value;
  b.counter_rate = p.counter_rate;
  b.n_gauge = c->n_gauge; b.gauge_slot = p.gauge_slot; b.gauge_value = p.gauge_value;
  b.n_histo = c->n_histo; b.histo_slot = p.histo_slot; b.histo_value = p.histo_value; b.histo_rate = p.histo_rate;
  b.n_set = c->n_set; b.set_slot = p.set_slot; b.set_member_off = p.set_member_off;
  b.set_member_bytes = p.set_member_bytes;
  return guarded(e, [&] {
    window_open(e, e->st);
    ingest_host(e, &b);
    // the caller refills the engine-owned pinned stage right after this returns: wait until the
    // DMA engine has read it (the kernels keep running)
    VN_HIP_CHECK(hipEventSynchronize(e->ev_h2d));
  });
}

int vn_ingest_host(vn_engine* e, const vn_batch* b) {
  if (!e || !b) return VN_EINVAL;
  return guarded(e, [&] {
    window_open(e, e->st);
    ingest_host(e, b);
  });
}

int vn_ingest(vn_engine* e, const vn_batch* b) {
  if (!e || !b) return VN_EINVAL;
  return guarded(e, [&] {
#ifdef VN_HOST_PROF
    const auto t0 = std::chrono::steady_clock::now();
    for (double& w : e->host_wait_ms) w = 0.0;
#endif
    if (over_class_caps(e, b))
      throw std::invalid_argument("batch larger than max_batch_records");
    validate_device_batch(e, b);
    window_open(e, e->st);
    ingest_device(e, b);
#ifdef VN_HOST_PROF
    const double tot = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "[vn_host] %p validate %.2f group %.2f plan %.2f total %.2f ms\n", (void*)e, e->host_wait_ms[0],
            e->host_wait_ms[1], e->host_wait_ms[2], tot);
#endif
  });
}

int vn_import_counters(vn_engine* e, const uint32_t* slot, const int64_t* value, uint64_t n) {
  if (!e) return VN_EINVAL;
  return guarded(e, [&] {
    if (n > e->max_cls[VN_COUNTER]) throw std::invalid_argument("import batch too large");
    check_slots_host(slot, n, e->cap[VN_COUNTER], "counter");
    ensure_device_stage(e);
    h2d(e->dstage.c_slot, slot, n, e->st);
    h2d(reinterpret_cast<int64_t*>(e->dstage.c_val), value, n, e->st);
    side_begin(e);
    import_counters(e, n, e->dstage.c_slot, reinterpret_cast<const int64_t*>(e->dstage.c_val));
    side_join(e);
    e->imported += n;
  });
}

int vn_import_gauges(vn_engine* e, const uint32_t* slot, const double* value, uint64_t n) {
  if (!e) return VN_EINVAL;
  return guarded(e, [&] {
    if (n > e->max_cls[VN_GAUGE]) throw std::invalid_argument("import batch too large");
    check_slots_host(slot, n, e->cap[VN_GAUGE], "gauge");
    ensure_device_stage(e);
    h2d(e->dstage.g_slot, slot, n, e->st);
    h2d(e->dstage.g_val, value, n, e->st);
    side_begin(e);
    ingest_gauges(e, n, e->dstage.g_slot, e->dstage.g_val);
    side_join(e);
    e->imported += n;
  });
}

int vn_import_histos(vn_engine* e, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes, uint64_t n) {
  if (!e || (n && (!slot || !off || !bytes))) return VN_EINVAL;
  return guarded(e, [&] {
    if (!n) return;
    stage_import(e, slot, off, bytes, n, e->cap[VN_HISTO]);
    import_histos(e, n, e->imp.in_slot, e->imp.in_off, e->imp.in_bytes);
    VN_HIP_CHECK(hipGetLastError());
    e->imported += n;
  });
}

// device-resident payloads: validate slots and offsets on the device
__global__ void k_check_payloads(uint64_t n, const uint32_t* __restrict__ slot, const uint64_t* __restrict__ off,
                                 uint32_t cap, uint32_t* __restrict__ err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (slot[i] >= cap || off[i + 1] < off[i]) atomicOr(err, kErrDecode);
}
void import_device(vn_engine* e, int cls, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes, uint64_t n) {
  if (n > e->max_records || (cls == VN_SET && n > e->max_cls[VN_SET]))
    throw std::invalid_argument("import batch larger than max_batch_records");
  ensure_import(e, n, 0);
  if (cls == VN_HISTO) {
    import_histos(e, n, slot, off, bytes);  // (its count pass validates slots and offsets)
    VN_HIP_CHECK(hipStreamSynchronize(e->st));  // the caller's payload arrays are read when this returns
  } else {
    hipLaunchKernelGGL(k_check_payloads, dim3(blocks_for(n, 256)), dim3(256), 0, e->st, n, slot, off, e->cap[cls],
                       e->h_err);
    VN_HIP_CHECK(hipStreamSynchronize(e->st));
    take_decode_error(e);
    import_sets(e, n, slot, off, bytes);
  }
  VN_HIP_CHECK(hipGetLastError());
  e->imported += n;
}

int vn_import_histos_device(vn_engine* e, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes, uint64_t n) {
  if (!e || (n && (!slot || !off || !bytes))) return VN_EINVAL;
  return guarded(e, [&] { if (n) import_device(e, VN_HISTO, slot, off, bytes, n); });
}

int vn_import_sets_device(vn_engine* e, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes, uint64_t n) {
  if (!e || (n && (!slot || !off || !bytes))) return VN_EINVAL;
  return guarded(e, [&] { if (n) import_device(e, VN_SET, slot, off, bytes, n); });
}

int vn_import_sets(vn_engine* e, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes, uint64_t n) {
  if (!e || (n && (!slot || !off || !bytes))) return VN_EINVAL;
  return guarded(e, [&] {
    if (!n) return;
    if (n > e->max_cls[VN_SET]) throw std::invalid_argument("import batch larger than the set class's record cap");
    stage_import(e, slot, off, bytes, n, e->cap[VN_SET]);
    import_sets(e, n, e->imp.in_slot, e->imp.in_off, e->imp.in_bytes);
    VN_HIP_CHECK(hipGetLastError());
    e->imported += n;
  });
}

int vn_histo_query(vn_engine* e, int kind, const uint32_t* slot, const double* arg, uint64_t n, double* out) {
  if (!e || (kind != 0 && kind != 1) || (n && (!slot || !arg || !out))) return VN_EINVAL;
  return guarded(e, [&] {
    if (!n) return;
    check_slots_host(slot, n, e->cap[VN_HISTO], "histo");
    if (kind == 0)
      for (uint64_t i = 0; i < n; i++)
        if (!(arg[i] >= 0.0 && arg[i] <= 1.0)) throw std::invalid_argument("quantile out of bounds");  // 284-286
    histo_imports_drain(e);
    std::vector<uint32_t> keys(slot, slot + n);
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    uint32_t *dk = nullptr, *ds = nullptr;
    double *da = nullptr, *dout = nullptr;
    dalloc(dk, keys.size());
    dalloc(ds, n);
    dalloc(da, n);
    dalloc(dout, n);
    try {
      h2d(dk, keys.data(), keys.size(), e->st);
      h2d(ds, slot, n, e->st);
      h2d(da, arg, n, e->st);
      histo_merge_pending(e, dk, (uint32_t)keys.size());
      histo_query(e, kind, ds, da, n, dout);
      VN_HIP_CHECK(hipMemcpyAsync(out, dout, n * sizeof(double), hipMemcpyDeviceToHost, e->st));
      VN_HIP_CHECK(hipStreamSynchronize(e->st));
    } catch (...) {
      dfree(dk); dfree(ds); dfree(da); dfree(dout);
      throw;
    }
    dfree(dk); dfree(ds); dfree(da); dfree(dout);
  });
}

int vn_export_histos(vn_engine* e, const uint32_t* slot, uint64_t n, vn_export* out) {
  if (!e || !out || (n && !slot)) return VN_EINVAL;
  return guarded(e, [&] { export_impl(e, VN_HISTO, slot, n, out); });
}

int vn_export_sets(vn_engine* e, const uint32_t* slot, uint64_t n, vn_export* out) {
  if (!e || !out || (n && !slot)) return VN_EINVAL;
  return guarded(e, [&] { export_impl(e, VN_SET, slot, n, out); });
}

int vn_hot_detect(vn_engine* e, uint32_t stride) {
  if (!e) return VN_EINVAL;
  return guarded(e, [&] { hot_enable(e, stride); });
}

int vn_hot_keys(vn_engine* e, int cls, uint64_t min_count, uint32_t cap, uint32_t* slot, uint64_t* count,
                uint32_t* n) {
  if (!e || !n || cls < 0 || cls >= VN_NCLASS || cls == VN_GAUGE) return VN_EINVAL;
  return guarded(e, [&] { *n = hot_collect(e, cls, min_count, cap, slot, count); });
}

int vn_flush(vn_engine* e, vn_flush_result* out) { return vn_flush_masked(e, nullptr, nullptr, out); }

int vn_flush_masked(vn_engine* e, const uint8_t* histo_quantile_mask, const uint8_t* set_estimate_mask,
                    vn_flush_result* out) {
  if (!e || !out) return VN_EINVAL;
  return guarded(e, [&] {
    const auto h0 = std::chrono::steady_clock::now();
    histo_imports_drain(e);
    if (e->w_open) VN_HIP_CHECK(hipEventRecord(e->ev_wmain, e->st));
    if (e->timing) VN_HIP_CHECK(hipEventRecord(e->ev[5], e->st));
    split_flush(e);  // split (hot) keys meet on their owner ranks first
    const auto h1 = std::chrono::steady_clock::now();
    flush_all(e, out, histo_quantile_mask, set_estimate_mask);
    VN_HIP_CHECK(hipGetLastError());
    if (e->timing) VN_HIP_CHECK(hipEventRecord(e->ev[6], e->st));
    hot_rotate(e);  // (first: the detector's window closes on every exit path, a thrown flag included)
    const uint32_t caller = check_error_flags(e);
    if (e->timing) {
      VN_HIP_CHECK(hipEventSynchronize(e->ev[6]));
      vn_timing& t = e->last;
      t = vn_timing{};
      // (a window with no vn_ingest -- imports only -- recorded none of the ingest events)
      auto span = [&](float* o, int a, int b) {
        if ((e->ev_rec >> a & 1u) && (e->ev_rec >> b & 1u)) VN_HIP_CHECK(hipEventElapsedTime(o, e->ev[a], e->ev[b]));
      };
      span(&t.ms_ingest_counter, 0, 1);
      span(&t.ms_ingest_gauge, 1, 2);
      span(&t.ms_ingest_set, 2, 3);
      span(&t.ms_ingest_histo, 3, 4);
      e->ev_rec = 0;
      VN_HIP_CHECK(hipEventElapsedTime(&t.ms_flush, e->ev[5], e->ev[6]));
      t.sort_passes_histo = e->rstat_h.launches;
      t.sort_passes_set = e->rstat_s.launches;
      float tot = 0;
      for (int i = 0; i + 1 < e->pool.used; i += 2) {
        float ms = 0;
        VN_HIP_CHECK(hipEventElapsedTime(&ms, e->pool.ev[i], e->pool.ev[i + 1]));
        tot += ms;
      }
      t.ms_radix_scatter_total = tot;
      t.radix_scatter_launches = e->rstat_h.launches + e->rstat_s.launches;
      t.radix_scatter_bytes = e->rstat_h.bytes + e->rstat_s.bytes;
      auto pool_ms = [](EventPool& p) {
        float tot = 0;
        for (int i = 0; i + 1 < p.used; i += 2) {
          float ms = 0;
          VN_HIP_CHECK(hipEventElapsedTime(&ms, p.ev[i], p.ev[i + 1]));
          tot += ms;
        }
        return tot;
      };
      t.ms_histo_replay = pool_ms(e->pool_rp);
      t.histo_replay_launches = e->kstat_rp.launches;
      t.histo_replay_bytes = e->kstat_rp.bytes;
      t.ms_set_segments = pool_ms(e->pool_ss);
      t.set_segment_launches = e->kstat_ss.launches;
      t.set_segment_bytes = e->kstat_ss.bytes;
      t.ms_part_scatter = pool_ms(e->pool_ps);
      t.ms_import_decode = pool_ms(e->pool_id);
      t.ms_import_drain = pool_ms(e->pool_im);
      e->pool_id.used = e->pool_im.used = 0;
      t.part_scatter_launches = e->rstat_c.launches;
      t.part_scatter_bytes = e->rstat_c.bytes;
    }
    const auto h2 = std::chrono::steady_clock::now();
    e->last.ms_flush_host = std::chrono::duration<float, std::milli>(h2 - h0).count();
    e->last.ms_split_host = std::chrono::duration<float, std::milli>(h1 - h0).count();
    e->last.ms_main_ready = e->last.ms_split_ready = 0.0f;
    e->last.ms_split_histo_ready = e->last.ms_split_set_prefix_ready = 0.0f;
    if (e->w_open) {  // (flush_all synchronised both streams)
      VN_HIP_CHECK(hipEventElapsedTime(&e->last.ms_main_ready, e->ev_w0, e->ev_wmain));
      if (e->sp.ran) {
        VN_HIP_CHECK(hipEventElapsedTime(&e->last.ms_split_ready, e->ev_w0, e->sp.ev_done));
        VN_HIP_CHECK(hipEventElapsedTime(&e->last.ms_split_histo_ready, e->ev_w0, e->sp.ev_histo));
        VN_HIP_CHECK(hipEventElapsedTime(&e->last.ms_split_set_prefix_ready, e->ev_w0, e->sp.ev_set_prefix));
      }
      e->w_open = false;
    }
    e->sp.ran = false;
    out->warn_flags = caller;  // (the window is flushed; the misuse is reported, not thrown)
  });
}

int vn_import_counts(vn_engine* e, uint64_t* out5, int reset) {
  if (!e || !out5) return VN_EINVAL;
  return guarded(e, [&] {
    unsigned long long d[2] = {0, 0};
    if (e->d_imp_counts) {
      VN_HIP_CHECK(hipMemcpyAsync(d, e->d_imp_counts, sizeof d, hipMemcpyDeviceToHost, e->st));
      VN_HIP_CHECK(hipStreamSynchronize(e->st));
    }
    e->imp_counts[3] = d[0];
    e->imp_counts[4] = d[1];
    for (int i = 0; i < 5; i++) out5[i] = e->imp_counts[i];
    if (reset) {
      for (uint64_t& c : e->imp_counts) c = 0;
      if (e->d_imp_counts) VN_HIP_CHECK(hipMemsetAsync(e->d_imp_counts, 0, sizeof d, e->st));
    }
  });
}

int vn_sync(vn_engine* e) {
  if (!e) return VN_EINVAL;
  return guarded(e, [&] {
    histo_imports_drain(e);
    VN_HIP_CHECK(hipStreamSynchronize(e->st));
    throw_caller_errors(check_error_flags(e));
  });
}

int vn_timing_enable(vn_engine* e, int enable) {
  if (!e) return VN_EINVAL;
  return guarded(e, [&] {
    e->timing = enable != 0;
    if (e->timing && !e->ev[0]) {
      for (auto& ev : e->ev) VN_HIP_CHECK(hipEventCreate(&ev));
      e->pool_storage.resize(256);
      for (auto& ev : e->pool_storage) VN_HIP_CHECK(hipEventCreate(&ev));
      e->pool.ev = e->pool_storage.data();
      e->pool.cap = (int)e->pool_storage.size();
      for (auto* ps : {&e->pool_rp_storage, &e->pool_ss_storage, &e->pool_ps_storage}) {
        ps->resize(64);
        for (auto& ev : *ps) VN_HIP_CHECK(hipEventCreate(&ev));
      }
      for (auto* ps : {&e->pool_id_storage, &e->pool_im_storage}) {
        ps->resize(256);
        for (auto& ev : *ps) VN_HIP_CHECK(hipEventCreate(&ev));
      }
      e->pool_id.ev = e->pool_id_storage.data();
      e->pool_id.cap = (int)e->pool_id_storage.size();
      e->pool_im.ev = e->pool_im_storage.data();
      e->pool_im.cap = (int)e->pool_im_storage.size();
      e->pool_rp.ev = e->pool_rp_storage.data();
      e->pool_rp.cap = (int)e->pool_rp_storage.size();
      e->pool_ss.ev = e->pool_ss_storage.data();
      e->pool_ss.cap = (int)e->pool_ss_storage.size();
      e->pool_ps.ev = e->pool_ps_storage.data();
      e->pool_ps.cap = (int)e->pool_ps_storage.size();
    }
  });
}

int vn_get_timing(vn_engine* e, vn_timing* out) {
  if (!e || !out) return VN_EINVAL;
  *out = e->last;
  return VN_OK;
}

int vn_read_histo(vn_engine* e, uint32_t slot, double* means, double* weights, uint32_t cap, uint32_t* n_centroids,
                  double* stats) {
  if (!e || slot >= e->cap[VN_HISTO]) return VN_EINVAL;
  return guarded(e, [&] {
    histo_imports_drain(e);
    VN_HIP_CHECK(hipStreamSynchronize(e->st));
    uint32_t nc = 0;
    uint8_t cur = 0;
    VN_HIP_CHECK(hipMemcpy(&nc, e->hncent + slot, 4, hipMemcpyDeviceToHost));
    VN_HIP_CHECK(hipMemcpy(&cur, e->hcur + slot, 1, hipMemcpyDeviceToHost));
    if (n_centroids) *n_centroids = nc;
    uint32_t m = std::min(nc, cap);
    size_t off = (size_t)slot * e->cap_cent;
    if (means && m) VN_HIP_CHECK(hipMemcpy(means, e->cmean[cur] + off, m * 8, hipMemcpyDeviceToHost));
    if (weights && m) VN_HIP_CHECK(hipMemcpy(weights, e->cw[cur] + off, m * 8, hipMemcpyDeviceToHost));
    if (stats)
      VN_HIP_CHECK(hipMemcpy(stats, e->hst + (size_t)slot * VN_HISTO_STATS, VN_HISTO_STATS * 8, hipMemcpyDeviceToHost));
  });
}

int vn_read_set(vn_engine* e, uint32_t slot, vn_set_state* st, uint32_t* list_codes, uint32_t list_cap,
                uint32_t* tmp_codes, uint32_t tmp_cap, uint8_t* registers) {
  if (!e || slot >= e->cap[VN_SET] || !st) return VN_EINVAL;
  return guarded(e, [&] {
    VN_HIP_CHECK(hipStreamSynchronize(e->st));
    uint32_t touch = 0;
    VN_HIP_CHECK(hipMemcpy(&touch, e->stouch + slot, 4, hipMemcpyDeviceToHost));
    uint8_t mode = 0, b = 0;
    VN_HIP_CHECK(hipMemcpy(&mode, e->smode + slot, 1, hipMemcpyDeviceToHost));
    VN_HIP_CHECK(hipMemcpy(&b, e->sbase + slot, 1, hipMemcpyDeviceToHost));
    st->touched = touch != 0;
    st->sparse = mode == 0;
    st->b = b;
    VN_HIP_CHECK(hipMemcpy(&st->nz, e->snz + slot, 4, hipMemcpyDeviceToHost));
    VN_HIP_CHECK(hipMemcpy(&st->list_count, e->slc + slot, 4, hipMemcpyDeviceToHost));
    VN_HIP_CHECK(hipMemcpy(&st->list_bytes, e->slb + slot, 4, hipMemcpyDeviceToHost));
    VN_HIP_CHECK(hipMemcpy(&st->list_last, e->slast + slot, 4, hipMemcpyDeviceToHost));
    VN_HIP_CHECK(hipMemcpy(&st->tmp_count, e->stc + slot, 4, hipMemcpyDeviceToHost));
    const uint32_t* ar = e->sarena + (size_t)slot * kArenaWords;
    if (mode == 0) {
      uint32_t m = std::min(st->list_count, list_cap);
      if (list_codes && m) VN_HIP_CHECK(hipMemcpy(list_codes, ar, m * 4, hipMemcpyDeviceToHost));
      uint32_t mt = std::min(st->tmp_count, tmp_cap);
      if (tmp_codes && mt)
        VN_HIP_CHECK(hipMemcpy(tmp_codes, e->stmp + (size_t)slot * kTmpCap, mt * 4, hipMemcpyDeviceToHost));
    } else if (registers) {
      VN_HIP_CHECK(hipMemcpy(registers, ar, kHllM, hipMemcpyDeviceToHost));
    }
  });
}

int vn_metro64(int device, const uint8_t* bytes, const uint32_t* off, uint64_t n, uint64_t seed, uint64_t* out) {
  try {
    VN_HIP_CHECK(hipSetDevice(device));
    if (n == 0) return VN_OK;
    uint64_t nb = off[n];
    uint8_t* db = nullptr;
    uint32_t* doff = nullptr;
    uint64_t* dout = nullptr;
    VN_HIP_CHECK(hipMalloc(&db, nb ? nb : 1));
    VN_HIP_CHECK(hipMalloc(&doff, (n + 1) * 4));
    VN_HIP_CHECK(hipMalloc(&dout, n * 8));
    if (nb) VN_HIP_CHECK(hipMemcpy(db, bytes, nb, hipMemcpyHostToDevice));
    VN_HIP_CHECK(hipMemcpy(doff, off, (n + 1) * 4, hipMemcpyHostToDevice));
    metro64_batch(db, doff, n, seed, dout, nullptr);
    VN_HIP_CHECK(hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost));
    (void)hipFree(db);
    (void)hipFree(doff);
    (void)hipFree(dout);
    return VN_OK;
  } catch (const HipError&) {
    return VN_EHIP;
  }
}

int vn_device_alloc(int device, uint64_t bytes, void** out) {
  if (hipSetDevice(device) != hipSuccess) return VN_EHIP;
  return hipMalloc(out, bytes ? bytes : 1) == hipSuccess ? VN_OK : VN_ENOMEM;
}
int vn_device_free(void* p) { return hipFree(p) == hipSuccess ? VN_OK : VN_EHIP; }
int vn_copy_to_device(int device, void* dst, const void* src, uint64_t bytes) {
  if (hipSetDevice(device) != hipSuccess) return VN_EHIP;
  return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? VN_OK : VN_EHIP;
}
int vn_copy_to_host(int device, void* dst, const void* src, uint64_t bytes) {
  if (hipSetDevice(device) != hipSuccess) return VN_EHIP;
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? VN_OK : VN_EHIP;
}
int vn_device_copy(int device, void* dst, const void* src, uint64_t bytes) {
  if (hipSetDevice(device) != hipSuccess) return VN_EHIP;
  // a device-to-device hipMemcpy may return before the copy is done, and the null stream it runs
  // on does not order against the engines' non-blocking streams: the caller may reuse src (an
  // engine's export buffer) or read dst from an engine stream as soon as this returns, so wait
  if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, nullptr) != hipSuccess) return VN_EHIP;
  return hipStreamSynchronize(nullptr) == hipSuccess ? VN_OK : VN_EHIP;
}
int vn_device_count(int* n) { return hipGetDeviceCount(n) == hipSuccess ? VN_OK : VN_EHIP; }
int vn_device_synchronize(int device) {
  if (hipSetDevice(device) != hipSuccess) return VN_EHIP;
  return hipDeviceSynchronize() == hipSuccess ? VN_OK : VN_EHIP;
}

}  // extern "C"

// ingest_set.hip -- Set.Sample -> axiomhq/hyperloglog Sketch.Insert, bit-exact.
//
// Reference (vendor/github.com/axiomhq/hyperloglog/hyperloglog.go):
//   Insert (186-200): x = metro64(member, 1337).  Sparse: tmpSet.add(encodeHash(x)); when
//     len(tmpSet)*100 > m (len >= 164): mergeSparse (229-267: sorted union into the
//     compressed list) and, if the list's varint byte length > m, toNormal (152-166).
//     Dense: insert(getPosVal(x)) (168-183) -- 4-bit registers over a base b; a value that
//     does not fit (uint8(r-b) >= 16) rebases by regs.min(), which is non-zero only once
//     every register is non-zero (nz == 0).
//
// MI355X formulation:
//   k_set_keys   one lane per record: metro64 + encodeHash -> (slot<<32 | code)
//   radix sort   stable by slot: every key's codes contiguous, in arrival order
//   k_set_segments  one workgroup per key touched in the batch, replaying the reference
//     state machine exactly:
//       sparse: the tmpSet is an LDS hash; one lane walks the arrival order to the next
//         164th distinct code (the only order-dependent decision), then the workgroup
//         merges the sorted tmpSet into the LDS copy of the sorted list in parallel and
//         recomputes the varint byte length; > 16384 bytes -> registers built from the list.
//       dense: registers live in LDS (one u32 per register).  Per 4096-record chunk the
//         workgroup finds T_full (the record that fills the last zero register -- first
//         filler per register via LDS atomic max on a marker) and the first rebase candidate
//         after it; records before that point are plain commutative max updates (LDS atomic
//         max), the rebase itself is a parallel min + subtract.  Identical to the
//         sequential semantics, rebase epochs included.
#include "set_dense.h"

namespace vn {

struct SetCtx {
  const uint32_t* cnt;  // touched keys (device count)
  const uint64_t* order;  // slot of the i-th key to merge (low 32 bits), most records first
  const uint32_t* tl;
  const uint32_t* start;
  const uint32_t* end;
  const uint64_t* R;
  uint8_t* mode;
  uint8_t* base;
  uint32_t* nz;
  uint32_t* lc;
  uint32_t* lb;
  uint32_t* last;
  uint32_t* tc;
  uint32_t* tmp;
  uint32_t* arena;
  uint32_t* err;
  uint32_t skip_small;  // keys k_set_small took (sparse, no mergeSparse trigger possible) are skipped
  uint32_t* bt;         // touched flags: k_set_small marks the keys it took with 2
};

// mergeSparse's move: list U[0, lc) shifted up by the new codes inserted below each element
// (s_lbs: the new codes' insertion points, ascending); thread t moves rows [t*jmax, (t+1)*jmax),
// KP >= jmax of them staged in registers before the barrier and written after it
template <int KP>
__device__ __forceinline__ void shift_list_up(uint32_t* U, uint32_t lc, uint32_t nnew, const uint32_t* s_lbs, int jmax,
                                              uint32_t t) {
  const uint32_t i0 = t * (uint32_t)jmax;
  uint32_t keep[KP];
#pragma unroll
  for (int j = 0; j < KP; j++) {
    if (j >= jmax) break;
    const uint32_t i = i0 + (uint32_t)j;
    keep[j] = i < lc ? U[i] : 0u;
  }
  uint32_t r = 0;  // new codes inserted at or before i0
  {
    uint32_t l = 0, h = nnew;
    while (l < h) {
      const uint32_t m = (l + h) >> 1;
      if (s_lbs[m] <= i0) l = m + 1;
      else h = m;
    }
    r = l;
  }
  uint32_t nextlb = r < nnew ? s_lbs[r] : 0xffffffffu;
  lds_barrier();
#pragma unroll
  for (int j = 0; j < KP; j++) {
    if (j >= jmax) break;
    const uint32_t i = i0 + (uint32_t)j;
    if (i < lc) {
      while (nextlb <= i) {
        r++;
        nextlb = r < nnew ? s_lbs[r] : 0xffffffffu;
      }
      U[i + r] = keep[j];
    }
  }
}

// A key that stays sparse and cannot reach a mergeSparse trigger in this batch (tmpSet codes +
// batch records < 164): Insert only adds the batch's new codes to the tmpSet (hyperloglog.go:
// 186-200), in arrival order as k_set_segments stores them.  One wave per key, 2.6 KiB of LDS,
// instead of a 256-thread workgroup holding 70 KiB: the Zipf tail -- half the keys of a C4
// window -- no longer waits for the heavy kernel's two workgroups per CU.
__device__ __forceinline__ bool set_small(uint8_t mode, uint32_t tc, uint32_t n) {
  return mode == 0 && tc + n < kHllTmpTrigger;
}

__global__ __launch_bounds__(256) void k_set_small(SetCtx x) {
  __shared__ uint32_t s_old[4][kHllTmpTrigger];
  __shared__ uint32_t s_rec[4][kHllTmpTrigger];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + w;
  if (i >= *x.cnt) return;
  const uint32_t slot = (uint32_t)x.order[i];
  const uint32_t lo = x.start[slot], n = x.end[slot] - lo;
  const uint32_t tc = x.tc[slot];
  if (!set_small(x.mode[slot], tc, n)) return;
  uint32_t* tmp = x.tmp + (uint64_t)slot * kTmpCap;
  for (uint32_t j = lane; j < tc; j += 64) s_old[w][j] = tmp[j];
  for (uint32_t j = lane; j < n; j += 64) s_rec[w][j] = (uint32_t)x.R[lo + j];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t add = tc;
  for (uint32_t g = 0; g < n; g += 64) {
    const uint32_t p = g + lane;
    bool fresh = false;
    uint32_t c = 0;
    if (p < n) {
      c = s_rec[w][p];
      fresh = true;
      for (uint32_t j = 0; j < tc && fresh; j++) fresh = s_old[w][j] != c;
      for (uint32_t j = 0; j < p && fresh; j++) fresh = s_rec[w][j] != c;
    }
    const uint64_t bal = __ballot(fresh);
    if (fresh) tmp[add + (uint32_t)__popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))))] = c;
    add += (uint32_t)__popcll(bal);
  }
  if (lane == 0) {
    x.tc[slot] = add;
    x.bt[slot] = 2;  // taken: k_set_segments skips it (its tc no longer shows that it was small)
  }
}

__global__ void k_set_keys(uint64_t n, const uint32_t* __restrict__ slot, const uint32_t* __restrict__ off,
                           const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ hashes,
                           uint64_t* __restrict__ R) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = slot[i];
  uint64_t x = hashes ? hashes[i] : metro64(bytes + off[i], off[i + 1] - off[i], kMetroSeed);
  R[i] = ((uint64_t)s << 32) | (uint64_t)encode_hash(x);
}

// after the grouping sort: segment bounds, and each key marked batch- and window-touched once
// (not once per record)
__global__ void k_set_seg_mark(uint64_t n, const uint64_t* __restrict__ R, uint32_t* __restrict__ start,
                               uint32_t* __restrict__ end, uint32_t* __restrict__ bt, uint32_t* __restrict__ stouch) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;  // neighbours' keys from the adjacent lanes
  const uint32_t s = i < n ? (uint32_t)(R[i] >> 32) : 0xFFFFFFFFu;
  uint32_t prev = __shfl_up(s, 1, 64), next = __shfl_down(s, 1, 64);
  if (lane == 0 && i > 0 && i < n) prev = (uint32_t)(R[i - 1] >> 32);
  if (lane == 63 && i + 1 < n) next = (uint32_t)(R[i + 1] >> 32);
  if (i >= n) return;
  if (i == 0 || prev != s) {
    start[s] = (uint32_t)i;
    bt[s] = 1;
    stouch[s] = 1;
  }
  if (i == n - 1 || next != s) end[s] = (uint32_t)(i + 1);
}

#ifdef VN_SET_PROF
// profiling build only (tools/set_profile.py): k_set_segments cycles per phase, summed over
// workgroups: 0 setup, 1 sparse scan, 2 sparse merge, 3 toNormal, 4 dense, 5 write-back,
// 6 triggers, 7 heavy keys, 8 records of heavy keys, 9 whole workgroups
__device__ unsigned long long g_set_prof[32];  // 16 + i: workgroup 0 alone (the key with the most records)
#define SPROF_T(v) const long long v = clock64()
#define SPROF_ADD(i, a, b)                                                                     \
  if (threadIdx.x == 0) {                                                                      \
    atomicAdd(&g_set_prof[i], (unsigned long long)((b) - (a)));                                \
    if (blockIdx.x == 0) atomicAdd(&g_set_prof[16 + (i)], (unsigned long long)((b) - (a)));    \
  }
#define SPROF_INC(i, v) \
  if (threadIdx.x == 0) atomicAdd(&g_set_prof[i], (unsigned long long)(v))
// the longest workgroup's cycles (slot 14) and its record count (15, the latest such key's)
#define SPROF_MAX(a, b, nrec)                                                                  \
  if (threadIdx.x == 0) {                                                                      \
    const unsigned long long _c = (unsigned long long)((b) - (a));                             \
    if (atomicMax(&g_set_prof[14], _c) < _c) g_set_prof[15] = (unsigned long long)(nrec);      \
  }
#else
#define SPROF_MAX(a, b, nrec)
#define SPROF_T(v)
#define SPROF_ADD(i, a, b)
#define SPROF_INC(i, v)
#endif

constexpr uint32_t kScanStage = 1024;  // records staged in LDS per scan window (a trigger needs ~170)
constexpr uint32_t kHashSlots = 512;  // LDS open-addressing table for the tmpSet (<= 163 codes)
#ifndef VN_SET_GROUP
#define VN_SET_GROUP 0
#endif
constexpr bool kSetGroup = VN_SET_GROUP;   // grouped mergeSparse (set_segment)
constexpr uint32_t kSetGroupCap = 1024;    // pending codes of a group: six triggers' tmpSets
// codes per thread per chunk of a key's dense phase (the C4 window's largest set key, 5.3M
// records, is the kernel's critical path); measured: 32 (twice the bytes in flight, half the
// barriers per code) 25.5M cycles for that key against 24.1M with 16 (profiles/r06_t_setprof*)
#ifndef VN_SET_DENSE_ITEMS
#define VN_SET_DENSE_ITEMS 16
#endif
constexpr int kSetDenseItems = VN_SET_DENSE_ITEMS;

__device__ __forceinline__ uint32_t hslot(uint32_t c) { return (c * 2654435761u) >> 23; }  // 9 bits

// lookup (read only)
__device__ __forceinline__ bool hash_contains(const uint32_t* h, uint32_t c) {
  uint32_t i = hslot(c);
  for (;;) {
    uint32_t v = h[i];
    if (v == c) return true;
    if (v == kHllNoCode) return false;
    i = (i + 1) & (kHashSlots - 1);
  }
}
// parallel insert; returns the entry index holding c
__device__ __forceinline__ uint32_t hash_claim(uint32_t* h, uint32_t c) {
  uint32_t i = hslot(c);
  for (;;) {
    uint32_t prev = atomicCAS(&h[i], kHllNoCode, c);
    if (prev == kHllNoCode || prev == c) return i;
    i = (i + 1) & (kHashSlots - 1);
  }
}
// parallel insert of distinct codes
__device__ __forceinline__ void hash_insert_par(uint32_t* h, uint32_t c) {
  uint32_t i = hslot(c);
  for (;;) {
    uint32_t prev = atomicCAS(&h[i], kHllNoCode, c);
    if (prev == kHllNoCode || prev == c) return;
    i = (i + 1) & (kHashSlots - 1);
  }
}

__device__ __forceinline__ void set_segment(const SetCtx& x, const uint32_t slot) {
  __shared__ uint32_t U[kArenaWords];   // sparse list (sorted codes) or dense registers (u32 each)
  __shared__ uint32_t s_hash[kHashSlots];
  __shared__ uint32_t s_first[kHashSlots];  // lowest lane of the current group holding the entry
  __shared__ uint32_t s_tmp[256];       // tmpSet codes in insertion order, then sorted
  __shared__ uint32_t s_new[256];       // tmp codes not yet in the list (sorted)
  __shared__ uint32_t s_lbs[256];       // their insertion points in the old list
  __shared__ uint32_t s_red[4];
  __shared__ uint32_t s_rec[kScanStage];  // the records of the current scan window
  __shared__ uint32_t s_pos, s_trig, s_tc, s_lc, s_mode, s_b, s_nz, s_wbase, s_wend;
  __shared__ uint32_t s_filled, s_tfull, s_pstar, s_newfill, s_min, s_take;

  SPROF_T(p_begin);
  const uint32_t t = threadIdx.x;
  const uint32_t lo = x.start[slot], n = x.end[slot] - lo;
  const uint64_t* R = x.R + lo;
  SPROF_INC(7, 1);
  SPROF_INC(8, n);
  uint32_t* arena = x.arena + (uint64_t)slot * kArenaWords;
  uint8_t* regs8 = reinterpret_cast<uint8_t*>(arena);

  if (t == 0) {
    s_mode = x.mode[slot];
    s_b = x.base[slot];
    s_nz = x.nz[slot];
    s_tc = x.tc[slot];
    s_lc = x.lc[slot];
    s_pos = 0;
    s_wbase = s_wend = 0;  // no window staged
  }
  lds_barrier();
  bool list_in_lds = false, list_dirty = false;
  uint32_t lbytes = x.lb[slot];
  SPROF_T(p_setup);
  SPROF_ADD(0, p_begin, p_setup);

  if (s_mode == 0) {
    // ------------------------------------------------------------ sparse phase
    for (uint32_t i = t; i < kHashSlots; i += kBlock) {
      s_hash[i] = kHllNoCode;
      s_first[i] = 0xffffffffu;
    }
    lds_barrier();
    const uint32_t tc0 = s_tc;
    if (t < tc0) {
      uint32_t c = x.tmp[(uint64_t)slot * kTmpCap + t];
      s_tmp[t] = c;
      hash_insert_par(s_hash, c);
    }
    lds_barrier();
    // Grouped mergeSparse: the list after triggers k..k+g is the list before them united with
    // their tmpSets, and its varint byte length only grows as codes are added, so while the
    // union stays within m no trigger in between reached toNormal -- one merge of the union
    // (sorted and deduplicated) replaces g of them.  The trigger scan is unchanged.  The pending
    // codes and the merge's new codes and insertion points live in the top 2 kSetGroup words of
    // U, above the list and its growth (lc + 3 kSetGroup <= kArenaWords).  A group whose union
    // passes m is scanned again from its first record with one merge per trigger, so toNormal
    // comes at the same record as in the reference.  Measured (C4 window, tools/set_profile.py):
    // see DESIGN.md §5.
    bool gmode = kSetGroup > 0, gfirst = true;
    uint32_t np = 0, gpos = 0, plast = 0;
    uint32_t* const GP = U + kArenaWords - 2 * kSetGroupCap;  // pending codes, then the new ones
    uint32_t* const GL = U + kArenaWords - kSetGroupCap;      // the new codes' insertion points
    auto group_flush = [&]() -> bool {
      if (!list_in_lds) {
        for (uint32_t i = t; i < s_lc; i += kBlock) U[i] = arena[i];
        list_in_lds = true;
        lds_barrier();
      }
      // the pending tmpSets are sorted runs of kHllTmpTrigger distinct codes (sorted as they
      // joined): each code's place in the merged order is its index in its run plus, per other
      // run, the codes below it there (<= for runs before its own, so ties keep run order)
      const uint32_t g = np / kHllTmpTrigger;
      const uint32_t* S = GP;
      if (g > 1) {
        for (uint32_t i = t; i < np; i += kBlock) {
          const uint32_t xc = GP[i], a = i / kHllTmpTrigger;
          uint32_t rank = i - a * kHllTmpTrigger;
          for (uint32_t r = 0; r < g; r++) {
            if (r == a) continue;
            const uint32_t* run = GP + r * kHllTmpTrigger;
            uint32_t lo = 0, hi = kHllTmpTrigger;
            while (lo < hi) {
              const uint32_t m = (lo + hi) >> 1;
              const uint32_t v = run[m];
              if (r < a ? v <= xc : v < xc) lo = m + 1;
              else hi = m;
            }
            rank += lo;
          }
          if (VN_BAD(rank < np, "set group merge rank", rank, np)) continue;
          GL[rank] = xc;
        }
        lds_barrier();
        S = GL;
      }
      // distinct codes not in the list, in order (four adjacent entries per thread)
      const uint32_t lc = s_lc;
      uint32_t code[4], lb[4], cnt = 0;
      bool nw[4];
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t i = 4 * t + q;
        code[q] = i < np ? S[i] : kHllNoCode;
        const bool first = i < np && (i == 0 || S[i - 1] != code[q]);
        lb[q] = first ? lower_bound_u32(U, lc, code[q]) : 0u;
        nw[q] = first && !(lb[q] < lc && U[lb[q]] == code[q]);
        cnt += nw[q] ? 1u : 0u;
      }
      const uint32_t lane = t & 63, w = t >> 6;
      uint32_t inc = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if ((int)lane >= d) inc += o;
      }
      if (lane == 63) s_red[w] = inc;
      lds_barrier();
      uint32_t excl = inc - cnt, nnew = 0;
#pragma unroll
      for (uint32_t i = 0; i < 4; i++) {
        excl += i < w ? s_red[i] : 0u;
        nnew += s_red[i];
      }
      lds_barrier();  // (every pending code read before the new ones overwrite them)
      {
        uint32_t r = excl;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++)
          if (nw[q]) {
            if (VN_BAD(r < kSetGroupCap && lb[q] <= lc, "set group new code", r, lb[q])) continue;
            GP[r] = code[q];
            GL[r] = lb[q];
            r++;
          }
      }
      lds_barrier();
      // the list's varint byte length after the union (as the one-trigger merge below counts it)
      uint32_t dbytes = 0;
      {
        uint32_t r = excl;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++)
          if (nw[q]) {
            const uint32_t c = code[q], l = lb[q];
            const uint32_t predS = l > 0 ? U[l - 1] : 0u, succS = l < lc ? U[l] : 0u;
            const uint32_t predM = (r > 0 && GL[r - 1] == l) ? GP[r - 1] : predS;
            dbytes += varint_len(c - predM);
            const bool last_in_gap = !(r + 1 < nnew && GL[r + 1] == l);
            if (last_in_gap && l < lc) dbytes += varint_len(succS - c) - varint_len(succS - predS);
            r++;
          }
      }
      const uint32_t bytes = lbytes + block_allreduce_u32_sum(dbytes, s_red);
      if (VN_BAD(lc + nnew + 2 * kSetGroupCap <= kArenaWords, "set group list growth", lc + nnew, kArenaWords))
        return false;
      SPROF_INC(10, 1);
      SPROF_INC(11, np);
      if (bytes > kHllM) return false;  // (uniform)
      constexpr int kPer = (kArenaWords + kBlock - 1) / kBlock;
      const int jmax = (int)((lc + kBlock - 1) / kBlock);
      if (jmax <= 8) shift_list_up<8>(U, lc, nnew, GL, jmax, t);
      else shift_list_up<kPer>(U, lc, nnew, GL, jmax, t);
      {
        uint32_t r = excl;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++)
          if (nw[q]) {
            U[lb[q] + r] = code[q];
            r++;
          }
      }
      lds_barrier();
      lbytes = bytes;
      list_dirty = true;
      if (t == 0) s_lc = lc + nnew;
      np = 0;
      gpos = plast;
      gfirst = false;
      lds_barrier();
      return true;
    };
    // the group's union passed m: its triggers again from its first record, one merge each
    auto group_fallback = [&]() {
      SPROF_INC(12, 1);
      gmode = false;
      np = 0;
      for (uint32_t i = t; i < kHashSlots; i += kBlock) {
        s_hash[i] = kHllNoCode;
        s_first[i] = 0xffffffffu;
      }
      lds_barrier();
      if (gfirst && t < tc0) {
        const uint32_t c = x.tmp[(uint64_t)slot * kTmpCap + t];
        s_tmp[t] = c;
        hash_insert_par(s_hash, c);
      }
      if (t == 0) {
        s_pos = gpos;
        s_tc = gfirst ? tc0 : 0u;
        s_wbase = s_wend = 0;  // (the scan window is staged again from there)
      }
      lds_barrier();
    };
    for (;;) {
    while (s_pos < n && s_mode == 0) {
      SPROF_T(p_scan0);
      // the records are staged in LDS kScanStage at a time by the whole workgroup (coalesced);
      // a window serves the scans of several triggers
      if (s_pos >= s_wend) {
        const uint32_t b0 = s_pos, e0 = min(n, b0 + kScanStage);
        for (uint32_t i = t; i < e0 - b0; i += kBlock) s_rec[i] = (uint32_t)R[b0 + i];
        lds_barrier();
        if (t == 0) {
          s_wbase = b0;
          s_wend = e0;
        }
      }
      lds_barrier();
      const uint32_t wbase = s_wbase, wend = s_wend;
#ifdef VN_SET_WAVESCAN  // (A/B build: round 4's scan, wave 0 alone, 64 records per step)
      // wave 0 advances to the next mergeSparse trigger -- the record that makes the tmpSet
      // hold kHllTmpTrigger distinct codes -- 64 records per step: a record counts if its
      // code is neither in the tmpSet nor held by a lower lane of the same step.
      if (t < 64) {
        uint32_t pos = s_pos, tc = s_tc, trig = 0;
        const uint64_t below = (t == 0) ? 0ull : (~0ull >> (64 - t));
        while (pos < wend) {
          const uint32_t p = pos + t;
          const bool valid = p < wend;
          const uint32_t c = valid ? s_rec[p - wbase] : kHllNoCode;
          const bool fresh = valid && !hash_contains(s_hash, c);
          uint32_t hi = 0;
          if (fresh) {
            hi = hash_claim(s_hash, c);
            atomicMin(&s_first[hi], t);
          }
          const bool first = fresh && s_first[hi] == t;
          const uint64_t bal = __ballot(first);
          const uint32_t cnt = (uint32_t)__popcll(bal);
          const uint32_t need = kHllTmpTrigger - tc;
          uint32_t take = 64, add = cnt;
          if (cnt >= need) {  // the need-th first occurrence triggers the merge
            uint64_t b = bal;
            for (uint32_t q = 1; q < need; q++) b &= b - 1;
            const uint32_t L = (uint32_t)__builtin_ctzll(b);
            take = L + 1;
            add = need;
            trig = 1;
          }
          if (first && t < take) s_tmp[tc + (uint32_t)__popcll(bal & below)] = c;
          tc += add;
          pos = min(pos + take, wend);
          if (trig) break;
        }
        if (t == 0) {
          s_pos = pos;
          s_tc = tc;
          s_trig = trig;
        }
      }
#else
      // the workgroup advances kBlock records per step to the next mergeSparse trigger -- the
      // record that makes the tmpSet hold kHllTmpTrigger distinct codes: a record counts if its
      // code is neither in the tmpSet nor held by a lower thread of the same step (the lowest
      // claimer of a new code's hash entry), its rank among the step's counted records a
      // block-wide prefix count
      {
        uint32_t pos = s_pos, tc = s_tc;
        bool trig = false;
        const uint32_t lane = t & 63, w = t >> 6;
        const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        while (pos < wend) {
          const uint32_t p = pos + t;
          const bool valid = p < wend;
          const uint32_t c = valid ? s_rec[p - wbase] : kHllNoCode;
          const bool fresh = valid && !hash_contains(s_hash, c);
          lds_barrier();  // every lookup before any claim of this step
          uint32_t hi = 0;
          if (fresh) {
            hi = hash_claim(s_hash, c);
            atomicMin(&s_first[hi], t);
          }
          lds_barrier();
          const bool first = fresh && s_first[hi] == t;
          const uint64_t bal = __ballot(first);
          if (lane == 0) s_red[w] = (uint32_t)__popcll(bal);
          lds_barrier();
          uint32_t before = 0, cnt = 0;
#pragma unroll
          for (uint32_t i = 0; i < 4; i++) {
            before += i < w ? s_red[i] : 0u;
            cnt += s_red[i];
          }
          const uint32_t rank = before + (uint32_t)__popcll(bal & below);
          const uint32_t need = kHllTmpTrigger - tc;
          if (first && rank < need) s_tmp[tc + rank] = c;
          uint32_t take = kBlock;
          if (cnt >= need) {  // the need-th counted record triggers the merge
            if (first && rank == need - 1) s_take = t + 1;
            trig = true;
          }
          lds_barrier();  // (s_red and s_take are read before the next step writes them)
          if (trig) take = s_take;
          tc += min(cnt, need);
          pos = min(pos + take, wend);
          if (trig) break;
        }
        if (t == 0) {
          s_pos = pos;
          s_tc = tc;
          s_trig = trig ? 1u : 0u;
        }
      }
#endif
      lds_barrier();
      SPROF_T(p_scan1);
      SPROF_ADD(1, p_scan0, p_scan1);
      if (!s_trig) continue;  // window done without a trigger: the next window, or the end
      SPROF_INC(6, 1);
      if (gmode) {
        if (np + kHllTmpTrigger > kSetGroupCap) {
          SPROF_T(p_g0);
          const bool ok = group_flush();
          SPROF_T(p_g1);
          SPROF_ADD(2, p_g0, p_g1);
          if (!ok) {
            group_fallback();
            continue;
          }
        }
        if (s_lc + 3 * kSetGroupCap <= kArenaWords) {  // this trigger's tmpSet joins the group
          if (t < kHllTmpTrigger) {  // (sorted by rank: the tmpSet's codes are distinct)
            const uint32_t mine = s_tmp[t];
            uint32_t rk = 0;
            for (uint32_t j = 0; j < kHllTmpTrigger; j++) rk += s_tmp[j] < mine ? 1u : 0u;
            if (!VN_BAD(np + rk < kSetGroupCap, "set group append", np + rk, kSetGroupCap)) GP[np + rk] = mine;
          }
          np += kHllTmpTrigger;
          plast = s_pos;
          if (t == 0) s_tc = 0;
          for (uint32_t i = t; i < kHashSlots; i += kBlock) {
            s_hash[i] = kHllNoCode;
            s_first[i] = 0xffffffffu;
          }
          lds_barrier();
          continue;
        }
        // (the list leaves no room for a group: this trigger merges alone, as every later one)
        gmode = false;
      }
      // mergeSparse: sorted union of the list and the tmpSet
      SPROF_INC(13, 1);
      if (!list_in_lds) {
        for (uint32_t i = t; i < s_lc; i += kBlock) U[i] = arena[i];
        list_in_lds = true;
      }
      // the full tmpSet (kHllTmpTrigger distinct codes) sorted by rank: one pass, two barriers
      {
        uint32_t mine = 0, rk = 0;
        if (t < kHllTmpTrigger) {
          mine = s_tmp[t];
          for (uint32_t j = 0; j < kHllTmpTrigger; j++) rk += s_tmp[j] < mine ? 1u : 0u;
        }
        lds_barrier();
        if (t < kHllTmpTrigger) s_tmp[rk] = mine;
      }
      lds_barrier();
      const uint32_t lc = s_lc;
      uint32_t isnew = 0, lb = 0, code = 0;
      if (t < kHllTmpTrigger) {
        code = s_tmp[t];
        lb = lower_bound_u32(U, lc, code);
        isnew = !(lb < lc && U[lb] == code);
      }
      // exclusive rank among new codes (ascending)
      uint64_t bal = __ballot(isnew);
      const int lane = t & 63, w = t >> 6;
      if (lane == 0) s_red[w] = (uint32_t)__popcll(bal);
      lds_barrier();
      uint32_t before = 0;
      for (int i = 0; i < w; i++) before += s_red[i];
      const uint32_t nnew = s_red[0] + s_red[1] + s_red[2] + s_red[3];
      uint32_t rank = before + (uint32_t)__popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
      // the list around each new code (before anything moves): its neighbours in the old list
      const uint32_t predS = (isnew && lb > 0) ? U[lb - 1] : 0u;
      const uint32_t succS = (isnew && lb < lc) ? U[lb] : 0u;
      if (isnew) {
        s_new[rank] = code;
        s_lbs[rank] = lb;
      }
      lds_barrier();
      // varint byte length of the delta-encoded list, updated around the insertions: a new code
      // adds its delta from its predecessor in the merged list, and the last new code of a gap
      // changes the delta of the old element after it (the first delta is from 0)
      uint32_t dbytes = 0;
      if (isnew) {
        const bool prev_same = rank > 0 && s_lbs[rank - 1] == lb;
        const uint32_t predM = prev_same ? s_new[rank - 1] : predS;
        dbytes = varint_len(code - predM);
        const bool last_in_gap = !(rank + 1 < nnew && s_lbs[rank + 1] == lb);
        if (last_in_gap && lb < lc) dbytes += varint_len(succS - code) - varint_len(succS - predS);
      }
      // move list elements up by the number of new codes below them: thread t moves the
      // contiguous rows [t*jmax, (t+1)*jmax), walking the insertion points alongside (staged in
      // registers: 8 rows per thread while the list holds at most 2048 codes -- the 65-row staging
      // of a full list lives partly in scratch)
      constexpr int kPer = (kArenaWords + kBlock - 1) / kBlock;
      const int jmax = (int)((lc + kBlock - 1) / kBlock);  // list elements per thread (uniform)
      if (jmax <= 8) shift_list_up<8>(U, lc, nnew, s_lbs, jmax, t);
      else shift_list_up<kPer>(U, lc, nnew, s_lbs, jmax, t);
      if (isnew) U[lb + rank] = code;
      lds_barrier();
      const uint32_t nlc = lc + nnew;
      const uint32_t bytes = lbytes + block_allreduce_u32_sum(dbytes, s_red);
      lbytes = bytes;
      list_dirty = true;
      if (t == 0) {
        s_lc = nlc;
        s_tc = 0;
      }
      for (uint32_t i = t; i < kHashSlots; i += kBlock) {
        s_hash[i] = kHllNoCode;
        s_first[i] = 0xffffffffu;
      }
      lds_barrier();
      SPROF_T(p_merge1);
      SPROF_ADD(2, p_scan1, p_merge1);
      if (bytes > kHllM) {
        // toNormal: registers from the merged list (b stays; nz > 0 so no rebase can occur)
        uint32_t keep[kPer];
#pragma unroll
        for (int j = 0; j < kPer; j++) {
          uint32_t i = t + j * kBlock;
          keep[j] = i < nlc ? U[i] : kHllNoCode;
        }
        lds_barrier();
        for (uint32_t i = t; i < kHllM; i += kBlock) U[i] = 0;
        lds_barrier();
        const uint32_t b = s_b;
#pragma unroll
        for (int j = 0; j < kPer; j++) {
          if (keep[j] != kHllNoCode) {
            uint32_t ri, r;
            decode_hash(keep[j], &ri, &r);
            if (r > b) atomicMax(&U[ri], min(r - b, kHllCapacity - 1));
          }
        }
        lds_barrier();
        uint32_t z = 0;
        for (uint32_t i = t; i < kHllM; i += kBlock) z += U[i] == 0;
        z = block_allreduce_u32_sum(z, s_red);
        if (t == 0) {
          s_nz = z;
          s_mode = 1;
        }
        list_in_lds = false;
        list_dirty = false;
        lds_barrier();
        SPROF_T(p_norm1);
        SPROF_ADD(3, p_merge1, p_norm1);
      }
    }
    lds_barrier();
    if (gmode && np > 0) {  // the triggers pending at the key's last record
      SPROF_T(p_g0);
      const bool ok = group_flush();
      SPROF_T(p_g1);
      SPROF_ADD(2, p_g0, p_g1);
      if (!ok) {
        group_fallback();
        continue;
      }
    }
    break;
    }
    if (s_mode == 0) {
      // write back the sparse state
      SPROF_T(p_wb0);
      const uint32_t tc = s_tc;
      if (t < tc) x.tmp[(uint64_t)slot * kTmpCap + t] = s_tmp[t];
      if (list_dirty)
        for (uint32_t i = t; i < s_lc; i += kBlock) arena[i] = U[i];
      if (t == 0) {
        x.tc[slot] = tc;
        x.lc[slot] = s_lc;
        x.lb[slot] = lbytes;
        if (list_dirty && s_lc) x.last[slot] = U[s_lc - 1];
      }
      SPROF_T(p_wb1);
      SPROF_ADD(5, p_wb0, p_wb1);
      SPROF_ADD(9, p_begin, p_wb1);
      SPROF_MAX(p_begin, p_wb1, n);
      return;
    }
  } else {
    // ------------------------------------------------------------ dense: registers to LDS
    for (uint32_t i = t; i < kHllM; i += kBlock) U[i] = regs8[i];
    lds_barrier();
  }

  // -------------------------------------------------------------- dense phase
  SPROF_T(p_dense0);
  {
    const DenseLds S{U, &s_b, &s_nz, &s_filled, &s_tfull, &s_pstar, &s_newfill, &s_min, s_red};
    dense_insert_codes<kSetDenseItems>(S, [R](uint32_t p) { return (uint32_t)R[p]; }, s_pos, n, x.err);
  }
  lds_barrier();
  SPROF_T(p_dense1);
  SPROF_ADD(4, p_dense0, p_dense1);
  for (uint32_t i = t; i < kHllM; i += kBlock) regs8[i] = (uint8_t)U[i];
  if (t == 0) {
    x.mode[slot] = 1;
    x.base[slot] = (uint8_t)s_b;
    x.nz[slot] = s_nz;
    x.tc[slot] = 0;
    x.lc[slot] = 0;
    x.lb[slot] = 0;
  }
  SPROF_T(p_end);
  SPROF_ADD(5, p_dense1, p_end);
  SPROF_ADD(9, p_begin, p_end);
  SPROF_MAX(p_begin, p_end, n);
}

// One workgroup per touched key; with an order, workgroup i takes the key with the i-th most
// records (longest-processing-time first: the biggest keys do not start last).
__global__ __launch_bounds__(kBlock) void k_set_segments(SetCtx x) {
  const uint32_t i = blockIdx.x;
  if (i >= *x.cnt) return;
  const uint32_t slot = x.order ? (uint32_t)x.order[i] : x.tl[i];
  if (x.skip_small && x.bt[slot] == 2) return;
  set_segment(x, slot);
}

// longest-first order: key = (0xFFFFF - min(records, 0xFFFFF)) << 32 | slot; untouched -> ~0
__global__ void k_set_lpt_keys(uint32_t n, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ tl,
                               const uint32_t* __restrict__ start, const uint32_t* __restrict__ end,
                               uint64_t* __restrict__ out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  if (k >= *cnt) {
    out[k] = ~0ull;
    return;
  }
  const uint32_t s = tl[k], c = min(end[s] - start[s], 0xFFFFFu);
  out[k] = ((uint64_t)(0xFFFFFu - c) << 32) | s;
}

__global__ void k_set_clear_flags(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ list,
                                  uint32_t* __restrict__ flags) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < *cnt) flags[list[k]] = 0;
}

void ingest_sets(vn_engine* e, uint64_t n, const uint32_t* slot, const uint32_t* off, const uint8_t* bytes,
                 const uint64_t* hashes) {
  if (!n) return;
  hipStream_t st = e->side;
  const uint32_t caps = e->cap[VN_SET];
  hipLaunchKernelGGL(k_set_keys, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, slot, off, bytes, hashes, e->sR0);
  RadixPass passes[4];
  int np = 0;
  np = make_passes(passes, false, 32, e->slot_bits[VN_SET]);
  bool fl = radix_sort(e->sR0, nullptr, e->sR1, nullptr, n, passes, np, *e->side_rs, st,
                       e->timing ? &e->rstat_s : nullptr);
  const uint64_t* R = fl ? e->sR1 : e->sR0;
  hipLaunchKernelGGL(k_set_seg_mark, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, R, e->s_start, e->s_end, e->s_bt,
                     e->stouch);
  compact_flags(e->s_bt, e->s_pos, e->s_tl, e->s_cnt, caps, *e->side_ss, st);
  // no host round trip: the touched-key count stays on the device and the grid is its upper
  // bound, so the whole set path is queued before the histogram path blocks the host
  const uint32_t nk = (uint32_t)std::min<uint64_t>(caps, n);  // >= touched keys
  const uint64_t* order = nullptr;  // most records first (longest-processing-time order)
  {  // ordered now, before the replays fill the CUs; only the merge is deferred
    hipLaunchKernelGGL(k_set_lpt_keys, dim3(blocks_for(nk, 256)), dim3(256), 0, st, nk, e->s_cnt, e->s_tl, e->s_start,
                       e->s_end, e->s_lpt0);
    RadixPass lp[4];
    const int nlp = make_passes(lp, false, 32, 20);
    order = radix_sort(e->s_lpt0, nullptr, e->s_lpt1, nullptr, nk, lp, nlp, *e->side_rs, st, nullptr) ? e->s_lpt1
                                                                                                     : e->s_lpt0;
  }
  e->set_pending = true;
  e->set_pending_n = n;
  e->set_pending_R = R;
  e->set_pending_order = order;
  if (!e->set_defer) set_finish(e);
}

// The exact Sketch.Insert replay of k_set_segments over arbitrary per-slot record ranges:
// R holds (slot << 32 | sparse code) records, key list[k] (k < *dev_count <= grid) covers
// R[e->s_start[slot], e->s_end[slot]) in insertion order (split.hip: a split set's gathered
// first records).
void set_replay_ranges(vn_engine* e, const uint64_t* R, const uint32_t* dev_count, const uint32_t* list,
                       uint32_t grid, hipStream_t st) {
  if (!grid) return;
  SetCtx x;
  x.cnt = dev_count;
  x.order = nullptr;
  x.tl = list;
  x.start = e->s_start;
  x.end = e->s_end;
  x.R = R;
  x.mode = e->smode;
  x.base = e->sbase;
  x.nz = e->snz;
  x.lc = e->slc;
  x.lb = e->slb;
  x.last = e->slast;
  x.tc = e->stc;
  x.tmp = e->stmp;
  x.arena = e->sarena;
  x.err = e->h_err;
  x.skip_small = 0;
  x.bt = nullptr;
  hipLaunchKernelGGL(k_set_segments, dim3(grid), dim3(kBlock), 0, st, x);
}

void set_finish(vn_engine* e) {
  if (!e->set_pending) return;
  e->set_pending = false;
  hipStream_t st = e->side;
  const uint32_t nk = (uint32_t)std::min<uint64_t>(e->cap[VN_SET], e->set_pending_n);  // >= touched keys
  const uint64_t* order = e->set_pending_order;
  const uint32_t grid = nk;  // >= touched keys
  SetCtx x;
  x.cnt = e->s_cnt;
  x.order = order;
  x.tl = e->s_tl;
  x.start = e->s_start;
  x.end = e->s_end;
  x.R = e->set_pending_R;
  x.mode = e->smode;
  x.base = e->sbase;
  x.nz = e->snz;
  x.lc = e->slc;
  x.lb = e->slb;
  x.last = e->slast;
  x.tc = e->stc;
  x.tmp = e->stmp;
  x.arena = e->sarena;
  x.err = e->h_err;
  x.skip_small = order ? 1u : 0u;
  x.bt = e->s_bt;
  hipEvent_t ea = e->timing ? e->pool_ss.next() : nullptr, eb = e->timing ? e->pool_ss.next() : nullptr;
  if (ea && eb) VN_HIP_CHECK(hipEventRecord(ea, st));
  // the small keys (the tail of the longest-first order) take one wave each; the heavy kernel,
  // queued behind, skips them -- both kernels only read the state that decides which runs a key
  if (order) hipLaunchKernelGGL(k_set_small, dim3(blocks_for(grid, 4)), dim3(256), 0, st, x);
  hipLaunchKernelGGL(k_set_segments, dim3(grid), dim3(kBlock), 0, st, x);
  if (ea && eb) VN_HIP_CHECK(hipEventRecord(eb, st));
  if (e->timing) {
    e->kstat_ss.launches++;
    e->kstat_ss.bytes += 8ull * e->set_pending_n;
  }
  hipLaunchKernelGGL(k_set_clear_flags, dim3(blocks_for(nk, 256)), dim3(256), 0, st, e->s_cnt, e->s_tl, e->s_bt);
}

#ifdef VN_SET_PROF
extern "C" int vn_prof_set_read(unsigned long long* out40, int reset) {
  if (hipMemcpyFromSymbol(out40, HIP_SYMBOL(g_set_prof), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out40 + 32, HIP_SYMBOL(g_dense_prof), sizeof(unsigned long long) * 8) != hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_set_prof), z, sizeof z) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dense_prof), z, sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  }
  return 0;
}
#endif
}  // namespace vn

// Device intake: DogStatsD datagram lines in HBM -> Worker.ProcessMetric on the GPU.
//
// What server.go:693-722 (ReadMetricSocket -> HandleMetricPacket -> ParseMetric) and
// worker.go:187-227 (ProcessMetric: Upsert the MetricKey into one of the ten type x scope maps of
// worker.go:81-138, then Sample) do per line, done for a whole buffer:
//   1. vn_parse_dogstatsd_device (parse_device.hip): one parsed record per non-empty line;
//   2. k_in_class: the Upsert map of each line that parses (worker.go:81-138: counters/gauges with
//      veneurglobalonly -> global maps, histograms/timers/sets with veneurlocalonly -> local
//      maps); histogram/timer lines whose sample rate is NaN are dropped (the parser lets NaN
//      through, parser.go:265; Go's digest would never finish its next merge, DESIGN.md §4 -- the
//      host Worker drops them too); a counter's NaN rate is sampled as Go does (MinInt64 factor);
//   3. the window's key table, a device hash table MetricKey -> slot with linear probing:
//      k_in_probe finds resident keys; k_in_claim makes each missing key one pending entry by
//      compare-and-swap (lines that find a pending entry compare their key with the pending line's
//      own bytes -- no lane ever waits on another) and keeps the first line of every new key
//      (atomicMin); k_in_commit gives every new key the next slot of its class in line order (the
//      order Upsert sees them), stores its bytes in the key arena and makes the entry resident;
//   4. k_in_emit: the records of each class in line order -- the staged batch of ProcessMetric
//      calls -- and one vn_ingest.
// One host round trip per buffer (the line count inside the parse, then the new-key / record counts
// that size the commit and the ingest).  vn_intake_upsert runs step 3 for keys the host hands in
// (ImportMetric's Upsert, worker.go:230-268), so both paths share one slot table; vn_intake_keys
// gives the host the window's keys for Flush (InterMetric names and tags).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "engine.h"
#include "primitives.h"

namespace vn {
namespace {

constexpr uint32_t kMiss = 0xffffffffu;
constexpr uint32_t kResident = 0x80000000u;  // tstate: resident | key index; else 1 + pending line; 0 empty
constexpr uint8_t kNoMap = 0xff;
__constant__ uint8_t c_map_class[10] = {0, 0, 1, 1, 2, 2, 2, 2, 3, 3};

// Upsert's map (worker.go:81-138); type: counter gauge histogram timer set, scope: mixed local global
__device__ __forceinline__ uint8_t map_for(uint8_t type, uint8_t scope) {
  switch (type) {
    case 0: return scope == 2 ? 1 : 0;
    case 1: return scope == 2 ? 3 : 2;
    case 2: return scope == 1 ? 5 : 4;
    case 3: return scope == 1 ? 7 : 6;
    case 4: return scope == 1 ? 9 : 8;
  }
  return kNoMap;
}

__device__ __forceinline__ uint32_t key_hash(uint32_t digest, uint8_t map) {
  uint32_t h = digest ^ (0x9E3779B9u * (uint32_t)(map + 1));
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// A batch of keys to upsert (SoA): bytes of the name at name_base + name_off, joined tags at
// tags_base + tags_off.
struct KeyBatch {
  uint32_t n;
  const uint8_t* name_base;
  const uint8_t* tags_base;
  uint8_t* map;        // kNoMap: skip
  uint32_t* name_off;
  uint32_t* name_len;
  uint32_t* tags_off;
  uint32_t* tags_len;
  uint32_t* n_tags;
  uint32_t* digest;
};

struct Table {
  uint32_t mask;
  uint32_t* state;
  uint32_t* first;
  // resident keys, by key index
  uint8_t* kmap;
  uint32_t* kslot;
  uint32_t* kntags;
  uint32_t* kdigest;
  uint32_t* kname_len;
  uint32_t* ktags_len;
  uint64_t* kname_off;  // arena offset; the tags follow the name
  uint8_t* arena;
};

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}

__device__ __forceinline__ bool eq_resident(const KeyBatch& kb, uint32_t i, const Table& t, uint32_t kid) {
  if (t.kmap[kid] != kb.map[i] || t.kdigest[kid] != kb.digest[i] || t.kname_len[kid] != kb.name_len[i] ||
      t.ktags_len[kid] != kb.tags_len[i])
    return false;
  const uint8_t* a = t.arena + t.kname_off[kid];
  return bytes_eq(a, kb.name_base + kb.name_off[i], kb.name_len[i]) &&
         bytes_eq(a + kb.name_len[i], kb.tags_base + kb.tags_off[i], kb.tags_len[i]);
}

__device__ __forceinline__ bool eq_lines(const KeyBatch& kb, uint32_t i, uint32_t j) {
  if (kb.map[i] != kb.map[j] || kb.digest[i] != kb.digest[j] || kb.name_len[i] != kb.name_len[j] ||
      kb.tags_len[i] != kb.tags_len[j])
    return false;
  return bytes_eq(kb.name_base + kb.name_off[i], kb.name_base + kb.name_off[j], kb.name_len[i]) &&
         bytes_eq(kb.tags_base + kb.tags_off[i], kb.tags_base + kb.tags_off[j], kb.tags_len[i]);
}

// parsed lines -> key batch + the valid-record flags (class-major: vflag[c * n + i])
__global__ __launch_bounds__(256) void k_in_class(const vn_parsed_line* __restrict__ lines, uint32_t n, KeyBatch kb,
                                                  uint32_t* __restrict__ vflag, uint32_t* __restrict__ mlen,
                                                  uint32_t* __restrict__ dropped) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const vn_parsed_line o = lines[i];
  uint8_t m = kNoMap;
  if (o.status == VN_PARSE_OK) {
    m = map_for(o.type, o.scope);
    const uint8_t c = c_map_class[m];
    if (c == 2 && o.rate != o.rate) {  // a histogram/timer with a NaN sample rate
      m = kNoMap;
      atomicAdd(dropped, 1u);
    }
  }
  kb.map[i] = m;
  kb.name_off[i] = (uint32_t)o.name_off;
  kb.name_len[i] = o.name_len;
  kb.tags_off[i] = (uint32_t)o.tags_off;
  kb.tags_len[i] = o.tags_len;
  kb.n_tags[i] = o.n_tags;
  kb.digest[i] = o.digest;
  const uint8_t c = m == kNoMap ? 4 : c_map_class[m];
#pragma unroll
  for (int k = 0; k < 4; k++) vflag[k * n + i] = (c == k) ? 1u : 0u;
  mlen[i] = c == 3 ? o.value_len : 0u;  // set members: the value chunk's bytes
}

__global__ __launch_bounds__(256) void k_in_probe(KeyBatch kb, Table t, uint32_t* __restrict__ kid_out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kb.n) return;
  uint32_t r = kMiss;
  if (kb.map[i] != kNoMap) {
    uint32_t h = key_hash(kb.digest[i], kb.map[i]) & t.mask;
    for (uint32_t step = 0; step <= t.mask; step++, h = (h + 1) & t.mask) {
      const uint32_t s = t.state[h];
      if (s == 0) break;
      if ((s & kResident) && eq_resident(kb, i, t, s & ~kResident)) {
        r = s & ~kResident;
        break;
      }
    }
  }
  kid_out[i] = r;
}

// missing keys: claim an empty entry (pending = 1 + line) or join the pending entry of an equal key
__global__ __launch_bounds__(256) void k_in_claim(KeyBatch kb, Table t, const uint32_t* __restrict__ kid,
                                                  uint32_t* __restrict__ ent, uint32_t* __restrict__ err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kb.n) return;
  ent[i] = kMiss;
  if (kb.map[i] == kNoMap || kid[i] != kMiss) return;
  uint32_t h = key_hash(kb.digest[i], kb.map[i]) & t.mask;
  for (uint32_t step = 0; step <= t.mask; step++) {
    uint32_t s = t.state[h];
    if (s == 0) {
      const uint32_t prev = atomicCAS(&t.state[h], 0u, 1u + i);
      if (prev == 0) {
        atomicMin(&t.first[h], i);
        ent[i] = h;
        return;
      }
      s = prev;  // someone else took it: look at what they put there
    }
    if (!(s & kResident) && eq_lines(kb, i, s - 1u)) {
      atomicMin(&t.first[h], i);
      ent[i] = h;
      return;
    }
    h = (h + 1) & t.mask;
  }
  atomicOr(err, 1u);  // table full (cannot happen: it holds twice the slots)
}

// new-key flags (class-major) and the key bytes of each new key's first line
__global__ __launch_bounds__(256) void k_in_newflags(KeyBatch kb, Table t, const uint32_t* __restrict__ ent,
                                                     uint32_t* __restrict__ nflag, uint32_t* __restrict__ nbytes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kb.n) return;
  const uint32_t h = ent[i];
  const bool first = h != kMiss && t.first[h] == i;
  const uint8_t c = first ? c_map_class[kb.map[i]] : 4;
#pragma unroll
  for (int k = 0; k < 4; k++) nflag[k * kb.n + i] = (c == k) ? 1u : 0u;
  nbytes[i] = first ? kb.name_len[i] + kb.tags_len[i] : 0u;
}

// a batch that does not fit the capacity: every pending entry back to empty
__global__ __launch_bounds__(256) void k_in_revert(KeyBatch kb, Table t, const uint32_t* __restrict__ ent) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kb.n) return;
  const uint32_t h = ent[i];
  if (h != kMiss && t.first[h] == i) {
    t.state[h] = 0u;
    t.first[h] = kMiss;
  }
}

struct CommitCtx {
  uint32_t nk0;             // keys before this batch
  uint32_t next_slot[4];    // per class, before this batch
  uint64_t arena0;          // arena bytes before this batch
};

__global__ __launch_bounds__(256) void k_in_commit(KeyBatch kb, Table t, const uint32_t* __restrict__ ent,
                                                   const uint32_t* __restrict__ nscan,
                                                   const uint32_t* __restrict__ bscan, CommitCtx cc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kb.n) return;
  const uint32_t h = ent[i];
  if (h == kMiss || t.first[h] != i) return;
  const uint8_t m = kb.map[i];
  const uint8_t c = c_map_class[m];
  const uint32_t rank_all = nscan[c * kb.n + i];        // class-major: new keys of lower classes first
  const uint32_t rank_c = rank_all - nscan[c * kb.n];   // among this class's new keys, in line order
  const uint32_t k = cc.nk0 + rank_all;
  const uint64_t a = cc.arena0 + bscan[i];
  t.kmap[k] = m;
  t.kslot[k] = cc.next_slot[c] + rank_c;
  t.kntags[k] = kb.n_tags[i];
  t.kdigest[k] = kb.digest[i];
  t.kname_len[k] = kb.name_len[i];
  t.ktags_len[k] = kb.tags_len[i];
  t.kname_off[k] = a;
  const uint8_t* nm = kb.name_base + kb.name_off[i];
  for (uint32_t b = 0; b < kb.name_len[i]; b++) t.arena[a + b] = nm[b];
  const uint8_t* tg = kb.tags_base + kb.tags_off[i];
  for (uint32_t b = 0; b < kb.tags_len[i]; b++) t.arena[a + kb.name_len[i] + b] = tg[b];
  t.first[h] = kMiss;
  __threadfence();
  t.state[h] = kResident | k;
}

// every upserted key's slot (resident from the probe, or committed by this batch)
__global__ __launch_bounds__(256) void k_in_slots(KeyBatch kb, Table t, const uint32_t* __restrict__ kid,
                                                  const uint32_t* __restrict__ ent, uint32_t* __restrict__ slot) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kb.n) return;
  uint32_t k = kid[i];
  if (k == kMiss && ent[i] != kMiss) k = t.state[ent[i]] & ~kResident;
  slot[i] = k == kMiss ? kMiss : t.kslot[k];
}

struct Staged {
  uint32_t* slot;   // class segments [base[c], base[c] + n[c]) in line order
  double* value;
  float* rate;
  uint32_t* moff;   // set member offsets, by set rank (+ the total at n_set)
  uint8_t* mbytes;
};

__global__ __launch_bounds__(256) void k_in_emit(const vn_parsed_line* __restrict__ lines, KeyBatch kb,
                                                 const uint32_t* __restrict__ slot, const uint32_t* __restrict__ vscan,
                                                 const uint32_t* __restrict__ mscan, const uint8_t* __restrict__ buf,
                                                 Staged s) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kb.n) return;
  const uint8_t m = kb.map[i];
  if (m == kNoMap) return;
  const uint8_t c = c_map_class[m];
  const uint32_t pos = vscan[c * kb.n + i];  // class-major rank: the class segment's base is built in
  const vn_parsed_line& o = lines[i];
  s.slot[pos] = slot[i];
  if (c == 3) {
    const uint32_t r = pos - vscan[3 * kb.n];
    const uint32_t mo = mscan[i];
    s.moff[r] = mo;
    const uint8_t* src = buf + (uint32_t)o.value_off;
    for (uint32_t b = 0; b < o.value_len; b++) s.mbytes[mo + b] = src[b];
  } else {
    s.value[pos] = o.value;
    s.rate[pos] = o.rate;
  }
}

template <class T>
void dalloc(T*& p, uint64_t n) {
  VN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p), std::max<uint64_t>(n, 1) * sizeof(T)));
}

}  // namespace
}  // namespace vn

using namespace vn;

struct vn_intake {
  vn_engine* eng = nullptr;
  vn_parser* parser = nullptr;
  uint64_t max_bytes = 0, max_lines = 0;
  uint32_t cap[4] = {0, 0, 0, 0};
  // the window's key table
  Table t{};
  uint64_t nkeys_cap = 0, arena_cap = 0;
  uint32_t nkeys = 0;
  uint64_t arena_top = 0;
  uint32_t next_slot[4] = {0, 0, 0, 0};
  // per call
  vn_parsed_line* lines = nullptr;
  uint8_t* tags = nullptr;
  uint8_t* ubytes = nullptr;   // vn_intake_upsert: the host keys' bytes
  uint64_t ubytes_cap = 0;
  KeyBatch kb{};
  uint32_t *kid = nullptr, *ent = nullptr, *slot = nullptr;
  uint32_t *vflag = nullptr, *vscan = nullptr, *nflag = nullptr, *nscan = nullptr;
  uint32_t *nbytes = nullptr, *bscan = nullptr, *mlen = nullptr, *mscan = nullptr;
  uint32_t* dcnt = nullptr;    // [0] dropped, [1] table-full flag
  uint32_t* h_cnt = nullptr;   // pinned read-back
  Staged s{};
  ScanScratch scan;
  vn_intake_stats last{};
  std::string err;
};

namespace {

int in_fail(vn_intake* in, int code, const std::string& msg) {
  in->err = msg;
  return code;
}

template <class F>
int in_guard(vn_intake* in, F&& f) {
  try {
    f();
    return VN_OK;
  } catch (const HipError& h) {
    return in_fail(in, VN_EHIP, std::string(hipGetErrorString(h.err)) + " at " + h.file + ":" +
                                    std::to_string(h.line));
  } catch (const std::invalid_argument& x) {
    return in_fail(in, VN_EINVAL, x.what());
  } catch (const std::bad_alloc&) {
    return in_fail(in, VN_ENOMEM, "out of memory");
  } catch (const std::exception& x) {
    return in_fail(in, VN_EINVAL, x.what());
  }
}

void ensure_arena(vn_intake* in, uint64_t need, hipStream_t st) {
  if (need <= in->arena_cap) return;
  uint64_t cap = std::max<uint64_t>(need, in->arena_cap * 2);
  uint8_t* a = nullptr;
  dalloc(a, cap);
  if (in->arena_top) VN_HIP_CHECK(hipMemcpyAsync(a, in->t.arena, in->arena_top, hipMemcpyDeviceToDevice, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
  if (in->t.arena) VN_HIP_CHECK(hipFree(in->t.arena));
  in->t.arena = a;
  in->arena_cap = cap;
}

// Upsert the n keys of in->kb (device arrays filled): probe, claim, commit.  Returns per class the
// records (vflag counts) in h_cnt[0..3] and their member bytes in h_cnt[4] when emit is set.
void upsert(vn_intake* in, uint32_t n, bool emit) {
  hipStream_t st = in->eng->st;
  KeyBatch& kb = in->kb;
  kb.n = n;
  const int g = blocks_for(n, 256);
  hipLaunchKernelGGL(k_in_probe, dim3(g), dim3(256), 0, st, kb, in->t, in->kid);
  VN_HIP_CHECK(hipMemsetAsync(in->dcnt + 1, 0, 4, st));
  hipLaunchKernelGGL(k_in_claim, dim3(g), dim3(256), 0, st, kb, in->t, in->kid, in->ent, in->dcnt + 1);
  hipLaunchKernelGGL(k_in_newflags, dim3(g), dim3(256), 0, st, kb, in->t, in->ent, in->nflag, in->nbytes);
  scan_exclusive_u32(in->nflag, in->nscan, 4ull * n, in->scan, st);
  scan_exclusive_u32(in->nbytes, in->bscan, n, in->scan, st);
  // one read-back: new keys per class, their bytes, records per class, member bytes, flags
  uint32_t* h = in->h_cnt;
  for (int c = 0; c <= 4; c++)
    VN_HIP_CHECK(hipMemcpyAsync(h + c, in->nscan + (uint64_t)c * n, 4, hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipMemcpyAsync(h + 5, in->bscan + n, 4, hipMemcpyDeviceToHost, st));
  if (emit) {
    for (int c = 0; c <= 4; c++)
      VN_HIP_CHECK(hipMemcpyAsync(h + 6 + c, in->vscan + (uint64_t)c * n, 4, hipMemcpyDeviceToHost, st));
    VN_HIP_CHECK(hipMemcpyAsync(h + 11, in->mscan + n, 4, hipMemcpyDeviceToHost, st));
  }
  VN_HIP_CHECK(hipMemcpyAsync(h + 12, in->dcnt, 8, hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
  uint32_t nnew[4];
  for (int c = 0; c < 4; c++) nnew[c] = h[c + 1] - h[c];
  bool over = h[13] != 0;
  for (int c = 0; c < 4; c++)
    if ((uint64_t)in->next_slot[c] + nnew[c] > in->cap[c]) over = true;
  if (over) {
    hipLaunchKernelGGL(k_in_revert, dim3(g), dim3(256), 0, st, kb, in->t, in->ent);
    VN_HIP_CHECK(hipStreamSynchronize(st));
    static const char* names[4] = {"counter", "gauge", "histo", "set"};
    for (int c = 0; c < 4; c++)
      if ((uint64_t)in->next_slot[c] + nnew[c] > in->cap[c])
        throw std::invalid_argument(std::string("more ") + names[c] +
                                    " keys in one window than the engine's capacity (" + std::to_string(in->cap[c]) +
                                    ")");
    throw std::runtime_error("intake key table full");
  }
  const uint32_t total_new = h[4];
  ensure_arena(in, in->arena_top + h[5], st);
  CommitCtx cc;
  cc.nk0 = in->nkeys;
  for (int c = 0; c < 4; c++) cc.next_slot[c] = in->next_slot[c];
  cc.arena0 = in->arena_top;
  hipLaunchKernelGGL(k_in_commit, dim3(g), dim3(256), 0, st, kb, in->t, in->ent, in->nscan, in->bscan, cc);
  hipLaunchKernelGGL(k_in_slots, dim3(g), dim3(256), 0, st, kb, in->t, in->kid, in->ent, in->slot);
  in->nkeys += total_new;
  in->arena_top += h[5];
  for (int c = 0; c < 4; c++) in->next_slot[c] += nnew[c];
  in->last.new_keys = total_new;
}

void make_batch(vn_intake* in, uint64_t n) {
  KeyBatch& kb = in->kb;
  dalloc(kb.map, n);
  dalloc(kb.name_off, n);
  dalloc(kb.name_len, n);
  dalloc(kb.tags_off, n);
  dalloc(kb.tags_len, n);
  dalloc(kb.n_tags, n);
  dalloc(kb.digest, n);
  dalloc(in->kid, n);
  dalloc(in->ent, n);
  dalloc(in->slot, n);
  dalloc(in->vflag, 4 * n + 1);
  dalloc(in->vscan, 4 * n + 1);
  dalloc(in->nflag, 4 * n + 1);
  dalloc(in->nscan, 4 * n + 1);
  dalloc(in->nbytes, n + 1);
  dalloc(in->bscan, n + 1);
  dalloc(in->mlen, n + 1);
  dalloc(in->mscan, n + 1);
  dalloc(in->s.slot, n);
  dalloc(in->s.value, n);
  dalloc(in->s.rate, n);
  dalloc(in->s.moff, n + 1);
}

}  // namespace

extern "C" {

int vn_intake_create(vn_engine* eng, uint64_t max_bytes, uint64_t max_lines, vn_intake** out) {
  if (!eng || !out || !max_bytes || !max_lines || max_bytes >= (1ull << 32) || max_lines > *std::min_element(eng->max_cls, eng->max_cls + VN_NCLASS))
    return VN_EINVAL;
  *out = nullptr;
  vn_intake* in = new vn_intake;
  in->eng = eng;
  in->max_bytes = max_bytes;
  in->max_lines = max_lines;
  int rc = in_guard(in, [&] {
    VN_HIP_CHECK(hipSetDevice(eng->device));
    if (vn_parser_create(eng->device, max_bytes, max_lines, &in->parser) != VN_OK)
      throw std::bad_alloc();
    uint64_t nk = 0;
    for (int c = 0; c < 4; c++) {
      in->cap[c] = eng->cap[c];
      nk += eng->cap[c];
    }
    uint64_t tc = 1024;
    while (tc < 2 * nk) tc <<= 1;
    if (tc > (1ull << 31)) throw std::invalid_argument("key table too large");
    in->t.mask = (uint32_t)(tc - 1);
    dalloc(in->t.state, tc);
    dalloc(in->t.first, tc);
    VN_HIP_CHECK(hipMemset(in->t.state, 0, tc * 4));
    VN_HIP_CHECK(hipMemset(in->t.first, 0xff, tc * 4));
    in->nkeys_cap = std::max<uint64_t>(nk, 1);
    dalloc(in->t.kmap, in->nkeys_cap);
    dalloc(in->t.kslot, in->nkeys_cap);
    dalloc(in->t.kntags, in->nkeys_cap);
    dalloc(in->t.kdigest, in->nkeys_cap);
    dalloc(in->t.kname_len, in->nkeys_cap);
    dalloc(in->t.ktags_len, in->nkeys_cap);
    dalloc(in->t.kname_off, in->nkeys_cap);
    in->arena_cap = std::max<uint64_t>(in->nkeys_cap * 48, 1 << 16);
    dalloc(in->t.arena, in->arena_cap);
    dalloc(in->lines, max_lines);
    dalloc(in->tags, max_bytes);
    dalloc(in->s.mbytes, max_bytes);
    make_batch(in, max_lines);
    dalloc(in->dcnt, 2);
    VN_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&in->h_cnt), 16 * sizeof(uint32_t)));
  });
  if (rc != VN_OK) {
    vn_intake_destroy(in);
    return rc;
  }
  *out = in;
  return VN_OK;
}

void vn_intake_destroy(vn_intake* in) {
  if (!in) return;
  (void)hipSetDevice(in->eng->device);
  (void)hipDeviceSynchronize();
  if (in->parser) vn_parser_destroy(in->parser);
  void* ps[] = {in->t.state, in->t.first, in->t.kmap, in->t.kslot, in->t.kntags, in->t.kdigest, in->t.kname_len,
                in->t.ktags_len, in->t.kname_off, in->t.arena, in->lines, in->tags, in->ubytes, in->kb.map,
                in->kb.name_off, in->kb.name_len, in->kb.tags_off, in->kb.tags_len, in->kb.n_tags, in->kb.digest,
                in->kid, in->ent, in->slot, in->vflag, in->vscan, in->nflag, in->nscan, in->nbytes, in->bscan,
                in->mlen, in->mscan, in->s.slot, in->s.value, in->s.rate, in->s.moff, in->s.mbytes, in->dcnt,
                in->scan.partials};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  if (in->h_cnt) (void)hipHostFree(in->h_cnt);
  delete in;
}

const char* vn_intake_last_error(const vn_intake* in) { return in ? in->err.c_str() : "null intake"; }

int vn_intake_process(vn_intake* in, const char* buf, uint64_t len, vn_intake_stats* stats) {
  if (!in || (len && !buf)) return VN_EINVAL;
  if (len > in->max_bytes) return in_fail(in, VN_EINVAL, "buffer longer than the intake's max_bytes");
  return in_guard(in, [&] {
    VN_HIP_CHECK(hipSetDevice(in->eng->device));
    in->last = vn_intake_stats{};
    uint64_t n = 0;
    const int prc = vn_parse_dogstatsd_device(in->parser, buf, len, in->lines, in->max_lines,
                                              reinterpret_cast<char*>(in->tags), in->max_bytes, &n);
    if (prc != VN_OK) throw std::invalid_argument(std::string("parse: ") + vn_parser_last_error(in->parser));
    in->last.lines = n;
    if (n) {
      hipStream_t st = in->eng->st;
      KeyBatch& kb = in->kb;
      kb.name_base = reinterpret_cast<const uint8_t*>(buf);
      kb.tags_base = in->tags;
      VN_HIP_CHECK(hipMemsetAsync(in->dcnt, 0, 4, st));
      const int g = blocks_for(n, 256);
      hipLaunchKernelGGL(k_in_class, dim3(g), dim3(256), 0, st, in->lines, (uint32_t)n, kb, in->vflag, in->mlen,
                         in->dcnt);
      scan_exclusive_u32(in->vflag, in->vscan, 4 * n, in->scan, st);
      scan_exclusive_u32(in->mlen, in->mscan, n, in->scan, st);
      upsert(in, (uint32_t)n, true);
      const uint32_t* h = in->h_cnt;
      uint64_t nc[4];
      for (int c = 0; c < 4; c++) nc[c] = h[7 + c] - h[6 + c];
      in->last.processed = h[10];
      in->last.dropped = h[12];
      hipLaunchKernelGGL(k_in_emit, dim3(g), dim3(256), 0, st, in->lines, kb, in->slot, in->vscan, in->mscan,
                         reinterpret_cast<const uint8_t*>(buf), in->s);
      // member offsets end with the total (n_set + 1 entries)
      VN_HIP_CHECK(hipMemcpyAsync(in->s.moff + nc[3], in->mscan + n, 4, hipMemcpyDeviceToDevice, st));
      vn_batch b{};
      b.n_counter = nc[0];
      b.counter_slot = in->s.slot + h[6];
      b.counter_value = in->s.value + h[6];
      b.counter_rate = in->s.rate + h[6];
      b.n_gauge = nc[1];
      b.gauge_slot = in->s.slot + h[7];
      b.gauge_value = in->s.value + h[7];
      b.n_histo = nc[2];
      b.histo_slot = in->s.slot + h[8];
      b.histo_value = in->s.value + h[8];
      b.histo_rate = in->s.rate + h[8];
      b.n_set = nc[3];
      b.set_slot = in->s.slot + h[9];
      b.set_member_off = in->s.moff;
      b.set_member_bytes = in->s.mbytes;
      const int irc = vn_ingest(in->eng, &b);
      if (irc != VN_OK) throw std::invalid_argument(std::string("ingest: ") + vn_last_error(in->eng));
    }
    in->last.parse_errors = in->last.lines - in->last.processed - in->last.dropped;
    if (stats) *stats = in->last;
  });
}

int vn_intake_upsert(vn_intake* in, uint64_t n, const uint8_t* map, const uint32_t* n_tags, const uint32_t* digest,
                     const uint32_t* name_off, const uint32_t* name_len, const uint32_t* tags_off,
                     const uint32_t* tags_len, const uint8_t* bytes, uint64_t nbytes, uint32_t* slot_out) {
  if (!in || (n && (!map || !n_tags || !digest || !name_off || !name_len || !tags_off || !tags_len || !slot_out)) ||
      (nbytes && !bytes))
    return VN_EINVAL;
  if (n > in->max_lines) return in_fail(in, VN_EINVAL, "more keys than the intake's max_lines");
  return in_guard(in, [&] {
    if (!n) return;
    for (uint64_t i = 0; i < n; i++) {
      if (map[i] > 9) throw std::invalid_argument("map id out of range");
      if ((uint64_t)name_off[i] + name_len[i] > nbytes || (uint64_t)tags_off[i] + tags_len[i] > nbytes)
        throw std::invalid_argument("key bytes out of range");
    }
    VN_HIP_CHECK(hipSetDevice(in->eng->device));
    hipStream_t st = in->eng->st;
    if (nbytes > in->ubytes_cap) {
      VN_HIP_CHECK(hipStreamSynchronize(st));
      if (in->ubytes) VN_HIP_CHECK(hipFree(in->ubytes));
      in->ubytes = nullptr;
      dalloc(in->ubytes, nbytes);
      in->ubytes_cap = nbytes;
    }
    KeyBatch& kb = in->kb;
    if (nbytes) VN_HIP_CHECK(hipMemcpyAsync(in->ubytes, bytes, nbytes, hipMemcpyHostToDevice, st));
    VN_HIP_CHECK(hipMemcpyAsync(kb.map, map, n, hipMemcpyHostToDevice, st));
    VN_HIP_CHECK(hipMemcpyAsync(kb.n_tags, n_tags, n * 4, hipMemcpyHostToDevice, st));
    VN_HIP_CHECK(hipMemcpyAsync(kb.digest, digest, n * 4, hipMemcpyHostToDevice, st));
    VN_HIP_CHECK(hipMemcpyAsync(kb.name_off, name_off, n * 4, hipMemcpyHostToDevice, st));
    VN_HIP_CHECK(hipMemcpyAsync(kb.name_len, name_len, n * 4, hipMemcpyHostToDevice, st));
    VN_HIP_CHECK(hipMemcpyAsync(kb.tags_off, tags_off, n * 4, hipMemcpyHostToDevice, st));
    VN_HIP_CHECK(hipMemcpyAsync(kb.tags_len, tags_len, n * 4, hipMemcpyHostToDevice, st));
    kb.name_base = in->ubytes;
    kb.tags_base = in->ubytes;
    upsert(in, (uint32_t)n, false);
    VN_HIP_CHECK(hipMemcpyAsync(slot_out, in->slot, n * 4, hipMemcpyDeviceToHost, st));
    VN_HIP_CHECK(hipStreamSynchronize(st));
  });
}

int vn_intake_keys_info(vn_intake* in, vn_intake_info* info) {
  if (!in || !info) return VN_EINVAL;
  info->n_keys = in->nkeys;
  info->arena_bytes = in->arena_top;
  for (int c = 0; c < 4; c++) info->next_slot[c] = in->next_slot[c];
  return VN_OK;
}

int vn_intake_read_keys(vn_intake* in, uint8_t* map, uint32_t* slot, uint32_t* n_tags, uint64_t* name_off,
                        uint32_t* name_len, uint32_t* tags_len, uint8_t* arena) {
  if (!in) return VN_EINVAL;
  return in_guard(in, [&] {
    VN_HIP_CHECK(hipSetDevice(in->eng->device));
    hipStream_t st = in->eng->st;
    const uint64_t k = in->nkeys;
    if (k) {
      if (!map || !slot || !n_tags || !name_off || !name_len || !tags_len) throw std::invalid_argument("null array");
      VN_HIP_CHECK(hipMemcpyAsync(map, in->t.kmap, k, hipMemcpyDeviceToHost, st));
      VN_HIP_CHECK(hipMemcpyAsync(slot, in->t.kslot, k * 4, hipMemcpyDeviceToHost, st));
      VN_HIP_CHECK(hipMemcpyAsync(n_tags, in->t.kntags, k * 4, hipMemcpyDeviceToHost, st));
      VN_HIP_CHECK(hipMemcpyAsync(name_off, in->t.kname_off, k * 8, hipMemcpyDeviceToHost, st));
      VN_HIP_CHECK(hipMemcpyAsync(name_len, in->t.kname_len, k * 4, hipMemcpyDeviceToHost, st));
      VN_HIP_CHECK(hipMemcpyAsync(tags_len, in->t.ktags_len, k * 4, hipMemcpyDeviceToHost, st));
    }
    if (in->arena_top) {
      if (!arena) throw std::invalid_argument("null arena");
      VN_HIP_CHECK(hipMemcpyAsync(arena, in->t.arena, in->arena_top, hipMemcpyDeviceToHost, st));
    }
    VN_HIP_CHECK(hipStreamSynchronize(st));
  });
}

int vn_intake_reset(vn_intake* in) {
  if (!in) return VN_EINVAL;
  return in_guard(in, [&] {
    VN_HIP_CHECK(hipSetDevice(in->eng->device));
    hipStream_t st = in->eng->st;
    const uint64_t tc = (uint64_t)in->t.mask + 1;
    VN_HIP_CHECK(hipMemsetAsync(in->t.state, 0, tc * 4, st));
    VN_HIP_CHECK(hipMemsetAsync(in->t.first, 0xff, tc * 4, st));
    in->nkeys = 0;
    in->arena_top = 0;
    for (int c = 0; c < 4; c++) in->next_slot[c] = 0;
  });
}

}  // extern "C"

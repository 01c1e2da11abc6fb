// synth_device.hip -- the C4 stream generated in HBM (bench / tests; include/veneur_amd_synth.h).
//
// One global DogStatsD-shaped stream of n_samples positions over n_keys keys (Zipf popularity,
// alias-method draws from a counter-based RNG: position p's key and values depend on (seed, p)
// only), routed the way veneur routes it to workers -- key digest % nranks (server.go:655) --
// except for the split keys, whose records go round-robin by the key's window arrival index
// (record j of a split key to rank j % nranks, include/veneur_amd.h "multi-GPU").  Every rank
// generates the whole stream's keys and keeps its own records, in stream order, so the ranks
// together hold exactly one stream (no per-rank renormalisation of the popularity).
//
// Three passes over the positions, 4096 per block of one wave (lane l owns positions
// [64 l, 64 l + 64) of the block, so lane order is stream order):
//   1. per block, records of every split key                 -> base offsets by scan
//   2. per block, this rank's records per output stream      -> output offsets by scan
//   3. write the records (values drawn from the same RNG as the key)
#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "../../include/veneur_amd_synth.h"
#include "kernels.h"
#include "primitives.h"
#include "sketch.h"

namespace vn {
namespace {

constexpr uint32_t kGBlock = 4096;  // positions per block
constexpr uint32_t kGLane = 64;     // positions per lane
constexpr uint32_t kMaxSplit = 256; // split keys over all classes
constexpr uint32_t kNoSlot = 0xffffffffu;
enum { kOutC = 0, kOutG, kOutH, kOutS, kOutSH, kOutSS, kNOut };

__host__ __device__ __forceinline__ uint64_t smix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ double u01d(uint64_t x) { return (double)(x >> 11) * (1.0 / 9007199254740992.0); }

struct GenCtx {
  uint64_t seed, n;
  uint32_t K, nranks, rank, nsplit;
  const uint32_t* alias_thr;   // [K] coin threshold (2^32 scale)
  const uint32_t* alias_idx;   // [K]
  const uint8_t* cls;          // [K] class of the key
  const uint32_t* owner;       // [K] digest % nranks
  const uint32_t* slot;        // [K] local slot on this rank (kNoSlot: not here)
  const uint32_t* split;       // [K] split index (kNoSlot: not split)
  const uint32_t* split_key;   // [nsplit] class-local split key index (for the split batches)
  uint64_t universe;
  double rate_half, rate_tenth, mu, sigma;
};

__device__ __forceinline__ uint32_t draw_key(const GenCtx& g, uint64_t r0) {
  const uint32_t col = (uint32_t)((r0 >> 32) % g.K);
  return (uint32_t)r0 < g.alias_thr[col] ? col : g.alias_idx[col];
}

// 1. records of each split key per block: bc[s * nblocks + b]
__global__ __launch_bounds__(64) void k_gen_split_counts(GenCtx g, uint32_t nblocks, uint32_t* __restrict__ bc) {
  __shared__ uint32_t cnt[kMaxSplit];
  const uint32_t b = blockIdx.x, l = threadIdx.x;
  for (uint32_t s = l; s < g.nsplit; s += 64) cnt[s] = 0;
  __syncthreads();
  const uint64_t p0 = (uint64_t)b * kGBlock + (uint64_t)l * kGLane;
  for (uint32_t i = 0; i < kGLane; i++) {
    const uint64_t p = p0 + i;
    if (p >= g.n) break;
    const uint32_t s = g.split[draw_key(g, smix(g.seed * 0x100000001B3ull + p))];
    if (s != kNoSlot) atomicAdd(&cnt[s], 1u);
  }
  __syncthreads();
  for (uint32_t s = l; s < g.nsplit; s += 64) bc[(uint64_t)s * nblocks + b] = cnt[s];
}

// per lane: the window arrival index of each of its split records, from the block base and the
// counts of the lanes before it (LDS [64][nsplit] u16 prefix)
struct LaneSplit {
  uint16_t* c;  // [64][kMaxSplit]
};

// output stream of position p on this rank (or kNOut), with its split index
__device__ __forceinline__ uint32_t route(const GenCtx& g, uint32_t key, uint32_t s, uint64_t j) {
  const uint32_t c = g.cls[key];
  if (s != kNoSlot) {
    if (j % g.nranks != g.rank) return kNOut;
    return c == 0 ? kOutC : (c == 2 ? kOutSH : kOutSS);  // split counters ingest as counters
  }
  if (g.owner[key] != g.rank) return kNOut;
  return c;  // kOutC, kOutG, kOutH, kOutS
}

template <bool kWrite>
struct Sink;

struct Outs {
  uint32_t* c_slot; double* c_val; float* c_rate;
  uint32_t* g_slot; double* g_val;
  uint32_t* h_slot; double* h_val; float* h_rate;
  uint32_t* s_slot; uint32_t* s_off; uint8_t* s_bytes;
  uint32_t* sh_key; double* sh_val; float* sh_rate;
  uint32_t* ss_key; uint32_t* ss_off; uint8_t* ss_bytes;
  unsigned long long* counter_sum;  // this rank's sum of int64(v) * int64(float32(1/rate)) (wrapping)
  double* histo_weight;             // this rank's sum of histo weights
};

// 2 / 3. one pass over the block: count (kWrite false) or write (kWrite true) this rank's records
template <bool kWrite>
__global__ __launch_bounds__(64) void k_gen_route(GenCtx g, uint32_t nblocks, const uint32_t* __restrict__ sbase,
                                                  uint32_t* __restrict__ oc, const uint64_t* __restrict__ obase,
                                                  Outs o) {
  __shared__ uint16_t lc[64][kMaxSplit];
  __shared__ uint32_t ocnt[64][kNOut];
  const uint32_t b = blockIdx.x, l = threadIdx.x;
  const uint64_t p0 = (uint64_t)b * kGBlock + (uint64_t)l * kGLane;
  // lane-local split counts, then exclusive prefix over the lanes
  for (uint32_t s = 0; s < g.nsplit; s++) lc[l][s] = 0;
  for (uint32_t i = 0; i < kGLane && g.nsplit; i++) {
    const uint64_t p = p0 + i;
    if (p >= g.n) break;
    const uint32_t s = g.split[draw_key(g, smix(g.seed * 0x100000001B3ull + p))];
    if (s != kNoSlot) lc[l][s]++;
  }
  __syncthreads();
  for (uint32_t s = l; s < g.nsplit; s += 64) {
    uint16_t run = 0;
    for (uint32_t q = 0; q < 64; q++) {
      const uint16_t v = lc[q][s];
      lc[q][s] = run;
      run += v;
    }
  }
  __syncthreads();
  uint32_t cnt[kNOut];
  for (int k = 0; k < kNOut; k++) cnt[k] = 0;
  unsigned long long csum = 0;
  double hw = 0.0;
  if (kWrite) {
    // this lane's first output of each stream: block base + the lanes before it
    for (int k = 0; k < kNOut; k++) ocnt[l][k] = oc[((uint64_t)b * 64 + l) * kNOut + k];
  }
  for (uint32_t i = 0; i < kGLane; i++) {
    const uint64_t p = p0 + i;
    if (p >= g.n) break;
    const uint64_t r0 = smix(g.seed * 0x100000001B3ull + p);
    const uint32_t key = draw_key(g, r0);
    const uint32_t s = g.split[key];
    uint64_t j = 0;
    if (s != kNoSlot) j = (uint64_t)sbase[(uint64_t)s * nblocks + b] + lc[l][s]++;
    const uint32_t d = route(g, key, s, j);
    if (d == kNOut) continue;
    if (!kWrite) {
      cnt[d]++;
      continue;
    }
    const uint64_t w = obase[(uint64_t)d * nblocks + b] + ocnt[l][d]++;
    const uint64_t r1 = smix(r0), r2 = smix(r1), r3 = smix(r2);
    const double ur = u01d(r2);
    const float rate = ur < g.rate_tenth ? 0.1f : (ur < g.rate_tenth + g.rate_half ? 0.5f : 1.0f);
    const uint32_t slot = g.slot[key];
    if (d == kOutC) {
      const double v = (double)(1 + (r1 % 10));
      o.c_slot[w] = slot;
      o.c_val[w] = v;
      o.c_rate[w] = rate;
      csum += (unsigned long long)((int64_t)v * (int64_t)(1.0f / rate));
    } else if (d == kOutG) {
      o.g_slot[w] = slot;
      o.g_val[w] = u01d(r1) * 1000.0;
    } else if (d == kOutH || d == kOutSH) {
      double a = u01d(r1), bb = u01d(r3);
      if (a < 1e-300) a = 1e-300;
      const double z = sqrt(-2.0 * log(a)) * cos(6.283185307179586 * bb);
      const double v = exp(g.mu + g.sigma * z);
      hw += (double)(1.0f / rate);
      if (d == kOutH) {
        o.h_slot[w] = slot;
        o.h_val[w] = v;
        o.h_rate[w] = rate;
      } else {
        o.sh_key[w] = g.split_key[s];
        o.sh_val[w] = v;
        o.sh_rate[w] = rate;
      }
    } else {
      // member "m%010llu": 11 bytes
      unsigned long long m = g.universe ? (r1 % g.universe) : r1;
      uint8_t* dst = (d == kOutS ? o.s_bytes : o.ss_bytes) + w * 11;
      dst[0] = 'm';
      for (int q = 10; q >= 1; q--) {
        dst[q] = (uint8_t)('0' + m % 10);
        m /= 10;
      }
      if (d == kOutS) {
        o.s_slot[w] = slot;
        o.s_off[w] = (uint32_t)(w * 11);
      } else {
        o.ss_key[w] = g.split_key[s];
        o.ss_off[w] = (uint32_t)(w * 11);
      }
    }
  }
  if (!kWrite) {
    for (int k = 0; k < kNOut; k++) oc[((uint64_t)b * 64 + l) * kNOut + k] = cnt[k];
  } else {
    for (int d = 32; d >= 1; d >>= 1) {
      csum += (unsigned long long)__shfl_xor((long long)csum, d, 64);
      hw += __shfl_xor(hw, d, 64);
    }
    if (l == 0) {
      if (csum) atomicAdd(o.counter_sum, csum);
      if (hw != 0.0) atomicAdd(o.histo_weight, hw);
    }
  }
}

// per block: totals of the lane counts, and each lane's exclusive offset inside the block
__global__ __launch_bounds__(64) void k_gen_lane_scan(uint32_t nblocks, uint32_t* __restrict__ oc,
                                                      uint32_t* __restrict__ bt) {
  const uint32_t b = blockIdx.x, k = threadIdx.x;
  if (k >= kNOut) return;
  uint32_t run = 0;
  for (uint32_t l = 0; l < 64; l++) {
    uint32_t* p = oc + ((uint64_t)b * 64 + l) * kNOut + k;
    const uint32_t v = *p;
    *p = run;
    run += v;
  }
  bt[(uint64_t)k * nblocks + b] = run;
}
// per stream row (nblocks u32 counts) -> u64 exclusive bases; totals[k]
__global__ void k_gen_row_scan(uint32_t nrows, uint32_t nblocks, const uint32_t* __restrict__ cnt,
                               uint64_t* __restrict__ base, uint64_t* __restrict__ totals) {
  // one thread per row, sequential (nblocks ~ 244k for 1e9 positions; a few ms, setup only)
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  uint64_t run = 0;
  for (uint32_t b = 0; b < nblocks; b++) {
    base[(uint64_t)r * nblocks + b] = run;
    run += cnt[(uint64_t)r * nblocks + b];
  }
  totals[r] = run;
}
__global__ void k_u64_to_u32(uint64_t n, const uint64_t* __restrict__ a, uint32_t* __restrict__ b) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = (uint32_t)a[i];
}

uint32_t fnv(const char* s, size_t n, uint32_t h) {
  for (size_t i = 0; i < n; i++) {
    h ^= (uint8_t)s[i];
    h *= 16777619u;
  }
  return h;
}

template <class T>
T* dmalloc(size_t n) {
  void* p = nullptr;
  VN_HIP_CHECK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
  return static_cast<T*>(p);
}

// key table shared by vn_synth_device and vn_synth_key_counts
struct KeyTable {
  std::vector<uint8_t> cls;
  std::vector<uint32_t> digest, thr, idx;
};
KeyTable key_table(const vn_synth_dev_config* c) {
  const uint32_t K = c->n_keys;
  KeyTable t;
  t.cls.resize(K);
  t.digest.resize(K);
  static const char* kType[4] = {"counter", "gauge", "histogram", "set"};
  double cum[4], tot = c->mix[0] + c->mix[1] + c->mix[2] + c->mix[3], run = 0;
  for (int i = 0; i < 4; i++) cum[i] = (run += c->mix[i] / tot);
  char name[32];
  for (uint32_t k = 0; k < K; k++) {
    // class by key, as the host generator (synth.cpp) draws it
    const uint64_t x = smix(c->seed ^ (0xA5A5A5A5ull + (uint64_t)k * 0x9E3779B97F4A7C15ull));
    const double u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
    int cl = 0;
    while (cl < 3 && u >= cum[cl]) cl++;
    while (cl < 3 && c->mix[cl] == 0) cl++;
    t.cls[k] = (uint8_t)cl;
    const int n = snprintf(name, sizeof(name), "k%07u", k);
    t.digest[k] = fnv(kType[cl], strlen(kType[cl]), fnv(name, (size_t)n, 2166136261u));
  }
  // Vose alias table of the Zipf law p_k ~ 1 / (k + 1)^s
  std::vector<double> q(K);
  double z = 0;
  for (uint32_t k = 0; k < K; k++) z += (q[k] = c->zipf_s == 0 ? 1.0 : 1.0 / std::pow((double)k + 1.0, c->zipf_s));
  for (auto& v : q) v = v * K / z;
  t.thr.assign(K, 0xffffffffu);
  t.idx.resize(K);
  std::vector<uint32_t> small, large;
  for (uint32_t k = 0; k < K; k++) {
    t.idx[k] = k;
    (q[k] < 1.0 ? small : large).push_back(k);
  }
  while (!small.empty() && !large.empty()) {
    const uint32_t a = small.back(), g = large.back();
    small.pop_back();
    t.thr[a] = (uint32_t)std::min(4294967295.0, q[a] * 4294967296.0);
    t.idx[a] = g;
    q[g] = (q[g] + q[a]) - 1.0;
    if (q[g] < 1.0) {
      large.pop_back();
      small.push_back(g);
    }
  }
  return t;
}

__global__ void k_gen_key_counts(GenCtx g, uint64_t n, uint32_t* __restrict__ cnt) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[draw_key(g, smix(g.seed * 0x100000001B3ull + p))], 1u);
}

// ---- C5 host windows (vn_synth_hosts_device)
struct HostsGen {
  uint64_t seed;
  uint32_t host0, nh, H, S;
};
__device__ __forceinline__ uint64_t host_key_draw(const HostsGen& g, uint32_t h, uint32_t k, uint64_t salt) {
  return smix(g.seed ^ smix(((uint64_t)h << 32 | k) ^ salt));
}
__device__ __forceinline__ uint32_t histo_count(const HostsGen& g, uint32_t h, uint32_t k) {
  return 50u + (uint32_t)(host_key_draw(g, h, k, 0x1111) % 101u);
}
__device__ __forceinline__ uint32_t set_count(const HostsGen& g, uint32_t h, uint32_t k) {
  const double u = 1.0 - u01d(host_key_draw(g, h, k, 0x2222));  // (0, 1]
  const double x = pow(u, -1.0 / 1.2) - 1.0;                     // Lomax(1.2)
  return x * 50.0 >= 19999.0 ? 20000u : (uint32_t)(x * 50.0) + 1u;
}
__global__ void k_hosts_counts(HostsGen g, uint32_t* __restrict__ hc, uint32_t* __restrict__ sc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nH = (uint64_t)g.nh * g.H, nS = (uint64_t)g.nh * g.S;
  if (i < nH) hc[i] = histo_count(g, g.host0 + (uint32_t)(i / g.H), (uint32_t)(i % g.H));
  if (i < nS) sc[i] = set_count(g, g.host0 + (uint32_t)(i / g.S), (uint32_t)(i % g.S));
}
__global__ void k_hosts_histo(HostsGen g, const uint64_t* __restrict__ off, uint32_t* __restrict__ slot,
                              double* __restrict__ val, float* __restrict__ rate) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)g.nh * g.H) return;
  const uint32_t h = g.host0 + (uint32_t)(i / g.H), k = (uint32_t)(i % g.H);
  const double mu = 3.9 + 0.05 * (double)(h % 8u);
  for (uint64_t o = off[i], j = 0; o < off[i + 1]; o++, j++) {
    const uint64_t a = host_key_draw(g, h, k, 0x3333 + 2 * j), b = host_key_draw(g, h, k, 0x3334 + 2 * j);
    const double u1 = 1.0 - u01d(a), u2 = u01d(b);
    const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    slot[o] = (uint32_t)i;
    val[o] = exp(mu + z);
    rate[o] = (b & 0x3ffu) < 102u ? 0.5f : 1.0f;  // about 10% at rate 0.5
  }
}
__global__ void k_hosts_set(HostsGen g, const uint64_t* __restrict__ off, uint32_t* __restrict__ slot,
                            uint64_t* __restrict__ hash) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)g.nh * g.S) return;
  const uint32_t h = g.host0 + (uint32_t)(i / g.S), k = (uint32_t)(i % g.S);
  for (uint64_t o = off[i], j = 0; o < off[i + 1]; o++, j++) {
    slot[o] = (uint32_t)i;
    hash[o] = host_key_draw(g, h, k, 0x4444 + j);
  }
}

}  // namespace
}  // namespace vn

using namespace vn;

extern "C" {

int vn_synth_key_counts(const vn_synth_dev_config* c, uint64_t n_positions, uint32_t* counts) {
  if (!c || !counts || !c->n_keys) return -1;
  try {
    VN_HIP_CHECK(hipSetDevice(c->device));
    const KeyTable t = key_table(c);
    const uint32_t K = c->n_keys;
    uint32_t* thr = dmalloc<uint32_t>(K);
    uint32_t* idx = dmalloc<uint32_t>(K);
    uint32_t* cnt = dmalloc<uint32_t>(K);
    VN_HIP_CHECK(hipMemcpy(thr, t.thr.data(), K * 4, hipMemcpyHostToDevice));
    VN_HIP_CHECK(hipMemcpy(idx, t.idx.data(), K * 4, hipMemcpyHostToDevice));
    VN_HIP_CHECK(hipMemset(cnt, 0, K * 4));
    GenCtx g{};
    g.seed = c->seed;
    g.K = K;
    g.alias_thr = thr;
    g.alias_idx = idx;
    hipLaunchKernelGGL(k_gen_key_counts, dim3(4096), dim3(256), 0, 0, g, std::min(n_positions, c->n_samples), cnt);
    VN_HIP_CHECK(hipMemcpy(counts, cnt, K * 4, hipMemcpyDeviceToHost));
    (void)hipFree(thr);
    (void)hipFree(idx);
    (void)hipFree(cnt);
    return 0;
  } catch (const HipError&) {
    return -2;
  }
}

int vn_synth_device(const vn_synth_dev_config* c, vn_synth_dev_out* out) {
  if (!c || !out || !c->n_keys || !c->nranks || c->rank >= c->nranks) return -1;
  std::memset(out, 0, sizeof(*out));
  uint32_t nsplit = 0;
  for (int k = 0; k < 4; k++) nsplit += c->n_split[k];
  if (nsplit > kMaxSplit || c->n_split[1]) return -1;  // gauges are never split
  try {
    VN_HIP_CHECK(hipSetDevice(c->device));
    const uint32_t K = c->n_keys;
    const KeyTable t = key_table(c);
    // local slots: owned keys (not split), ascending key id, then the split keys of the class
    std::vector<uint32_t> owner(K), slot(K, kNoSlot), split(K, kNoSlot), skey;
    for (uint32_t k = 0; k < K; k++) owner[k] = t.digest[k] % c->nranks;
    for (int cl = 0, s = 0; cl < 4; cl++)
      for (uint32_t i = 0; i < c->n_split[cl]; i++, s++) {
        const uint32_t k = c->split_key[cl][i];
        if (k >= K || t.cls[k] != cl) return -3;
        split[k] = (uint32_t)s;
        skey.push_back(i);
      }
    std::vector<uint32_t> ks[4];
    for (uint32_t k = 0; k < K; k++)
      if (split[k] == kNoSlot && owner[k] == c->rank) ks[t.cls[k]].push_back(k);
    for (int cl = 0; cl < 4; cl++) {
      out->split_slot0[cl] = (uint32_t)ks[cl].size();
      for (uint32_t i = 0; i < c->n_split[cl]; i++) ks[cl].push_back(c->split_key[cl][i]);
      out->n_slots[cl] = (uint32_t)ks[cl].size();
      out->key_of_slot[cl] = (uint32_t*)malloc(std::max<size_t>(1, ks[cl].size()) * 4);
      out->digest_of_slot[cl] = (uint32_t*)malloc(std::max<size_t>(1, ks[cl].size()) * 4);
      for (size_t i = 0; i < ks[cl].size(); i++) {
        out->key_of_slot[cl][i] = ks[cl][i];
        out->digest_of_slot[cl][i] = t.digest[ks[cl][i]];
        slot[ks[cl][i]] = (uint32_t)i;
      }
    }
    // device tables
    uint32_t* d_thr = dmalloc<uint32_t>(K);
    uint32_t* d_idx = dmalloc<uint32_t>(K);
    uint8_t* d_cls = dmalloc<uint8_t>(K);
    uint32_t* d_own = dmalloc<uint32_t>(K);
    uint32_t* d_slot = dmalloc<uint32_t>(K);
    uint32_t* d_split = dmalloc<uint32_t>(K);
    uint32_t* d_skey = dmalloc<uint32_t>(std::max<size_t>(1, skey.size()));
    VN_HIP_CHECK(hipMemcpy(d_thr, t.thr.data(), K * 4, hipMemcpyHostToDevice));
    VN_HIP_CHECK(hipMemcpy(d_idx, t.idx.data(), K * 4, hipMemcpyHostToDevice));
    VN_HIP_CHECK(hipMemcpy(d_cls, t.cls.data(), K, hipMemcpyHostToDevice));
    VN_HIP_CHECK(hipMemcpy(d_own, owner.data(), K * 4, hipMemcpyHostToDevice));
    VN_HIP_CHECK(hipMemcpy(d_slot, slot.data(), K * 4, hipMemcpyHostToDevice));
    VN_HIP_CHECK(hipMemcpy(d_split, split.data(), K * 4, hipMemcpyHostToDevice));
    if (!skey.empty()) VN_HIP_CHECK(hipMemcpy(d_skey, skey.data(), skey.size() * 4, hipMemcpyHostToDevice));
    GenCtx g{};
    g.seed = c->seed;
    g.n = c->n_samples;
    g.K = K;
    g.nranks = c->nranks;
    g.rank = c->rank;
    g.nsplit = nsplit;
    g.alias_thr = d_thr;
    g.alias_idx = d_idx;
    g.cls = d_cls;
    g.owner = d_own;
    g.slot = d_slot;
    g.split = d_split;
    g.split_key = d_skey;
    g.universe = c->member_universe;
    g.rate_half = c->rate_half;
    g.rate_tenth = c->rate_tenth;
    g.mu = c->histo_mu;
    g.sigma = c->histo_sigma;
    const uint64_t nb64 = (c->n_samples + kGBlock - 1) / kGBlock;
    if (nb64 >= (1ull << 31)) return -1;
    const uint32_t nb = (uint32_t)std::max<uint64_t>(nb64, 1);
    // 1. split-key arrival bases
    uint32_t* sbase = dmalloc<uint32_t>((size_t)std::max(nsplit, 1u) * nb);
    if (nsplit) {
      uint32_t* bc = dmalloc<uint32_t>((size_t)nsplit * nb);
      uint64_t* b64 = dmalloc<uint64_t>((size_t)nsplit * nb);
      uint64_t* tots = dmalloc<uint64_t>(nsplit);
      hipLaunchKernelGGL(k_gen_split_counts, dim3(nb), dim3(64), 0, 0, g, nb, bc);
      hipLaunchKernelGGL(k_gen_row_scan, dim3(1), dim3(256), 0, 0, nsplit, nb, bc, b64, tots);
      hipLaunchKernelGGL(k_u64_to_u32, dim3(blocks_for((uint64_t)nsplit * nb, 256)), dim3(256), 0, 0,
                         (uint64_t)nsplit * nb, b64, sbase);
      VN_HIP_CHECK(hipDeviceSynchronize());
      (void)hipFree(bc);
      (void)hipFree(b64);
      (void)hipFree(tots);
    }
    // 2. this rank's records per output stream and lane
    uint32_t* oc = dmalloc<uint32_t>((size_t)nb * 64 * kNOut);
    uint32_t* bt = dmalloc<uint32_t>((size_t)nb * kNOut);
    uint64_t* obase = dmalloc<uint64_t>((size_t)nb * kNOut);
    uint64_t* otot = dmalloc<uint64_t>(kNOut);
    Outs o{};
    hipLaunchKernelGGL(k_gen_route<false>, dim3(nb), dim3(64), 0, 0, g, nb, sbase, oc, obase, o);
    hipLaunchKernelGGL(k_gen_lane_scan, dim3(nb), dim3(64), 0, 0, nb, oc, bt);
    hipLaunchKernelGGL(k_gen_row_scan, dim3(1), dim3(64), 0, 0, (uint32_t)kNOut, nb, bt, obase, otot);
    uint64_t tot[kNOut];
    VN_HIP_CHECK(hipMemcpy(tot, otot, sizeof(tot), hipMemcpyDeviceToHost));
    // 3. outputs
    o.c_slot = dmalloc<uint32_t>(tot[kOutC]); o.c_val = dmalloc<double>(tot[kOutC]); o.c_rate = dmalloc<float>(tot[kOutC]);
    o.g_slot = dmalloc<uint32_t>(tot[kOutG]); o.g_val = dmalloc<double>(tot[kOutG]);
    o.h_slot = dmalloc<uint32_t>(tot[kOutH]); o.h_val = dmalloc<double>(tot[kOutH]); o.h_rate = dmalloc<float>(tot[kOutH]);
    o.s_slot = dmalloc<uint32_t>(tot[kOutS]); o.s_off = dmalloc<uint32_t>(tot[kOutS] + 1);
    o.s_bytes = dmalloc<uint8_t>(tot[kOutS] * 11);
    o.sh_key = dmalloc<uint32_t>(tot[kOutSH]); o.sh_val = dmalloc<double>(tot[kOutSH]);
    o.sh_rate = dmalloc<float>(tot[kOutSH]);
    o.ss_key = dmalloc<uint32_t>(tot[kOutSS]); o.ss_off = dmalloc<uint32_t>(tot[kOutSS] + 1);
    o.ss_bytes = dmalloc<uint8_t>(tot[kOutSS] * 11);
    unsigned long long* sums = dmalloc<unsigned long long>(2);
    VN_HIP_CHECK(hipMemset(sums, 0, 16));
    o.counter_sum = sums;
    o.histo_weight = reinterpret_cast<double*>(sums + 1);
    if (tot[kOutS] * 11 >= (1ull << 32) || tot[kOutSS] * 11 >= (1ull << 32)) return -4;  // u32 member offsets
    hipLaunchKernelGGL(k_gen_route<true>, dim3(nb), dim3(64), 0, 0, g, nb, sbase, oc, obase, o);
    const uint32_t send = (uint32_t)(tot[kOutS] * 11), ssend = (uint32_t)(tot[kOutSS] * 11);
    VN_HIP_CHECK(hipMemcpy(o.s_off + tot[kOutS], &send, 4, hipMemcpyHostToDevice));
    VN_HIP_CHECK(hipMemcpy(o.ss_off + tot[kOutSS], &ssend, 4, hipMemcpyHostToDevice));
    unsigned long long hs[2];
    VN_HIP_CHECK(hipMemcpy(hs, sums, 16, hipMemcpyDeviceToHost));
    VN_HIP_CHECK(hipGetLastError());
    out->counter_sum = (int64_t)hs[0];
    std::memcpy(&out->histo_weight, &hs[1], 8);
    for (void* p : {(void*)d_thr, (void*)d_idx, (void*)d_cls, (void*)d_own, (void*)d_slot, (void*)d_split,
                    (void*)d_skey, (void*)sbase, (void*)oc, (void*)bt, (void*)obase, (void*)otot, (void*)sums})
      (void)hipFree(p);
    vn_batch& b = out->batch;
    b.n_counter = tot[kOutC]; b.counter_slot = o.c_slot; b.counter_value = o.c_val; b.counter_rate = o.c_rate;
    b.n_gauge = tot[kOutG]; b.gauge_slot = o.g_slot; b.gauge_value = o.g_val;
    b.n_histo = tot[kOutH]; b.histo_slot = o.h_slot; b.histo_value = o.h_val; b.histo_rate = o.h_rate;
    b.n_set = tot[kOutS]; b.set_slot = o.s_slot; b.set_member_off = o.s_off; b.set_member_bytes = o.s_bytes;
    b.set_hash = nullptr;
    vn_split_batch& sb = out->split;
    sb.n_histo = tot[kOutSH]; sb.histo_key = o.sh_key; sb.histo_value = o.sh_val; sb.histo_rate = o.sh_rate;
    sb.n_set = tot[kOutSS]; sb.set_key = o.ss_key; sb.set_member_off = o.ss_off; sb.set_member_bytes = o.ss_bytes;
    sb.set_hash = nullptr;
    out->n_member_bytes = tot[kOutS] * 11;
    out->n_split_member_bytes = tot[kOutSS] * 11;
    return 0;
  } catch (const HipError&) {
    return -2;
  }
}

int vn_synth_hosts_device(const vn_synth_hosts_config* c, vn_synth_hosts_out* out) {
  if (!c || !out || !c->n_hosts || (!c->n_histo_keys && !c->n_set_keys)) return -1;
  std::memset(out, 0, sizeof(*out));
  try {
    VN_HIP_CHECK(hipSetDevice(c->device));
    HostsGen g{c->seed, c->host0, c->n_hosts, c->n_histo_keys, c->n_set_keys};
    const uint64_t nH = (uint64_t)g.nh * g.H, nS = (uint64_t)g.nh * g.S, nmax = std::max(nH, nS);
    if (nH >= (1ull << 32) || nS >= (1ull << 32)) return -1;
    uint32_t* hc = dmalloc<uint32_t>(nH);
    uint32_t* sc = dmalloc<uint32_t>(nS);
    uint64_t* ho = dmalloc<uint64_t>(nH + 1);
    uint64_t* so = dmalloc<uint64_t>(nS + 1);
    hipLaunchKernelGGL(k_hosts_counts, dim3((uint32_t)((nmax + 255) / 256)), dim3(256), 0, 0, g, hc, sc);
    scan_sizes_u64(hc, ho, nH, 0);
    scan_sizes_u64(sc, so, nS, 0);
    VN_HIP_CHECK(hipMemcpy(&out->n_histo, ho + nH, 8, hipMemcpyDeviceToHost));
    VN_HIP_CHECK(hipMemcpy(&out->n_set, so + nS, 8, hipMemcpyDeviceToHost));
    out->h_slot = dmalloc<uint32_t>(out->n_histo);
    out->h_val = dmalloc<double>(out->n_histo);
    out->h_rate = dmalloc<float>(out->n_histo);
    out->s_slot = dmalloc<uint32_t>(out->n_set);
    out->s_hash = dmalloc<uint64_t>(out->n_set);
    if (nH)
      hipLaunchKernelGGL(k_hosts_histo, dim3((uint32_t)((nH + 255) / 256)), dim3(256), 0, 0, g, ho, out->h_slot,
                         out->h_val, out->h_rate);
    if (nS)
      hipLaunchKernelGGL(k_hosts_set, dim3((uint32_t)((nS + 255) / 256)), dim3(256), 0, 0, g, so, out->s_slot,
                         out->s_hash);
    VN_HIP_CHECK(hipDeviceSynchronize());
    for (void* q : {(void*)hc, (void*)sc, (void*)ho, (void*)so}) (void)hipFree(q);
    return 0;
  } catch (const HipError&) {
    vn_synth_hosts_free(out);
    return -2;
  }
}

void vn_synth_hosts_free(vn_synth_hosts_out* o) {
  if (!o) return;
  for (void* q : {(void*)o->h_slot, (void*)o->h_val, (void*)o->h_rate, (void*)o->s_slot, (void*)o->s_hash})
    if (q) (void)hipFree(q);
  std::memset(o, 0, sizeof(*o));
}

void vn_synth_device_free(vn_synth_dev_out* o) {
  if (!o) return;
  const vn_batch& b = o->batch;
  for (const void* p : {(const void*)b.counter_slot, (const void*)b.counter_value, (const void*)b.counter_rate,
                        (const void*)b.gauge_slot, (const void*)b.gauge_value, (const void*)b.histo_slot,
                        (const void*)b.histo_value, (const void*)b.histo_rate, (const void*)b.set_slot,
                        (const void*)b.set_member_off, (const void*)b.set_member_bytes})
    if (p) (void)hipFree(const_cast<void*>(p));
  const vn_split_batch& s = o->split;
  for (const void* p : {(const void*)s.histo_key, (const void*)s.histo_value, (const void*)s.histo_rate,
                        (const void*)s.set_key, (const void*)s.set_member_off, (const void*)s.set_member_bytes})
    if (p) (void)hipFree(const_cast<void*>(p));
  for (int k = 0; k < 4; k++) {
    free(o->key_of_slot[k]);
    free(o->digest_of_slot[k]);
  }
  std::memset(o, 0, sizeof(*o));
}

}  // extern "C"

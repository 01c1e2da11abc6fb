// partition.h -- one stable 8-bit radix partition pass with fused loaders.
//
// A pass reads records straight from the caller's SoA arrays (Src), ranks them stably by
// the digit (key >> shift) & 255 within each 4096-record tile (wave64 ballot match), and
// writes them digit-major through Dst, so each digit run leaves the tile contiguously.
// The per-digit bucket [start, end) of the output is read back from the scanned offsets.
#pragma once
#include "primitives.h"

namespace vn {

__device__ __forceinline__ uint64_t part_match8(uint32_t d, bool active) {
  uint64_t m = __ballot(active);
#pragma unroll
  for (int bit = 0; bit < 8; bit++) {
    uint64_t bb = __ballot(active && ((d >> bit) & 1u));
    m &= ((d >> bit) & 1u) ? bb : ~bb;
  }
  return m;
}

// Per-tile digit counts.  The lanes of a wave that share a digit add once, through their lowest
// lane (the wave's match mask): a Zipf-hot bucket -- most of a key-range partition's records --
// would otherwise serialise 64 LDS atomics on one address per load.
template <class Src>
__global__ __launch_bounds__(kBlock) void k_part_count(Src src, uint64_t n, int shift, uint32_t* __restrict__ counts,
                                                       uint32_t nblocks) {
  __shared__ uint32_t s_hist[4][256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4 * 256; i += kBlock) (&s_hist[0][0])[i] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t key[kItems];
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const uint64_t i = base + (uint64_t)j * kBlock + threadIdx.x;
    key[j] = i < n ? src.key(i) : 0u;
  }
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const bool active = base + (uint64_t)j * kBlock + threadIdx.x < n;
    const uint32_t d = (key[j] >> shift) & 0xffu;
    const uint64_t peers = part_match8(d, active);
    if (active && (peers & lt) == 0) atomicAdd(&s_hist[w][d], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  const uint32_t d = threadIdx.x;
  counts[(uint64_t)d * nblocks + blockIdx.x] = s_hist[0][d] + s_hist[1][d] + s_hist[2][d] + s_hist[3][d];
}

// Each wave owns a contiguous quarter of the tile: its records are loaded up front (all loads
// in flight together) and ranked with wave ballots against a per-wave running count per digit
// in LDS (a wave's DS operations execute in order: no workgroup barrier while ranking).
// A Dst with kPacked = true stores each record as the one dword pack() makes of it (its rare
// out-of-line payload written at once, at the record's final place): the tile is staged as
// those dwords alone, 16 KiB of LDS instead of 48, and more tiles fit a CU.
template <class Dst, class = void>
struct DstPacked {
  static constexpr bool value = false;
};
template <class Dst>
struct DstPacked<Dst, decltype((void)Dst::kPacked)> {
  static constexpr bool value = Dst::kPacked;
};

template <class Src, class Dst>
__global__ __launch_bounds__(kBlock) void k_part_scatter(Src src, Dst dst, uint64_t n, int shift,
                                                         const uint32_t* __restrict__ counts,
                                                         const uint32_t* __restrict__ offsets, uint32_t nblocks) {
  using P = typename Src::P;
  constexpr bool kPack = DstPacked<Dst>::value;
  __shared__ uint32_t s_key[kTile];
  __shared__ P s_pay[kPack ? 1 : kTile];
  __shared__ uint8_t s_dig[kPack ? kTile : 1];  // (packed: each record's digit beside its dword)
  __shared__ uint32_t s_run[4][256];
  __shared__ uint32_t s_loc[256];
  __shared__ uint32_t s_glob[256];
  __shared__ uint32_t s_wave[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  const uint32_t tile_n = (uint32_t)((n - base) < (uint64_t)kTile ? (n - base) : kTile);
  constexpr uint32_t kWaveTile = kTile / 4;
  const uint32_t wbase = (uint32_t)w * kWaveTile;
  uint32_t key[kItems];
  P pay[kItems];
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const uint32_t li = wbase + (uint32_t)j * 64 + lane;
    key[j] = 0;
    pay[j] = P{};
    if (li < tile_n) src.load(base + li, key[j], pay[j]);
  }
  {
    uint32_t c = counts[(uint64_t)t * nblocks + blockIdx.x];
    // exclusive scan of the tile's digit counts (4 waves)
    uint32_t inc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t o = __shfl_up(inc, d, 64);
      if (lane >= d) inc += o;
    }
    if (lane == 63) s_wave[w] = inc;
    __syncthreads();
    uint32_t b0 = 0;
    for (int i = 0; i < w; i++) b0 += s_wave[i];
    s_loc[t] = b0 + inc - c;
    s_glob[t] = offsets[(uint64_t)t * nblocks + blockIdx.x];
    s_run[0][t] = s_run[1][t] = s_run[2][t] = s_run[3][t] = 0;
  }
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t rank[kItems];
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const uint32_t li = wbase + (uint32_t)j * 64 + lane;
    const bool active = li < tile_n;
    const uint32_t d = active ? (key[j] >> shift) & 0xffu : 0u;
    const uint64_t peers = part_match8(d, active);
    const uint32_t before = active ? s_run[w][d] : 0u;
    rank[j] = before + (uint32_t)__popcll(peers & lt);
    asm volatile("" ::: "memory");  // the wave's reads of s_run precede its leaders' update
    if (active && (peers & lt) == 0) s_run[w][d] = before + (uint32_t)__popcll(peers);
    asm volatile("" ::: "memory");
  }
  __syncthreads();
  {
    const uint32_t c0 = s_run[0][t], c1 = s_run[1][t], c2 = s_run[2][t], l = s_loc[t];
    s_run[0][t] = l;
    s_run[1][t] = l + c0;
    s_run[2][t] = l + c0 + c1;
    s_run[3][t] = l + c0 + c1 + c2;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const uint32_t li = wbase + (uint32_t)j * 64 + lane;
    if (li < tile_n) {
      const uint32_t d = (key[j] >> shift) & 0xffu;
      const uint32_t pos = s_run[w][d] + rank[j];
      if constexpr (kPack) {
        s_key[pos] = dst.pack((uint64_t)s_glob[d] + (pos - s_loc[d]), key[j], pay[j]);
        s_dig[pos] = (uint8_t)d;
      } else {
        s_key[pos] = key[j];
        s_pay[pos] = pay[j];
      }
    }
  }
  __syncthreads();
  if constexpr (kPack) {
    for (uint32_t li = t; li < tile_n; li += kBlock) {
      const uint32_t d = s_dig[li];
      dst.key[(uint64_t)s_glob[d] + (li - s_loc[d])] = s_key[li];
    }
  } else {
    for (uint32_t li = t; li < tile_n; li += kBlock) {
      uint32_t k = s_key[li];
      uint32_t d = (k >> shift) & 0xffu;
      dst.store((uint64_t)s_glob[d] + (li - s_loc[d]), k, s_pay[li]);
    }
  }
}

// One partition pass: counts, digit-major scan, scatter.  After it, bucket d of the output
// is [offsets[d * nblocks], offsets[(d + 1) * nblocks]) (offsets[256 * nblocks] = n).
template <class Src, class Dst>
uint32_t partition_pass(const Src& src, const Dst& dst, uint64_t n, int shift, RadixScratch& s, hipStream_t st,
                        RadixStats* stats, uint64_t bytes_per_record) {
  radix_scratch_reserve(s, n);
  const uint32_t nblocks = (uint32_t)blocks_for(n, kTile);
  hipLaunchKernelGGL(k_part_count<Src>, dim3(nblocks), dim3(kBlock), 0, st, src, n, shift, s.counts, nblocks);
  scan_exclusive_u32(s.counts, s.offsets, (uint64_t)256 * nblocks, s.scan, st);
  hipEvent_t e0 = (stats && stats->pool) ? stats->pool->next() : nullptr;
  hipEvent_t e1 = (stats && stats->pool) ? stats->pool->next() : nullptr;
  if (e0 && e1) VN_HIP_CHECK(hipEventRecord(e0, st));
  hipLaunchKernelGGL((k_part_scatter<Src, Dst>), dim3(nblocks), dim3(kBlock), 0, st, src, dst, n, shift, s.counts,
                     s.offsets, nblocks);
  if (e0 && e1) VN_HIP_CHECK(hipEventRecord(e1, st));
  if (stats) {
    stats->launches += 1;
    stats->bytes += n * bytes_per_record;
  }
  return nblocks;
}

// Sources / destinations ---------------------------------------------------------------
struct KV64Dst {  // u32 key + u64 payload
  uint32_t* key;
  uint64_t* pay;
  __device__ __forceinline__ void store(uint64_t pos, uint32_t k, uint64_t p) const {
    key[pos] = k;
    pay[pos] = p;
  }
};
struct KV32Dst {  // u32 key + u32 payload
  uint32_t* key;
  uint32_t* pay;
  __device__ __forceinline__ void store(uint64_t pos, uint32_t k, uint32_t p) const {
    key[pos] = k;
    pay[pos] = p;
  }
};

}  // namespace vn

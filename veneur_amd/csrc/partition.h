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
// Digits are counted, not ranked, so the order a thread loads its records in is free: with V4 a
// lane reads four adjacent keys as one 16-byte load (the key array 16-byte aligned).  A block
// counts kCountTiles tiles in turn (fewer, longer workgroups), one count row entry per tile.
#ifndef VN_PART_COUNT_TILES
#define VN_PART_COUNT_TILES 4
#endif
constexpr uint32_t kCountTiles = VN_PART_COUNT_TILES;
template <class Src, bool V4>
__global__ __launch_bounds__(kBlock) void k_part_count(Src src, uint64_t n, int shift, uint32_t* __restrict__ counts,
                                                       uint32_t nblocks) {
  __shared__ uint32_t s_hist[kCountTiles][4][256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < (int)kCountTiles * 4 * 256; i += kBlock) (&s_hist[0][0][0])[i] = 0;
  __syncthreads();
  for (uint32_t tt = 0; tt < kCountTiles; tt++) {
    const uint64_t tile = (uint64_t)blockIdx.x * kCountTiles + tt;
    if (tile >= nblocks) break;
    const uint64_t base = tile * kTile;
    uint32_t key[kItems];
    bool act[kItems];
    if constexpr (V4) {
#pragma unroll
      for (int g = 0; g < kItems / 4; g++) {
        const uint64_t i0 = base + (uint64_t)g * (4 * kBlock) + 4 * threadIdx.x;
        if (i0 + 4 <= n) {
          const uint4 k4 = src.key4(i0);
          key[4 * g] = k4.x, key[4 * g + 1] = k4.y, key[4 * g + 2] = k4.z, key[4 * g + 3] = k4.w;
        } else {
#pragma unroll
          for (int q = 0; q < 4; q++) key[4 * g + q] = i0 + q < n ? src.key(i0 + q) : 0u;
        }
#pragma unroll
        for (int q = 0; q < 4; q++) act[4 * g + q] = i0 + q < n;
      }
    } else {
#pragma unroll
      for (int j = 0; j < kItems; j++) {
        const uint64_t i = base + (uint64_t)j * kBlock + threadIdx.x;
        key[j] = i < n ? src.key(i) : 0u;
        act[j] = i < n;
      }
    }
    // digit 0 -- the lowest slots, where the interning order puts the first-seen (usually the
    // hottest) keys -- counted by a wave ballot, every other digit one LDS add per record
    uint32_t h0 = 0;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
      const uint32_t d = (key[j] >> shift) & 0xffu;
      h0 += (uint32_t)__popcll(__ballot(act[j] && d == 0u));
      if (act[j] && d != 0u) atomicAdd(&s_hist[tt][w][d], 1u);
    }
    if (lane == 0 && h0) atomicAdd(&s_hist[tt][w][0], h0);
  }
  __syncthreads();
  const uint32_t d = threadIdx.x;
  for (uint32_t tt = 0; tt < kCountTiles; tt++) {
    const uint64_t tile = (uint64_t)blockIdx.x * kCountTiles + tt;
    if (tile < nblocks)
      counts[tile * 256 + d] = s_hist[tt][0][d] + s_hist[tt][1][d] + s_hist[tt][2][d] + s_hist[tt][3][d];
  }
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

// With V4 (a Src whose records may leave a tile in any order within their digit -- counters'
// wrapping sums -- and every array 16-byte aligned) a lane loads four adjacent records at once:
// item j of a lane is record wbase + 256 (j / 4) + 4 lane + j % 4 instead of wbase + 64 j + lane,
// and a record's rank within its digit is taken without the stable match (below).
template <class Src, class Dst, bool V4>
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
  auto li_of = [&](int j) -> uint32_t {
    return V4 ? wbase + (uint32_t)(j >> 2) * 256 + 4 * lane + (uint32_t)(j & 3) : wbase + (uint32_t)j * 64 + lane;
  };
  uint32_t key[kItems];
  P pay[kItems];
  if constexpr (V4) {
#pragma unroll
    for (int g = 0; g < kItems / 4; g++) {
      const uint32_t l0 = li_of(4 * g);
      if (l0 + 4 <= tile_n) {
        src.load4(base + l0, &key[4 * g], &pay[4 * g]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          key[4 * g + q] = 0;
          pay[4 * g + q] = P{};
          if (l0 + q < tile_n) src.load(base + l0 + q, key[4 * g + q], pay[4 * g + q]);
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kItems; j++) {
      const uint32_t li = li_of(j);
      key[j] = 0;
      pay[j] = P{};
      if (li < tile_n) src.load(base + li, key[j], pay[j]);
    }
  }
  {
    uint32_t c = counts[(uint64_t)blockIdx.x * 256 + t];
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
    s_glob[t] = offsets[(uint64_t)blockIdx.x * 256 + t];
    s_run[0][t] = s_run[1][t] = s_run[2][t] = s_run[3][t] = 0;
  }
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t rank[kItems];
  if constexpr (V4) {
    // (order-free records) a record's place within its wave's run of its digit: digit 0 by the
    // wave's ballot and a running count in a scalar register, any other digit the value an LDS
    // add returns -- no match over the digit's bits
    uint32_t h0 = 0;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
      const bool active = li_of(j) < tile_n;
      const uint32_t d = (key[j] >> shift) & 0xffu;
      const uint64_t z = __ballot(active && d == 0u);
      rank[j] = h0 + (uint32_t)__popcll(z & lt);
      if (active && d != 0u) rank[j] = atomicAdd(&s_run[w][d], 1u);
      h0 += (uint32_t)__popcll(z);
    }
    if (lane == 0) s_run[w][0] = h0;
  } else {
#pragma unroll
    for (int j = 0; j < kItems; j++) {
      const bool active = li_of(j) < tile_n;
      const uint32_t d = active ? (key[j] >> shift) & 0xffu : 0u;
      const uint64_t peers = part_match8(d, active);
      const uint32_t before = active ? s_run[w][d] : 0u;
      rank[j] = before + (uint32_t)__popcll(peers & lt);
      asm volatile("" ::: "memory");  // the wave's reads of s_run precede its leaders' update
      if (active && (peers & lt) == 0) s_run[w][d] = before + (uint32_t)__popcll(peers);
      asm volatile("" ::: "memory");
    }
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
    if (li_of(j) < tile_n) {
      const uint32_t d = (key[j] >> shift) & 0xffu;
      const uint32_t pos = s_run[w][d] + rank[j];
      if (VN_BAD(pos < kTile, "part_scatter tile position", pos, kTile)) continue;
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
      const uint64_t g = (uint64_t)s_glob[d] + (li - s_loc[d]);
      if (VN_BAD(g < n, "part_scatter store", g, n)) continue;
      dst.key[g] = s_key[li];
    }
  } else {
    for (uint32_t li = t; li < tile_n; li += kBlock) {
      uint32_t k = s_key[li];
      uint32_t d = (k >> shift) & 0xffu;
      const uint64_t g = (uint64_t)s_glob[d] + (li - s_loc[d]);
      if (VN_BAD(g < n, "part_scatter store", g, n)) continue;
      dst.store(g, k, s_pay[li]);
    }
  }
}

// The tile counts are tile-major (counts[tile * 256 + d]: a tile's 256 counts one coalesced row,
// written by k_part_count and read by k_part_scatter as such); the digit-major exclusive scan
// over them goes through tile groups: k_part_gsum sums each digit over a group of kScanTiles
// tiles (one row per step, coalesced), those 256 x groups sums are scanned digit-major, and
// k_part_goff walks each group again writing every tile's offset row.
constexpr uint32_t kScanTiles = 64;
__global__ __launch_bounds__(256) void k_part_gsum(const uint32_t* __restrict__ counts, uint32_t ntiles,
                                                    uint32_t* __restrict__ gs, uint32_t ngroups) {
  const uint32_t d = threadIdx.x, g = blockIdx.x, t0 = g * kScanTiles, t1 = min(ntiles, t0 + kScanTiles);
  uint32_t s = 0;
#pragma unroll 8
  for (uint32_t t = t0; t < t1; t++) s += counts[(uint64_t)t * 256 + d];
  gs[(uint64_t)d * ngroups + g] = s;
}
__global__ __launch_bounds__(256) void k_part_goff(const uint32_t* __restrict__ counts, uint32_t ntiles,
                                                    const uint32_t* __restrict__ gx, uint32_t ngroups,
                                                    uint32_t* __restrict__ offsets) {
  const uint32_t d = threadIdx.x, g = blockIdx.x, t0 = g * kScanTiles, t1 = min(ntiles, t0 + kScanTiles);
  uint32_t run = gx[(uint64_t)d * ngroups + g];
  for (uint32_t t = t0; t < t1; t++) {
    const uint64_t at = (uint64_t)t * 256 + d;
    const uint32_t c = counts[at];
    offsets[at] = run;
    run += c;
  }
}

// One partition pass: counts, digit-major scan, scatter.  Returns the bucket bounds: bucket d
// of the output is [b[d * stride], b[(d + 1) * stride]) with b = s.gsum + 256 * stride + 1
// (the scanned group sums; b[256 * stride] = n), stride the return value.
template <class Src, class Dst>
uint32_t partition_pass(const Src& src, const Dst& dst, uint64_t n, int shift, RadixScratch& s, hipStream_t st,
                        RadixStats* stats, uint64_t bytes_per_record) {
  radix_scratch_reserve(s, n);
  const uint32_t nblocks = (uint32_t)blocks_for(n, kTile);
  const uint32_t ngroups = (nblocks + kScanTiles - 1) / kScanTiles;
  const size_t gw = 2 * ((size_t)256 * ngroups + 1);
  if (s.gsum_cap < gw) {
    if (s.gsum) VN_HIP_CHECK(hipFree(s.gsum));
    VN_HIP_CHECK(hipMalloc(&s.gsum, gw * sizeof(uint32_t)));
    s.gsum_cap = gw;
  }
  uint32_t* gs = s.gsum;
  uint32_t* gx = s.gsum + (size_t)256 * ngroups + 1;
  const uint32_t cblocks = (nblocks + kCountTiles - 1) / kCountTiles;
  if (src.key16())
    hipLaunchKernelGGL((k_part_count<Src, true>), dim3(cblocks), dim3(kBlock), 0, st, src, n, shift, s.counts, nblocks);
  else
    hipLaunchKernelGGL((k_part_count<Src, false>), dim3(cblocks), dim3(kBlock), 0, st, src, n, shift, s.counts,
                       nblocks);
  hipLaunchKernelGGL(k_part_gsum, dim3(ngroups), dim3(256), 0, st, s.counts, nblocks, gs, ngroups);
  scan_exclusive_u32(gs, gx, (uint64_t)256 * ngroups, s.scan, st);
  hipLaunchKernelGGL(k_part_goff, dim3(ngroups), dim3(256), 0, st, s.counts, nblocks, gx, ngroups, s.offsets);
  hipEvent_t e0 = (stats && stats->pool) ? stats->pool->next() : nullptr;
  hipEvent_t e1 = (stats && stats->pool) ? stats->pool->next() : nullptr;
  if (e0 && e1) VN_HIP_CHECK(hipEventRecord(e0, st));
  if (src.vec16())
    hipLaunchKernelGGL((k_part_scatter<Src, Dst, true>), dim3(nblocks), dim3(kBlock), 0, st, src, dst, n, shift,
                       s.counts, s.offsets, nblocks);
  else
    hipLaunchKernelGGL((k_part_scatter<Src, Dst, false>), dim3(nblocks), dim3(kBlock), 0, st, src, dst, n, shift,
                       s.counts, s.offsets, nblocks);
  if (e0 && e1) VN_HIP_CHECK(hipEventRecord(e1, st));
  if (stats) {
    stats->launches += 1;
    stats->bytes += n * bytes_per_record;
  }
  return ngroups;
}
inline const uint32_t* partition_bounds(const RadixScratch& s, uint32_t stride) {
  return s.gsum + (size_t)256 * stride + 1;
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

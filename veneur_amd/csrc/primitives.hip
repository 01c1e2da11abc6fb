// primitives.hip -- scan, compaction and stable LSD radix sort for gfx950.
//
// Radix pass = reduce-then-scan:
//   count:   each 4096-record tile builds its 256-bin digit histogram in LDS
//   scan:    digit-major exclusive scan of the [256][tiles] histogram -> global offsets
//   scatter: the tile ranks its records stably (wave64 ballot match per digit, per-wave
//            counts in LDS), reorders them by digit in LDS, then writes each digit run
//            contiguously so consecutive lanes store consecutive addresses.
#include <cstdlib>
#include "primitives.h"

namespace vn {

// ---------------------------------------------------------------- block scan helpers
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// exclusive scan of one value per thread across a 256-thread block; returns the total.
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t* s_wave, uint32_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = wave_incl_scan_u32(v);
  if (lane == 63) s_wave[w] = inc;
  __syncthreads();
  uint32_t base = 0;
  for (int i = 0; i < w; i++) base += s_wave[i];
  total = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
  __syncthreads();
  return base + inc - v;
}

// ---------------------------------------------------------------- exclusive scan u32
// cond (may be null): when it points at 0 the kernels return at once (radix_sort's conditional
// passes)
__global__ __launch_bounds__(kBlock) void k_scan_reduce(const uint32_t* __restrict__ cond,
                                                        const uint32_t* __restrict__ in, uint64_t n,
                                                        uint32_t* __restrict__ partials) {
  if (cond && !*cond) return;
  __shared__ uint32_t s_wave[4];
  uint64_t base = (uint64_t)blockIdx.x * kTile;
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    uint64_t i = base + (uint64_t)j * kBlock + threadIdx.x;
    if (i < n) sum += in[i];
  }
  uint32_t total;
  (void)block_excl_scan_u32(sum, s_wave, total);
  if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

// single block: exclusive scan of the partials in place, total into partials[np]
__global__ __launch_bounds__(kBlock) void k_scan_partials(const uint32_t* __restrict__ cond, uint32_t* partials,
                                                          uint32_t np) {
  if (cond && !*cond) return;
  __shared__ uint32_t s_wave[4];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < np; base += kBlock) {
    uint32_t i = base + threadIdx.x;
    uint32_t v = i < np ? partials[i] : 0;
    uint32_t total;
    uint32_t ex = block_excl_scan_u32(v, s_wave, total);
    if (i < np) partials[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) partials[np] = carry;
}

__global__ __launch_bounds__(kBlock) void k_scan_down(const uint32_t* __restrict__ cond,
                                                      const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                      uint64_t n, const uint32_t* __restrict__ partials,
                                                      uint32_t np) {
  if (cond && !*cond) return;
  __shared__ uint32_t s_wave[4];
  // blocked layout: thread t owns items [t*16, t*16+16) of the tile
  uint64_t base = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
  uint32_t v[kItems];
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    uint64_t i = base + j;
    v[j] = i < n ? in[i] : 0;
    sum += v[j];
  }
  uint32_t total;
  uint32_t run = partials[blockIdx.x] + block_excl_scan_u32(sum, s_wave, total);
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    uint64_t i = base + j;
    if (i < n) out[i] = run;
    run += v[j];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = partials[np];
}

void scan_exclusive_u32(const uint32_t* in, uint32_t* out, uint64_t n, ScanScratch& s, hipStream_t st,
                        const uint32_t* cond) {
  uint32_t np = (uint32_t)blocks_for(n ? n : 1, kTile);
  if (s.cap < np + 1) {
    if (s.partials) VN_HIP_CHECK(hipFree(s.partials));
    s.cap = np + 1 + 1024;
    VN_HIP_CHECK(hipMalloc(&s.partials, s.cap * sizeof(uint32_t)));
  }
  if (n == 0) {
    VN_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(uint32_t), st));
    return;
  }
  hipLaunchKernelGGL(k_scan_reduce, dim3(np), dim3(kBlock), 0, st, cond, in, n, s.partials);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(kBlock), 0, st, cond, s.partials, np);
  hipLaunchKernelGGL(k_scan_down, dim3(np), dim3(kBlock), 0, st, cond, in, out, n, s.partials, np);
}

// ---------------------------------------------------------------- compaction
__global__ void k_flag_to_u32(const uint32_t* __restrict__ flag, uint32_t* __restrict__ f, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = flag[i] != 0;
}
__global__ void k_compact_scatter(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos, uint64_t n,
                                  uint32_t* __restrict__ list, uint32_t* __restrict__ count) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) list[pos[i]] = (uint32_t)i;
  if (i == 0) count[0] = pos[n];
}
void compact_flags(const uint32_t* flag, uint32_t* pos, uint32_t* list, uint32_t* count, uint64_t n,
                   ScanScratch& s, hipStream_t st) {
  // flags are 0/1 already (engine invariant), scan them directly
  scan_exclusive_u32(flag, pos, n, s, st);
  hipLaunchKernelGGL(k_compact_scatter, dim3(blocks_for(n ? n : 1, 256)), dim3(256), 0, st, flag, pos, n, list,
                     count);
}

// ---------------------------------------------------------------- radix sort
template <bool HASB>
__device__ __forceinline__ uint32_t digit_of(uint64_t a, uint64_t b, bool from_b, int shift, uint32_t mask) {
  uint64_t w = (HASB && from_b) ? b : a;
  return (uint32_t)(w >> shift) & mask;
}

template <bool HASB>
__global__ __launch_bounds__(kBlock) void k_radix_count(const uint64_t* __restrict__ A, const uint64_t* __restrict__ B,
                                                        uint64_t n, bool from_b, int shift, uint32_t mask,
                                                        uint32_t* __restrict__ counts, uint32_t nblocks,
                                                        const uint32_t* __restrict__ cond) {
  if (cond && !*cond) return;  // a conditional sort that is not needed (radix_sort)
  __shared__ uint32_t s_hist[4][256];
  const int w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4 * 256; i += kBlock) (&s_hist[0][0])[i] = 0;
  __syncthreads();
  const uint64_t* src = (HASB && from_b) ? B : A;
  uint64_t base = (uint64_t)blockIdx.x * kTile;
#pragma unroll 4
  for (int j = 0; j < kItems; j++) {
    uint64_t i = base + (uint64_t)j * kBlock + threadIdx.x;
    if (i < n) atomicAdd(&s_hist[w][(uint32_t)(src[i] >> shift) & mask], 1u);
  }
  __syncthreads();
  uint32_t d = threadIdx.x;
  if (d <= mask) counts[(uint64_t)d * nblocks + blockIdx.x] = s_hist[0][d] + s_hist[1][d] + s_hist[2][d] + s_hist[3][d];
}

// lanes of the wave holding the same digit (of `bits` bits) as this lane (among `active` lanes)
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool active, int bits) {
  uint64_t m = __ballot(active);
  for (int bit = 0; bit < bits; bit++) {
    uint64_t bb = __ballot(active && ((d >> bit) & 1u));
    m &= ((d >> bit) & 1u) ? bb : ~bb;
  }
  return m;
}

// Stable scatter of one tile (kTile records) by a digit of <= 8 bits.  NW waves per workgroup;
// each wave owns a contiguous 1/NW of the tile (kTile / (64 NW) records per lane, loaded up
// front so all global loads are in flight together) and ranks its records with wave ballots and
// a per-wave running count per digit in LDS -- DS operations of one wave execute in order, so no
// workgroup barrier is needed while ranking.  The per-(wave, digit) starts are a scan over the
// waves.  The tile is then reordered through one LDS word array -- for 16-byte records A words
// first, then B words, with each position's digit kept beside them -- and written out with
// consecutive lanes on consecutive records of a digit.  16-byte records use 8 waves and stage
// one word array at a time (~46 KiB of LDS, VGPR-bound at 6 waves/SIMD); 8-byte records use 4
// waves (~38 KiB, 4 workgroups per CU).
template <bool HASB, int NW>
__global__ __launch_bounds__(NW * 64) void k_radix_scatter(const uint64_t* __restrict__ A, const uint64_t* __restrict__ B,
                                                           uint64_t* __restrict__ A2, uint64_t* __restrict__ B2,
                                                           uint64_t n, bool from_b, int shift, int bits,
                                                           const uint32_t* __restrict__ counts,
                                                           const uint32_t* __restrict__ offsets, uint32_t nblocks,
                                                           const uint32_t* __restrict__ cond) {
  if (cond && !*cond) return;
  constexpr int kRWaves = NW, kRBlock = NW * 64, kRItems = kTile / kRBlock;
  __shared__ uint64_t s_x[kTile];
  __shared__ uint8_t s_dig[HASB ? kTile : 1];
  __shared__ uint32_t s_run[kRWaves][256];  // per wave: records of each digit ranked so far
  __shared__ uint32_t s_loc[256];           // tile-local start of each digit
  __shared__ uint32_t s_glob[256];          // global start of each digit for this tile
  __shared__ uint32_t s_wave[kRWaves];

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  const uint32_t tile_n = (uint32_t)((n - base) < (uint64_t)kTile ? (n - base) : kTile);
  constexpr uint32_t kWaveTile = kTile / kRWaves;

  uint64_t a[kRItems], b[kRItems];
  const uint32_t wbase = (uint32_t)w * kWaveTile;
#pragma unroll
  for (int j = 0; j < kRItems; j++) {
    const uint32_t li = wbase + (uint32_t)j * 64 + lane;
    a[j] = li < tile_n ? A[base + li] : 0;
    if (HASB) b[j] = li < tile_n ? B[base + li] : 0;
  }
  const uint32_t mask = (1u << bits) - 1u;
  {
    const bool dig = (uint32_t)t <= mask;
    uint32_t c = dig ? counts[(uint64_t)t * nblocks + blockIdx.x] : 0u;
    uint32_t total;
    const uint32_t loc = block_excl_scan_u32(c, s_wave, total);  // digits live in waves 0..3
    if (t < 256) {  // (NW = 4: every thread)
      s_loc[t] = loc;
      s_glob[t] = dig ? offsets[(uint64_t)t * nblocks + blockIdx.x] : 0u;
#pragma unroll
      for (int v = 0; v < kRWaves; v++) s_run[v][t] = 0;
    }
  }
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t rank[kRItems];
  uint8_t dg[kRItems];
#pragma unroll
  for (int j = 0; j < kRItems; j++) {
    const uint32_t li = wbase + (uint32_t)j * 64 + lane;
    const bool active = li < tile_n;
    const uint32_t d = active ? digit_of<HASB>(a[j], HASB ? b[j] : 0, from_b, shift, mask) : 0u;
    dg[j] = (uint8_t)d;
    const uint64_t peers = match_digit(d, active, bits);
    const uint32_t before = active ? s_run[w][d] : 0u;
    rank[j] = before + (uint32_t)__popcll(peers & lt);
    asm volatile("" ::: "memory");  // the wave's reads of s_run precede its leaders' update
    if (active && (peers & lt) == 0) s_run[w][d] = before + (uint32_t)__popcll(peers);
    asm volatile("" ::: "memory");
  }
  __syncthreads();
  if (t < 256) {  // per (wave, digit) start inside the tile: digit start + the earlier waves' counts
    uint32_t run = s_loc[t];
#pragma unroll
    for (int v = 0; v < kRWaves; v++) {
      const uint32_t c = s_run[v][t];
      s_run[v][t] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRItems; j++) {
    const uint32_t li = wbase + (uint32_t)j * 64 + lane;
    if (li < tile_n) {
      rank[j] += s_run[w][dg[j]];
      s_x[rank[j]] = a[j];
      if (HASB) s_dig[rank[j]] = dg[j];
    }
  }
  __syncthreads();
  for (uint32_t li = t; li < tile_n; li += kRBlock) {
    const uint64_t av = s_x[li];
    const uint32_t d = HASB ? (uint32_t)s_dig[li] : digit_of<false>(av, 0, false, shift, mask);
    A2[(uint64_t)s_glob[d] + (li - s_loc[d])] = av;
  }
  if (HASB) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRItems; j++) {
      const uint32_t li = wbase + (uint32_t)j * 64 + lane;
      if (li < tile_n) s_x[rank[j]] = b[j];
    }
    __syncthreads();
    for (uint32_t li = t; li < tile_n; li += kRBlock) {
      const uint32_t d = s_dig[li];
      B2[(uint64_t)s_glob[d] + (li - s_loc[d])] = s_x[li];
    }
  }
}

void radix_scratch_reserve(RadixScratch& s, uint64_t max_n) {
  size_t blocks = (size_t)blocks_for(max_n ? max_n : 1, kTile);
  if (s.blocks_cap >= blocks) return;
  radix_scratch_free(s);
  s.blocks_cap = blocks;
  VN_HIP_CHECK(hipMalloc(&s.counts, 256 * blocks * sizeof(uint32_t)));
  VN_HIP_CHECK(hipMalloc(&s.offsets, (256 * blocks + 1) * sizeof(uint32_t)));
}

void radix_scratch_free(RadixScratch& s) {
  if (s.counts) (void)hipFree(s.counts);
  if (s.offsets) (void)hipFree(s.offsets);
  if (s.scan.partials) (void)hipFree(s.scan.partials);
  if (s.gsum) (void)hipFree(s.gsum);
  s = RadixScratch{};
}


bool radix_sort(uint64_t* a0, uint64_t* b0, uint64_t* a1, uint64_t* b1, uint64_t n, const RadixPass* passes,
                int npasses, RadixScratch& s, hipStream_t st, RadixStats* stats, const uint32_t* cond) {
  if (n == 0 || npasses == 0) return false;
  radix_scratch_reserve(s, n);
  const uint32_t nblocks = (uint32_t)blocks_for(n, kTile);
  const bool hasb = b0 != nullptr;
  bool flipped = false;
  for (int p = 0; p < npasses; p++) {
    const RadixPass ps = passes[p];
    uint64_t* sa = flipped ? a1 : a0;
    uint64_t* sb = flipped ? b1 : b0;
    uint64_t* da = flipped ? a0 : a1;
    uint64_t* db = flipped ? b0 : b1;
    const uint32_t mask = (1u << ps.bits) - 1u;
    if (hasb)
      hipLaunchKernelGGL(k_radix_count<true>, dim3(nblocks), dim3(kBlock), 0, st, sa, sb, n, ps.from_b, ps.shift, mask,
                         s.counts, nblocks, cond);
    else
      hipLaunchKernelGGL(k_radix_count<false>, dim3(nblocks), dim3(kBlock), 0, st, sa, sb, n, ps.from_b, ps.shift,
                         mask, s.counts, nblocks, cond);
    scan_exclusive_u32(s.counts, s.offsets, (uint64_t)(mask + 1) * nblocks, s.scan, st, cond);
    hipEvent_t e0 = (stats && stats->pool) ? stats->pool->next() : nullptr;
    hipEvent_t e1 = (stats && stats->pool) ? stats->pool->next() : nullptr;
    if (e0 && e1) VN_HIP_CHECK(hipEventRecord(e0, st));
    if (hasb)
      hipLaunchKernelGGL((k_radix_scatter<true, 8>), dim3(nblocks), dim3(512), 0, st, sa, sb, da, db, n, ps.from_b,
                         ps.shift, ps.bits, s.counts, s.offsets, nblocks, cond);
    else  // 8-byte records also scatter with 8 waves (measured ~1% faster on C3 than 4)
      hipLaunchKernelGGL((k_radix_scatter<false, 8>), dim3(nblocks), dim3(512), 0, st, sa, sb, da, db, n, ps.from_b,
                         ps.shift, ps.bits, s.counts, s.offsets, nblocks, cond);
    if (e0 && e1) VN_HIP_CHECK(hipEventRecord(e1, st));
    if (stats) {
      stats->launches += 1;
      stats->bytes += n * (hasb ? 32ull : 16ull);  // read + write of every record
    }
    flipped = !flipped;
  }
  return flipped;
}

// ---------------------------------------------------------------- u32 sizes -> u64 offsets
// (export payload offsets may pass 4 GiB): per-tile sums, one-workgroup scan of the tile sums,
// then each tile writes its running offsets
__global__ __launch_bounds__(kBlock) void k_size_tiles(const uint32_t* __restrict__ size, uint64_t n,
                                                       uint64_t* __restrict__ tile) {
  __shared__ uint64_t s_w[4];
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  uint64_t sum = 0;
  for (uint32_t j = threadIdx.x; j < (uint32_t)kTile; j += kBlock)
    if (base + j < n) sum += size[base + j];
  for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) tile[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}
__global__ void k_size_tiles_scan(uint64_t* __restrict__ tile, uint32_t ntiles) {
  if (threadIdx.x != 0) return;
  uint64_t run = 0;
  for (uint32_t i = 0; i < ntiles; i++) {
    const uint64_t v = tile[i];
    tile[i] = run;
    run += v;
  }
  tile[ntiles] = run;
}
__global__ void k_size_offsets(const uint32_t* __restrict__ size, uint64_t n, const uint64_t* __restrict__ tile,
                               uint32_t ntiles, uint64_t* __restrict__ off) {
  if (threadIdx.x != 0) return;  // one lane walks its tile (export sizes: latency, not bandwidth)
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  uint64_t run = tile[blockIdx.x];
  for (uint32_t j = 0; j < (uint32_t)kTile && base + j < n; j++) {
    off[base + j] = run;
    run += size[base + j];
  }
  if (blockIdx.x == ntiles - 1) off[n] = tile[ntiles];
}
void scan_sizes_u64(const uint32_t* size, uint64_t* off, uint64_t n, hipStream_t st) {
  if (n == 0) {
    VN_HIP_CHECK(hipMemsetAsync(off, 0, sizeof(uint64_t), st));
    return;
  }
  const uint32_t ntiles = (uint32_t)blocks_for(n, kTile);
  uint64_t* tile = nullptr;
  VN_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&tile), (ntiles + 1) * sizeof(uint64_t), st));
  hipLaunchKernelGGL(k_size_tiles, dim3(ntiles), dim3(kBlock), 0, st, size, n, tile);
  hipLaunchKernelGGL(k_size_tiles_scan, dim3(1), dim3(64), 0, st, tile, ntiles);
  hipLaunchKernelGGL(k_size_offsets, dim3(ntiles), dim3(64), 0, st, size, n, tile, ntiles, off);
  VN_HIP_CHECK(hipFreeAsync(tile, st));
}

}  // namespace vn

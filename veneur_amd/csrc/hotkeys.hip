// hotkeys.hip -- the engine's own hot-key detector: the split list of the next window.
//
// The reference routes every record of a key to one worker (server.go:655, Digest % N); the
// split of a hot counter / timer / set key over the ranks (split.hip) is this build's addition,
// so it needs a live detector instead of a list picked ahead of time.  While detection is on
// (vn_hot_detect), every stride-th record of each ingest call -- vn_ingest / vn_ingest_host and
// the split records of vn_ingest_split, whose keys map through the split list to their slots --
// adds one to its slot's count.  vn_flush closes the window's counts; vn_hot_keys then returns
// the slots of a class whose estimated window count (count x stride) reaches a threshold,
// hottest first.  The counting is a strided sample, so one launch touches n / stride records
// with as many device atomics (stride 1: exact counts); the positions are fixed, so the same
// window gives the same list.
#include <algorithm>
#include <vector>

#include "kernels.h"

namespace vn {

namespace {

// one block: kHotItems samples per thread, counted in an LDS table first (a Zipf-hot slot
// would otherwise serialise one device atomic per sample), then one atomic per table entry
constexpr int kHotItems = 16;
constexpr uint32_t kHotTable = 2048, kHotEmpty = 0xffffffffu;
__global__ __launch_bounds__(256) void k_hot_sample(uint64_t n, const uint32_t* __restrict__ key,
                                                    const uint32_t* __restrict__ map, uint32_t nmap, uint32_t stride,
                                                    uint32_t cap, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t tk[kHotTable], tc[kHotTable];
  for (uint32_t h = threadIdx.x; h < kHotTable; h += 256) {
    tk[h] = kHotEmpty;
    tc[h] = 0;
  }
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * 256 * kHotItems;
#pragma unroll 4
  for (int j = 0; j < kHotItems; j++) {
    const uint64_t i = (b0 + (uint64_t)j * 256 + threadIdx.x) * stride;
    if (i >= n) break;
    uint32_t s = key[i];
    if (map) s = s < nmap ? map[s] : kHotEmpty;
    if (s >= cap) continue;
    uint32_t h = (s * 2654435761u) >> 21;  // 11 bits
    bool done = false;
    for (int p = 0; p < 8 && !done; p++, h = (h + 1) & (kHotTable - 1)) {
      uint32_t k = tk[h];
      if (k == kHotEmpty) k = atomicCAS(&tk[h], kHotEmpty, s);
      if (k == kHotEmpty || k == s) {
        atomicAdd(&tc[h], 1u);
        done = true;
      }
    }
    if (!done) atomicAdd(&cnt[s], 1u);
  }
  __syncthreads();
  for (uint32_t h = threadIdx.x; h < kHotTable; h += 256)
    if (tk[h] != kHotEmpty) atomicAdd(&cnt[tk[h]], tc[h]);
}

// candidates: (count << 32 | slot) of every slot with count >= thr, appended (any order)
__global__ void k_hot_compact(uint32_t cap, const uint32_t* __restrict__ cnt, uint32_t thr,
                              uint64_t* __restrict__ out, uint32_t* __restrict__ nout) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= cap) return;
  const uint32_t c = cnt[s];
  if (c && c >= thr) out[atomicAdd(nout, 1u)] = ((uint64_t)c << 32) | s;
}

}  // namespace

void hot_enable(vn_engine* e, uint32_t stride) {
  if (stride && !e->hk_list) {
    for (int w = 0; w < 2; w++)
      for (int c = 0; c < VN_NCLASS; c++) {
        const size_t n = std::max<uint32_t>(e->cap[c], 1u);
        VN_HIP_CHECK(hipMalloc(&e->hk_cnt[w][c], n * sizeof(uint32_t)));
        VN_HIP_CHECK(hipMemsetAsync(e->hk_cnt[w][c], 0, n * sizeof(uint32_t), e->st));
      }
    uint32_t mx = 1;
    for (int c = 0; c < VN_NCLASS; c++) mx = std::max(mx, e->cap[c]);
    VN_HIP_CHECK(hipMalloc(&e->hk_list, (size_t)mx * sizeof(uint64_t) + 8));
    VN_HIP_CHECK(hipStreamSynchronize(e->st));
  }
  e->hot_stride = stride;
}

void hot_sample(vn_engine* e, int cls, uint64_t n, const uint32_t* key, const uint32_t* map, uint32_t nmap,
                hipStream_t st) {
  const uint32_t stride = e->hot_stride;
  if (!stride || !n || !key || !e->cap[cls]) return;
  const uint64_t m = (n + stride - 1) / stride;
  hipLaunchKernelGGL(k_hot_sample, dim3(blocks_for(m, 256 * kHotItems)), dim3(256), 0, st, n, key, map, nmap, stride, e->cap[cls],
                     e->hk_cnt[e->hk_cur][cls]);
}

void hot_rotate(vn_engine* e) {
  if (!e->hk_list) return;
  e->hk_prev_stride = e->hot_stride;
  e->hk_cur ^= 1;
  // the split records of the next window count on the split engine's stream: the clear is done
  // before vn_flush returns
  for (int c = 0; c < VN_NCLASS; c++)
    if (e->cap[c]) VN_HIP_CHECK(hipMemsetAsync(e->hk_cnt[e->hk_cur][c], 0, e->cap[c] * sizeof(uint32_t), e->st));
  VN_HIP_CHECK(hipStreamSynchronize(e->st));
}

uint32_t hot_collect(vn_engine* e, int cls, uint64_t min_count, uint32_t cap, uint32_t* slot, uint64_t* count) {
  if (!e->hk_list || !e->hk_prev_stride || !e->cap[cls]) return 0;
  const uint64_t stride = e->hk_prev_stride;
  const uint64_t thr64 = (min_count + stride - 1) / stride;  // count * stride >= min_count
  const uint32_t thr = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(thr64, 1), 0xffffffffull);
  uint32_t* nout = reinterpret_cast<uint32_t*>(e->hk_list);  // first 8 bytes: the count
  uint64_t* list = e->hk_list + 1;
  hipStream_t st = e->st;
  VN_HIP_CHECK(hipMemsetAsync(nout, 0, sizeof(uint32_t), st));
  hipLaunchKernelGGL(k_hot_compact, dim3(blocks_for(e->cap[cls], 256)), dim3(256), 0, st, e->cap[cls],
                     e->hk_cnt[e->hk_cur ^ 1][cls], thr, list, nout);
  uint32_t n = 0;
  VN_HIP_CHECK(hipMemcpyAsync(&n, nout, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
  std::vector<uint64_t> h(n);
  if (n) {
    VN_HIP_CHECK(hipMemcpyAsync(h.data(), list, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    VN_HIP_CHECK(hipStreamSynchronize(st));
  }
  // hottest first, ties by ascending slot
  std::sort(h.begin(), h.end(), [](uint64_t a, uint64_t b) {
    const uint32_t ca = (uint32_t)(a >> 32), cb = (uint32_t)(b >> 32);
    return ca != cb ? ca > cb : (uint32_t)a < (uint32_t)b;
  });
  const uint32_t k = std::min<uint32_t>(n, cap);
  for (uint32_t i = 0; i < k; i++) {
    if (slot) slot[i] = (uint32_t)h[i];
    if (count) count[i] = (h[i] >> 32) * stride;
  }
  return k;
}

void hot_destroy(vn_engine* e) {
  for (int w = 0; w < 2; w++)
    for (int c = 0; c < VN_NCLASS; c++)
      if (e->hk_cnt[w][c]) {
        (void)hipFree(e->hk_cnt[w][c]);
        e->hk_cnt[w][c] = nullptr;
      }
  if (e->hk_list) (void)hipFree(e->hk_list);
  e->hk_list = nullptr;
}

}  // namespace vn

// primitives.h -- device-wide building blocks of the engine (HIP, gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vn {

// Debug builds (VN_DEBUG_CHECKS) guard the indices of the round-6 kernels: a bad one is printed
// and its access skipped, so a broken invariant is named instead of faulting the GPU.
#ifdef VN_DEBUG_CHECKS
__device__ inline bool vn_bad(bool ok, const char* what, unsigned long long a, unsigned long long b) {
  if (!ok) printf("VN_CHECK %s: %llu vs %llu (block %u thread %u)\n", what, a, b, blockIdx.x, threadIdx.x);
  return !ok;
}
#define VN_BAD(ok, what, a, b) ::vn::vn_bad((ok), (what), (unsigned long long)(a), (unsigned long long)(b))
#else
#define VN_BAD(ok, what, a, b) false
#endif

constexpr int kBlock = 256;               // 4 waves
constexpr int kItems = 16;                // items per thread in a tile
constexpr int kTile = kBlock * kItems;    // 4096 records per tile / chunk

// ---- exclusive scan of u32 (out may alias nothing); out[n] receives the total.
struct ScanScratch {
  uint32_t* partials = nullptr;  // >= ceil(n / kTile) + 1
  size_t cap = 0;
};
void scan_exclusive_u32(const uint32_t* in, uint32_t* out, uint64_t n, ScanScratch& s, hipStream_t st,
                        const uint32_t* cond = nullptr);

// ---- stable LSD radix sort over 64-bit words.
// Records are (A[i], B[i]) pairs (B may be null for key-only sorts).  Each pass sorts
// stably by an 8-bit digit taken from A (from_b = false) or B (from_b = true) at `shift`.
struct RadixPass {
  bool from_b;
  int shift;
  int bits = 8;  // digit width (<= 8): fewer buckets give longer contiguous write runs
};
// Split the key field [lo, lo + nbits) of A (from_b false) or B into the fewest passes of
// <= 8 bits, all of the same width (e.g. 18 slot bits -> 3 passes of 6 bits); returns the count.
inline int make_passes(RadixPass* out, bool from_b, int lo, int nbits) {
  if (nbits <= 0) return 0;
  const int np = (nbits + 7) / 8, w = (nbits + np - 1) / np;
  for (int p = 0; p < np; p++) out[p] = RadixPass{from_b, lo + p * w, w};
  return np;
}
struct RadixScratch {
  uint32_t* counts = nullptr;    // 256 * blocks
  uint32_t* offsets = nullptr;   // 256 * blocks + 1
  ScanScratch scan;
  size_t blocks_cap = 0;
  uint32_t* gsum = nullptr;      // partition.h: per (digit, tile group) sums, then their scan
  size_t gsum_cap = 0;           //   (2 * (256 * groups + 1) words)
};
// Sorts n records; ping-pongs between (a0,b0) and (a1,b1).  Returns true if the result
// ended in (a1, b1).  If timing events are supplied, the scatter kernels are bracketed.
// Optional timing: the scatter launches are bracketed by events taken from a pool that the
// caller resolves after its own synchronisation (no sync inside the sort).
struct EventPool {
  hipEvent_t* ev = nullptr;
  int cap = 0, used = 0;
  hipEvent_t next() { return used < cap ? ev[used++] : nullptr; }
};
struct RadixStats {
  EventPool* pool = nullptr;     // pairs (begin, end) appended per scatter launch
  uint64_t launches = 0;
  uint64_t bytes = 0;            // algorithmic bytes of those launches (read + write)
};
bool radix_sort(uint64_t* a0, uint64_t* b0, uint64_t* a1, uint64_t* b1, uint64_t n,
                const RadixPass* passes, int npasses, RadixScratch& s, hipStream_t st,
                RadixStats* stats, const uint32_t* cond = nullptr);
// cond (device word, may be null): every kernel of the sort returns at once when it reads 0, so
// the sort is queued without a host round trip and runs only when a kernel before it set the
// word.  With an even pass count the result is in (a0, b0) either way.

void radix_scratch_reserve(RadixScratch& s, uint64_t max_n);
void radix_scratch_free(RadixScratch& s);

// ---- compaction: list[] receives the indices i < n with flag[i] != 0 (ascending);
// count[0] receives the number of them.  pos must hold n+1 u32.
void compact_flags(const uint32_t* flag, uint32_t* pos, uint32_t* list, uint32_t* count, uint64_t n,
                   ScanScratch& s, hipStream_t st);

inline int blocks_for(uint64_t n, int per_block) { return (int)((n + per_block - 1) / per_block); }

}  // namespace vn

#define VN_HIP_CHECK(expr)                                                   \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) throw vn::HipError(_e, #expr, __FILE__, __LINE__); \
  } while (0)

namespace vn {
struct HipError {
  hipError_t err;
  const char* expr;
  const char* file;
  int line;
  HipError(hipError_t e, const char* x, const char* f, int l) : err(e), expr(x), file(f), line(l) {}
};
}  // namespace vn

// set_dense.h -- axiomhq Sketch.insert over a stream of sparse codes for one key whose dense
// registers sit in LDS, run by one 256-thread workgroup.  Shared by Set.Sample ingest
// (ingest_set.hip) and Set.Combine of a sparse sketch into a dense one (import_set.hip).
//
// Reference: vendor/github.com/axiomhq/hyperloglog/hyperloglog.go:168-183 (insert) with
// registers.go:56-123 (rebase, set, min).  Per chunk of kTile codes the workgroup finds T_full
// (the code that fills the last zero register -- first filler per register via an LDS atomic
// max on a marker) and the first rebase candidate after it; codes before that point are plain
// commutative max updates (LDS atomic max), the rebase itself is a parallel min + subtract.
// Identical to the sequential semantics, rebase epochs included.
#pragma once
#include "kernels.h"

namespace vn {

constexpr uint32_t kMark = 0x80000000u;

// profiling build only (VN_SET_PROF, tools/set_profile.py): workgroup 0's dense phase by path --
// 0 chunks, 1 passes, 2 fill-path cycles, 3 exact-marking cycles, 4 full-path cycles (T_full,
// candidates, plain max), 5 rebases, 6 rebase cycles, 7 chunk-top cycles (decode, prefetch issue)
#ifdef VN_SET_PROF
static __device__ unsigned long long g_dense_prof[8];
#define DPROF_T(v) const long long v = clock64()
#define DPROF_ADD(i, a, b) \
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_dense_prof[i], (unsigned long long)((b) - (a)))
#define DPROF_INC(i) \
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_dense_prof[i], 1ull)
#else
#define DPROF_T(v)
#define DPROF_ADD(i, a, b)
#define DPROF_INC(i)
#endif

// bitonic sort of 256 u32 in LDS, ascending (all 256 threads).  A step with j < 64 pairs lanes of
// one wave, whose LDS accesses complete in order: unless the next step pairs across waves (j = 64
// or 128) or the sort ends, it ends with a wave wait instead of a workgroup barrier (6 barriers
// instead of 36)
__device__ __forceinline__ void bitonic256(uint32_t* a) {
  const uint32_t t = threadIdx.x;
  for (uint32_t k = 2; k <= 256; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      uint32_t ixj = t ^ j;
      if (ixj > t) {
        uint32_t x = a[t], y = a[ixj];
        bool up = (t & k) == 0;
        if ((x > y) == up) {
          a[t] = y;
          a[ixj] = x;
        }
      }
      if (j >= 64 || (j == 1 && k >= 64)) __syncthreads();
      else wave_lds_sync();
    }
  }
}

__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* a, uint32_t n, uint32_t v) {
  uint32_t l = 0, h = n;
  while (l < h) {
    uint32_t m = (l + h) >> 1;
    if (a[m] < v) l = m + 1;
    else h = m;
  }
  return l;
}


// LDS state of the key (all pointers into __shared__ memory of the calling kernel)
struct DenseLds {
  uint32_t* U;  // kHllM registers, one u32 each
  uint32_t *b, *nz;
  uint32_t *filled, *tfull, *pstar, *newfill, *mn;
  uint32_t* red;  // 4
};

// insert(decode(src(p))) for p in [pos0, n), in order; src(p) -> sparse code (u32).  DI codes per
// thread per chunk; the next chunk's codes are loaded while a chunk is processed, so a key's
// stream runs at one workgroup's memory parallelism: bigger chunks keep more bytes in flight
// (and take fewer barriers per code)
#ifndef VN_SET_DENSE_BUFS
// chunks of codes in flight in the dense phase (2 or 3).  Three measured not better: the heavy
// key's workgroup 7.66 ms either way, C4 74.4 / 73.7 ms per window with two against 74.7 / 75.2
// with three (profiles/r06_sets/)
#define VN_SET_DENSE_BUFS 2
#endif
template <int DI, class Src>
__device__ __forceinline__ void dense_insert_codes(const DenseLds& S, const Src& src, uint32_t pos0, uint32_t n,
                                                   uint32_t* err) {
  const uint32_t t = threadIdx.x;
  constexpr uint32_t kDT = DI * kBlock;  // records per chunk
  uint32_t* U = S.U;
  // kBufs chunks in flight: chunk k's codes sit in buffer k % kBufs, loaded kBufs chunks ahead,
  // so a load has that many chunks' phases to land in (a heavy key's workgroup is otherwise bound
  // by its loads' latency: round 6, two buffers, ~5.2k cycles per 4096-code chunk waiting at the top)
  constexpr uint32_t kBufs = VN_SET_DENSE_BUFS >= 3 ? 3u : 2u;
  uint32_t rawA[DI], rawB[DI];
#if VN_SET_DENSE_BUFS >= 3
  uint32_t rawC[DI];
#endif
  auto load = [&](uint32_t (&raw)[DI], uint32_t c0) {
#pragma unroll
    for (int j = 0; j < DI; j++) {
      const uint32_t p = c0 + j * kBlock + t;
      raw[j] = p < n ? src(p) : 0u;
    }
  };
  load(rawA, pos0);
  load(rawB, pos0 + kDT);
#if VN_SET_DENSE_BUFS >= 3
  load(rawC, pos0 + 2 * kDT);
#endif
  auto chunk = [&](uint32_t (&raw)[DI], const uint32_t cpos0) {
    DPROF_T(d_top);
    DPROF_INC(0);
    const uint32_t cend = min(n, cpos0 + kDT);
    uint32_t ri[DI], rr[DI];
#pragma unroll
    for (int j = 0; j < DI; j++) {
      uint32_t p = cpos0 + j * kBlock + t;
      ri[j] = 0;
      rr[j] = 0;
      if (p < cend) decode_hash(raw[j], &ri[j], &rr[j]);
    }
    load(raw, cpos0 + kBufs * kDT);  // kBufs chunks ahead, into the registers just decoded
    uint32_t cpos = cpos0;
    DPROF_T(d_loop);
    DPROF_ADD(7, d_top, d_loop);
    for (;;) {
      DPROF_T(d_p0);
      DPROF_INC(1);
      const uint32_t b = (*S.b);
      uint32_t tfull;
      if ((*S.nz) > 0) {
        // fast path: if the chunk cannot fill every zero register, no rebase can occur in it and
        // every update is a plain max.  First bound: a register fills only from a code with
        // r > b, so fewer such codes than zero registers cannot complete the fill (one wave
        // ballot count, no LDS pass -- most chunks of a long fill end here); else mark the zero
        // registers the chunk would fill and count them exactly
        if (t == 0) {
          (*S.filled) = 0;
          (*S.newfill) = 0;
        }
        lds_barrier();
        {
          uint32_t h = 0;
#pragma unroll
          for (int j = 0; j < DI; j++) {
            const uint32_t p = cpos0 + j * kBlock + t;
            h += (uint32_t)__popcll(__ballot(p >= cpos && p < cend && rr[j] > b));
          }
          if ((t & 63) == 0 && h) atomicAdd(&(*S.filled), h);
        }
        lds_barrier();
        bool completes = false;
        DPROF_T(d_m0);
        const bool maybe = (*S.filled) >= (*S.nz);  // (every wave reads it before it is reset)
        if (maybe) {
          lds_barrier();
          if (t == 0) (*S.filled) = 0;
          lds_barrier();
#pragma unroll
          for (int j = 0; j < DI; j++) {
            uint32_t p = cpos0 + j * kBlock + t;
            if (p >= cpos && p < cend && rr[j] > b && U[ri[j]] == 0)
              if (atomicOr(&U[ri[j]], kMark) == 0) atomicAdd(&(*S.filled), 1u);
          }
          lds_barrier();
          completes = (*S.filled) >= (*S.nz);
#pragma unroll
          for (int j = 0; j < DI; j++) {
            uint32_t p = cpos0 + j * kBlock + t;
            if (p >= cpos && p < cend && (U[ri[j]] & kMark)) U[ri[j]] = 0;
          }
          lds_barrier();
        }
        DPROF_T(d_m1);
        DPROF_ADD(3, d_m0, d_m1);
        if (!completes) {
#pragma unroll
          for (int j = 0; j < DI; j++) {
            uint32_t p = cpos0 + j * kBlock + t;
            if (p >= cpos && p < cend && rr[j] > b) {
              uint32_t old = atomicMax(&U[ri[j]], min(rr[j] - b, kHllCapacity - 1));
              if (old == 0) atomicAdd(&(*S.newfill), 1u);
            }
          }
          lds_barrier();
          if (t == 0) (*S.nz) -= (*S.newfill);
          lds_barrier();
          DPROF_T(d_f1);
          DPROF_ADD(2, d_p0, d_f1);
          break;
        }
        if (t == 0) {
          (*S.filled) = 0;
          (*S.tfull) = 0;
        }
        // phase A: mark the first filler of every zero register
#pragma unroll
        for (int j = 0; j < DI; j++) {
          uint32_t p = cpos0 + j * kBlock + t;
          if (p >= cpos && p < cend && rr[j] > b) {
            uint32_t v = U[ri[j]];
            if (v == 0 || (v & kMark)) atomicMax(&U[ri[j]], kMark | (0x7fffffffu - p));
          }
        }
        lds_barrier();
        // phase B: count first fillers, latest fill position
#pragma unroll
        for (int j = 0; j < DI; j++) {
          uint32_t p = cpos0 + j * kBlock + t;
          if (p >= cpos && p < cend && rr[j] > b && U[ri[j]] == (kMark | (0x7fffffffu - p))) {
            atomicAdd(&(*S.filled), 1u);
            atomicMax(&(*S.tfull), p);
          }
        }
        lds_barrier();
        tfull = ((*S.filled) == (*S.nz)) ? (*S.tfull) : 0xffffffffu;
#pragma unroll
        for (int j = 0; j < DI; j++) {
          uint32_t p = cpos0 + j * kBlock + t;
          if (p >= cpos && p < cend && (U[ri[j]] & kMark)) U[ri[j]] = 0;
        }
        lds_barrier();
      } else {
        tfull = cpos - 1;  // already full (cpos >= 1 whenever nz == 0 inside a key's stream)
        if (cpos == 0) tfull = 0xfffffffeu;
      }
      if (t == 0) {
        (*S.pstar) = 0xffffffffu;
        (*S.newfill) = 0;
      }
      lds_barrier();
      // phase C: first rebase candidate strictly after T_full
      if (tfull != 0xffffffffu) {
#pragma unroll
        for (int j = 0; j < DI; j++) {
          uint32_t p = cpos0 + j * kBlock + t;
          bool after = (tfull == 0xfffffffeu) ? true : (p > tfull);
          if (p >= cpos && p < cend && after && ((rr[j] - b) & 0xffu) >= kHllCapacity) atomicMin(&(*S.pstar), p);
        }
      }
      lds_barrier();
      const uint32_t pstar = (*S.pstar);
      // phase D: plain max updates before the rebase point
#pragma unroll
      for (int j = 0; j < DI; j++) {
        uint32_t p = cpos0 + j * kBlock + t;
        if (p >= cpos && p < cend && p < pstar && rr[j] > b) {
          uint32_t old = atomicMax(&U[ri[j]], min(rr[j] - b, kHllCapacity - 1));
          if (old == 0) atomicAdd(&(*S.newfill), 1u);
        }
      }
      lds_barrier();
      if (t == 0) (*S.nz) -= (*S.newfill);
      lds_barrier();
      DPROF_T(d_c1);
      DPROF_ADD(4, d_p0, d_c1);
      if (pstar == 0xffffffffu) break;
      DPROF_INC(5);
      // rebase at pstar (nz == 0 here): b += min(regs); regs -= min
      if (t == 0) (*S.mn) = 0xffffffffu;
      lds_barrier();
      {
        uint32_t mn = 0xffffffffu;
        for (uint32_t i = t; i < kHllM; i += kBlock) mn = min(mn, U[i]);
        atomicMin(&(*S.mn), mn);
      }
      lds_barrier();
      const uint32_t db = (*S.mn);
      uint32_t z = 0;
      for (uint32_t i = t; i < kHllM; i += kBlock) {
        uint32_t v = U[i] - db;
        U[i] = v;
        z += v == 0;
      }
      z = block_allreduce_u32_sum(z, S.red);
      if (t == 0) {
        if (db == 0 || db == 0xffffffffu) atomicOr(err, 2u);
        uint32_t nb = b + db;
        (*S.b) = nb;
        (*S.nz) = z;
        // the candidate record itself, after the rebase
        uint32_t pi, pr;
        decode_hash(src(pstar), &pi, &pr);
        if (pr > nb) {
          uint32_t v = min(pr - nb, kHllCapacity - 1);
          if (v > U[pi]) {
            if (U[pi] == 0) (*S.nz) -= 1;
            U[pi] = v;
          }
        }
      }
      lds_barrier();
      DPROF_T(d_r1);
      DPROF_ADD(6, d_c1, d_r1);
      cpos = pstar + 1;
      if (cpos >= cend) break;
    }
  };
  for (uint32_t c = pos0; c < n; c += kBufs * kDT) {
    chunk(rawA, c);
    if (c + kDT < n) chunk(rawB, c + kDT);
#if VN_SET_DENSE_BUFS >= 3
    if (c + 2 * kDT < n) chunk(rawC, c + 2 * kDT);
#endif
  }
}

}  // namespace vn

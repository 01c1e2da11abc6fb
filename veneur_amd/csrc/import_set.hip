// import_set.hip -- Worker.ImportMetric for sets (worker.go:248-252), bit-exact.
//
// Set.Combine (samplers/samplers.go:313-325) = hyperloglog.New() + UnmarshalBinary
// (vendor/github.com/axiomhq/hyperloglog/hyperloglog.go:318-376) + Sketch.Merge (92-149):
//   sparse <- sparse   every tmpSet code and list code of the other joins the tmpSet, then
//                      maybeToNormal (80-87): if len(tmpSet)*100 > m, mergeSparse (229-267)
//                      and, if the list's byte length > m, toNormal (152-166)
//   sparse <- dense    toNormal, then dense <- dense
//   dense  <- sparse   insert(decodeHash(code)) for the other's tmpSet codes (map order in Go;
//                      ascending here and in the oracle) and then its list, in order
//   dense  <- dense    align the bases: the lower side is rebase()d by the difference
//                      (registers.go:56-74: registers below it are left alone), then a
//                      per-register max with registers.set's nz bookkeeping
// A payload whose precision is not 14 makes Merge return "precisions must be equal"; the
// worker logs it and moves on (worker.go:248-252) -- the key is still Upserted, nothing merges.
// A payload UnmarshalBinary would panic on (truncated) fails the whole call (VN_EDECODE).
//
// MI355X formulation: one wave per payload parses and validates it (k_hll_parse); payloads
// are grouped by key with a stable radix sort; one 256-thread workgroup per key then applies
// its payloads in arrival order with the key's list or registers in LDS: varint lists decode
// in parallel (scan of terminator bytes, then a scan of the deltas), unions are merge-path
// merges staged in registers, registers are LDS atomic maxes, and inserts into a dense key
// run the exact insert machinery of set_dense.h (rebase epochs included).
#include "set_dense.h"
#include "wave_dpp.h"

namespace vn {

namespace {

struct HllPart {
  uint32_t kind;      // 0 sparse, 1 dense, 2 skipped (precision != 14)
  uint32_t b;
  uint32_t ntmp;      // tmpSet codes (big-endian u32) at tmp_off
  uint32_t list_len;  // varint list bytes at list_off
  uint32_t regs_len;  // dense: tailcut bytes at regs_off (<= 8192; missing bytes are zero registers)
  uint32_t rr;        // sparse: min rho | max rho << 8 over its codes (0xff: no codes)
  uint32_t ncodes;    // sparse: tmpSet + list codes
  uint64_t tmp_off, list_off, regs_off;
};
static_assert(sizeof(HllPart) <= 64, "ImportScratch.parts holds 64 bytes per payload");

constexpr uint32_t kMaxImportTmp = 256;   // tmpSet codes per payload (Go keeps < 164)
constexpr uint32_t kPer = (kArenaWords + kBlock - 1) / kBlock;  // 65 codes per thread
constexpr uint32_t kCWords = kArenaWords + 512;                 // payload codes + the key's tmpSet
constexpr uint32_t kCPer = (kCWords + kBlock - 1) / kBlock;     // 67
#ifdef VN_SET_LANE_RUNS
constexpr uint32_t kLaneBytes = 2048;  // a dense key's plain run: longer sparse payloads go block-wide
#endif

__device__ __forceinline__ uint32_t be32(const uint8_t* d) {
  return ((uint32_t)d[0] << 24) | ((uint32_t)d[1] << 16) | ((uint32_t)d[2] << 8) | d[3];
}

// f(byte) over global bytes [p, p + len) in order, read as aligned 16-byte blocks, G of them per
// step with the next G blocks' loads in flight while these are consumed (one lane walking its own
// payload: with one block ahead, a lane waited a memory latency every 16 bytes).  The blocks never
// leave the 16-byte-aligned span holding the bytes (so no page the bytes do not touch).
template <uint32_t G = 1, class F>
__device__ __forceinline__ void for_bytes(const uint8_t* p, uint32_t len, F&& f) {
  if (!len) return;
  const uintptr_t s = reinterpret_cast<uintptr_t>(p), a0 = s & ~(uintptr_t)15;
  const uint32_t lo = (uint32_t)(s - a0), end = lo + len, nblk = (end + 15u) >> 4;
  const uint4* b = reinterpret_cast<const uint4*>(a0);
  uint4 cur[G];
#pragma unroll
  for (uint32_t g = 0; g < G; g++) cur[g] = b[min(g, nblk - 1u)];
  for (uint32_t k = 0; k < nblk; k += G) {
    uint4 nxt[G];
#pragma unroll
    for (uint32_t g = 0; g < G; g++) nxt[g] = b[min(k + G + g, nblk - 1u)];
#pragma unroll
    for (uint32_t g = 0; g < G; g++) {
      const uint32_t base = (k + g) << 4;
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint32_t w = j < 4 ? cur[g].x : j < 8 ? cur[g].y : j < 12 ? cur[g].z : cur[g].w;
        const uint32_t pos = base + (uint32_t)j;
        if (pos >= lo && pos < end) f((w >> ((j & 3) * 8)) & 0xffu);
      }
    }
#pragma unroll
    for (uint32_t g = 0; g < G; g++) cur[g] = nxt[g];
  }
}

// The codes of a compressedList's varint bytes [p, p + len), by one whole wave (lanes in step, exec
// full), 256 bytes per step, four bytes per lane; f(code, prev, has_prev) at each code (PREV: the
// code before it in the list, if any).  compressedList.decode (compressed.go:157-165) makes a code
// the running uint32 sum of the varint values, and a varint's value the OR of (byte & 0x7f) << 7 d
// over its bytes (d = the byte's place in it; from d = 5 on Go's uint32 shift adds nothing).  The
// bit ranges are disjoint, so a code is the sum, over every list byte up to its terminator, of that
// byte's contribution: each byte finds where its varint starts (the last terminator before it:
// within the lane, else a wave max-scan of the lanes' last terminators, else the one carried from
// the previous step), and the codes are a wave sum-scan of the contributions read at the
// terminators.  A trailing unterminated varint gives no code.  Returns the number of codes.
template <bool PREV, class F>
__device__ __forceinline__ uint32_t wave_list_codes(const uint8_t* p, uint32_t len, F&& f) {
  const uint32_t lane = threadIdx.x & 63u;
  if (!len) return 0;
  const uintptr_t s = reinterpret_cast<uintptr_t>(p), a0 = s & ~(uintptr_t)3;
  const uint32_t lo = (uint32_t)(s - a0), end = lo + len;  // positions relative to a0
  const uint32_t* w32 = reinterpret_cast<const uint32_t*>(a0);
  uint32_t carry = 0, vstart = lo;  // the code so far; the first byte of the varint in progress
  uint32_t lastc = 0, ncodes = 0;   // (PREV) the last code of the steps before
  bool haslast = false;
  uint32_t nxt = 4 * lane < end ? w32[lane] : 0u;
  for (uint32_t base = 0; base < end; base += 256) {
    const uint32_t p0 = base + 4 * lane, w = nxt;
    nxt = p0 + 256 < end ? w32[(p0 + 256) >> 2] : 0u;  // the next step's dword in flight
    uint32_t tm = 0;  // bit j: byte j is a list byte and a terminator
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t pos = p0 + (uint32_t)j;
      if (pos >= lo && pos < end && !((w >> (8 * j)) & 0x80u)) tm |= 1u << j;
    }
    const uint32_t mine = tm ? p0 + 32u - (uint32_t)__builtin_clz(tm) : 0u;  // my last terminator + 1
    const uint32_t upto = wave_incl_max(mine);
    uint32_t st = max(wave_shr1(upto), vstart);
    uint32_t c[4], sum = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t pos = p0 + (uint32_t)j, by = (w >> (8 * j)) & 0xffu, d = pos - st;
      c[j] = (pos >= lo && pos < end && d < 5u) ? (by & 0x7fu) << (7u * d) : 0u;
      sum += c[j];
      if (tm & (1u << j)) st = pos + 1;
    }
    const uint32_t incl = wave_incl_add_u32(sum);
    uint32_t ph = 0, pc = 0;  // (PREV) the last code at or below this lane, if any
    if (PREV) {
      uint32_t run = incl - sum + carry;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        run += c[j];
        if (tm & (1u << j)) pc = run;
      }
      ph = tm != 0;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t oh = (uint32_t)__shfl_up((int)ph, d, 64), oc = (uint32_t)__shfl_up((int)pc, d, 64);
        if ((int)lane >= d && !ph) {
          ph = oh;
          pc = oc;
        }
      }
    }
    uint32_t eh = PREV ? (uint32_t)__shfl_up((int)ph, 1, 64) : 0u, ec = PREV ? (uint32_t)__shfl_up((int)pc, 1, 64) : 0u;
    if (lane == 0 || !eh) {
      eh = haslast;
      ec = lastc;
    }
    uint32_t run = incl - sum + carry;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      run += c[j];
      if (tm & (1u << j)) {
        f(run, ec, eh != 0);
        ec = run;
        eh = 1;
      }
    }
    ncodes += (uint32_t)__shfl((int)wave_incl_add_u32((uint32_t)__builtin_popcount(tm)), 63);
    if (PREV && __shfl((int)ph, 63)) {
      haslast = true;
      lastc = (uint32_t)__shfl((int)pc, 63);
    }
    carry += (uint32_t)__shfl((int)incl, 63);
    vstart = max(vstart, (uint32_t)__shfl((int)upto, 63));
  }
  return ncodes;
}

// ins(code) for every code of a sparse payload, by one whole wave: the tmpSet's big-endian codes a
// lane each, then the list (wave_list_codes)
template <class Ins>
__device__ __forceinline__ void wave_insert_sparse(const uint8_t* bytes, const HllPart& R, Ins&& ins) {
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t i = lane; i < R.ntmp; i += 64) ins(be32(bytes + R.tmp_off + 4ull * i));
  (void)wave_list_codes<false>(bytes + R.list_off, R.list_len, [&](uint32_t c, uint32_t, bool) { ins(c); });
}

// parse + validate one MarshalBinary payload per wave (hyperloglog.go:318-376, compressed.go:83-97):
// the header by every lane, the tmpSet's codes a lane each, the list by wave_list_codes; the rho
// range and the checks (the list decodes completely into strictly increasing codes) reduced over
// the wave.  (A lane per payload walked 8.5 ms of C5's payloads byte by byte.)
__global__ __launch_bounds__(256) void k_hll_parse(uint64_t n, const uint64_t* __restrict__ off,
                                                   const uint8_t* __restrict__ bytes, HllPart* __restrict__ parts,
                                                   uint32_t* __restrict__ err) {
  const uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;  // (wave-uniform)
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t o = off[i], len = off[i + 1] - o;
  const uint8_t* d = bytes + o;
  HllPart p{};
  p.kind = 2;
  bool bad = len < 4;
  if (!bad && d[1] == kHllP) {
    p.b = d[2];
    if (d[3] == 1) {  // sparse: tmpSet, then the compressed list (count, last, byte length, bytes)
      bad = len < 8;
      if (!bad) {
        const uint64_t tssz = be32(d + 4), last = 8 + 4 * tssz;
        bad = tssz > kMaxImportTmp || len < last + 12;
        if (!bad) {
          const uint64_t sz = be32(d + last + 8);
          bad = sz > kHllM || len < last + 12 + sz;
          if (!bad) {
            const uint8_t* lb = d + last + 12;
            uint32_t rlo = 0, rmax = 0;  // (rlo: 255 - the smallest rho, so both reduce by max)
            bool lbad = false;
            for (uint32_t t = lane; t < (uint32_t)tssz; t += 64) {
              uint32_t ri, r;
              decode_hash(be32(d + 8 + 4ull * t), &ri, &r);
              rlo = max(rlo, 255u - r);
              rmax = max(rmax, r);
            }
            const uint32_t k = wave_list_codes<true>(lb, (uint32_t)sz, [&](uint32_t c, uint32_t prev, bool has_prev) {
              if (has_prev && c <= prev) lbad = true;  // the list must be strictly increasing
              uint32_t ri, r;
              decode_hash(c, &ri, &r);
              rlo = max(rlo, 255u - r);
              rmax = max(rmax, r);
            });
            if (sz && (lb[sz - 1] & 0x80u)) lbad = true;  // a code without its last byte
            bad = __any(lbad);
            rlo = (uint32_t)__shfl((int)wave_incl_max(rlo), 63);
            rmax = (uint32_t)__shfl((int)wave_incl_max(rmax), 63);
            p.kind = 0;
            p.ntmp = (uint32_t)tssz;
            p.tmp_off = o + 8;
            p.list_off = o + last + 12;
            p.list_len = (uint32_t)sz;
            p.rr = (rlo || rmax ? 255u - rlo : 0xffu) | (rmax << 8);
            p.ncodes = (uint32_t)tssz + k;
          }
        }
      }
    } else {  // dense: m/2 tailcut bytes
      bad = len < 8 || be32(d + 4) != kHllM / 2 || len - 8 > kHllM / 2;
      if (!bad) {
        p.kind = 1;
        p.regs_off = o + 8;
        p.regs_len = (uint32_t)(len - 8);
      }
    }
  }
  if (lane == 0) {
    if (bad) atomicOr(err, kErrDecode);
    parts[i] = p;
  }
}

__global__ void k_hll_keys(uint64_t n, const uint32_t* __restrict__ slot, uint64_t* __restrict__ keys,
                           uint32_t* __restrict__ bt, uint32_t* __restrict__ stouch) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slot[i];
  keys[i] = ((uint64_t)s << 32) | (uint64_t)i;
  bt[s] = 1;
  stouch[s] = 1;  // Upsert happens before Combine (worker.go:241), even if the merge fails
}

// ---- block-wide helpers (256 threads)
__device__ __forceinline__ uint32_t upper_bound_u32(const uint32_t* a, uint32_t n, uint32_t v) {
  uint32_t l = 0, h = n;
  while (l < h) {
    uint32_t m = (l + h) >> 1;
    if (a[m] <= v) l = m + 1;
    else h = m;
  }
  return l;
}

// exclusive scan (sum or max) of one u32 per thread; s_red holds 4 u32
template <bool MAX>
__device__ __forceinline__ uint32_t block_scan_u32(uint32_t v, uint32_t* s_red, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if ((int)lane >= d) inc = MAX ? max(inc, o) : inc + o;
  }
  if (lane == 63) s_red[w] = inc;
  __syncthreads();
  uint32_t base = 0;
  for (uint32_t i = 0; i < w; i++) base = MAX ? max(base, s_red[i]) : base + s_red[i];
  total = 0;
  for (uint32_t i = 0; i < 4; i++) total = MAX ? max(total, s_red[i]) : total + s_red[i];
  __syncthreads();
  uint32_t ex = __shfl_up(inc, 1, 64);
  if (lane == 0) ex = 0;
  return MAX ? max(base, ex) : base + ex;
}

// compressedList bytes (a validated payload) -> codes in out[], ascending; returns the count
__device__ uint32_t decode_list(const uint8_t* g, uint32_t L, uint32_t* out, uint32_t* s_red) {
  const uint32_t t = threadIdx.x;
  const uint32_t per = (L + kBlock - 1) / kBlock, lo = min(L, t * per), hi = min(L, lo + per);
  uint32_t ends = 0, last_end = 0;  // last_end: position + 1 of my last terminator (0: none)
  for (uint32_t k = lo; k < hi; k++)
    if (!(g[k] & 0x80u)) {
      ends++;
      last_end = k + 1;
    }
  uint32_t total, tmax;
  const uint32_t ci0 = block_scan_u32<false>(ends, s_red, total);
  const uint32_t prev_end = block_scan_u32<true>(last_end, s_red, tmax);
  for (uint32_t k = t; k < total; k += kBlock) out[k] = 0;
  __syncthreads();
  uint32_t ci = ci0, start = prev_end;  // first byte of the code my first byte belongs to
  for (uint32_t k = lo; k < hi; k++) {
    const uint32_t b = g[k], j = k - start;
    if (7 * j < 32) atomicOr(&out[ci], (b & 0x7fu) << (7 * j));
    if (!(b & 0x80u)) {
      ci++;
      start = k + 1;
    }
  }
  __syncthreads();
  // deltas -> codes: prefix sum (uint32 arithmetic, as compressedList.decode)
  const uint32_t per2 = (total + kBlock - 1) / kBlock, lo2 = min(total, t * per2), hi2 = min(total, lo2 + per2);
  uint32_t sum = 0;
  for (uint32_t k = lo2; k < hi2; k++) sum += out[k];
  uint32_t tt;
  uint32_t run = block_scan_u32<false>(sum, s_red, tt);
  for (uint32_t k = lo2; k < hi2; k++) {
    run += out[k];
    out[k] = run;
  }
  __syncthreads();
  return total;
}

// Remove repeats from sorted A[0..n) in place (register-staged); returns the new length.
template <int K>
__device__ uint32_t unique_sorted(uint32_t* A, uint32_t n, uint32_t* s_red) {
  const uint32_t t = threadIdx.x;
  const uint32_t per = (n + kBlock - 1) / kBlock, lo = min(n, t * per), hi = min(n, lo + per);
  uint32_t v[K];
  bool keep[K];
  uint32_t kept = 0;
#pragma unroll
  for (int q = 0; q < K; q++) {
    const uint32_t k = lo + q;
    keep[q] = false;
    v[q] = 0;
    if (k < hi) {
      v[q] = A[k];
      keep[q] = k == 0 || A[k - 1] != v[q];
      kept += keep[q];
    }
  }
  uint32_t total;
  uint32_t pos = block_scan_u32<false>(kept, s_red, total);  // its barriers order the reads above
#pragma unroll
  for (int q = 0; q < K; q++)
    if (keep[q]) A[pos++] = v[q];
  __syncthreads();
  return total;
}

// lower_bound of v in sorted a[0..n) knowing it is at least l (the bound of a smaller value): a
// thread's elements are consecutive, so the next bound is usually a step or two on -- up to four
// linear steps, then a binary search over the rest (a search per element from 0 was ~14
// dependent LDS reads each for a 16k-code list)
__device__ __forceinline__ uint32_t lower_bound_after(const uint32_t* a, uint32_t l, uint32_t n, uint32_t v) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (l >= n || a[l] >= v) return l;
    l++;
  }
  uint32_t h = n;
  while (l < h) {
    const uint32_t m = (l + h) >> 1;
    if (a[m] < v) l = m + 1;
    else h = m;
  }
  return l;
}

// OUT = sorted A[0..na) U sorted B[0..nb), both free of repeats.  An element's place is its index
// plus the elements of the other list below it, minus the common elements below it (an exclusive
// scan of the "also in the other list" flags).  OUT may be A (ALIAS 1) or B (ALIAS 2): that side's
// values are staged in registers before anything is written, the other side is read again after
// the scan's barriers; places are kept as u16 pairs (< 2^16: na + nb <= 256 (KA + KB)) and the
// flags as bits, so the 16k-code union (KA = 65, KB = 67) stays in registers.  A union of more
// than cap codes writes nothing and returns its size.
template <int KA, int KB, int ALIAS>
__device__ uint32_t union_unique(const uint32_t* A, uint32_t na, const uint32_t* B, uint32_t nb, uint32_t* OUT,
                                 uint32_t* s_red, uint32_t cap = 0xffffffffu) {
  static_assert(kBlock * (KA + KB) <= 65536, "u16 places");
  const uint32_t t = threadIdx.x;
  const uint32_t pa = (na + kBlock - 1) / kBlock, loA = min(na, t * pa), hiA = min(na, loA + pa);
  const uint32_t pb = (nb + kBlock - 1) / kBlock, loB = min(nb, t * pb), hiB = min(nb, loB + pb);
  uint32_t av[ALIAS == 1 ? KA : 1], bv[ALIAS == 2 ? KB : 1];
  uint32_t apos[(KA + 1) / 2], bpos[(KB + 1) / 2], ain[(KA + 31) / 32], bin[(KB + 31) / 32];
#pragma unroll
  for (int q = 0; q < (KA + 1) / 2; q++) apos[q] = 0;
#pragma unroll
  for (int q = 0; q < (KB + 1) / 2; q++) bpos[q] = 0;
#pragma unroll
  for (int q = 0; q < (KA + 31) / 32; q++) ain[q] = 0;
#pragma unroll
  for (int q = 0; q < (KB + 31) / 32; q++) bin[q] = 0;
  uint32_t ca = 0, cb = 0, l = 0;
#pragma unroll
  for (int q = 0; q < KA; q++) {
    const uint32_t i = loA + q;
    if (i < hiA) {
      const uint32_t v = A[i];
      if (ALIAS == 1) av[q] = v;
      l = q == 0 ? lower_bound_u32(B, nb, v) : lower_bound_after(B, l, nb, v);
      const uint32_t in = l < nb && B[l] == v;
      ain[q >> 5] |= in << (q & 31);
      apos[q >> 1] |= (i + l) << (16 * (q & 1));
      ca += in;
    }
  }
  l = 0;
#pragma unroll
  for (int q = 0; q < KB; q++) {
    const uint32_t j = loB + q;
    if (j < hiB) {
      const uint32_t v = B[j];
      if (ALIAS == 2) bv[q] = v;
      l = q == 0 ? lower_bound_u32(A, na, v) : lower_bound_after(A, l, na, v);
      const uint32_t in = l < na && A[l] == v;
      bin[q >> 5] |= in << (q & 31);
      bpos[q >> 1] |= (j + l) << (16 * (q & 1));
      cb += in;
    }
  }
  uint32_t common, common2;
  uint32_t exa = block_scan_u32<false>(ca, s_red, common);
  uint32_t exb = block_scan_u32<false>(cb, s_red, common2);
  if (na + nb - common > cap) {  // over the output's capacity: the size only, nothing written
    __syncthreads();
    return na + nb - common;
  }
#pragma unroll
  for (int q = 0; q < KA; q++)
    if (loA + q < hiA) {
      const uint32_t v = ALIAS == 1 ? av[q] : A[loA + q];
      OUT[((apos[q >> 1] >> (16 * (q & 1))) & 0xffffu) - exa] = v;
      exa += (ain[q >> 5] >> (q & 31)) & 1u;
    }
#pragma unroll
  for (int q = 0; q < KB; q++)
    if (loB + q < hiB) {
      const uint32_t in = (bin[q >> 5] >> (q & 31)) & 1u;
      if (!in) OUT[((bpos[q >> 1] >> (16 * (q & 1))) & 0xffffu) - exb] = ALIAS == 2 ? bv[q] : B[loB + q];
      exb += in;
    }
  __syncthreads();
  return na + nb - common;
}

// a tmpSet-sized A (<= 256 codes) with B: one element per thread when B fits too (the unrolled
// 67-element staging costs ~10k cycles even for a few codes)
template <int ALIAS>
__device__ __forceinline__ uint32_t union_small(const uint32_t* A, uint32_t na, const uint32_t* B, uint32_t nb,
                                                uint32_t* OUT, uint32_t* s_red) {
  if (nb <= kBlock) return union_unique<1, 1, ALIAS>(A, na, B, nb, OUT, s_red);
  return union_unique<1, kCPer, ALIAS>(A, na, B, nb, OUT, s_red);
}

// varint byte length of sorted unique codes (compressedList.Append deltas from 0)
__device__ uint32_t list_bytes(const uint32_t* U, uint32_t n, uint32_t* s_red) {
  uint32_t bytes = 0;
  for (uint32_t i = threadIdx.x; i < n; i += kBlock) bytes += varint_len(U[i] - (i ? U[i - 1] : 0u));
  return block_allreduce_u32_sum(bytes, s_red);
}

// toNormal (hyperloglog.go:152-166): registers from the codes of A and B (duplicates harmless:
// with nz > 0 every insert is a plain max of min(r - b, 15)); the registers replace U.
// A and B may live in U.  Returns nz.
__device__ uint32_t to_normal(uint32_t* U, const uint32_t* A, uint32_t na, const uint32_t* B, uint32_t nb, uint32_t b,
                              uint32_t* s_red) {
  const uint32_t t = threadIdx.x;
  uint32_t ka[kPer], kb[kPer];
#pragma unroll
  for (int q = 0; q < (int)kPer; q++) {
    const uint32_t i = t + q * kBlock;
    ka[q] = i < na ? A[i] : kHllNoCode;
    kb[q] = i < nb ? B[i] : kHllNoCode;
  }
  __syncthreads();
  for (uint32_t i = t; i < kHllM; i += kBlock) U[i] = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < (int)kPer; q++) {
    uint32_t ri, r;
    if (ka[q] != kHllNoCode) {
      decode_hash(ka[q], &ri, &r);
      if (r > b) atomicMax(&U[ri], min(r - b, kHllCapacity - 1));
    }
    if (kb[q] != kHllNoCode) {
      decode_hash(kb[q], &ri, &r);
      if (r > b) atomicMax(&U[ri], min(r - b, kHllCapacity - 1));
    }
  }
  __syncthreads();
  uint32_t z = 0;
  for (uint32_t i = t; i < kHllM; i += kBlock) z += U[i] == 0;
  return block_allreduce_u32_sum(z, s_red);
}

#ifdef VN_SET_PROF
// profiling build only (tools/c5_set_profile.py): k_set_merge cycles and counts, summed over
// workgroups: 0 workgroup, 1 sparse <- sparse payloads (2 count), 3 dense runs of sparse payloads
// (4 runs, 5 payloads in them), 6 dense <- sparse one at a time (7 count), 8 dense payloads (9 count),
// 10 toNormal count, 11 payloads in all; sparse <- sparse phases: 12 tmpSet load and sort, 13 list
// decode, 14 unique + the two unions (payload, then tmpSet), 15 mergeSparse triggers; of which 16 (none
// now), 17 the list union; 18 the tmpSet copy of the other payloads
__device__ unsigned long long g_imp_prof[24];
#define IPROF_T(v) const long long v = clock64()
#define IPROF_ADD(i, a, b) \
  if (threadIdx.x == 0) atomicAdd(&g_imp_prof[i], (unsigned long long)((b) - (a)))
#define IPROF_INC(i, v) \
  if (threadIdx.x == 0) atomicAdd(&g_imp_prof[i], (unsigned long long)(v))
#else
#define IPROF_T(v)
#define IPROF_ADD(i, a, b)
#define IPROF_INC(i, v)
#endif

struct MergeCtx {
  const uint32_t* tl;
  const uint32_t* start;
  const uint32_t* end;
  const uint64_t* keys;   // sorted (slot << 32 | payload index)
  const HllPart* parts;
  const uint8_t* bytes;
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
};

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_set_merge(MergeCtx x) {
  __shared__ uint32_t U[kArenaWords];  // the key: sorted list codes, or registers (u32 each)
  __shared__ uint32_t Cb[kCWords];     // the payload's list codes / unions
  __shared__ uint32_t s_tmp[256];      // the key's tmpSet, sorted (kHllNoCode padding)
  __shared__ uint32_t s_ptmp[256];     // the payload's tmpSet, sorted
  __shared__ uint32_t s_red[4];
  __shared__ uint32_t s_b, s_nz, s_filled, s_tfull, s_pstar, s_newfill, s_min, s_nh;
  const uint32_t k = blockIdx.x, t = threadIdx.x;
  IPROF_T(w0);
  const uint32_t slot = x.tl[k];
  const uint32_t p0 = x.start[slot], p1 = x.end[slot];
  IPROF_INC(11, p1 - p0);
  uint32_t* arena = x.arena + (uint64_t)slot * kArenaWords;
  uint8_t* regs8 = reinterpret_cast<uint8_t*>(arena);

  bool dense = x.mode[slot] != 0;
  uint32_t lc = x.lc[slot], tc = x.tc[slot], lbytes = x.lb[slot];
  bool list_dirty = false;
  if (t == 0) {
    s_b = x.base[slot];
    s_nz = x.nz[slot];
  }
  if (dense) {
    for (uint32_t i = t; i < kHllM; i += kBlock) U[i] = regs8[i];
  } else {
    for (uint32_t i = t; i < lc; i += kBlock) U[i] = arena[i];
    s_tmp[t] = t < tc ? x.tmp[(uint64_t)slot * kTmpCap + t] : kHllNoCode;
  }
  __syncthreads();
  if (!dense) bitonic256(s_tmp);
  const DenseLds S{U, &s_b, &s_nz, &s_filled, &s_tfull, &s_pstar, &s_newfill, &s_min, s_red};

  for (uint32_t q = p0; q < p1; q++) {
    IPROF_T(q0);
    if (dense) {
      // A dense key and a run of sparse payloads none of whose inserts can rebase: a rebase
      // needs an overflow code (uint8(rho - b) >= capacity, hyperloglog.go:169-176) while no
      // register is zero, so a payload whose codes all have b <= rho < b + 16, or one that
      // starts while more zero registers remain than codes arrive before its end, only does
      // plain register maxes -- commutative, so the run's payloads apply at once, one per
      // lane (the long ones block-wide), and nz is recounted after.
      const uint32_t b = s_b, nz = s_nz;
      HllPart R{};
      R.kind = 1;
      if (q + t < p1) R = x.parts[(uint32_t)x.keys[q + t]];
      const uint32_t rmin = R.rr & 0xffu, rmax = R.rr >> 8;
      const bool cand = R.kind == 0 && (rmin < b || rmax >= b + kHllCapacity);
      uint32_t tot;
      const uint32_t before = block_scan_u32<false>(R.kind == 0 ? R.ncodes : 0u, s_red, tot);
      const bool safe = R.kind == 2 || (R.kind == 0 && (!cand || before + R.ncodes < nz));
      if (t == 0) {
        s_min = kBlock;
        s_nh = 0;
      }
      __syncthreads();
      if (!safe) atomicMin(&s_min, t);
      __syncthreads();
      const uint32_t nrun = s_min;
      if (nrun) {
        auto ins = [&](uint32_t code) {
          uint32_t ri, r;
          decode_hash(code, &ri, &r);
          if (r > b) atomicMax(&U[ri], min(r - b, kHllCapacity - 1));
        };
#ifdef VN_SET_LANE_RUNS
        if (t < nrun && R.kind == 0) {
          if (4u * R.ntmp + R.list_len > kLaneBytes) {
            s_ptmp[atomicAdd(&s_nh, 1u)] = t;
          } else {
            uint32_t c = 0, nb = 0;
            for_bytes<8>(x.bytes + R.tmp_off, 4u * R.ntmp, [&](uint32_t by) {
              c = (c << 8) | by;
              if (++nb == 4) {
                ins(c);
                nb = 0;
              }
            });
            uint32_t prev = 0, v = 0, sh = 0;
            for_bytes<8>(x.bytes + R.list_off, R.list_len, [&](uint32_t by) {
              if (sh < 32) v |= (by & 0x7fu) << sh;
              sh += 7;
              if (!(by & 0x80u)) {
                prev += v;
                ins(prev);
                v = 0;
                sh = 0;
              }
            });
          }
        }
        __syncthreads();
        const uint32_t nh = s_nh;
        for (uint32_t h = 0; h < nh; h++) {  // the long payloads, block-wide
          const HllPart H = x.parts[(uint32_t)x.keys[q + s_ptmp[h]]];
          if (t < H.ntmp) ins(be32(x.bytes + H.tmp_off + 4ull * t));
          const uint32_t nl = decode_list(x.bytes + H.list_off, H.list_len, Cb, s_red);
          for (uint32_t i = t; i < nl; i += kBlock) ins(Cb[i]);
          __syncthreads();
        }
#else
        // the run's payloads a wave each, drawn in turn from s_nh (a lane per payload walked its
        // whole list alone: the run waited for its longest payload, ≈40 cycles per byte)
        for (;;) {
          uint32_t i = 0;
          if ((t & 63u) == 0) i = atomicAdd(&s_nh, 1u);
          i = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)__shfl((int)i, 0));
          if (i >= nrun) break;
          const HllPart H = x.parts[(uint32_t)x.keys[q + i]];
          if (H.kind == 0) wave_insert_sparse(x.bytes, H, ins);
        }
        __syncthreads();
#endif
        uint32_t z = 0;
        for (uint32_t i = t; i < kHllM; i += kBlock) z += U[i] == 0;
        z = block_allreduce_u32_sum(z, s_red);
        if (t == 0) s_nz = z;
        __syncthreads();
        q += nrun - 1;
        IPROF_T(q1);
        IPROF_ADD(3, q0, q1);
        IPROF_INC(4, 1);
        IPROF_INC(5, nrun);
        continue;
      }
    }
    const HllPart P = x.parts[(uint32_t)x.keys[q]];
    if (P.kind == 2) continue;
    if (P.kind == 0) {
      // ---- the payload's codes: tmpSet (sorted) and decoded list
      s_ptmp[t] = t < P.ntmp ? be32(x.bytes + P.tmp_off + 4ull * t) : kHllNoCode;
      __syncthreads();
      bitonic256(s_ptmp);
      IPROF_T(qa);
      const uint32_t nl = decode_list(x.bytes + P.list_off, P.list_len, Cb, s_red);
      IPROF_T(qb);
      if (!dense) {
        // sparse <- sparse: tmpSet gets every code, then maybeToNormal
        const uint32_t npt = unique_sorted<1>(s_ptmp, P.ntmp, s_red);
        const uint32_t nd = union_small<2>(s_ptmp, npt, Cb, nl, Cb, s_red);
        // the new tmpSet, tmpSet U the payload's codes, in Cb (its 512 spare words hold the tmpSet)
        const uint32_t total = union_small<2>(s_tmp, tc, Cb, nd, Cb, s_red);
        IPROF_T(qc);
        IPROF_ADD(12, q0, qa);
        IPROF_ADD(13, qa, qb);
        IPROF_ADD(14, qb, qc);
        IPROF_INC(15, total * 100u > kHllM ? 1 : 0);
        if (total * 100u > kHllM) {
          // mergeSparse: list = list U tmpSet; then toNormal if its byte length > m
          s_tmp[t] = kHllNoCode;
          tc = 0;
          IPROF_T(qd);
          IPROF_ADD(16, qc, qd);
          // (staging sized to the operands: a list or payload of at most 2048 codes takes 8 per thread)
          const uint32_t cnt =
              lc <= 8 * kBlock
                  ? (total <= 8 * kBlock ? union_unique<8, 8, 1>(U, lc, Cb, total, U, s_red, kArenaWords)
                                         : union_unique<8, kCPer, 1>(U, lc, Cb, total, U, s_red, kArenaWords))
                  : (total <= 8 * kBlock ? union_unique<kPer, 8, 1>(U, lc, Cb, total, U, s_red, kArenaWords)
                                         : union_unique<kPer, kCPer, 1>(U, lc, Cb, total, U, s_red, kArenaWords));
          IPROF_T(qe);
          IPROF_ADD(17, qd, qe);
          if (cnt <= kArenaWords) {
            lc = cnt;
            lbytes = list_bytes(U, lc, s_red);
            list_dirty = true;
            if (lbytes > kHllM) {
              const uint32_t z = to_normal(U, U, lc, nullptr, 0, s_b, s_red);
              if (t == 0) s_nz = z;
              dense = true;
            }
          } else {  // more codes than a sparse list can hold (U untouched): certainly over m bytes
            const uint32_t z = to_normal(U, U, lc, Cb, total, s_b, s_red);
            if (t == 0) s_nz = z;
            dense = true;
          }
          __syncthreads();
          IPROF_INC(10, dense ? 1 : 0);
        } else {
          tc = total;
          s_tmp[t] = t < tc ? Cb[t] : kHllNoCode;
          __syncthreads();
          IPROF_T(qf);
          IPROF_ADD(18, qc, qf);
        }
        IPROF_T(q1);
        IPROF_ADD(1, q0, q1);
        IPROF_INC(2, 1);
      } else {
        // dense <- sparse: insert every code, tmpSet first (ascending), then the list
        const uint32_t nt = P.ntmp;
        const uint32_t* pt = s_ptmp;
        const uint32_t* cl = Cb;
        dense_insert_codes<kItems>(S, [pt, cl, nt](uint32_t p) { return p < nt ? pt[p] : cl[p - nt]; }, 0, nt + nl, x.err);
        __syncthreads();
        IPROF_T(q1);
        IPROF_ADD(6, q0, q1);
        IPROF_INC(7, 1);
      }
      continue;
    }
    // ---- dense payload
    if (!dense) {  // toNormal first (mergeSparse of the tmpSet included)
      const uint32_t z = to_normal(U, U, lc, s_tmp, tc, s_b, s_red);
      if (t == 0) s_nz = z;
      s_tmp[t] = kHllNoCode;
      tc = 0;
      dense = true;
      __syncthreads();
    }
    const uint32_t kb = s_b, pb = P.b;
    uint32_t changed = 0, fills = 0;
    if (kb < pb) {
      // sk.regs.rebase(pb - kb): registers >= d drop by d, nz counts those left above zero
      const uint32_t d = pb - kb;
      for (uint32_t i = t; i < kHllM; i += kBlock) {
        const uint32_t v = U[i];
        if (v >= d) {
          U[i] = v - d;
          changed += (v - d) > 0;
        }
      }
      changed = block_allreduce_u32_sum(changed, s_red);
      if (t == 0) {
        s_nz = kHllM - changed;
        s_b = pb;
      }
    }
    __syncthreads();
    const uint32_t d2 = kb > pb ? kb - pb : 0u;  // cpOther.regs.rebase(kb - pb) on the copy
    const uint8_t* rg = x.bytes + P.regs_off;
    for (uint32_t i = t; i < kHllM; i += kBlock) {
      const uint32_t byte = (i >> 1) < P.regs_len ? rg[i >> 1] : 0u;
      uint32_t v = (i & 1) ? (byte & 15u) : (byte >> 4);
      if (v >= d2) v -= d2;
      const uint32_t cur = U[i];
      if (v > cur) {
        fills += cur == 0;
        U[i] = v;
      }
    }
    fills = block_allreduce_u32_sum(fills, s_red);
    if (t == 0) s_nz -= fills;
    __syncthreads();
    IPROF_T(q1);
    IPROF_ADD(8, q0, q1);
    IPROF_INC(9, 1);
  }
  __syncthreads();
  IPROF_T(w1);
  IPROF_ADD(0, w0, w1);
  // ---- write back
  if (dense) {
    for (uint32_t i = t; i < kHllM; i += kBlock) regs8[i] = (uint8_t)U[i];
    if (t == 0) {
      x.mode[slot] = 1;
      x.base[slot] = (uint8_t)s_b;
      x.nz[slot] = s_nz;
      x.tc[slot] = 0;
      x.lc[slot] = 0;
      x.lb[slot] = 0;
    }
    return;
  }
  if (t < tc) x.tmp[(uint64_t)slot * kTmpCap + t] = s_tmp[t];
  if (list_dirty)
    for (uint32_t i = t; i < lc; i += kBlock) arena[i] = U[i];
  if (t == 0) {
    x.tc[slot] = tc;
    x.lc[slot] = lc;
    x.lb[slot] = lbytes;
    if (list_dirty && lc) x.last[slot] = U[lc - 1];
  }
}

__global__ void k_imp_seg_mark(uint64_t n, const uint64_t* __restrict__ K, uint32_t* __restrict__ start,
                               uint32_t* __restrict__ end) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = (uint32_t)(K[i] >> 32);
  if (i == 0 || (uint32_t)(K[i - 1] >> 32) != s) start[s] = (uint32_t)i;
  if (i == n - 1 || (uint32_t)(K[i + 1] >> 32) != s) end[s] = (uint32_t)(i + 1);
}

__global__ void k_set_clear_bt(uint32_t n, const uint32_t* __restrict__ list, uint32_t* __restrict__ flags) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) flags[list[k]] = 0;
}

}  // namespace

#ifdef VN_SET_PROF
extern "C" int vn_prof_import_set_read(unsigned long long* out24, int reset) {
  if (hipMemcpyFromSymbol(out24, HIP_SYMBOL(g_imp_prof), sizeof(unsigned long long) * 24) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[24] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_imp_prof), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// timing mode: dense payloads and sparse codes of a parsed batch (vn_import_counts)
__global__ void k_hll_counts(uint64_t n, const HllPart* __restrict__ parts, unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long d = 0, c = 0;
  if (i < n) {
    d = parts[i].kind == 1u ? 1ull : 0ull;
    c = parts[i].kind == 0u ? parts[i].ncodes : 0ull;
  }
  for (int s = 32; s >= 1; s >>= 1) {
    d += __shfl_xor(d, s, 64);
    c += __shfl_xor(c, s, 64);
  }
  if ((threadIdx.x & 63) == 0 && (d || c)) {
    atomicAdd(out, d);
    atomicAdd(out + 1, c);
  }
}

void import_sets(vn_engine* e, uint64_t n, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes) {
  if (!n) return;
  hipStream_t st = e->st;
  HllPart* parts = reinterpret_cast<HllPart*>(e->imp.parts);
  hipLaunchKernelGGL(k_hll_parse, dim3(blocks_for(n, 4)), dim3(256), 0, st, n, off, bytes, parts, e->h_err);  // a wave each
  VN_HIP_CHECK(hipStreamSynchronize(st));
  take_decode_error(e);  // a truncated payload: nothing is applied
  if (e->timing) {
    if (!e->d_imp_counts) {
      VN_HIP_CHECK(hipMalloc(&e->d_imp_counts, 2 * sizeof(unsigned long long)));
      VN_HIP_CHECK(hipMemsetAsync(e->d_imp_counts, 0, 2 * sizeof(unsigned long long), st));
    }
    e->imp_counts[2] += n;
    hipLaunchKernelGGL(k_hll_counts, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, parts, e->d_imp_counts);
  }
  // group the payloads by key, arrival order kept
  hipLaunchKernelGGL(k_hll_keys, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, slot, e->sR0, e->s_bt, e->stouch);
  RadixPass passes[4];
  int np = 0;
  np = make_passes(passes, false, 32, e->slot_bits[VN_SET]);
  const bool fl = radix_sort(e->sR0, nullptr, e->sR1, nullptr, n, passes, np, e->rs, st, nullptr);
  const uint64_t* keys = fl ? e->sR1 : e->sR0;
  hipLaunchKernelGGL(k_imp_seg_mark, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, keys, e->s_start, e->s_end);
  compact_flags(e->s_bt, e->s_pos, e->s_tl, e->s_cnt, e->cap[VN_SET], e->ss, st);
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 10, e->s_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
  const uint32_t ntouched = e->hf_cnt[10];
  if (!ntouched) return;
  MergeCtx x;
  x.tl = e->s_tl;
  x.start = e->s_start;
  x.end = e->s_end;
  x.keys = keys;
  x.parts = parts;
  x.bytes = bytes;
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
  hipLaunchKernelGGL(k_set_merge, dim3(ntouched), dim3(kBlock), 0, st, x);
  hipLaunchKernelGGL(k_set_clear_bt, dim3(blocks_for(ntouched, 256)), dim3(256), 0, st, ntouched, e->s_tl, e->s_bt);
}

}  // namespace vn

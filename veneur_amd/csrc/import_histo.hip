// import_histo.hip -- Worker.ImportMetric for histograms and timers (worker.go:230-268).
//
// Histo.Combine (samplers/samplers.go:519-526) decodes the forwarded digest --
// tdigest.NewMerging(100) + GobDecode (tdigest/merging_digest.go:382-412) -- and calls
// MergingDigest.Merge (344-356), which Add()s every centroid of the other digest.  Local*
// statistics are not touched.  Merge visits the centroids in rand.Perm order, seeded from the
// clock (trace/trace.go:30-32), so not even the reference reproduces itself; the engine Adds
// them in their stored order (ascending mean), which the parity tests hand the oracle as the
// permutation.
//
// The payloads are the JSONMetric.Value bytes a global veneur receives (after the JSON,
// base64 and zlib decode of handlers_global.go:110-188).  One lane per payload parses the gob
// stream (count pass, scan, emit pass); the centroids then join the ordinary histo ingest as
// records tagged kTagImport, so the exact replay / hot-key batch merge applies them in Add
// order, and they count for the digest (min/max, weight) but not for Local*.
#include "histo.h"

namespace vn {

namespace {

// encoding/gob reader over one payload (the subset MergingDigest.GobEncode writes).  One lane
// walks its own payload: bytes come from 16-byte-aligned blocks held in registers, the next
// block's load in flight while this one is parsed (a byte-at-a-time global load per step would
// leave every lane waiting on memory latency once per byte).  The blocks never leave the
// 16-byte-aligned span holding the payload.
struct GobIn {
  const uint4* blk;  // the aligned blocks covering the payload
  uint32_t lo;       // payload start within blk[0]
  uint32_t n, i;
  bool err;
  uint32_t nb, cb;   // blocks; the first held block
  uint64_t c0, c1, n0, n1, m0, m1;  // blocks cb, cb + 1, cb + 2 (low, high 8 bytes; clamped to nb - 1)
  __device__ __forceinline__ void load(uint32_t k, uint64_t& a, uint64_t& b) const {
    const uint4 v = blk[min(k, nb - 1u)];
    a = (uint64_t)v.x | ((uint64_t)v.y << 32);
    b = (uint64_t)v.z | ((uint64_t)v.w << 32);
  }
  __device__ GobIn(const uint8_t* d, uint32_t len) : n(len), i(0), err(false) {
    const uintptr_t s = reinterpret_cast<uintptr_t>(d), a0 = s & ~(uintptr_t)15;
    blk = reinterpret_cast<const uint4*>(a0);
    lo = (uint32_t)(s - a0);
    nb = (lo + len + 15u) >> 4;
    cb = 0;
    c0 = c1 = n0 = n1 = m0 = m1 = 0;
    if (nb) {
      load(0, c0, c1);
      load(1, n0, n1);
      load(2, m0, m1);
    }
  }
  // (a reader placed at byte pos: its first three blocks are those around pos)
  __device__ GobIn(const uint8_t* d, uint32_t len, uint32_t pos) : n(len), i(pos), err(false) {
    const uintptr_t s = reinterpret_cast<uintptr_t>(d), a0 = s & ~(uintptr_t)15;
    blk = reinterpret_cast<const uint4*>(a0);
    lo = (uint32_t)(s - a0);
    nb = (lo + len + 15u) >> 4;
    cb = (lo + pos) >> 4;
    load(cb, c0, c1);
    load(cb + 1, n0, n1);
    load(cb + 2, m0, m1);
  }
  // hold blocks k, k + 1, k + 2 (the two after the current one in flight while it is parsed)
  __device__ __forceinline__ void seek(uint32_t k) {
    if (k == cb) return;
    if (k == cb + 1) {
      c0 = n0;
      c1 = n1;
      n0 = m0;
      n1 = m1;
      load(k + 2, m0, m1);
    } else if (k == cb + 2) {
      c0 = m0;
      c1 = m1;
      load(k + 1, n0, n1);
      load(k + 2, m0, m1);
    } else {
      load(k, c0, c1);
      load(k + 1, n0, n1);
      load(k + 2, m0, m1);
    }
    cb = k;
  }
  __device__ __forceinline__ uint32_t at(uint32_t pos) {  // byte pos (< n)
    const uint32_t a = lo + pos;
    seek(a >> 4);
    // mask blend, not a select: a select of two fields can become a load through a selected
    // pointer, which keeps the reader in scratch memory
    const uint64_t m = 0ull - (uint64_t)((a >> 3) & 1u), h = (c0 & ~m) | (c1 & m);
    return (uint32_t)(h >> ((a & 7u) * 8u)) & 0xffu;
  }
  // 8 bytes from byte o (< 24) of the held blocks c0:c1 (this one) and n0:n1 (the next), by
  // mask blends (no register indexing: it would put the reader in scratch)
  __device__ __forceinline__ uint64_t win64(uint32_t o) const {
    const uint32_t w = o >> 3, s = (o & 7u) * 8u;
    const uint64_t m0_ = 0ull - (uint64_t)(w == 0), m1_ = 0ull - (uint64_t)(w == 1), m2_ = 0ull - (uint64_t)(w == 2);
    const uint64_t lo_w = (c0 & m0_) | (c1 & m1_) | (n0 & m2_) | (n1 & ~(m0_ | m1_ | m2_));
    const uint64_t hi_w = (c1 & m0_) | (n0 & m1_) | (n1 & m2_);
    return s ? (lo_w >> s) | (hi_w << (64u - s)) : lo_w;
  }
  // One centroid in the layout GobEncode gives a tdigest Centroid {Mean, Weight float64, ...}
  // whose type lists Mean and Weight first: {1, mean, 1, weight, 0}, or {2, weight, 0} when the
  // mean is zero (gob omits zero fields). Parsed from a 24-byte window at byte i without
  // per-token branches; false (nothing consumed) for any other form, which the general field
  // loop then reads -- so both give the same values and the same errors.
  __device__ __forceinline__ bool centroid(double& mean, double& weight) {
    const uint32_t a = lo + i;
    seek(a >> 4);
    const uint32_t o = a & 15u, sh = (o & 7u) * 8u;
    const uint64_t mk = 0ull - (uint64_t)(o >> 3);  // the window starts in c1
    const uint64_t w0 = (c0 & ~mk) | (c1 & mk), w1 = (c1 & ~mk) | (n0 & mk), w2 = (n0 & ~mk) | (n1 & mk),
                   w3 = (n1 & ~mk) | (m0 & mk);
    const uint64_t W0 = sh ? (w0 >> sh) | (w1 << (64u - sh)) : w0, W1 = sh ? (w1 >> sh) | (w2 << (64u - sh)) : w1,
                   W2 = sh ? (w2 >> sh) | (w3 << (64u - sh)) : w2;
    auto byte = [&](uint32_t p) -> uint32_t {  // byte p < 24 of the window
      const uint64_t q0 = 0ull - (uint64_t)((p >> 3) == 0), q1 = 0ull - (uint64_t)((p >> 3) == 1);
      const uint64_t x = (W0 & q0) | (W1 & q1) | (W2 & ~(q0 | q1));
      return (uint32_t)(x >> ((p & 7u) * 8u)) & 0xffu;
    };
    // a gob unsigned at p read as float64 bits (f(): the value's bytes reversed); its length, 0 if
    // the count byte is over 8
    auto fl = [&](uint32_t p, uint64_t& bits) -> uint32_t {
      const uint32_t b = byte(p);
      if (b < 0x80u) {
        bits = (uint64_t)b << 56;
        return 1;
      }
      const uint32_t cnt = 256u - b, q = p + 1, s2 = (q & 7u) * 8u;  // q <= 12
      const uint64_t qm = 0ull - (uint64_t)(q >> 3);
      const uint64_t lw = (W0 & ~qm) | (W1 & qm), hw = (W1 & ~qm) | (W2 & qm);
      const uint64_t y = s2 ? (lw >> s2) | (hw << (64u - s2)) : lw;  // the cnt bytes, little-endian
      bits = cnt <= 8u ? y << (64u - 8u * cnt) : 0ull;
      return cnt <= 8u ? 1u + cnt : 0u;
    };
    const uint32_t d1 = byte(0);
    uint64_t mb = 0, wb = 0;
    uint32_t p = 1;
    if (d1 == 1u) {
      const uint32_t lm = fl(1, mb);
      if (!lm || byte(1 + lm) != 1u) return false;
      p = 2 + lm;
    } else if (d1 != 2u) {
      return false;
    }
    const uint32_t lw = fl(p, wb);
    if (!lw || byte(p + lw) != 0u) return false;
    const uint32_t len = p + lw + 1;
    if (len > n - i) return false;
    i += len;
    mean = bitsd(mb);
    weight = bitsd(wb);
    return true;
  }
  __device__ __forceinline__ uint64_t u() {  // gob unsigned integer
    if (i >= n) {
      err = true;
      return 0;
    }
    const uint32_t b = at(i);  // (also moves the held blocks to byte i)
    i++;
    if (b < 0x80u) return b;
    const uint32_t cnt = 256u - b;  // byte count, sent negated
    if (cnt > 8u || cnt > n - i) {
      err = true;
      return 0;
    }
    // the cnt big-endian bytes after the count byte, read at once: they lie within the held
    // blocks (byte offset <= 16 + 8 of the current block's start)
    const uint64_t y = win64(((lo + i - 1) & 15u) + 1u);
    i += cnt;
    return __builtin_bswap64(y) >> (64u - 8u * cnt);
  }
  __device__ __forceinline__ int64_t s() {  // gob signed integer: sign in bit 0
    const uint64_t x = u();
    return (x & 1) ? ~(int64_t)(x >> 1) : (int64_t)(x >> 1);
  }
  __device__ __forceinline__ double f() {  // gob float64: IEEE bits byte-reversed, sent as an unsigned integer
    uint64_t x = u(), v = 0;
    for (int k = 0; k < 8; k++) {
      v = (v << 8) | (x & 0xffu);
      x >>= 8;
    }
    return bitsd(v);
  }
  __device__ __forceinline__ void skip_string() {
    const uint64_t l = u();
    if (l > n - i) {
      err = true;
      return;
    }
    i += (uint32_t)l;
  }
  __device__ __forceinline__ int field_name() {  // 1 = "Mean", 2 = "Weight", 0 = any other name
    const uint64_t l = u();
    if (l > n - i) {
      err = true;
      return 0;
    }
    int r = 0;
    if (l == 4 && at(i) == 'M' && at(i + 1) == 'e' && at(i + 2) == 'a' && at(i + 3) == 'n') r = 1;
    if (l == 6 && at(i) == 'W' && at(i + 1) == 'e' && at(i + 2) == 'i' && at(i + 3) == 'g' && at(i + 4) == 'h' &&
        at(i + 5) == 't')
      r = 2;
    i += (uint32_t)l;
    return r;
  }
  __device__ __forceinline__ int64_t common_type() {  // CommonType {Name string; Id typeId} -> Id
    int64_t id = 0, f = -1;
    for (;;) {
      const uint64_t dl = u();
      if (err || dl == 0) break;
      f += (int64_t)dl;
      if (f == 0) skip_string();
      else if (f == 1) id = s();
      else {
        err = true;
        break;
      }
    }
    return id;
  }
};

constexpr int kGobSlices = 4, kGobFields = 6;
// the type definitions of a digest stream: slice types (id -> elem) and one struct type
struct GobTypes {
  int ns = 0;
  int64_t sid[kGobSlices], selem[kGobSlices];
  int64_t st = -1;
  int nf = 0;
  int fname[kGobFields];
  int64_t fid[kGobFields];
};

// one wireType message (encoding/gob type.go: ArrayT 0, SliceT 1, StructT 2)
__device__ __forceinline__ void gob_wiretype(GobIn& r, GobTypes& T) {
  int64_t f = -1;
  for (;;) {
    const uint64_t dl = r.u();
    if (r.err || dl == 0) return;
    f += (int64_t)dl;
    if (f == 0 || f == 1) {  // {CommonType; Elem; [Len]}
      int64_t sf = -1, id = 0, elem = 0;
      for (;;) {
        const uint64_t d2 = r.u();
        if (r.err || d2 == 0) break;
        sf += (int64_t)d2;
        if (sf == 0) id = r.common_type();
        else if (sf == 1) elem = r.s();
        else if (sf == 2) (void)r.s();
        else {
          r.err = true;
          return;
        }
      }
      if (T.ns >= kGobSlices) {
        r.err = true;
        return;
      }
      T.sid[T.ns] = id;
      T.selem[T.ns] = elem;
      T.ns++;
    } else if (f == 2) {  // {CommonType; Field []*fieldType{Name; Id}}
      int64_t sf = -1;
      for (;;) {
        const uint64_t d2 = r.u();
        if (r.err || d2 == 0) break;
        sf += (int64_t)d2;
        if (sf == 0) {
          T.st = r.common_type();
        } else if (sf == 1) {
          const uint64_t nf = r.u();
          if (nf > (uint64_t)kGobFields) {
            r.err = true;
            return;
          }
          T.nf = (int)nf;
          for (int k = 0; k < (int)nf; k++) {
            T.fname[k] = 0;
            T.fid[k] = 0;
            int64_t ff = -1;
            for (;;) {
              const uint64_t d3 = r.u();
              if (r.err || d3 == 0) break;
              ff += (int64_t)d3;
              if (ff == 0) T.fname[k] = r.field_name();
              else if (ff == 1) T.fid[k] = r.s();
              else {
                r.err = true;
                return;
              }
            }
          }
        } else {
          r.err = true;
          return;
        }
      }
    } else {
      r.err = true;
      return;
    }
  }
}

// skip one field value of type id tid: builtin scalars, strings, or a slice of scalars
// (Centroid.Samples []float64, only sent by debug digests)
__device__ __forceinline__ void gob_skip(GobIn& r, const GobTypes& T, int64_t tid) {
  if (tid >= 1 && tid <= 4) {  // bool, int, uint, float
    (void)r.u();
    return;
  }
  if (tid == 5 || tid == 6) {  // []byte, string
    r.skip_string();
    return;
  }
  for (int k = 0; k < T.ns; k++)
    if (T.sid[k] == tid && T.selem[k] >= 1 && T.selem[k] <= 4) {
      const uint64_t c = r.u();
      for (uint64_t j = 0; j < c && !r.err; j++) (void)r.u();
      return;
    }
  r.err = true;
}

// One GobEncode()d MergingDigest ([]Centroid, then compression, min, max as float64):
// the number of centroids, written to mean/w when EMIT; -1 if the stream is malformed.
// Counting (!EMIT), *fast_at gets the byte where the centroids start when every one of them took
// the one-window parse (GobIn::centroid), else ~0u: k_gob_emit_fast then emits them from there.
// ... and ckpt[q] the byte of centroid kSeg q (q < kSegs; a payload of more centroids, or of 64 KiB
// or more, is not "fast")
constexpr uint32_t kSeg = 16, kSegs = 16;
template <bool EMIT>
__device__ __forceinline__ int64_t gob_digest(const uint8_t* d, uint32_t n, double* mean, double* w,
                                              uint32_t* fast_at = nullptr, uint16_t* ckpt = nullptr) {
  GobIn r(d, n);
  GobTypes T;
  bool have = false, allfast = false;
  uint32_t at = ~0u;
  int floats = 0;
  int64_t cnt = 0;
  // EMIT: the centroids go out eight at a time from a register queue.  On gfx950 one counter
  // (vmcnt) tracks loads and stores in issue order, so the wait for the reader's next block
  // also waits for every store issued before that block's load: with a store per centroid the
  // reader stalled on store latency every 16 bytes (the emit pass ran ~5x slower than the count
  // pass over the same bytes); batched, it stalls once per eight centroids
  constexpr int kQ = 8;
  double qm[kQ], qw[kQ];
  int nq = 0;
  while (r.i < r.n && floats < 3) {
    const uint64_t mlen = r.u();
    if (r.err || mlen > r.n - r.i) return -1;
    const uint32_t end = r.i + (uint32_t)mlen;
    const int64_t id = r.s();
    if (id < 0) {
      gob_wiretype(r, T);
    } else {
      if (r.u() != 0) return -1;  // a non-struct value starts with a zero delta
      if (!have) {
        int si = -1;
        for (int k = 0; k < T.ns; k++)
          if (T.sid[k] == id) si = k;
        if (si < 0 || T.selem[si] != T.st) return -1;
        uint32_t fk = 0;  // per field: 1 Mean, 2 Weight (float64), 0 skipped -- 2 bits each
        for (int k = 0; k < T.nf; k++)
          fk |= (uint32_t)(T.fid[k] == 4 ? (T.fname[k] == 1 ? 1 : T.fname[k] == 2 ? 2 : 0) : 0) << (2 * k);
        const bool common = T.nf >= 2 && (fk & 15u) == (1u | 2u << 2);  // Mean, Weight first
        const uint64_t c = r.u();
        at = r.i;
        allfast = common && c <= kSeg * kSegs && n < 65536u;
        for (uint64_t j = 0; j < c && !r.err; j++) {
          double m = 0.0, wt = 0.0;  // gob omits zero fields
          int64_t f = -1;
          if (!EMIT && ckpt && allfast && j % kSeg == 0) ckpt[j / kSeg] = (uint16_t)r.i;
          const bool fast = common && r.i < r.n && r.centroid(m, wt);
          allfast &= fast;
          if (!fast) for (;;) {
            const uint64_t dl = r.u();
            if (r.err || dl == 0) break;
            f += (int64_t)dl;
            if (f >= T.nf) {
              r.err = true;
              break;
            }
            const uint32_t kind = (fk >> (2 * f)) & 3u;
            if (kind == 1) m = r.f();
            else if (kind == 2) wt = r.f();
            else gob_skip(r, T, T.fid[f]);
          }
          if (EMIT) {
#pragma unroll
            for (int q = 0; q < kQ - 1; q++) {
              qm[q] = qm[q + 1];
              qw[q] = qw[q + 1];
            }
            qm[kQ - 1] = m;
            qw[kQ - 1] = wt;
            if (++nq == kQ) {  // centroids cnt - 7 .. cnt
#pragma unroll
              for (int q = 0; q < kQ; q++) {
                mean[cnt - (kQ - 1) + q] = qm[q];
                w[cnt - (kQ - 1) + q] = qw[q];
              }
              nq = 0;
            }
          } else if (d_isnan(m) || d_isinf(m) || wt <= 0.0) {
            return -1;  // Merge's Add would panic (merging_digest.go:98-100)
          }
          cnt++;
        }
        if (EMIT) {  // the queue's last nq centroids: cnt - nq .. cnt - 1
#pragma unroll
          for (int q = 0; q < kQ; q++)
            if (q >= kQ - nq) {
              mean[cnt - kQ + q] = qm[q];
              w[cnt - kQ + q] = qw[q];
            }
          nq = 0;
        }
        have = true;
      } else {
        if (id != 4) return -1;  // compression, min, max: float64
        (void)r.f();
        floats++;
      }
    }
    if (r.err || r.i != end) return -1;
  }
  if (!(have && floats == 3)) return -1;
  if (fast_at) *fast_at = allfast ? at : ~0u;
  return cnt;
}

// per payload: its centroid count, the whole payload validated (slot in range, offsets
// non-decreasing, a well-formed digest, every centroid a valid Add), so the emit cannot fail
__global__ void k_gob_count(uint64_t n, const uint32_t* __restrict__ slot, uint32_t cap,
                            const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                            uint32_t* __restrict__ cnt, uint32_t* __restrict__ cpos, uint16_t* __restrict__ ckpt,
                            uint32_t* __restrict__ err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t len = off[i + 1] - off[i];
  const bool ok = slot[i] < cap && off[i + 1] >= off[i] && len <= 0xffffffffull;
  uint32_t at = ~0u;
  const int64_t c =
      ok ? gob_digest<false>(bytes + off[i], (uint32_t)len, nullptr, nullptr, &at, ckpt + (uint64_t)i * kSegs) : -1;
  cpos[i] = c < 0 ? ~0u : at;
  if (c < 0 || c > (int64_t)kTagIndex) {
    atomicOr(err, kErrDecode);
    cnt[i] = 0;
  } else {
    cnt[i] = (uint32_t)c;
  }
}

// the centroids of payloads 0..n-1 appended to the run at base + coff[i]; each payload's slot and
// first centroid into the run's payload table at pb + i
__global__ void k_gob_emit(uint64_t n, const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                           const uint32_t* __restrict__ slot, const uint32_t* __restrict__ coff,
                           const uint32_t* __restrict__ cpos, uint64_t base,
                           double* __restrict__ omean, double* __restrict__ ow, uint32_t* __restrict__ pslot,
                           uint32_t* __restrict__ pbeg, uint64_t pb, uint32_t* __restrict__ err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || cpos[i] != ~0u) return;  // (those: k_gob_emit_fast)
  const uint64_t o = base + coff[i];
  pslot[pb + i] = slot[i];
  pbeg[pb + i] = (uint32_t)o;
  // k_gob_count validated the payload (every centroid a valid Add), so this pass only writes
  const int64_t c = gob_digest<true>(bytes + off[i], (uint32_t)(off[i + 1] - off[i]), omean + o, ow + o);
  if (c < 0) atomicOr(err, kErrDecode);
}

// The payloads whose centroids all take the one-window parse (cpos: where they start), kSeg
// centroids per thread from the count pass's checkpoints, kSegs threads per payload: a payload's
// threads are adjacent lanes writing adjacent kSeg-centroid runs, so the wave completes its output
// lines within a few stores (one lane per payload left every lane's line half written across
// long stretches of its parse: the stores, not the parse, set that kernel's time)
__global__ void k_gob_emit_seg(uint64_t n, const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                               const uint32_t* __restrict__ slot, const uint32_t* __restrict__ coff,
                               const uint32_t* __restrict__ cpos, const uint16_t* __restrict__ ckpt, uint64_t base,
                               double* __restrict__ omean, double* __restrict__ ow, uint32_t* __restrict__ pslot,
                               uint32_t* __restrict__ pbeg, uint64_t pb) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, i = t / kSegs;
  const uint32_t q = (uint32_t)(t % kSegs);
  if (i >= n || cpos[i] == ~0u) return;
  const uint32_t c0 = coff[i], c = coff[i + 1] - c0;
  const uint64_t o = base + c0;
  if (q == 0) {
    pslot[pb + i] = slot[i];
    pbeg[pb + i] = (uint32_t)o;
  }
  if (q * kSeg >= c) return;
  const uint32_t m = min(kSeg, c - q * kSeg);
  GobIn r(bytes + off[i], (uint32_t)(off[i + 1] - off[i]), ckpt[i * kSegs + q]);
  double* const dm = omean + o + q * kSeg;
  double* const dw = ow + o + q * kSeg;
  // two halves of eight: parsed into registers, then stored (fewer registers than one queue of
  // sixteen: more waves per SIMD; each half still fills 64 contiguous bytes per array)
#pragma unroll
  for (uint32_t h = 0; h < kSeg; h += 8) {
    double qm[8], qw[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) {
      qm[j] = 0.0;
      qw[j] = 0.0;
      if (h + j < m) (void)r.centroid(qm[j], qw[j]);
    }
#pragma unroll
    for (uint32_t j = 0; j < 8; j++)
      if (h + j < m) {
        dm[h + j] = qm[j];
        dw[h + j] = qw[j];
      }
  }
}

// Worker.ImportMetric Upserts the key before Combine (worker.go:241): every payload's key is in the
// window, a digest without centroids included (it makes no record, so no segment marks it)
__global__ void k_import_touch(uint64_t n, const uint32_t* __restrict__ slot, uint32_t* __restrict__ touch) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) touch[slot[i]] = 1;
}

// A call's payloads [b0, n) cut greedily into slices of whole payloads, each at most cap centroids
// and cap_pay payloads (the run): one thread, a binary search over the centroid scan co per slice.
// out: cuts[j] = first payload of slice j, cuts[kImportCuts + 1 + j] = co at it, j <= count; then
// the count and a flag (1: a payload alone is over cap).  At most kImportCuts slices per pass.
__global__ void k_import_cuts(const uint32_t* __restrict__ co, uint64_t n, uint64_t b0, uint64_t cap, uint64_t cap_pay,
                              uint32_t* __restrict__ out) {
  uint32_t* const cc = out + kImportCuts + 1;
  uint32_t j = 0, flag = 0;
  while (b0 < n && j < kImportCuts) {
    const uint32_t c0 = co[b0];
    if (co[b0 + 1] - c0 > cap) {
      flag = 1;
      break;
    }
    uint64_t lo = b0 + 1, hi = min(n, b0 + cap_pay);  // the largest b1 in [lo, hi] with co[b1] - c0 <= cap
    while (lo < hi) {
      const uint64_t m = (lo + hi + 1) >> 1;
      if (co[m] - c0 <= cap) lo = m;
      else hi = m - 1;
    }
    out[j] = (uint32_t)b0;
    cc[j] = c0;
    j++;
    b0 = lo;
  }
  out[j] = (uint32_t)b0;
  cc[j] = co[b0];
  out[2 * (kImportCuts + 1)] = j;
  out[2 * (kImportCuts + 1) + 1] = flag;
}

// ---- the drain's grouping: payloads sorted by key (stable), then their centroids moved
__global__ void k_pay_keys(uint64_t n, const uint32_t* __restrict__ pslot, uint64_t* __restrict__ key,
                           uint32_t* __restrict__ pbeg, uint32_t total) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) key[i] = ((uint64_t)pslot[i] << 32) | i;
  if (i == 0) pbeg[n] = total;  // (the end of the last payload)
}
__global__ void k_pay_counts(uint64_t n, const uint64_t* __restrict__ key, const uint32_t* __restrict__ pbeg,
                             uint32_t* __restrict__ cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = (uint32_t)key[i];
  cnt[i] = pbeg[p + 1] - pbeg[p];
}
// the key segments of the grouped run at payload granularity (the payloads in key order, pdst
// their places): a key starts at its first payload's place and ends after its last payload, both
// among the payloads with centroids -- what k_seg_mark finds from every record
__global__ void k_pay_seg_mark(uint64_t n, const uint64_t* __restrict__ key, const uint32_t* __restrict__ pdst,
                               const uint32_t* __restrict__ pcnt, uint32_t* __restrict__ start, uint32_t* __restrict__ end,
                               uint32_t* __restrict__ bt, uint32_t* __restrict__ touch) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !pcnt[i]) return;  // (a digest without centroids makes no record: no segment)
  const uint32_t s = (uint32_t)(key[i] >> 32);
  // the key's first and last payload with centroids (empty digests are rare: short walks)
  uint64_t j = i;
  while (j > 0 && (uint32_t)(key[j - 1] >> 32) == s && !pcnt[j - 1]) j--;
  if (j == 0 || (uint32_t)(key[j - 1] >> 32) != s) {
    start[s] = pdst[i];
    bt[s] = 1;
    touch[s] = 1;
  }
  j = i + 1;
  while (j < n && (uint32_t)(key[j] >> 32) == s && !pcnt[j]) j++;
  if (j == n || (uint32_t)(key[j] >> 32) != s) end[s] = pdst[i] + pcnt[i];
}
// one wave per payload in key order: its centroids as grouped histo records (A = mean bits,
// B = slot << 32 | kTagImport | run index, the record k_histo_keys_raw makes of an import)
__global__ __launch_bounds__(256) void k_pay_move(uint64_t n, const uint64_t* __restrict__ key,
                                                  const uint32_t* __restrict__ pbeg, const uint32_t* __restrict__ dst,
                                                  const double* __restrict__ mean, uint64_t* __restrict__ A,
                                                  uint64_t* __restrict__ B) {
  const uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t k = key[i];
  const uint32_t p = (uint32_t)k, b = pbeg[p], c = pbeg[p + 1] - b, d = dst[i];
  const uint64_t hi = k & 0xffffffff00000000ull;
  for (uint32_t r = lane; r < c; r += 64) {
    A[d + r] = dbits(mean[b + r]);
    B[d + r] = hi | (uint64_t)(kTagImport | (b + r));
  }
}

}  // namespace

// Histo.Combine of a batch of forwarded digests: decoded and validated now (one host round
// trip: the centroid count), their centroids appended in arrival order to the engine's import
// run, which is merged -- re-Add of every centroid through the exact replay / hot remainder
// -- in one ingest when it fills or before anything reads or adds to a histogram
// (histo_imports_drain).  Merging a run of imports at once equals merging them one call
// after another: the replay is the same ordered stream of Adds.  A batch holding more
// centroids than the run (a global veneur's whole fleet in one call) is cut into slices of
// whole payloads of at most the run each (one more round trip for the offsets), each appended
// and drained in arrival order.
void import_histos(vn_engine* e, uint64_t n, const uint32_t* slot, const uint64_t* off, const uint8_t* bytes) {
  if (!n) return;
  hipStream_t st = e->st;
  ImportScratch& s = e->imp;
  // (timing: each decode kernel between a pair of events)
  auto ev_pair = [&](EventPool& p, auto&& launch) {
    hipEvent_t a = e->timing ? p.next() : nullptr, b = e->timing ? p.next() : nullptr;
    if (a && b) VN_HIP_CHECK(hipEventRecord(a, st));
    launch();
    if (a && b) VN_HIP_CHECK(hipEventRecord(b, st));
  };
  ev_pair(e->pool_id, [&] {
    hipLaunchKernelGGL(k_gob_count, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, slot, e->cap[VN_HISTO], off, bytes,
                       s.cnt, s.cpos, s.ckpt, e->h_err);
  });
  scan_exclusive_u32(s.cnt, s.coff, n, e->ss, st);
  VN_HIP_CHECK(hipMemcpyAsync(e->hf_cnt + 9, s.coff + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
  take_decode_error(e);
  const uint64_t nc = e->hf_cnt[9];
  if (e->timing) {
    e->imp_counts[0] += n;
    e->imp_counts[1] += nc;
  }
  // (once the call can no longer be refused: after the validation, and in the sliced path after
  // the oversize check)
  auto touch_all = [&] {
    hipLaunchKernelGGL(k_import_touch, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, slot, e->htouch);
  };
  if (!nc) {
    touch_all();
    return;
  }
  // The emits run on their own stream (in timing mode on st, between their events): once the
  // previous drain has read the run (ev_imp_free, after its k_pay_move), a slice's emit goes on
  // beside that drain's replay, filling the other weights buffer; the next drain waits for it
  // (ev_imp_emit).  The count pass, the scan and the cuts above ran on st and were waited for.
  if (!e->st_imp) {
    // created at the first histo import, not with the engine: hardware queues are dealt to streams
    // in creation order, and one more stream per engine made two engines' streams share a queue
    // (windows in flight then ran in lock step: C4 80.6 -> 140.9 ms per window)
    VN_HIP_CHECK(hipStreamCreateWithFlags(&e->st_imp, hipStreamNonBlocking));
    VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_imp_free, hipEventDisableTiming));
    VN_HIP_CHECK(hipEventCreateWithFlags(&e->ev_imp_emit, hipEventDisableTiming));
  }
  hipStream_t se = e->timing ? st : e->st_imp;
  auto emit = [&](uint64_t m, uint64_t b0, uint64_t base) {
    VN_HIP_CHECK(hipStreamWaitEvent(se, e->ev_imp_free, 0));
    ev_pair(e->pool_id, [&] {
      hipLaunchKernelGGL(k_gob_emit_seg, dim3(blocks_for(m * kSegs, 256)), dim3(256), 0, se, m, off + b0, bytes,
                         slot + b0, s.coff + b0, s.cpos + b0, s.ckpt + b0 * kSegs, base, s.cmean, s.cw, s.pslot,
                         s.pbeg, s.npay);
      hipLaunchKernelGGL(k_gob_emit, dim3(blocks_for(m, 256)), dim3(256), 0, se, m, off + b0, bytes, slot + b0,
                         s.coff + b0, s.cpos + b0, base, s.cmean, s.cw, s.pslot, s.pbeg, s.npay, e->h_err);
    });
    VN_HIP_CHECK(hipEventRecord(e->ev_imp_emit, se));
  };
  if (nc <= s.cap_cent && n <= s.cap_pay) {
    touch_all();
    if (s.acc + nc > s.cap_cent || s.npay + n > s.cap_pay) histo_imports_drain(e);
    emit(n, 0, s.acc);
    s.acc += nc;
    s.npay += n;
    VN_HIP_CHECK(hipStreamWaitEvent(st, e->ev_imp_emit, 0));  // (later work on st -- a staging copy
    return;                                                    // over these payloads -- after the emits)
  }
  // slices of whole payloads in arrival order, each at most the run, cut greedily on the device
  // (k_import_cuts: only the cuts come back, not the 4-byte scan of every payload -- that copy and
  // a host loop over it held the GPU idle ≈9 ms per C5 window); a payload larger than the run is
  // refused before anything is emitted
  const size_t ncut = 2 * (kImportCuts + 1) + 2;
  std::vector<std::pair<uint32_t, uint32_t>> cuts;  // (first payload, its first centroid); n last
  for (uint64_t b0 = 0; b0 < n;) {
    hipLaunchKernelGGL(k_import_cuts, dim3(1), dim3(1), 0, st, s.coff, n, b0, s.cap_cent, s.cap_pay, s.cuts);
    VN_HIP_CHECK(hipMemcpyAsync(s.hcuts, s.cuts, ncut * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    VN_HIP_CHECK(hipStreamSynchronize(st));
    const uint32_t j = s.hcuts[2 * (kImportCuts + 1)];
    if (s.hcuts[2 * (kImportCuts + 1) + 1])
      throw std::invalid_argument("one imported digest holds more centroids than max_batch_records");
    for (uint32_t q = 0; q < j; q++) cuts.emplace_back(s.hcuts[q], s.hcuts[kImportCuts + 1 + q]);
    b0 = s.hcuts[j];
    if (b0 >= n) cuts.emplace_back((uint32_t)n, s.hcuts[kImportCuts + 1 + j]);
  }
  touch_all();
  for (size_t q = 0; q + 1 < cuts.size(); q++) {
    const uint64_t b0 = cuts[q].first, b1 = cuts[q + 1].first, c0 = cuts[q].second, c1 = cuts[q + 1].second;
    if (c1 > c0) {
      if (s.acc + (c1 - c0) > s.cap_cent || s.npay + (b1 - b0) > s.cap_pay) histo_imports_drain(e);
      emit(b1 - b0, b0, s.acc - c0);
      s.acc += c1 - c0;
      s.npay += b1 - b0;
    }
  }
  VN_HIP_CHECK(hipStreamWaitEvent(st, e->ev_imp_emit, 0));
}

// The run merges as one histo ingest.  Its centroids are grouped by key through their payloads:
// the payload table (slot, first centroid; arrival order) sorted stably by slot, each payload's
// place the scan of the counts in that order, then one wave per payload moves its centroids
// there -- the order a stable sort of the centroids by slot gives (a payload's centroids stay
// together and in order), at one read and one write per centroid instead of a radix sort of
// every centroid record.
void histo_imports_drain(vn_engine* e) {
  ImportScratch& s = e->imp;
  if (!s.acc) {
    s.npay = 0;
    return;
  }
  const uint64_t n = s.acc, np = s.npay;
  s.acc = 0;
  s.npay = 0;
  hipStream_t st = e->st;
  if (e->ev_imp_emit) VN_HIP_CHECK(hipStreamWaitEvent(st, e->ev_imp_emit, 0));  // the run's emits (st_imp) are done
  hipEvent_t a = e->timing ? e->pool_im.next() : nullptr, b = e->timing ? e->pool_im.next() : nullptr;
  if (a && b) VN_HIP_CHECK(hipEventRecord(a, st));
  hipLaunchKernelGGL(k_pay_keys, dim3(blocks_for(np, 256)), dim3(256), 0, st, np, s.pslot, s.pkey, s.pbeg,
                     (uint32_t)n);
  RadixPass passes[4];
  const int npass = make_passes(passes, false, 32, e->slot_bits[VN_HISTO]);
  const uint64_t* key =
      radix_sort(s.pkey, nullptr, s.pkey + s.cap_pay, nullptr, np, passes, npass, e->rs, st, nullptr) ? s.pkey + s.cap_pay
                                                                                                    : s.pkey;
  hipLaunchKernelGGL(k_pay_counts, dim3(blocks_for(np, 256)), dim3(256), 0, st, np, key, s.pbeg, s.pcnt);
  scan_exclusive_u32(s.pcnt, s.pdst, np, e->ss, st);
  hipLaunchKernelGGL(k_pay_move, dim3(blocks_for(np, 4)), dim3(256), 0, st, np, key, s.pbeg, s.pdst, s.cmean, e->hA0,
                     e->hB0);
  hipLaunchKernelGGL(k_pay_seg_mark, dim3(blocks_for(np, 256)), dim3(256), 0, st, np, key, s.pdst, s.pcnt, e->h_start,
                     e->h_end, e->h_bt, e->htouch);
  if (e->ev_imp_free) VN_HIP_CHECK(hipEventRecord(e->ev_imp_free, st));  // the payload table and the means are read
  double* const w = s.cw;
  std::swap(s.cw, s.cw_alt);  // the next emits fill the other weights buffer while this replay reads w
  histo_process(e, n, histo_group_sorted(e, n, e->hA0, e->hB0, e->hA1, e->hB1, true), w);
  if (a && b) VN_HIP_CHECK(hipEventRecord(b, st));
}

}  // namespace vn

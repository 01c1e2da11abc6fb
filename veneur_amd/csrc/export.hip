// export.hip -- the forward encoders of a local veneur (flusher.go:264-353 flushForward):
//   Histo.Export (samplers/samplers.go:501-514) = MergingDigest.GobEncode
//     (tdigest/merging_digest.go:361-380): mergeAllTemps, then gob of []Centroid, compression,
//     min, max -- the byte stream fixtures/import.uncompressed holds
//   Set.Export (samplers.go:296-310) = Sketch.MarshalBinary (hyperloglog.go:270-315); the
//     tmpSet is written in ascending order where Go follows map iteration order
// They also carry the multi-GPU exchange of hot keys: a rank exports a key's partial state,
// the bytes travel by RCCL all-gather, and the owner imports them (veneur_amd/dist.py).
// Sizes first (one lane per digest: a dry run of the writer; sets: from the state), an
// exclusive scan, then the bytes (histos: one lane per digest; sets: one workgroup per key,
// the varint list written in parallel from a scan of the per-code lengths).
#include "histo.h"

namespace vn {

namespace {

// encoding/gob writer; W = false only counts bytes
template <bool W>
struct GobOut {
  uint8_t* d;
  uint32_t n;
  __device__ void byte(uint32_t b) {
    if (W) d[n] = (uint8_t)b;
    n++;
  }
  __device__ void u(uint64_t x) {
    if (x < 0x80) {
      byte((uint32_t)x);
      return;
    }
    int nb = 0;
    for (uint64_t y = x; y; y >>= 8) nb++;
    byte(256u - (uint32_t)nb);
    for (int k = nb - 1; k >= 0; k--) byte((uint32_t)(x >> (8 * k)) & 0xffu);
  }
  __device__ void s(int64_t i) { u(i < 0 ? ((uint64_t)(~i) << 1) | 1u : (uint64_t)i << 1); }
  __device__ void f(double x) {  // IEEE bits byte-reversed
    uint64_t v = dbits(x), r = 0;
    for (int k = 0; k < 8; k++) {
      r = (r << 8) | (v & 0xffu);
      v >>= 8;
    }
    u(r);
  }
  __device__ void str(const char* p, uint32_t len) {
    u(len);
    for (uint32_t k = 0; k < len; k++) byte((uint8_t)p[k]);
  }
};

// message bodies of the digest stream (type ids 66 Centroid, 67 []float64, 68 []Centroid, as Go
// assigns them for MergingDigest: encoding/gob type.go)
template <bool W>
__device__ void body_slice_type(GobOut<W>& o) {
  o.s(-68); o.u(2); o.u(1); o.u(2); o.s(68); o.u(0); o.u(1); o.s(66); o.u(0); o.u(0);
}
template <bool W>
__device__ void body_struct_type(GobOut<W>& o) {
  o.s(-66); o.u(3); o.u(1); o.u(1); o.str("Centroid", 8); o.u(1); o.s(66); o.u(0); o.u(1); o.u(3);
  o.u(1); o.str("Mean", 4); o.u(1); o.s(4); o.u(0);
  o.u(1); o.str("Weight", 6); o.u(1); o.s(4); o.u(0);
  o.u(1); o.str("Samples", 7); o.u(1); o.s(67); o.u(0);
  o.u(0); o.u(0);
}
template <bool W>
__device__ void body_floats_type(GobOut<W>& o) {
  o.s(-67); o.u(2); o.u(1); o.u(1); o.str("[]float64", 9); o.u(1); o.s(67); o.u(0); o.u(1); o.s(4); o.u(0); o.u(0);
}
template <bool W>
__device__ void body_centroids(GobOut<W>& o, const double* m, const double* w, uint32_t nc) {
  o.s(68); o.u(0); o.u(nc);
  for (uint32_t i = 0; i < nc; i++) {
    int64_t last = -1;  // gob omits zero fields
    if (m[i] != 0.0) { o.u((uint64_t)(0 - last)); o.f(m[i]); last = 0; }
    if (w[i] != 0.0) { o.u((uint64_t)(1 - last)); o.f(w[i]); last = 1; }
    o.u(0);
  }
}
template <bool W>
__device__ void body_float(GobOut<W>& o, double v) {
  o.s(4); o.u(0); o.f(v);
}

// one message = uint(len(body)) + body
template <bool W, class F>
__device__ void message(GobOut<W>& o, F body) {
  GobOut<false> c{nullptr, 0};
  body(c);
  o.u(c.n);
  body(o);
}

template <bool W>
__device__ uint32_t gob_digest_write(uint8_t* out, const double* m, const double* w, uint32_t nc, double compression,
                                     double mn, double mx) {
  GobOut<W> o{out, 0};
  message(o, [](auto& b) { body_slice_type(b); });
  message(o, [](auto& b) { body_struct_type(b); });
  message(o, [](auto& b) { body_floats_type(b); });
  message(o, [&](auto& b) { body_centroids(b, m, w, nc); });
  message(o, [&](auto& b) { body_float(b, compression); });
  message(o, [&](auto& b) { body_float(b, mn); });
  message(o, [&](auto& b) { body_float(b, mx); });
  return o.n;
}

struct HistoView {
  const double* hst;
  const uint32_t* hncent;
  const uint8_t* hcur;
  const double *cm0, *cm1, *cw0, *cw1;
  uint32_t capc;
  double compression;
};

template <bool W>
__global__ void k_gob_encode(uint64_t n, const uint32_t* __restrict__ slot, HistoView v, uint32_t* __restrict__ size,
                             const uint64_t* __restrict__ off, uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slot[i];
  const uint8_t c = v.hcur[s];
  const double* m = (c ? v.cm1 : v.cm0) + (uint64_t)s * v.capc;
  const double* w = (c ? v.cw1 : v.cw0) + (uint64_t)s * v.capc;
  const double* h = v.hst + (uint64_t)s * VN_HISTO_STATS;
  const uint32_t len = gob_digest_write<W>(W ? out + off[i] : nullptr, m, w, v.hncent[s], v.compression, h[5], h[6]);
  if (!W) size[i] = len;
}

// ---- sets
struct SetView {
  const uint8_t* mode;
  const uint8_t* base;
  const uint32_t* lc;
  const uint32_t* lb;
  const uint32_t* last;
  const uint32_t* tc;
  const uint32_t* tmp;
  const uint32_t* arena;
};

__global__ void k_marshal_size(uint64_t n, const uint32_t* __restrict__ slot, SetView v, uint32_t* __restrict__ size) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slot[i];
  size[i] = v.mode[s] ? 8u + kHllM / 2 : 8u + 4u * v.tc[s] + 12u + v.lb[s];
}

__device__ __forceinline__ void put_be32(uint8_t* d, uint32_t x) {
  d[0] = (uint8_t)(x >> 24);
  d[1] = (uint8_t)(x >> 16);
  d[2] = (uint8_t)(x >> 8);
  d[3] = (uint8_t)x;
}

__global__ __launch_bounds__(kBlock) void k_marshal(const uint32_t* __restrict__ slot, SetView v,
                                                    const uint64_t* __restrict__ off, uint8_t* __restrict__ out) {
  __shared__ uint32_t s_tmp[256];
  __shared__ uint32_t s_wave[4];
  const uint32_t i = blockIdx.x, t = threadIdx.x;
  const uint32_t s = slot[i];
  uint8_t* d = out + off[i];
  const uint32_t* ar = v.arena + (uint64_t)s * kArenaWords;
  if (t == 0) {
    d[0] = 1;  // version (hyperloglog.go:11)
    d[1] = (uint8_t)kHllP;
    d[2] = v.base[s];
    d[3] = v.mode[s] ? 0 : 1;
  }
  if (v.mode[s]) {  // dense: m/2 tailcut bytes, high nibble = even register
    if (t == 0) put_be32(d + 4, kHllM / 2);
    const uint8_t* regs = reinterpret_cast<const uint8_t*>(ar);
    for (uint32_t k = t; k < kHllM / 2; k += kBlock) d[8 + k] = (uint8_t)((regs[2 * k] << 4) | (regs[2 * k + 1] & 15u));
    return;
  }
  // sparse: tmpSet (ascending), then count, last, byte length, varint deltas
  const uint32_t tc = v.tc[s], lc = v.lc[s];
  s_tmp[t] = t < tc ? v.tmp[(uint64_t)s * kTmpCap + t] : 0xffffffffu;
  __syncthreads();
  for (uint32_t k = 2; k <= 256; k <<= 1)  // bitonic sort of the tmpSet codes
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      const uint32_t ixj = t ^ j;
      if (ixj > t) {
        const uint32_t a = s_tmp[t], b = s_tmp[ixj];
        if ((a > b) == ((t & k) == 0)) {
          s_tmp[t] = b;
          s_tmp[ixj] = a;
        }
      }
      __syncthreads();
    }
  if (t == 0) put_be32(d + 4, tc);
  if (t < tc) put_be32(d + 8 + 4 * t, s_tmp[t]);
  uint8_t* L = d + 8 + 4 * tc;
  if (t == 0) {
    put_be32(L, lc);
    put_be32(L + 4, v.last[s]);
    put_be32(L + 8, v.lb[s]);
  }
  uint8_t* B = L + 12;
  // varint deltas (compressedList.Append, compressed.go:114-118, 167-173): per-thread runs
  const uint32_t per = (lc + kBlock - 1) / kBlock, lo = min(lc, t * per), hi = min(lc, lo + per);
  uint32_t bytes = 0;
  for (uint32_t k = lo; k < hi; k++) bytes += varint_len(ar[k] - (k ? ar[k - 1] : 0u));
  uint32_t total;
  uint32_t pos = block_scan_sum_u32(bytes, s_wave, total);
  for (uint32_t k = lo; k < hi; k++) {
    uint32_t x = ar[k] - (k ? ar[k - 1] : 0u);
    while (x & 0xffffff80u) {
      B[pos++] = (uint8_t)((x & 0x7fu) | 0x80u);
      x >>= 7;
    }
    B[pos++] = (uint8_t)(x & 0x7fu);
  }
}

}  // namespace

// sizes -> offsets (host copy) -> bytes (device), then the host copies of both
static void finish_export(vn_engine* e, uint64_t n, ExportBuffers& x) {
  VN_HIP_CHECK(hipMemcpyAsync(x.h_off, x.d_off, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, e->st));
  VN_HIP_CHECK(hipStreamSynchronize(e->st));
}

void export_histos(vn_engine* e, const uint32_t* dev_slot, uint64_t n, ExportBuffers& x) {
  hipStream_t st = e->st;
  HistoView v{e->hst, e->hncent, e->hcur, e->cmean[0], e->cmean[1], e->cw[0], e->cw[1], e->cap_cent,
              e->cfg.compression};
  hipLaunchKernelGGL(k_gob_encode<false>, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, dev_slot, v, x.d_size,
                     nullptr, nullptr);
  scan_sizes_u64(x.d_size, x.d_off, n, st);
  finish_export(e, n, x);
  ensure_export_bytes(e, x, x.h_off[n]);
  hipLaunchKernelGGL(k_gob_encode<true>, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, dev_slot, v, nullptr, x.d_off,
                     x.d_bytes);
  VN_HIP_CHECK(hipMemcpyAsync(x.h_bytes, x.d_bytes, x.h_off[n], hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
}

void export_sets(vn_engine* e, const uint32_t* dev_slot, uint64_t n, ExportBuffers& x) {
  hipStream_t st = e->st;
  SetView v{e->smode, e->sbase, e->slc, e->slb, e->slast, e->stc, e->stmp, e->sarena};
  hipLaunchKernelGGL(k_marshal_size, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, dev_slot, v, x.d_size);
  scan_sizes_u64(x.d_size, x.d_off, n, st);
  finish_export(e, n, x);
  ensure_export_bytes(e, x, x.h_off[n]);
  hipLaunchKernelGGL(k_marshal, dim3((uint32_t)n), dim3(kBlock), 0, st, dev_slot, v, x.d_off, x.d_bytes);
  VN_HIP_CHECK(hipMemcpyAsync(x.h_bytes, x.d_bytes, x.h_off[n], hipMemcpyDeviceToHost, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
}

}  // namespace vn

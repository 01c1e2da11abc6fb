// DogStatsD metric lines -> parsed records on the GPU.
//
// Restates samplers/parser.go:186-307 (ParseMetric) for every line of a datagram buffer already in
// HBM, split on '\n' (server.go:706-714; empty packets skipped, server.go:612-616), with the same
// output as the host parse vn_parse_dogstatsd (csrc/parse.cpp) -- the checker in the GPU tests.
//
//   k_ls_count / k_ls_emit   line starts: byte i starts a line when it is not '\n' and i == 0 or
//                            buf[i-1] == '\n'; per-4 KiB-tile counts, a scan, then each tile writes
//                            its starts in byte order (ballot ranks per wave, LDS ranks per tile)
//   k_parse_lines            one lane per line: name / value / type sections, Go 1.9 ParseFloat
//                            (gofloat.h: exact fast paths inline, the 800-digit decimal path
//                            deferred to k_parse_slow), sample rate, tag section bounds, the scope
//                            tag Go removes (the smallest tag with a veneurglobalonly /
//                            veneurlocalonly prefix: every global one sorts before every local
//                            one), joined-tag length, FNV-1a of name and type
//   k_parse_slow             the deferred numbers, one 816-byte decimal per lane of a small grid
//   scan                     joined-tag offsets of the lines that parse (tags_out is the host
//                            parse's tags_out byte for byte)
//   k_parse_tags             sort.Strings by rank (tag j before tag i when it is smaller, or equal
//                            and earlier), each kept tag written at its rank's offset, then
//                            FNV-1a over the joined tags (UDPMetric.Digest)
// HBM traffic: the buffer is read about twice (starts, then the parse), tags read again and
// written once; per line a 64-byte vn_parsed_line.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "gofloat.h"
#include "primitives.h"
#include "veneur_amd.h"

using vn::gofloat::Decimal;

struct vn_parser {
  int device = 0;
  hipStream_t st = nullptr;
  uint64_t max_bytes = 0, max_lines = 0;
  uint32_t* tile_cnt = nullptr;   // per 4 KiB tile, then its exclusive scan (+ total)
  uint32_t* tile_off = nullptr;
  uint32_t* starts = nullptr;     // line start offsets
  uint32_t* tsec = nullptr;       // per line: tag section offset, length
  int32_t* removed = nullptr;     // per line: index of the removed scope tag or -1
  uint32_t* tlen = nullptr;       // per line: joined tag bytes (0 unless the line parses with tags)
  uint32_t* toff = nullptr;       // its exclusive scan
  uint32_t* slow = nullptr;       // [0] count, then the lines with a deferred number
  Decimal* dec = nullptr;         // k_parse_slow scratch
  uint32_t* h_total = nullptr;    // pinned
  vn::ScanScratch scan;
  std::string err;
};

namespace vn {
namespace {

constexpr int kLsBlock = 256;
constexpr int kLsPer = 16;
constexpr uint32_t kLsTile = kLsBlock * kLsPer;  // 4096 bytes
constexpr int kSlowLanes = 2048;

__device__ __forceinline__ bool is_start(const uint8_t* __restrict__ buf, uint64_t i) {
  return buf[i] != '\n' && (i == 0 || buf[i - 1] == '\n');
}

__global__ __launch_bounds__(kLsBlock) void k_ls_count(const uint8_t* __restrict__ buf, uint64_t len,
                                                       uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s_w[kLsBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kLsTile;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kLsPer; j++) {
    const uint64_t i = base + (uint64_t)j * kLsBlock + threadIdx.x;
    c += (i < len && is_start(buf, i)) ? 1u : 0u;
  }
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ __launch_bounds__(kLsBlock) void k_ls_emit(const uint8_t* __restrict__ buf, uint64_t len,
                                                      const uint32_t* __restrict__ off, uint32_t* __restrict__ starts) {
  __shared__ uint32_t s_c[kLsPer][kLsBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kLsTile;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint64_t masks[kLsPer];
#pragma unroll
  for (int j = 0; j < kLsPer; j++) {
    const uint64_t i = base + (uint64_t)j * kLsBlock + threadIdx.x;
    masks[j] = __ballot(i < len && is_start(buf, i));
    if (lane == 0) s_c[j][w] = (uint32_t)__popcll(masks[j]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // byte order within the tile is (j, wave, lane)
    uint32_t run = off[blockIdx.x];
    for (int j = 0; j < kLsPer; j++)
      for (int q = 0; q < kLsBlock / 64; q++) {
        const uint32_t c = s_c[j][q];
        s_c[j][q] = run;
        run += c;
      }
  }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int j = 0; j < kLsPer; j++) {
    if ((masks[j] >> lane) & 1ull)
      starts[s_c[j][w] + (uint32_t)__popcll(masks[j] & lt)] = (uint32_t)(base + (uint64_t)j * kLsBlock + threadIdx.x);
  }
}

__device__ __forceinline__ uint32_t fnv(uint32_t h, const uint8_t* p, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x01000193u;
  return h;
}

__device__ __forceinline__ uint32_t find(const uint8_t* p, uint32_t from, uint32_t to, uint8_t c) {
  for (uint32_t i = from; i < to; i++)
    if (p[i] == c) return i;
  return to;
}

__device__ __forceinline__ bool has_prefix(const uint8_t* p, uint32_t n, const char* w, uint32_t m) {
  if (n < m) return false;
  for (uint32_t i = 0; i < m; i++)
    if (p[i] != (uint8_t)w[i]) return false;
  return true;
}

// Go's string order: bytes, then length
__device__ __forceinline__ int str_cmp(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb) {
  const uint32_t m = na < nb ? na : nb;
  for (uint32_t i = 0; i < m; i++)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return na < nb ? -1 : (na > nb ? 1 : 0);
}

// deferred-number marks in the status word while the slow kernel is pending
constexpr int32_t kValueDeferred = 1 << 16;
constexpr int32_t kRateDeferred = 1 << 17;

__global__ __launch_bounds__(256) void k_parse_lines(const uint8_t* __restrict__ buf, uint64_t len,
                                                     const uint32_t* __restrict__ starts, uint32_t n,
                                                     vn_parsed_line* __restrict__ out, uint32_t* __restrict__ tsec,
                                                     int32_t* __restrict__ removed, uint32_t* __restrict__ tlen,
                                                     uint32_t* __restrict__ slow) {
  const uint32_t li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= n) return;
  const uint32_t p = starts[li];
  const uint32_t end = find(buf, p, (uint32_t)len, '\n');
  vn_parsed_line o;
  o.line_off = p;
  o.line_len = end - p;
  o.name_off = o.value_off = 0;
  o.name_len = o.value_len = 0;
  o.tags_off = 0;
  o.tags_len = 0;
  o.n_tags = 0;
  o.digest = 0;
  o.value = 0.0;
  o.rate = 1.0f;
  o.type = 0;
  o.scope = 0;
  o.has_tags = 0;
  o.pad = 0;
  int32_t status = VN_PARSE_OK;
  uint32_t sec_off = 0, sec_len = 0, jl = 0;
  int32_t rm = -1;
  const uint32_t ln = end - p;
  do {
    if (ln >= 3 && buf[p] == '_' &&
        ((buf[p + 1] == 'e' && buf[p + 2] == '{') || (buf[p + 1] == 's' && buf[p + 2] == 'c'))) {
      status = VN_PARSE_NOT_METRIC;
      break;
    }
    const uint32_t pipe = find(buf, p, end, '|');
    const uint32_t colon = find(buf, p, pipe, ':');
    if (colon == pipe) { status = VN_PARSE_NO_COLON; break; }
    if (colon == p) { status = VN_PARSE_EMPTY_NAME; break; }
    o.name_off = p;
    o.name_len = colon - p;
    o.value_off = colon + 1;
    o.value_len = pipe - colon - 1;
    if (pipe == end) { status = VN_PARSE_NO_PIPE; break; }
    const uint32_t t = pipe + 1;
    const uint32_t tend = find(buf, t, end, '|');
    if (tend == t) { status = VN_PARSE_NO_TYPE; break; }
    const char* tname;
    uint32_t tn;
    switch (buf[t]) {
      case 'c': o.type = 0; tname = "counter"; tn = 7; break;
      case 'g': o.type = 1; tname = "gauge"; tn = 5; break;
      case 'h': o.type = 2; tname = "histogram"; tn = 9; break;
      case 'm': o.type = 3; tname = "timer"; tn = 5; break;
      case 's': o.type = 4; tname = "set"; tn = 3; break;
      default: tname = nullptr; tn = 0; break;
    }
    if (!tname) { status = VN_PARSE_BAD_TYPE; break; }
    uint32_t h = fnv(0x811C9DC5u, buf + p, o.name_len);
    h = fnv(h, reinterpret_cast<const uint8_t*>(tname), tn);
    o.digest = h;
    if (o.type != 4) {
      double v = 0.0;
      const int r = gofloat::parse_float(reinterpret_cast<const char*>(buf) + o.value_off, o.value_len, 64, &v,
                                         nullptr);
      if (r == gofloat::kDefer) {
        status |= kValueDeferred;
      } else if (r != gofloat::kOk || v != v || v - v != 0.0) {
        status = VN_PARSE_BAD_VALUE;
        break;
      } else {
        o.value = v;
      }
    }
    bool found_rate = false;
    uint32_t s = tend;
    int32_t sec = VN_PARSE_OK;
    while (s < end) {  // s is the '|' before the next section
      const uint32_t c = s + 1;
      const uint32_t cend = find(buf, c, end, '|');
      const uint32_t cn = cend - c;
      if (cn == 0) { sec = VN_PARSE_EMPTY_SECTION; break; }
      if (buf[c] == '@') {
        if (found_rate) { sec = VN_PARSE_MULTI_RATE; break; }
        double r = 0.0;
        const int rc = gofloat::parse_float(reinterpret_cast<const char*>(buf) + c + 1, cn - 1, 32, &r, nullptr);
        found_rate = true;
        if (rc == gofloat::kDefer) {
          status |= kRateDeferred;  // its range check follows in k_parse_slow
          o.value_off = (o.value_off & 0xffffffffull) | ((uint64_t)(c + 1) << 32);  // (parked: rate offset)
        } else {
          if (rc != gofloat::kOk) { sec = VN_PARSE_BAD_RATE; break; }
          if (r <= 0 || r > 1) { sec = VN_PARSE_RATE_RANGE; break; }  // NaN passes, as in Go
          o.rate = (float)r;
        }
      } else if (buf[c] == '#') {
        if (o.has_tags) { sec = VN_PARSE_MULTI_TAGS; break; }
        o.has_tags = 1;
        sec_off = c + 1;
        sec_len = cn - 1;
        // tags: count, bytes, and the scope tag Go's loop removes (parser.go:278-292)
        const uint8_t* q = buf + sec_off;
        uint32_t nt = 0, tb = 0, a = 0;
        int32_t best_g = -1, best_l = -1;
        uint32_t bg_o = 0, bg_n = 0, bl_o = 0, bl_n = 0;
        for (uint32_t k = 0; k <= sec_len; k++) {
          if (k == sec_len || q[k] == ',') {
            const uint32_t tl = k - a;
            if (has_prefix(q + a, tl, "veneurglobalonly", 16)) {
              if (best_g < 0 || str_cmp(q + a, tl, q + bg_o, bg_n) < 0) { best_g = (int32_t)nt; bg_o = a; bg_n = tl; }
            } else if (has_prefix(q + a, tl, "veneurlocalonly", 15)) {
              if (best_l < 0 || str_cmp(q + a, tl, q + bl_o, bl_n) < 0) { best_l = (int32_t)nt; bl_o = a; bl_n = tl; }
            }
            tb += tl;
            nt++;
            a = k + 1;
          }
        }
        uint32_t kept = nt, kb = tb;
        if (best_g >= 0) { rm = best_g; o.scope = 2; kept--; kb -= bg_n; }
        else if (best_l >= 0) { rm = best_l; o.scope = 1; kept--; kb -= bl_n; }
        o.n_tags = kept;
        jl = kb + (kept ? kept - 1 : 0);
      } else {
        sec = VN_PARSE_UNKNOWN_SECTION;
        break;
      }
      s = cend;
    }
    status |= sec;
  } while (false);
  const int32_t base = status & 0xffff;
  if (status & (kValueDeferred | kRateDeferred)) slow[1 + atomicAdd(&slow[0], 1u)] = li;
  o.status = status;
  out[li] = o;
  tsec[2 * li] = sec_off;
  tsec[2 * li + 1] = sec_len;
  removed[li] = rm;
  tlen[li] = (base == VN_PARSE_OK && o.has_tags && !(status & (kValueDeferred | kRateDeferred))) ? jl : 0;
  // deferred lines set their tag length once their numbers are known (k_parse_slow)
  if ((status & (kValueDeferred | kRateDeferred)) && base == VN_PARSE_OK && o.has_tags) tlen[li] = jl | 0x80000000u;
}

// The deferred numbers (more than 19 significant digits or a far exponent): Go's decimal path.
// Each lane owns one Decimal and strides over the list; a line's value is resolved before its
// rate (value errors precede every section error, as ParseMetric returns at the value).
__global__ __launch_bounds__(256) void k_parse_slow(const uint8_t* __restrict__ buf, vn_parsed_line* __restrict__ out,
                                                    const uint32_t* __restrict__ slow, uint32_t* __restrict__ tlen,
                                                    Decimal* __restrict__ dec) {
  const uint32_t cnt = slow[0];
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  Decimal* d = dec + tid;
  for (uint32_t k = tid; k < cnt; k += gridDim.x * blockDim.x) {
    const uint32_t li = slow[1 + k];  // one entry per line: its value, then its rate
    vn_parsed_line o = out[li];
    const bool vdef = (o.status & kValueDeferred) != 0, rdef = (o.status & kRateDeferred) != 0;
    int32_t st = o.status & 0xffff;
    bool value_failed = false;
    if (vdef) {
      double v = 0.0;
      const int r = gofloat::parse_float(reinterpret_cast<const char*>(buf) + (uint32_t)o.value_off,
                                         (uint32_t)o.value_len, 64, &v, d);
      if (r != gofloat::kOk || v != v || v - v != 0.0) {
        st = VN_PARSE_BAD_VALUE;
        value_failed = true;
      } else {
        o.value = v;
      }
    }
    if (rdef && !value_failed) {
      // the rate section: from its offset to the next '|' or the line end
      const uint32_t c = (uint32_t)(o.value_off >> 32);
      const uint32_t lend = (uint32_t)o.line_off + o.line_len;
      uint32_t ce = c;
      while (ce < lend && buf[ce] != '|') ce++;
      double r = 0.0;
      const int rc = gofloat::parse_float(reinterpret_cast<const char*>(buf) + c, ce - c, 32, &r, d);
      if (rc != gofloat::kOk) st = VN_PARSE_BAD_RATE;
      else if (r <= 0 || r > 1) st = VN_PARSE_RATE_RANGE;
      else o.rate = (float)r;
    }
    o.value_off &= 0xffffffffull;
    o.status = st;
    out[li] = o;
    const uint32_t tl = tlen[li];
    tlen[li] = (st == VN_PARSE_OK && (tl & 0x80000000u)) ? (tl & 0x7fffffffu) : 0u;
  }
}

__global__ __launch_bounds__(256) void k_parse_tags(const uint8_t* __restrict__ buf, uint32_t n,
                                                    vn_parsed_line* __restrict__ out,
                                                    const uint32_t* __restrict__ tsec,
                                                    const int32_t* __restrict__ removed,
                                                    const uint32_t* __restrict__ toff, uint8_t* __restrict__ tags_out) {
  const uint32_t li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= n) return;
  const uint32_t to = toff[li];
  const uint32_t jl = toff[li + 1] - to;
  vn_parsed_line& o = out[li];
  o.tags_off = to;
  if (o.status != VN_PARSE_OK || !o.has_tags) {
    if (o.status == VN_PARSE_OK) o.tags_len = 0;
    return;
  }
  o.tags_len = jl;
  const uint8_t* q = buf + tsec[2 * li];
  const uint32_t L = tsec[2 * li + 1];
  const int32_t rm = removed[li];
  // tag i at its sorted position: the bytes (+ comma) of every kept tag ranked before it
  uint32_t ai = 0, i = 0;
  for (uint32_t ki = 0; ki <= L; ki++) {
    if (ki != L && q[ki] != ',') continue;
    const uint32_t ni = ki - ai;
    if ((int32_t)i != rm) {
      uint32_t pos = 0, aj = 0, j = 0;
      for (uint32_t kj = 0; kj <= L; kj++) {
        if (kj != L && q[kj] != ',') continue;
        const uint32_t nj = kj - aj;
        if ((int32_t)j != rm && j != i) {
          const int c = str_cmp(q + aj, nj, q + ai, ni);
          if (c < 0 || (c == 0 && j < i)) pos += nj + 1;
        }
        aj = kj + 1;
        j++;
      }
      uint8_t* dst = tags_out + to + pos;
      for (uint32_t b = 0; b < ni; b++) dst[b] = q[ai + b];
      if (pos + ni < jl) dst[ni] = ',';
    }
    ai = ki + 1;
    i++;
  }
  o.digest = fnv(o.digest, tags_out + to, jl);
}

void check_rc(vn_parser* p, hipError_t rc, const char* what) {
  if (rc != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(rc));
}

}  // namespace
}  // namespace vn

using namespace vn;

extern "C" {

int vn_parser_create(int device, uint64_t max_bytes, uint64_t max_lines, vn_parser** out) {
  if (!out || max_bytes >= (1ull << 32) || max_lines >= (1ull << 31)) return VN_EINVAL;
  *out = nullptr;
  vn_parser* p = new vn_parser;
  p->device = device;
  p->max_bytes = max_bytes ? max_bytes : 1;
  p->max_lines = max_lines ? max_lines : 1;
  try {
    check_rc(p, hipSetDevice(device), "hipSetDevice");
    check_rc(p, hipStreamCreateWithFlags(&p->st, hipStreamNonBlocking), "hipStreamCreate");
    const uint64_t ntiles = (p->max_bytes + kLsTile - 1) / kLsTile;
    check_rc(p, hipMalloc(&p->tile_cnt, (ntiles + 1) * 4), "hipMalloc");
    check_rc(p, hipMalloc(&p->tile_off, (ntiles + 1) * 4), "hipMalloc");
    check_rc(p, hipMalloc(&p->starts, p->max_lines * 4), "hipMalloc");
    check_rc(p, hipMalloc(&p->tsec, p->max_lines * 8), "hipMalloc");
    check_rc(p, hipMalloc(&p->removed, p->max_lines * 4), "hipMalloc");
    check_rc(p, hipMalloc(&p->tlen, (p->max_lines + 1) * 4), "hipMalloc");
    check_rc(p, hipMalloc(&p->toff, (p->max_lines + 1) * 4), "hipMalloc");
    check_rc(p, hipMalloc(&p->slow, (p->max_lines + 1) * 4), "hipMalloc");
    check_rc(p, hipMalloc(&p->dec, (uint64_t)kSlowLanes * sizeof(Decimal)), "hipMalloc");
    check_rc(p, hipHostMalloc(&p->h_total, 8), "hipHostMalloc");
  } catch (const std::exception&) {
    vn_parser_destroy(p);
    return VN_ENOMEM;
  }
  *out = p;
  return VN_OK;
}

void vn_parser_destroy(vn_parser* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  if (p->st) (void)hipStreamSynchronize(p->st);
  for (void* q : {(void*)p->tile_cnt, (void*)p->tile_off, (void*)p->starts, (void*)p->tsec, (void*)p->removed,
                  (void*)p->tlen, (void*)p->toff, (void*)p->slow, (void*)p->dec, (void*)p->scan.partials})
    if (q) (void)hipFree(q);
  if (p->h_total) (void)hipHostFree(p->h_total);
  if (p->st) (void)hipStreamDestroy(p->st);
  delete p;
}

const char* vn_parser_last_error(const vn_parser* p) { return p ? p->err.c_str() : "null parser"; }

int vn_parse_dogstatsd_device(vn_parser* p, const char* buf, uint64_t len, vn_parsed_line* out, uint64_t max_lines,
                              char* tags_out, uint64_t tags_cap, uint64_t* n_lines) {
  if (!p || !n_lines) return VN_EINVAL;
  if (len > p->max_bytes || (len && !buf) || tags_cap < len || (len && !tags_out)) {
    p->err = "buffer longer than the parser's max_bytes, or tags_out smaller than the buffer";
    return VN_EINVAL;
  }
  *n_lines = 0;
  if (len == 0) return VN_OK;
  try {
    check_rc(p, hipSetDevice(p->device), "hipSetDevice");
    const uint8_t* b = reinterpret_cast<const uint8_t*>(buf);
    const uint32_t ntiles = (uint32_t)((len + kLsTile - 1) / kLsTile);
    hipLaunchKernelGGL(k_ls_count, dim3(ntiles), dim3(kLsBlock), 0, p->st, b, len, p->tile_cnt);
    scan_exclusive_u32(p->tile_cnt, p->tile_off, ntiles, p->scan, p->st);
    check_rc(p, hipMemcpyAsync(p->h_total, p->tile_off + ntiles, 4, hipMemcpyDeviceToHost, p->st), "hipMemcpy");
    check_rc(p, hipStreamSynchronize(p->st), "line count");
    const uint32_t n = p->h_total[0];
    if (n > max_lines || n > p->max_lines || (n && !out)) {
      p->err = "more lines than max_lines (" + std::to_string(n) + ")";
      return VN_EINVAL;
    }
    *n_lines = n;
    if (!n) return VN_OK;
    hipLaunchKernelGGL(k_ls_emit, dim3(ntiles), dim3(kLsBlock), 0, p->st, b, len, p->tile_off, p->starts);
    check_rc(p, hipMemsetAsync(p->slow, 0, 4, p->st), "hipMemset");
    hipLaunchKernelGGL(k_parse_lines, dim3(blocks_for(n, 256)), dim3(256), 0, p->st, b, len, p->starts, n, out,
                       p->tsec, p->removed, p->tlen, p->slow);
    hipLaunchKernelGGL(k_parse_slow, dim3(kSlowLanes / 256), dim3(256), 0, p->st, b, out, p->slow, p->tlen, p->dec);
    scan_exclusive_u32(p->tlen, p->toff, n, p->scan, p->st);
    hipLaunchKernelGGL(k_parse_tags, dim3(blocks_for(n, 256)), dim3(256), 0, p->st, b, n, out, p->tsec, p->removed,
                       p->toff, reinterpret_cast<uint8_t*>(tags_out));
    check_rc(p, hipGetLastError(), "launch");
    check_rc(p, hipStreamSynchronize(p->st), "parse");
    return VN_OK;
  } catch (const std::exception& x) {
    p->err = x.what();
    return VN_EHIP;
  }
}

// The device ParseFloat run on the host (known-answer / fuzz checks against strtod, strtof).
int vn_go_parse_float(const char* s, uint64_t n, int bits, double* out) {
  if ((!s && n) || !out || (bits != 32 && bits != 64) || n >= (1ull << 31)) return VN_EINVAL;
  static thread_local Decimal d;
  return gofloat::parse_float(s, (uint32_t)n, bits, out, &d);
}

}  // extern "C"

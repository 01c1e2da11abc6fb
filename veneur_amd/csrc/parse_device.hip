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
constexpr uint32_t kLsTile = kLsBlock * 16;  // 4096 bytes: 16 per thread
constexpr int kSlowLanes = 2048;

// Line starts of thread t's 16 bytes [base + 16t, +16) as a 16-bit mask: byte j starts a line when
// it is not '\n' and the byte before it is '\n' (or it is the buffer's first byte).  The bytes come
// in one 16-byte load (the buffer's last partial chunk byte by byte); the byte before them is the
// previous lane's last byte, or one load for lane 0 of each wave.
__device__ __forceinline__ uint32_t start_mask(const uint8_t* __restrict__ buf, uint64_t len, uint64_t pos) {
  uint32_t w[4] = {0x0a0a0a0au, 0x0a0a0a0au, 0x0a0a0a0au, 0x0a0a0a0au};  // past the end: '\n' (no starts)
  if (pos + 16 <= len && !(reinterpret_cast<uintptr_t>(buf) & 15u)) {
    const uint4 v = *reinterpret_cast<const uint4*>(buf + pos);
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else if (pos < len) {  // the last partial chunk, or a buffer that is not 16-byte aligned
    for (uint32_t j = 0; j < 16 && pos + j < len; j++)
      w[j >> 2] = (w[j >> 2] & ~(0xffu << (8 * (j & 3)))) | ((uint32_t)buf[pos + j] << (8 * (j & 3)));
  }
  const int lane = threadIdx.x & 63;
  uint32_t prev = __shfl_up(w[3] >> 24, 1, 64);
  if (lane == 0) prev = pos == 0 ? '\n' : (pos - 1 < len ? buf[pos - 1] : '\n');
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xffu;
    m |= (c != '\n' && prev == '\n') ? (1u << j) : 0u;
    prev = c;
  }
  return m;
}

__global__ __launch_bounds__(kLsBlock) void k_ls_count(const uint8_t* __restrict__ buf, uint64_t len,
                                                       uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s_w[kLsBlock / 64];
  const uint64_t pos = (uint64_t)blockIdx.x * kLsTile + 16u * threadIdx.x;
  uint32_t c = __popc(start_mask(buf, len, pos));
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ __launch_bounds__(kLsBlock) void k_ls_emit(const uint8_t* __restrict__ buf, uint64_t len,
                                                      const uint32_t* __restrict__ off, uint32_t* __restrict__ starts) {
  __shared__ uint32_t s_w[kLsBlock / 64];
  const uint64_t pos = (uint64_t)blockIdx.x * kLsTile + 16u * threadIdx.x;
  const uint32_t m = start_mask(buf, len, pos);
  const uint32_t c = __popc(m);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = c;  // inclusive scan over the wave
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_w[w] = incl;
  __syncthreads();
  uint32_t run = off[blockIdx.x];
  for (int q = 0; q < w; q++) run += s_w[q];
  run += incl - c;
  uint32_t mm = m;
  while (mm) {
    const int j = __ffs(mm) - 1;
    mm &= mm - 1;
    starts[run++] = (uint32_t)(pos + j);
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

// One line: buf[p, ...) up to the next '\n' or wend.  buf is the LDS window of the block's lines
// (off0 = the window's offset in the datagram buffer) or the buffer itself (off0 = 0).
__device__ __forceinline__ void parse_one(const uint8_t* buf, uint32_t off0, uint32_t p, uint32_t wend, uint32_t li,
                                          vn_parsed_line* __restrict__ out, uint32_t* __restrict__ tsec,
                                          int32_t* __restrict__ removed, uint32_t* __restrict__ tlen,
                                          uint32_t* __restrict__ slow) {
  const uint32_t end = find(buf, p, wend, '\n');
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
  o.line_off += off0;
  if (o.name_len || o.value_off) {
    o.name_off += off0;
    o.value_off = (o.value_off & 0xffffffff00000000ull) | ((o.value_off & 0xffffffffull) + off0);
  }
  if (status & kRateDeferred) o.value_off += (uint64_t)off0 << 32;
  if (o.has_tags) sec_off += off0;
  out[li] = o;
  tsec[2 * li] = sec_off;
  tsec[2 * li + 1] = sec_len;
  removed[li] = rm;
  tlen[li] = (base == VN_PARSE_OK && o.has_tags && !(status & (kValueDeferred | kRateDeferred))) ? jl : 0;
  // deferred lines set their tag length once their numbers are known (k_parse_slow)
  if ((status & (kValueDeferred | kRateDeferred)) && base == VN_PARSE_OK && o.has_tags) tlen[li] = jl | 0x80000000u;
}

// one block = 256 consecutive lines; their bytes are staged in LDS when they fit (the usual case:
// lines of up to 64 bytes on average), else the lanes read the buffer directly
constexpr uint32_t kWin = 16384;

// copies buf[lo, hi) to win from the word at lo & ~3 (full words, then the tail bytes); returns that base
__device__ __forceinline__ uint32_t stage_window(const uint8_t* __restrict__ buf, uint64_t len, uint32_t lo,
                                                 uint32_t hi, uint8_t* win) {
  const uint32_t wlo = lo & ~3u;
  // full words (a buffer that is not 4-byte aligned: bytes only)
  const uint32_t whi = (reinterpret_cast<uintptr_t>(buf) & 3u) ? wlo : min((hi + 3u) & ~3u, (uint32_t)len & ~3u);
  for (uint32_t w = wlo + 4u * threadIdx.x; w < whi; w += 4u * blockDim.x)
    *reinterpret_cast<uint32_t*>(win + (w - wlo)) = *reinterpret_cast<const uint32_t*>(buf + w);
  for (uint32_t i = max(whi, wlo) + threadIdx.x; i < hi; i += blockDim.x) win[i - wlo] = buf[i];
  return wlo;
}

__global__ __launch_bounds__(256) void k_parse_lines(const uint8_t* __restrict__ buf, uint64_t len,
                                                     const uint32_t* __restrict__ starts, uint32_t n,
                                                     vn_parsed_line* __restrict__ out, uint32_t* __restrict__ tsec,
                                                     int32_t* __restrict__ removed, uint32_t* __restrict__ tlen,
                                                     uint32_t* __restrict__ slow) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[kWin];
  const uint32_t first = blockIdx.x * blockDim.x;
  const uint32_t last = min(first + blockDim.x, n);
  const uint32_t lo = starts[first];
  const uint32_t hi = last < n ? starts[last] : (uint32_t)len;
  const uint32_t li = first + threadIdx.x;
  if (hi - (lo & ~3u) <= kWin) {  // block-uniform
    const uint32_t wlo = stage_window(buf, len, lo, hi, s_win);
    __syncthreads();
    if (li < n) parse_one(s_win, wlo, starts[li] - wlo, hi - wlo, li, out, tsec, removed, tlen, slow);
  } else if (li < n) {
    parse_one(buf, 0, starts[li], (uint32_t)len, li, out, tsec, removed, tlen, slow);
  }
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

// Tags of one line: q = its tag section (L bytes), written joined at dst; returns the FNV-1a of them
// continued from h.
__device__ __forceinline__ uint32_t join_tags(const uint8_t* q, uint32_t L, int32_t rm, uint32_t jl, uint8_t* dst,
                                              uint32_t h) {
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
      for (uint32_t b = 0; b < ni; b++) dst[pos + b] = q[ai + b];
      if (pos + ni < jl) dst[pos + ni] = ',';
    }
    ai = ki + 1;
    i++;
  }
  return fnv(h, dst, jl);
}

__global__ __launch_bounds__(256) void k_parse_tags(const uint8_t* __restrict__ buf, uint64_t len, uint32_t n,
                                                    vn_parsed_line* __restrict__ out,
                                                    const uint32_t* __restrict__ tsec,
                                                    const int32_t* __restrict__ removed,
                                                    const uint32_t* __restrict__ toff, uint8_t* __restrict__ tags_out) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[kWin];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kWin];
  const uint32_t first = blockIdx.x * blockDim.x;
  const uint32_t last = min(first + blockDim.x, n);
  const uint32_t li = first + threadIdx.x;
  const uint32_t lo = (uint32_t)out[first].line_off;
  const uint32_t hi = last < n ? (uint32_t)out[last].line_off : (uint32_t)len;
  const uint32_t t0 = toff[first], t1 = toff[last];  // this block's joined tags: tags_out[t0, t1)
  const bool staged = hi - (lo & ~3u) <= kWin;       // block-uniform (t1 - t0 <= hi - lo)
  uint32_t wlo = 0;
  if (staged) {
    wlo = stage_window(buf, len, lo, hi, s_win);
    __syncthreads();
  }
  if (li < n) {
    const uint32_t to = toff[li];
    const uint32_t jl = toff[li + 1] - to;
    vn_parsed_line& o = out[li];
    o.tags_off = to;
    if (o.status == VN_PARSE_OK) o.tags_len = o.has_tags ? jl : 0;
    if (o.status == VN_PARSE_OK && o.has_tags) {
      const uint32_t so = tsec[2 * li], L = tsec[2 * li + 1];
      o.digest = staged ? join_tags(s_win + (so - wlo), L, removed[li], jl, s_out + (to - t0), o.digest)
                        : join_tags(buf + so, L, removed[li], jl, tags_out + to, o.digest);
    }
  }
  if (staged) {  // the block's joined tags, written out with consecutive lanes on consecutive bytes
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < t1 - t0; i += blockDim.x) tags_out[t0 + i] = s_out[i];
  }
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
    hipLaunchKernelGGL(k_parse_tags, dim3(blocks_for(n, 256)), dim3(256), 0, p->st, b, len, n, out, p->tsec,
                       p->removed, p->toff, reinterpret_cast<uint8_t*>(tags_out));
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

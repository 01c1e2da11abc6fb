// Flush egress, native: InterMetric materialisation and the Datadog
// sink's request bodies straight from a flush result, with no per-key host objects.
//
//   flusher.go:168-230          generateInterMetrics: the maps in the reference's order, is_local
//                               rules (no percentiles for mixed histograms/timers on a local; mixed
//                               sets, global counters and global gauges flushed by a global only)
//   samplers/samplers.go:136-498  Counter/Gauge/Set/Histo.Flush: names ("%s.max", ...,
//                               "%s.%dpercentile" with int(p*100)), types, aggregate guards,
//                               routeInfo (veneursinkonly: tags)
//   sinks/datadog/datadog.go:77-106,160-213   Flush chunking (flushMaxPerBody) and finalizeMetrics:
//                               IsAcceptableMetric, counters as rates (value / interval), the
//                               sink's tags first, host: / device: magic tags, default hostname
//   http/http.go:116-135        PostHelper's body: json.NewEncoder(w).Encode({"series": chunk}) --
//                               Go 1.9 encoding/json: DDMetric field order and omitempty, floats
//                               as ES6 numbers (shortest round-trip digits, 'e' below 1e-6 and from
//                               1e21, "e-07" -> "e-7"), strings with HTML escaping, and a chunk
//                               holding NaN or Inf fails to encode (UnsupportedValueError: nothing
//                               is posted for it)
// Key order inside a map is the keys' creation order (Go iterates maps in random order).
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "veneur_amd.h"

struct vn_sink {
  std::string bytes;
  std::vector<uint64_t> off;
  std::vector<int32_t> status;
  std::string err;
};

namespace {

const char kHex[] = "0123456789abcdef";

// utf8.DecodeRuneInString: (rune, size); invalid -> (0xFFFD, 1)
uint32_t decode_rune(const uint8_t* p, size_t n, size_t* size) {
  const uint8_t c0 = p[0];
  *size = 1;
  if (c0 < 0x80) return c0;
  auto cont = [&](size_t i) { return i < n && (p[i] & 0xC0) == 0x80; };
  if (c0 >= 0xC2 && c0 <= 0xDF) {
    if (!cont(1)) return 0xFFFD;
    *size = 2;
    return ((c0 & 0x1Fu) << 6) | (p[1] & 0x3Fu);
  }
  if (c0 >= 0xE0 && c0 <= 0xEF) {
    if (!cont(1) || !cont(2)) return 0xFFFD;
    const uint32_t r = ((c0 & 0x0Fu) << 12) | ((p[1] & 0x3Fu) << 6) | (p[2] & 0x3Fu);
    if (r < 0x800 || (r >= 0xD800 && r <= 0xDFFF)) return 0xFFFD;
    *size = 3;
    return r;
  }
  if (c0 >= 0xF0 && c0 <= 0xF4) {
    if (!cont(1) || !cont(2) || !cont(3)) return 0xFFFD;
    const uint32_t r = ((c0 & 0x07u) << 18) | ((p[1] & 0x3Fu) << 12) | ((p[2] & 0x3Fu) << 6) | (p[3] & 0x3Fu);
    if (r < 0x10000 || r > 0x10FFFF) return 0xFFFD;
    *size = 4;
    return r;
  }
  return 0xFFFD;
}

// encodeState.string(s, escapeHTML = true), Go 1.9 encoding/json/encode.go
void json_string(std::string& o, const uint8_t* p, size_t n) {
  o.push_back('"');
  size_t i = 0;
  while (i < n) {
    const uint8_t b = p[i];
    if (b < 0x80) {
      if (b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&') {
        o.push_back((char)b);
      } else if (b == '"' || b == '\\') {
        o.push_back('\\');
        o.push_back((char)b);
      } else if (b == '\n') {
        o += "\\n";
      } else if (b == '\r') {
        o += "\\r";
      } else if (b == '\t') {
        o += "\\t";
      } else {
        o += "\\u00";
        o.push_back(kHex[b >> 4]);
        o.push_back(kHex[b & 0xF]);
      }
      i++;
      continue;
    }
    size_t sz;
    const uint32_t r = decode_rune(p + i, n - i, &sz);
    if (r == 0xFFFD && sz == 1) {
      o += "\\ufffd";
    } else if (r == 0x2028 || r == 0x2029) {
      o += "\\u202";
      o.push_back(kHex[r & 0xF]);
    } else {
      o.append(reinterpret_cast<const char*>(p + i), sz);
    }
    i += sz;
  }
  o.push_back('"');
}

// floatEncoder (Go 1.8+): ES6 number formatting of a finite float64
void json_float(std::string& o, double f) {
  char dig[40];
  // shortest round-trip digits in scientific form d[.ddd]e[+-]XX
  const auto r = std::to_chars(dig, dig + sizeof dig, f, std::chars_format::scientific);
  *r.ptr = 0;
  const double a = std::fabs(f);
  const bool efmt = a != 0 && (a < 1e-6 || a >= 1e21);
  const char* s = dig;
  std::string m;  // mantissa digits without the point
  bool neg = false;
  if (*s == '-') {
    neg = true;
    s++;
  }
  const char* e = strchr(s, 'e');
  for (const char* q = s; q < e; q++)
    if (*q != '.') m.push_back(*q);
  const int x = atoi(e + 1);  // value = 0.m * 10^(x+1) = m[0].m[1..] * 10^x
  if (neg) o.push_back('-');
  if (efmt) {  // AppendFloat 'e', -1: d[.ddd]e±dd, then "e-0d" -> "e-d"
    o.push_back(m[0]);
    if (m.size() > 1) {
      o.push_back('.');
      o.append(m, 1, std::string::npos);
    }
    o.push_back('e');
    o.push_back(x < 0 ? '-' : '+');
    const int ax = x < 0 ? -x : x;
    if (ax < 10 && x >= 0) {
      o.push_back('0');
      o.push_back((char)('0' + ax));
    } else if (ax < 10) {  // e-07 -> e-7
      o.push_back((char)('0' + ax));
    } else {
      o += std::to_string(ax);
    }
    return;
  }
  // AppendFloat 'f', -1: digits with the point placed, no exponent
  if (f == 0) {
    o.push_back('0');
    return;
  }
  const int dp = x + 1;  // digits before the point
  if (dp <= 0) {
    o += "0.";
    o.append((size_t)-dp, '0');
    o += m;
  } else if ((size_t)dp >= m.size()) {
    o += m;
    o.append((size_t)dp - m.size(), '0');
  } else {
    o.append(m, 0, (size_t)dp);
    o.push_back('.');
    o.append(m, (size_t)dp, std::string::npos);
  }
}

struct Str {
  const uint8_t* p;
  size_t n;
  bool starts(const char* w) const {
    const size_t k = strlen(w);
    return n >= k && memcmp(p, w, k) == 0;
  }
};

struct InterMetric {  // samplers.go:45-56 (only what the Datadog sink reads)
  uint64_t key;     // index into the key list (name, tags, route info)
  double value;
  bool counter;     // CounterMetric, else GaugeMetric
  uint8_t suffix;   // name suffix: kNone or a Histo.Flush aggregate / percentile
  int64_t pint;     // int(p*100) of a percentile
};
enum { kNone = 0, kSfxMax, kSfxMin, kSfxSum, kSfxAvg, kSfxCount, kSfxMedian, kSfxHmean, kSfxPct };
const char* const kSuffix[] = {"", ".max", ".min", ".sum", ".avg", ".count", ".median", ".hmean"};

// fn(lo, hi) over [0, n) in contiguous ranges on up to 16 host threads
template <class F>
void parallel_ranges(uint64_t n, F&& fn) {
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const uint64_t t = std::min<uint64_t>(hw, std::max<uint64_t>(1, n / 4096));
  if (t <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> th;
  for (uint64_t i = 0; i < t; i++) th.emplace_back([&, i] { fn(n * i / t, n * (i + 1) / t); });
  for (auto& x : th) x.join();
}

enum { kMax = 2, kMin = 1, kMedian = 4, kAvg = 8, kCount = 16, kSum = 32, kHmean = 64 };  // samplers.go:60-68

}  // namespace

extern "C" {

int vn_sink_create(vn_sink** out) {
  if (!out) return VN_EINVAL;
  *out = new vn_sink;
  return VN_OK;
}

void vn_sink_destroy(vn_sink* s) { delete s; }

const char* vn_sink_last_error(const vn_sink* s) { return s ? s->err.c_str() : "null sink"; }

int vn_datadog_flush(vn_sink* sk, const vn_flush_result* f, const vn_keys* keys, const vn_dd_config* cfg,
                     vn_dd_payload* out) {
  if (!sk || !f || !keys || !cfg || !out || (keys->n_keys && (!keys->map || !keys->slot || !keys->n_tags ||
                                                               !keys->name_off || !keys->name_len ||
                                                               !keys->tags_len || !keys->arena)))
    return VN_EINVAL;
  if (cfg->n_percentiles > VN_MAX_PERCENTILES || f->n_percentiles > VN_MAX_PERCENTILES ||
      (f->n_percentiles && !cfg->engine_percentiles) || cfg->flush_max_per_body == 0) {
    sk->err = "bad percentile lists or flush_max_per_body";
    return VN_EINVAL;
  }
  // slot -> row of the flush result, per class
  std::vector<int64_t> row[4];
  const uint64_t nrow[4] = {f->n_counter, f->n_gauge, f->n_histo, f->n_set};
  const uint32_t* rslot[4] = {f->counter_slot, f->gauge_slot, f->histo_slot, f->set_slot};
  for (int c = 0; c < 4; c++) {
    uint32_t mx = 0;
    for (uint64_t i = 0; i < nrow[c]; i++) mx = std::max(mx, rslot[c][i] + 1);
    for (uint64_t k = 0; k < keys->n_keys; k++)
      if (keys->map[k] <= 9) mx = std::max(mx, keys->slot[k] + 1);
    row[c].assign(mx, -1);
    for (uint64_t i = 0; i < nrow[c]; i++) row[c][rslot[c][i]] = (int64_t)i;
  }
  // percentile -> quantile column of the flush result
  auto qcol = [&](double p) -> int {
    for (uint32_t j = 0; j < f->n_percentiles; j++)
      if (cfg->engine_percentiles[j] == p) return (int)j;
    return -1;
  };
  const double nan = std::nan("");
  // the keys of each map in creation order
  std::vector<uint64_t> bymap[10];
  for (uint64_t k = 0; k < keys->n_keys; k++)
    if (keys->map[k] <= 9) bymap[keys->map[k]].push_back(k);
  static const int kClass[10] = {0, 0, 1, 1, 2, 2, 2, 2, 3, 3};
  std::vector<InterMetric> im;
  std::vector<double> hp(cfg->percentiles, cfg->percentiles + cfg->n_percentiles);
  std::vector<double> none;
  auto flush_map = [&](int m, const std::vector<double>* pct) {
    const int c = kClass[m];
    for (uint64_t k : bymap[m]) {
      const uint32_t s = keys->slot[k];
      const int64_t r = s < row[c].size() ? row[c][s] : -1;
      if (c == 0) {  // Counter.Flush: float64(value)
        im.push_back({k, r < 0 ? 0.0 : (double)f->counter_value[r], true, kNone, 0});
      } else if (c == 1) {
        im.push_back({k, r < 0 ? 0.0 : f->gauge_value[r], false, kNone, 0});
      } else if (c == 3) {  // Set.Flush: float64(Estimate()) as a gauge
        im.push_back({k, r < 0 ? 0.0 : (double)f->set_estimate[r], false, kNone, 0});
      } else {  // Histo.Flush
        double st[5] = {0.0, INFINITY, -INFINITY, 0.0, 0.0};
        if (r >= 0)
          for (int j = 0; j < 5; j++) st[j] = f->histo_stats[r * VN_HISTO_STATS + j];
        const double W = st[0], mn = st[1], mx = st[2], sum = st[3], rsum = st[4];
        auto q = [&](double p) {
          const int col = qcol(p);
          return (r < 0 || col < 0) ? nan : f->histo_quantiles[r * f->n_percentiles + col];
        };
        const uint32_t a = cfg->aggregates;
        if ((a & kMax) && !std::isinf(mx)) im.push_back({k, mx, false, kSfxMax, 0});
        if ((a & kMin) && !std::isinf(mn)) im.push_back({k, mn, false, kSfxMin, 0});
        if ((a & kSum) && sum != 0) im.push_back({k, sum, false, kSfxSum, 0});
        if ((a & kAvg) && sum != 0 && W != 0) im.push_back({k, sum / W, false, kSfxAvg, 0});
        if ((a & kCount) && W != 0) im.push_back({k, W, true, kSfxCount, 0});
        if (a & kMedian) im.push_back({k, q(0.5), false, kSfxMedian, 0});
        if ((a & kHmean) && rsum != 0 && W != 0) im.push_back({k, W / rsum, false, kSfxHmean, 0});
        for (double p : *pct) {
          volatile double p100 = p * 100.0;  // int(p*100): one float64 multiply, truncated
          im.push_back({k, q(p), false, kSfxPct, (int64_t)(double)p100});
        }
      }
    }
  };
  // generateInterMetrics (flusher.go:168-230)
  flush_map(0, nullptr);                                   // counters
  flush_map(2, nullptr);                                   // gauges
  flush_map(4, cfg->is_local ? &none : &hp);               // histograms
  flush_map(6, cfg->is_local ? &none : &hp);               // timers
  flush_map(5, &hp);                                       // local histograms
  flush_map(9, nullptr);                                   // local sets
  flush_map(7, &hp);                                       // local timers
  if (!cfg->is_local) {
    flush_map(8, nullptr);                                 // sets
    flush_map(1, nullptr);                                 // global counters
    flush_map(3, nullptr);                                 // global gauges
  }
  // finalizeMetrics (datadog.go:160-213) + the JSON object of each DDMetric
  const Str host_default{reinterpret_cast<const uint8_t*>(cfg->hostname ? cfg->hostname : ""),
                         cfg->hostname ? strlen(cfg->hostname) : 0};
  std::vector<Str> sink_tags;
  if (cfg->n_sink_tags) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(cfg->sink_tags ? cfg->sink_tags : "");
    const size_t n = cfg->sink_tags ? strlen(cfg->sink_tags) : 0;
    size_t a = 0;
    for (size_t i = 0; i <= n; i++)
      if (i == n || p[i] == ',') {
        sink_tags.push_back({p + a, i - a});
        a = i + 1;
      }
    if (sink_tags.size() != cfg->n_sink_tags) {
      sk->err = "sink_tags does not hold n_sink_tags tags";
      return VN_EINVAL;
    }
  }
  const int32_t interval_i = (int32_t)cfg->interval;  // int32(dd.interval)
  // one JSON object per InterMetric the sink accepts, built in parallel
  std::vector<std::string> objs(im.size());
  std::vector<uint8_t> acc(im.size()), fin(im.size());
  parallel_ranges(im.size(), [&](uint64_t lo, uint64_t hi) {
    std::vector<Str> tags;
    std::string tj, nm;
    for (uint64_t idx = lo; idx < hi; idx++) {
      const InterMetric& m = im[idx];
      const uint64_t k = m.key;
      tags.clear();
      const uint8_t* tp = keys->arena + keys->name_off[k] + keys->name_len[k];
      const size_t tn = keys->tags_len[k];
      if (keys->n_tags[k]) {
        size_t a = 0;
        for (size_t i = 0; i <= tn; i++)
          if (i == tn || tp[i] == ',') {
            tags.push_back({tp + a, i - a});
            a = i + 1;
          }
      }
      // routeInfo (samplers.go:106-122) + IsAcceptableMetric (sinks/sinks.go:32-37)
      bool routed = false, to_dd = false;
      for (const Str& t : tags)
        if (t.starts("veneursinkonly:")) {
          routed = true;
          if (t.n == 15 + 7 && memcmp(t.p + 15, "datadog", 7) == 0) to_dd = true;
        }
      if (routed && !to_dd) continue;
      acc[idx] = 1;
      nm.assign(reinterpret_cast<const char*>(keys->arena + keys->name_off[k]), keys->name_len[k]);
      if (m.suffix == kSfxPct) nm += "." + std::to_string((long long)m.pint) + "percentile";
      else nm += kSuffix[m.suffix];
      const double v = m.counter ? m.value / cfg->interval : m.value;  // counters are rates
      Str host{nullptr, 0}, device{nullptr, 0};
      std::string& o = objs[idx];
      o = "{\"metric\":";
      json_string(o, reinterpret_cast<const uint8_t*>(nm.data()), nm.size());
      o += ",\"points\":[[";
      json_float(o, (double)cfg->timestamp);
      o.push_back(',');
      const bool ok = std::isfinite(v);
      if (ok) json_float(o, v);
      o += "]]";
      size_t ntag = 0;
      tj.clear();
      for (const Str& t : sink_tags) {
        if (ntag++) tj.push_back(',');
        json_string(tj, t.p, t.n);
      }
      for (const Str& t : tags) {
        if (t.starts("host:")) {
          host = {t.p + 5, t.n - 5};
        } else if (t.starts("device:")) {
          device = {t.p + 7, t.n - 7};
        } else {
          if (ntag++) tj.push_back(',');
          json_string(tj, t.p, t.n);
        }
      }
      if (ntag) o += ",\"tags\":[" + tj + "]";
      o += m.counter ? ",\"type\":\"rate\"" : ",\"type\":\"gauge\"";
      if (!host.p || host.n == 0) host = host_default;  // an empty host: tag leaves the default too
      if (host.n) {
        o += ",\"host\":";
        json_string(o, host.p, host.n);
      }
      if (device.p && device.n) {
        o += ",\"device_name\":";
        json_string(o, device.p, device.n);
      }
      if (interval_i) o += ",\"interval\":" + std::to_string(interval_i);
      o.push_back('}');
      fin[idx] = ok;
    }
  });
  std::vector<uint64_t> sel;
  sel.reserve(im.size());
  for (uint64_t i = 0; i < im.size(); i++)
    if (acc[i]) sel.push_back(i);
  // Flush's chunks (datadog.go:83-101): rounding-up division, every chunk under the limit
  const int64_t n = (int64_t)sel.size(), mpb = cfg->flush_max_per_body;
  const int64_t workers = (n - 1) / mpb + 1;  // Go: -1 / mpb == 0 -> one (empty) chunk
  const int64_t chunk = (n - 1) / workers + 1;
  auto bounds = [&](int64_t w, int64_t* lo, int64_t* hi) {
    *lo = std::min(n, w * chunk);
    *hi = w < workers - 1 ? std::min(n, *lo + chunk) : n;
  };
  sk->off.assign(workers + 1, 0);
  sk->status.assign(workers, VN_OK);
  for (int64_t w = 0; w < workers; w++) {
    int64_t lo, hi;
    bounds(w, &lo, &hi);
    bool good = true;
    uint64_t sz = 11 + 3;  // {"series":[ ... ]}\n
    for (int64_t i = lo; i < hi; i++) {
      good = good && fin[sel[i]];
      sz += objs[sel[i]].size() + (i > lo ? 1 : 0);
    }
    sk->status[w] = good ? VN_OK : VN_EINVAL;  // json: unsupported value: NaN / +Inf / -Inf
    sk->off[w + 1] = sk->off[w] + (good ? sz : 0);
  }
  sk->bytes.resize(sk->off[workers]);
  parallel_ranges((uint64_t)workers, [&](uint64_t wlo, uint64_t whi) {
    for (uint64_t w = wlo; w < whi; w++) {
      if (sk->status[w] != VN_OK) continue;
      int64_t lo, hi;
      bounds((int64_t)w, &lo, &hi);
      char* d = &sk->bytes[0] + sk->off[w];
      memcpy(d, "{\"series\":[", 11);
      d += 11;
      for (int64_t i = lo; i < hi; i++) {
        if (i > lo) *d++ = ',';
        const std::string& o = objs[sel[i]];
        memcpy(d, o.data(), o.size());
        d += o.size();
      }
      memcpy(d, "]}\n", 3);
    }
  });
  out->n_intermetrics = im.size();
  out->n_metrics = (uint64_t)n;
  out->n_bodies = (uint32_t)workers;
  out->body_off = sk->off.data();
  out->body_status = sk->status.data();
  out->bytes = reinterpret_cast<const uint8_t*>(sk->bytes.data());
  return VN_OK;
}

}  // extern "C"

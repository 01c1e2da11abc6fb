// DogStatsD metric lines -> parsed records, native host side of the C-ABI (vn_parse_dogstatsd).
//
// Restates samplers/parser.go:186-307 (ParseMetric) over a whole datagram buffer split on '\n'
// (server.go:706-714; empty packets skipped as HandleMetricPacket does, server.go:612-616).  The
// Python mirror (veneur_amd/parser.py) is the checker: tests/test_parser.py compares the two on
// the reference's cases and on random and mutated lines.  Numbers follow Go 1.9's ParseFloat:
// the syntax is validated here (no spaces, underscores or hex; "inf"/"infinity"/"nan" parse),
// then glibc's strtod / strtof, which round the decimal correctly (strtof directly to float32,
// as ParseFloat(s, 32) does).
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <locale.h>
#include <string>
#include <vector>

#include "veneur_amd.h"

namespace {

inline uint32_t fnv1a(uint32_t h, const char* p, size_t n) {
  for (size_t i = 0; i < n; ++i) h = (h ^ (uint8_t)p[i]) * 0x01000193u;
  return h;
}

inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }

bool ieq(const char* p, size_t n, const char* w) {
  size_t m = strlen(w);
  if (n != m) return false;
  for (size_t i = 0; i < n; ++i)
    if (lower(p[i]) != w[i]) return false;
  return true;
}

// Go 1.9 atof.go special(): [+-]inf, [+-]infinity, nan (no sign)
int special(const char* p, size_t n, double* v) {
  if (ieq(p, n, "nan")) { *v = NAN; return 1; }
  double s = 1.0;
  if (n && (p[0] == '+' || p[0] == '-')) { s = p[0] == '-' ? -1.0 : 1.0; ++p; --n; }
  if (ieq(p, n, "inf") || ieq(p, n, "infinity")) { *v = s * INFINITY; return 1; }
  return 0;
}

// [+-]?(digits[.digits*] | .digits)([eE][+-]?digits)?
bool decimal_syntax(const char* p, size_t n) {
  size_t i = 0, d = 0;
  if (i < n && (p[i] == '+' || p[i] == '-')) ++i;
  while (i < n && p[i] >= '0' && p[i] <= '9') { ++i; ++d; }
  if (i < n && p[i] == '.') {
    ++i;
    while (i < n && p[i] >= '0' && p[i] <= '9') { ++i; ++d; }
  }
  if (d == 0) return false;
  if (i < n && (p[i] == 'e' || p[i] == 'E')) {
    ++i;
    if (i < n && (p[i] == '+' || p[i] == '-')) ++i;
    size_t e = 0;
    while (i < n && p[i] >= '0' && p[i] <= '9') { ++i; ++e; }
    if (e == 0) return false;
  }
  return i == n;
}

// 0 ok; 1 syntax; 2 out of range (±Inf after rounding)
int parse_float(const char* p, size_t n, bool f32, double* out) {
  if (special(p, n, out)) return 0;
  if (!decimal_syntax(p, n)) return 1;
  char small[128];
  std::string big;
  const char* z;
  if (n < sizeof(small)) { memcpy(small, p, n); small[n] = 0; z = small; }
  else { big.assign(p, n); z = big.c_str(); }
  // the "C" locale whatever LC_NUMERIC the host process set (Go's ParseFloat has no locale)
  static const locale_t c_locale = newlocale(LC_ALL_MASK, "C", (locale_t)0);
  char* end = nullptr;
  if (f32) {
    float v = strtof_l(z, &end, c_locale);
    if (end != z + n) return 1;
    if (std::isinf(v)) return 2;
    *out = (double)v;
  } else {
    double v = strtod_l(z, &end, c_locale);
    if (end != z + n) return 1;
    if (std::isinf(v)) return 2;
    *out = v;
  }
  return 0;
}

struct Range { const char* p; size_t n; };

bool range_less(const Range& a, const Range& b) {  // Go's string order: bytes, then length
  int c = memcmp(a.p, b.p, std::min(a.n, b.n));
  return c < 0 || (c == 0 && a.n < b.n);
}

bool has_prefix(const Range& r, const char* w) {
  size_t m = strlen(w);
  return r.n >= m && memcmp(r.p, w, m) == 0;
}

// One metric line; returns VN_PARSE_OK or an error code.  Writes joined tags at *tpos.
int parse_line(const char* base, const char* p, size_t n, char* tags_out, uint64_t tags_cap, uint64_t* tpos,
               std::vector<Range>& tags, vn_parsed_line* o) {
  o->rate = 1.0f;
  o->scope = 0;
  o->value = 0.0;
  o->tags_off = *tpos;
  o->tags_len = 0;
  o->has_tags = 0;
  const char* end = p + n;
  const char* pipe = (const char*)memchr(p, '|', n);
  const char* c0end = pipe ? pipe : end;
  const char* colon = (const char*)memchr(p, ':', (size_t)(c0end - p));
  if (!colon) return VN_PARSE_NO_COLON;
  if (colon == p) return VN_PARSE_EMPTY_NAME;
  o->name_off = (uint64_t)(p - base);
  o->name_len = (uint32_t)(colon - p);
  o->value_off = (uint64_t)(colon + 1 - base);
  o->value_len = (uint32_t)(c0end - colon - 1);
  if (!pipe) return VN_PARSE_NO_PIPE;
  const char* t = pipe + 1;
  const char* tend = (const char*)memchr(t, '|', (size_t)(end - t));
  if (!tend) tend = end;
  if (tend == t) return VN_PARSE_NO_TYPE;
  static const char* names[] = {"counter", "gauge", "histogram", "timer", "set"};
  switch (t[0]) {
    case 'c': o->type = 0; break;
    case 'g': o->type = 1; break;
    case 'h': o->type = 2; break;
    case 'm': o->type = 3; break;
    case 's': o->type = 4; break;
    default: return VN_PARSE_BAD_TYPE;
  }
  uint32_t h = fnv1a(0x811C9DC5u, p, o->name_len);
  h = fnv1a(h, names[o->type], strlen(names[o->type]));
  if (o->type != 4) {
    double v;
    if (parse_float(colon + 1, o->value_len, false, &v) || std::isnan(v) || std::isinf(v)) return VN_PARSE_BAD_VALUE;
    o->value = v;
  }
  bool found_rate = false;
  const char* s = tend;
  while (s < end) {  // s points at the '|' before the next section
    const char* c = s + 1;
    const char* cend = (const char*)memchr(c, '|', (size_t)(end - c));
    if (!cend) cend = end;
    size_t cn = (size_t)(cend - c);
    if (cn == 0) return VN_PARSE_EMPTY_SECTION;
    if (c[0] == '@') {
      if (found_rate) return VN_PARSE_MULTI_RATE;
      double r;
      if (parse_float(c + 1, cn - 1, true, &r)) return VN_PARSE_BAD_RATE;
      if (r <= 0 || r > 1) return VN_PARSE_RATE_RANGE;  // NaN passes, as in Go
      o->rate = (float)r;
      found_rate = true;
    } else if (c[0] == '#') {
      if (o->has_tags) return VN_PARSE_MULTI_TAGS;
      o->has_tags = 1;
      tags.clear();
      const char* q = c + 1;
      while (true) {
        const char* comma = (const char*)memchr(q, ',', (size_t)(cend - q));
        const char* qe = comma ? comma : cend;
        tags.push_back({q, (size_t)(qe - q)});
        if (!comma) break;
        q = comma + 1;
      }
      std::sort(tags.begin(), tags.end(), range_less);
      for (size_t i = 0; i < tags.size(); ++i) {
        if (has_prefix(tags[i], "veneurlocalonly")) { tags.erase(tags.begin() + i); o->scope = 1; break; }
        if (has_prefix(tags[i], "veneurglobalonly")) { tags.erase(tags.begin() + i); o->scope = 2; break; }
      }
      uint64_t w = *tpos;
      o->tags_off = w;
      o->n_tags = (uint32_t)tags.size();
      for (size_t i = 0; i < tags.size(); ++i) {
        if (w + tags[i].n + 1 > tags_cap) return VN_PARSE_TAGS_FULL;
        if (i) tags_out[w++] = ',';
        memcpy(tags_out + w, tags[i].p, tags[i].n);
        w += tags[i].n;
      }
      o->tags_len = (uint32_t)(w - o->tags_off);
      h = fnv1a(h, tags_out + o->tags_off, o->tags_len);
    } else {
      return VN_PARSE_UNKNOWN_SECTION;
    }
    s = cend;
  }
  o->digest = h;
  if (o->has_tags) *tpos = o->tags_off + o->tags_len;
  return VN_PARSE_OK;
}

}  // namespace

extern "C" int64_t vn_parse_dogstatsd(const char* buf, uint64_t len, vn_parsed_line* out, uint64_t max_lines,
                                      char* tags_out, uint64_t tags_cap) {
  if ((!buf && len) || (!out && max_lines)) return VN_EINVAL;
  std::vector<Range> tags;
  uint64_t n = 0, tpos = 0, pos = 0;
  while (true) {
    const char* p = buf + pos;
    const char* nl = len > pos ? (const char*)memchr(p, '\n', len - pos) : nullptr;
    uint64_t ln = nl ? (uint64_t)(nl - p) : len - pos;
    if (ln > 0) {  // HandleMetricPacket ignores an empty packet
      if (n == max_lines) return VN_EINVAL;
      vn_parsed_line* o = out + n++;
      memset(o, 0, sizeof(*o));
      o->line_off = pos;
      o->line_len = (uint32_t)ln;
      if (ln >= 3 && (memcmp(p, "_e{", 3) == 0 || memcmp(p, "_sc", 3) == 0)) o->status = VN_PARSE_NOT_METRIC;
      else o->status = parse_line(buf, p, ln, tags_out, tags_cap, &tpos, tags, o);
    }
    if (!nl) break;
    pos += ln + 1;
  }
  return (int64_t)n;
}

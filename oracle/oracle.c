/*
 * oracle.c -- CPU restatement of veneur's per-flush sketch path (see oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY: never linked into veneur_amd.  Compiled with
 * -ffp-contract=off so every float operation rounds like the Go reference on
 * amd64 (Go 1.9 never fuses multiply-adds on amd64).
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* =========================================================================
 * go-bits Clz (vendor/github.com/dgryski/go-bits/clz.go:6-37, clz_amd64.s:
 * BSR based, returns 64 for 0).
 * ========================================================================= */
uint64_t or_clz64(uint64_t x) { return x == 0 ? 64 : (uint64_t)__builtin_clzll(x); }

/* =========================================================================
 * MetroHash64 (vendor/github.com/dgryski/go-metro/metro64.go:7-85; the amd64
 * assembly in metro_amd64.s computes the same function).
 * ========================================================================= */
static inline uint64_t rotr64(uint64_t v, unsigned k) { return (v >> k) | (v << (64 - k)); }
static inline uint64_t ld64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint16_t ld16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }

uint64_t or_metro_hash64(const uint8_t* ptr, size_t len, uint64_t seed) {
  const uint64_t k0 = 0xD6D018F5ull, k1 = 0xA2AA033Bull, k2 = 0x62992FC1ull, k3 = 0x30BC5B29ull;
  uint64_t hash = (seed + k2) * k0;
  if (len >= 32) {
    uint64_t v0 = hash, v1 = hash, v2 = hash, v3 = hash;
    while (len >= 32) {
      v0 += ld64(ptr) * k0; ptr += 8; v0 = rotr64(v0, 29) + v2;
      v1 += ld64(ptr) * k1; ptr += 8; v1 = rotr64(v1, 29) + v3;
      v2 += ld64(ptr) * k2; ptr += 8; v2 = rotr64(v2, 29) + v0;
      v3 += ld64(ptr) * k3; ptr += 8; v3 = rotr64(v3, 29) + v1;
      len -= 32;
    }
    v2 ^= rotr64(((v0 + v3) * k0) + v1, 37) * k1;
    v3 ^= rotr64(((v1 + v2) * k1) + v0, 37) * k0;
    v0 ^= rotr64(((v0 + v2) * k0) + v3, 37) * k1;
    v1 ^= rotr64(((v1 + v3) * k1) + v2, 37) * k0;
    hash += v0 ^ v1;
  }
  if (len >= 16) {
    uint64_t v0 = hash + (ld64(ptr) * k2); ptr += 8; v0 = rotr64(v0, 29) * k3;
    uint64_t v1 = hash + (ld64(ptr) * k2); ptr += 8; v1 = rotr64(v1, 29) * k3;
    v0 ^= rotr64(v0 * k0, 21) + v1;
    v1 ^= rotr64(v1 * k3, 21) + v0;
    hash += v1;
    len -= 16;
  }
  if (len >= 8) { hash += ld64(ptr) * k3; ptr += 8; len -= 8; hash ^= rotr64(hash, 55) * k1; }
  if (len >= 4) { hash += (uint64_t)ld32(ptr) * k3; ptr += 4; len -= 4; hash ^= rotr64(hash, 26) * k1; }
  if (len >= 2) { hash += (uint64_t)ld16(ptr) * k3; ptr += 2; len -= 2; hash ^= rotr64(hash, 48) * k1; }
  if (len >= 1) { hash += (uint64_t)ptr[0] * k3; hash ^= rotr64(hash, 37) * k1; }
  hash ^= rotr64(hash, 28);
  hash *= k0;
  hash ^= rotr64(hash, 29);
  return hash;
}

/* FNV-1a 32 (hash/fnv) as used for MetricKey digests (samplers/parser.go:213-304). */
uint32_t or_fnv1a32(const uint8_t* buf, size_t len, uint32_t h) {
  for (size_t i = 0; i < len; i++) { h ^= buf[i]; h *= 16777619u; }
  return h;
}

/* =========================================================================
 * Go 1.9 math restatements.
 * ========================================================================= */
static double go_frexp(double x, int* e) {
  /* Go math.Frexp: special cases 0, Inf, NaN return (x, 0) */
  if (x == 0 || isinf(x) || isnan(x)) { *e = 0; return x; }
  return frexp(x, e); /* exact, same contract: frac in [0.5,1) */
}
static double go_ldexp(double frac, int e) { return ldexp(frac, e); } /* exact in normal range */

/* math.Log -- src/math/log.go (FreeBSD e_log.c); log_amd64.s evaluates the same
 * expression tree in the same order. */
double or_go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
               L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
               L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (isnan(x) || (isinf(x) && x > 0)) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = go_frexp(x, &ki);
  if (f1 < M_SQRT2 / 2) { f1 *= 2; ki--; }
  double f = f1 - 1;
  double k = (double)ki;
  double s = f / (2 + f);
  double s2 = s * s;
  double s4 = s2 * s2;
  double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  double R = t1 + t2;
  double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

static int go_is_odd_int(double x) {
  double xi;
  double xf = modf(x, &xi);
  return xf == 0 && ((int64_t)xi & 1) == 1;
}

/* math.Pow -- src/math/pow.go (Go 1.9).  Only the finite integer-exponent branch is
 * exercised by the sketch path (beta14's Pow(zl, k), k = 2..7, and Pow(2, v)). */
double or_go_pow(double x, double y) {
  if (y == 0 || x == 1) return 1;
  if (y == 1) return x;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0) {
    if (y < 0) return go_is_odd_int(y) ? copysign(INFINITY, x) : INFINITY;
    if (y > 0) return go_is_odd_int(y) ? x : 0;
  }
  if (isinf(y)) {
    if (x == -1) return 1;
    if ((fabs(x) < 1) == (y > 0)) return 0;
    return INFINITY;
  }
  if (isinf(x)) {
    if (x < 0) return or_go_pow(1 / x, -y);
    if (y < 0) return 0;
    if (y > 0) return INFINITY;
  }
  if (y == 0.5) return sqrt(x);
  if (y == -0.5) return 1 / sqrt(x);
  double absy = y;
  int flip = 0;
  if (absy < 0) { absy = -absy; flip = 1; }
  double yi;
  double yf = modf(absy, &yi);
  if (yf != 0 && x < 0) return NAN;
  if (yi >= 9.223372036854775808e18) {
    if (x == -1) return 1;
    if ((fabs(x) < 1) == (y > 0)) return 0;
    return INFINITY;
  }
  double a1 = 1.0;
  int ae = 0;
  if (yf != 0) {
    if (yf > 0.5) { yf--; yi++; }
    a1 = exp(yf * or_go_log(x)); /* not reached on the sketch path */
  }
  int xe;
  double x1 = go_frexp(x, &xe);
  for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
    if (xe < -(1 << 12) || (1 << 12) < xe) { ae += xe; break; }
    if (i & 1) { a1 *= x1; ae += xe; }
    x1 *= x1;
    xe <<= 1;
    if (x1 < .5) { x1 += x1; xe--; }
  }
  if (flip) { a1 = 1 / a1; ae = -ae; }
  return go_ldexp(a1, ae);
}

/* math.Asin -- src/math/asin.go + atan.go (Cephes). Used by indexEstimate
 * (tdigest/merging_digest.go:240-243). */
static double go_xatan(double x) {
  const double P0 = -8.750608600031904122785e-01, P1 = -1.615753718733365076637e+01,
               P2 = -7.500855792314704667340e+01, P3 = -1.228866684490136173410e+02,
               P4 = -6.485021904942025371773e+01, Q0 = +2.485846490142306297962e+01,
               Q1 = +1.650270098316988542046e+02, Q2 = +4.328810604912902668951e+02,
               Q3 = +4.853903996359136964868e+02, Q4 = +1.945506571482613964425e+02;
  double z = x * x;
  z = z * ((((P0 * z + P1) * z + P2) * z + P3) * z + P4) / (((((z + Q0) * z + Q1) * z + Q2) * z + Q3) * z + Q4);
  z = x * z + x;
  return z;
}
static double go_satan(double x) {
  const double Morebits = 6.123233995736765886130e-17, Tan3pio8 = 2.41421356237309504880;
  if (x <= 0.66) return go_xatan(x);
  if (x > Tan3pio8) return M_PI / 2 - go_xatan(1 / x) + Morebits;
  return M_PI / 4 + go_xatan((x - 1) / (x + 1)) + 0.5 * Morebits;
}
double or_go_asin(double x) {
  if (x == 0) return x;
  int sign = 0;
  if (x < 0) { x = -x; sign = 1; }
  if (x > 1) return NAN;
  double temp = sqrt(1 - x * x);
  if (x > 0.7) temp = M_PI / 2 - go_satan(temp / x);
  else temp = go_satan(x / temp);
  return sign ? -temp : temp;
}

/* int64(float64) on amd64: CVTTSD2SQ, "integer indefinite" for NaN / out of range. */
int64_t or_go_f64_to_i64(double x) {
  if (isnan(x) || x >= 9.223372036854775808e18 || x <= -9.223372036854775808e18) return INT64_MIN;
  return (int64_t)x;
}
/* uint64(float64) on amd64 (Go 1.9 SSA lowering): x < 2^63 -> CVTTSD2SQ;
 * else CVTTSD2SQ(x - 2^63) ^ (1<<63). */
uint64_t or_go_f64_to_u64(double x) {
  if (x < 9.223372036854775808e18) return (uint64_t)or_go_f64_to_i64(x);
  return (uint64_t)or_go_f64_to_i64(x - 9.223372036854775808e18) ^ 0x8000000000000000ull;
}

/* =========================================================================
 * Go 1.9 sort.Sort (src/sort/sort.go quickSort) over an abstract Less/Swap.
 * Restated so that the tie order of sort.Sort(centroidList) follows Go's.
 * ========================================================================= */
typedef struct {
  int (*less)(void* d, int64_t i, int64_t j);
  void (*swap)(void* d, int64_t i, int64_t j);
  void* d;
} go_sorter;
#define LESS(i, j) s->less(s->d, (i), (j))
#define SWAP(i, j) s->swap(s->d, (i), (j))
static void go_insertion_sort(go_sorter* s, int64_t a, int64_t b) {
  for (int64_t i = a + 1; i < b; i++)
    for (int64_t j = i; j > a && LESS(j, j - 1); j--) SWAP(j, j - 1);
}
static void go_sift_down(go_sorter* s, int64_t lo, int64_t hi, int64_t first) {
  int64_t root = lo;
  for (;;) {
    int64_t child = 2 * root + 1;
    if (child >= hi) return;
    if (child + 1 < hi && LESS(first + child, first + child + 1)) child++;
    if (!LESS(first + root, first + child)) return;
    SWAP(first + root, first + child);
    root = child;
  }
}
static void go_heap_sort(go_sorter* s, int64_t a, int64_t b) {
  int64_t first = a, lo = 0, hi = b - a;
  for (int64_t i = (hi - 1) / 2; i >= 0; i--) go_sift_down(s, i, hi, first);
  for (int64_t i = hi - 1; i >= 0; i--) { SWAP(first, first + i); go_sift_down(s, lo, i, first); }
}
static void go_median_of_three(go_sorter* s, int64_t m1, int64_t m0, int64_t m2) {
  if (LESS(m1, m0)) SWAP(m1, m0);
  if (LESS(m2, m1)) {
    SWAP(m2, m1);
    if (LESS(m1, m0)) SWAP(m1, m0);
  }
}
static void go_do_pivot(go_sorter* s, int64_t lo, int64_t hi, int64_t* midlo, int64_t* midhi) {
  int64_t m = lo + (hi - lo) / 2;
  if (hi - lo > 40) {
    int64_t t = (hi - lo) / 8;
    go_median_of_three(s, lo, lo + t, lo + 2 * t);
    go_median_of_three(s, m, m - t, m + t);
    go_median_of_three(s, hi - 1, hi - 1 - t, hi - 1 - 2 * t);
  }
  go_median_of_three(s, lo, m, hi - 1);
  int64_t pivot = lo;
  int64_t a = lo + 1, c = hi - 1;
  for (; a < c && LESS(a, pivot); a++) {}
  int64_t b = a;
  for (;;) {
    for (; b < c && !LESS(pivot, b); b++) {}
    for (; b < c && LESS(pivot, c - 1); c--) {}
    if (b >= c) break;
    SWAP(b, c - 1);
    b++;
    c--;
  }
  int protect = hi - c < 5;
  if (!protect && hi - c < (hi - lo) / 4) {
    int dups = 0;
    if (!LESS(pivot, hi - 1)) { SWAP(c, hi - 1); c++; dups++; }
    if (!LESS(b - 1, pivot)) { b--; dups++; }
    if (!LESS(m, pivot)) { SWAP(m, b - 1); b--; dups++; }
    protect = dups > 1;
  }
  if (protect) {
    for (;;) {
      for (; a < b && !LESS(b - 1, pivot); b--) {}
      for (; a < b && LESS(a, pivot); a++) {}
      if (a >= b) break;
      SWAP(a, b - 1);
      a++;
      b--;
    }
  }
  SWAP(pivot, b - 1);
  *midlo = b - 1;
  *midhi = c;
}
static void go_quick_sort(go_sorter* s, int64_t a, int64_t b, int max_depth) {
  while (b - a > 12) {
    if (max_depth == 0) { go_heap_sort(s, a, b); return; }
    max_depth--;
    int64_t mlo, mhi;
    go_do_pivot(s, a, b, &mlo, &mhi);
    if (mlo - a < b - mhi) { go_quick_sort(s, a, mlo, max_depth); a = mhi; }
    else { go_quick_sort(s, mhi, b, max_depth); b = mlo; }
  }
  if (b - a > 1) {
    for (int64_t i = a + 6; i < b; i++)
      if (LESS(i, i - 6)) SWAP(i, i - 6);
    go_insertion_sort(s, a, b);
  }
}
static void go_sort(go_sorter* s, int64_t n) {
  int depth = 0;
  for (int64_t i = n; i > 0; i >>= 1) depth++;
  go_quick_sort(s, 0, n, depth * 2);
}
#undef LESS
#undef SWAP

/* =========================================================================
 * axiomhq/hyperloglog (vendor/github.com/axiomhq/hyperloglog, rev 67c63c17)
 * ========================================================================= */
#define HLL_CAPACITY 16u
#define HLL_PP 25u
#define HLL_MP (1u << 25)
#define HLL_VERSION 1u

/* Go map[uint32]struct{} restated as an open-addressing set (iteration order is
 * irrelevant wherever the oracle iterates it: it sorts first). */
typedef struct { uint32_t* keys; uint8_t* used; size_t cap, len; } u32set;
static void u32set_init(u32set* s) { s->keys = NULL; s->used = NULL; s->cap = 0; s->len = 0; }
static void u32set_free(u32set* s) { free(s->keys); free(s->used); u32set_init(s); }
static inline size_t u32h(uint32_t k) { uint64_t x = k * 0x9E3779B97F4A7C15ull; return (size_t)(x >> 20); }
static void u32set_grow(u32set* s);
static int u32set_add(u32set* s, uint32_t k) {
  if ((s->len + 1) * 2 > s->cap) u32set_grow(s);
  size_t mask = s->cap - 1, i = u32h(k) & mask;
  while (s->used[i]) {
    if (s->keys[i] == k) return 0;
    i = (i + 1) & mask;
  }
  s->used[i] = 1; s->keys[i] = k; s->len++;
  return 1;
}
static int u32set_has(const u32set* s, uint32_t k) {
  if (!s->cap) return 0;
  size_t mask = s->cap - 1, i = u32h(k) & mask;
  while (s->used[i]) {
    if (s->keys[i] == k) return 1;
    i = (i + 1) & mask;
  }
  return 0;
}
static void u32set_grow(u32set* s) {
  size_t ncap = s->cap ? s->cap * 2 : 16;
  uint32_t* ok = s->keys; uint8_t* ou = s->used; size_t ocap = s->cap;
  s->keys = (uint32_t*)malloc(ncap * sizeof(uint32_t));
  s->used = (uint8_t*)calloc(ncap, 1);
  s->cap = ncap; s->len = 0;
  for (size_t i = 0; i < ocap; i++) if (ou[i]) u32set_add(s, ok[i]);
  free(ok); free(ou);
}
static int cmp_u32(const void* a, const void* b) {
  uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return x < y ? -1 : x > y;
}
static size_t u32set_sorted(const u32set* s, uint32_t* out) {
  size_t n = 0;
  for (size_t i = 0; i < s->cap; i++) if (s->used[i]) out[n++] = s->keys[i];
  qsort(out, n, sizeof(uint32_t), cmp_u32);
  return n;
}
static void u32set_clear(u32set* s) {
  if (s->cap) memset(s->used, 0, s->cap);
  s->len = 0;
}

/* compressedList (compressed.go) -- varint delta list */
typedef struct { uint32_t count, last; uint8_t* b; size_t len, cap; } clist;
static void clist_init(clist* l) { l->count = 0; l->last = 0; l->b = NULL; l->len = 0; l->cap = 0; }
static void clist_free(clist* l) { free(l->b); clist_init(l); }
static void clist_push(clist* l, uint8_t v) {
  if (l->len == l->cap) { l->cap = l->cap ? l->cap * 2 : 64; l->b = (uint8_t*)realloc(l->b, l->cap); }
  l->b[l->len++] = v;
}
static void clist_append(clist* l, uint32_t x) { /* compressedList.Append, compressed.go:114-118 */
  l->count++;
  uint32_t d = x - l->last;
  while (d & 0xffffff80u) { clist_push(l, (uint8_t)((d & 0x7f) | 0x80)); d >>= 7; }
  clist_push(l, (uint8_t)(d & 0x7f));
  l->last = x;
}
/* variableLengthList.decode (compressed.go:157-165) */
static uint32_t clist_decode(const clist* l, size_t* i, uint32_t last) {
  uint32_t x = 0;
  size_t j = *i;
  for (; l->b[j] & 0x80; j++) x |= (uint32_t)(l->b[j] & 0x7f) << ((j - *i) * 7);
  x |= (uint32_t)l->b[j] << ((j - *i) * 7);
  *i = j + 1;
  return x + last;
}

struct or_hll {
  int sparse;
  uint8_t p, b;
  uint32_t m;
  double alpha;
  u32set tmp;
  int has_list;
  clist list;
  int has_regs;
  uint8_t* tc; /* tailcuts: m/2 bytes */
  uint32_t ntc;
  uint32_t nz;
};

static double hll_alpha(double m) { /* utils.go:34-44 */
  if (m == 16) return 0.673;
  if (m == 32) return 0.697;
  if (m == 64) return 0.709;
  return 0.7213 / (1 + 1.079 / m);
}
static inline uint64_t bextr(uint64_t v, uint8_t start, uint8_t length) {
  return (v >> start) & ((length >= 64) ? ~0ull : ((1ull << length) - 1));
}
static inline uint32_t bextr32(uint32_t v, uint8_t start, uint8_t length) {
  return (v >> start) & ((length >= 32) ? ~0u : ((1u << length) - 1));
}
void or_hll_get_pos_val(uint64_t x, uint8_t p, uint64_t* idx, uint8_t* rho) { /* utils.go:46-51 */
  *idx = bextr(x, (uint8_t)(64 - p), p);
  uint64_t w = (x << p) | (1ull << (p - 1));
  *rho = (uint8_t)(or_clz64(w) + 1);
}
uint32_t or_hll_encode_hash(uint64_t x, uint8_t p, uint8_t pp) { /* sparse.go:14-22 */
  uint32_t idx = (uint32_t)bextr(x, (uint8_t)(64 - pp), pp);
  if (bextr(x, (uint8_t)(64 - pp), (uint8_t)(pp - p)) == 0) {
    uint64_t zeros = or_clz64((bextr(x, 0, (uint8_t)(64 - pp)) << pp) | ((1ull << pp) - 1)) + 1;
    return (idx << 7) | (uint32_t)(zeros << 1) | 1;
  }
  return idx << 1;
}
static uint32_t hll_get_index(uint32_t k, uint8_t p, uint8_t pp) { /* sparse.go:7-12 */
  if (k & 1) return bextr32(k, (uint8_t)(32 - p), p);
  return bextr32(k, (uint8_t)(pp - p + 1), p);
}
void or_hll_decode_hash(uint32_t k, uint8_t p, uint8_t pp, uint32_t* idx, uint8_t* r) { /* sparse.go:25-35 */
  uint8_t rr;
  if (k & 1) rr = (uint8_t)(bextr32(k, 1, 6) + pp - p);
  else rr = (uint8_t)(or_clz64((uint64_t)(uint32_t)(k << (32 - pp + p - 1))) - 31);
  *idx = hll_get_index(k, p, pp);
  *r = rr;
}

/* registers.go */
static uint8_t reg_get_nib(uint8_t r, uint8_t off) { return off == 0 ? (uint8_t)(r >> 4) : (uint8_t)((uint8_t)(r << 4) >> 4); }
static int reg_set_nib(uint8_t* r, uint8_t off, uint8_t val) { /* reg.set, registers.go:15-27 */
  int is_zero;
  if (off == 0) {
    is_zero = (uint8_t)(*r >> 4) == 0;
    uint8_t tmp = (uint8_t)((uint8_t)(*r << 4) >> 4);
    *r = (uint8_t)(tmp | (uint8_t)(val << 4));
  } else {
    is_zero = (uint8_t)((uint8_t)(*r << 4) >> 4) == 0;
    uint8_t tmp = (uint8_t)(*r >> 4);
    *r = (uint8_t)((uint8_t)(tmp << 4) | val);
  }
  return is_zero;
}
static void regs_new(or_hll* sk, uint32_t size) {
  free(sk->tc);
  sk->ntc = size / 2;
  sk->tc = (uint8_t*)calloc(sk->ntc ? sk->ntc : 1, 1);
  sk->nz = size;
  sk->has_regs = 1;
}
static void regs_set(or_hll* sk, uint32_t i, uint8_t val) {
  uint8_t off = (uint8_t)(i % 2);
  if (reg_set_nib(&sk->tc[i / 2], off, val)) sk->nz--;
}
static uint8_t regs_get(const or_hll* sk, uint32_t i) { return reg_get_nib(sk->tc[i / 2], (uint8_t)(i % 2)); }
static void regs_rebase(or_hll* sk, uint8_t delta) { /* registers.go:55-74 */
  uint32_t nz = sk->ntc * 2;
  for (uint32_t i = 0; i < sk->ntc; i++) {
    uint8_t val = reg_get_nib(sk->tc[i], 0);
    if (val >= delta) {
      reg_set_nib(&sk->tc[i], 0, (uint8_t)(val - delta));
      if ((uint8_t)(val - delta) > 0) nz--;
    }
    val = reg_get_nib(sk->tc[i], 1);
    if (val >= delta) {
      reg_set_nib(&sk->tc[i], 1, (uint8_t)(val - delta));
      if ((uint8_t)(val - delta) > 0) nz--;
    }
  }
  sk->nz = nz;
}
static uint8_t regs_min(const or_hll* sk) { /* registers.go:106-123 */
  if (sk->nz > 0) return 0;
  uint8_t mn = 255;
  for (uint32_t i = 0; i < sk->ntc; i++) {
    uint8_t r = sk->tc[i];
    uint8_t v = (uint8_t)((uint8_t)(r << 4) >> 4);
    if (v < mn) mn = v;
    v = (uint8_t)(r >> 4);
    if (v < mn) mn = v;
    if (mn == 0) break;
  }
  return mn;
}
/* sumAndZeros (registers.go:88-104), including its reference bug: ez counts the
 * high nibble twice and never the low one, and nz is overwritten with ez. */
static void regs_sum_and_zeros(or_hll* sk, uint8_t base, double* res_out, double* ez_out) {
  double res = 0, ez = 0;
  for (uint32_t i = 0; i < sk->ntc; i++) {
    uint8_t r = sk->tc[i];
    double v1 = (double)(uint8_t)(base + reg_get_nib(r, 0));
    if (v1 == 0) ez++;
    res += 1.0 / or_go_pow(2.0, v1);
    double v2 = (double)(uint8_t)(base + reg_get_nib(r, 0));
    if (v2 == 0) ez++;
    res += 1.0 / or_go_pow(2.0, (double)(uint8_t)(base + reg_get_nib(r, 1)));
  }
  sk->nz = (uint32_t)ez;
  *res_out = res;
  *ez_out = ez;
}

static or_hll* hll_alloc(void) {
  or_hll* sk = (or_hll*)calloc(1, sizeof(or_hll));
  u32set_init(&sk->tmp);
  clist_init(&sk->list);
  return sk;
}
or_hll* or_hll_new(uint8_t precision) { /* hyperloglog.go:49-63 */
  if (precision < 4 || precision > 18) return NULL;
  or_hll* sk = hll_alloc();
  sk->m = (uint32_t)or_go_pow(2, (double)precision);
  sk->p = precision;
  sk->alpha = hll_alpha((double)sk->m);
  sk->sparse = 1;
  sk->has_list = 1;
  return sk;
}
void or_hll_free(or_hll* sk) {
  if (!sk) return;
  u32set_free(&sk->tmp);
  clist_free(&sk->list);
  free(sk->tc);
  free(sk);
}
or_hll* or_hll_clone(const or_hll* s) {
  or_hll* sk = hll_alloc();
  sk->sparse = s->sparse; sk->p = s->p; sk->b = s->b; sk->m = s->m; sk->alpha = s->alpha;
  for (size_t i = 0; i < s->tmp.cap; i++) if (s->tmp.used[i]) u32set_add(&sk->tmp, s->tmp.keys[i]);
  sk->has_list = s->has_list;
  if (s->has_list) {
    sk->list.count = s->list.count; sk->list.last = s->list.last;
    for (size_t i = 0; i < s->list.len; i++) clist_push(&sk->list, s->list.b[i]);
  }
  sk->has_regs = s->has_regs;
  if (s->has_regs) {
    sk->ntc = s->ntc; sk->nz = s->nz;
    sk->tc = (uint8_t*)malloc(s->ntc ? s->ntc : 1);
    memcpy(sk->tc, s->tc, s->ntc);
  }
  return sk;
}

void or_hll_merge_sparse(or_hll* sk) { /* hyperloglog.go:229-267 */
  if (sk->tmp.len == 0) return;
  uint32_t* keys = (uint32_t*)malloc(sk->tmp.len * sizeof(uint32_t));
  size_t nk = u32set_sorted(&sk->tmp, keys);
  clist nl;
  clist_init(&nl);
  size_t it = 0;
  uint32_t last = 0;
  size_t i = 0;
  while (it < sk->list.len || i < nk) {
    if (!(it < sk->list.len)) { clist_append(&nl, keys[i]); i++; continue; }
    if (i >= nk) { last = clist_decode(&sk->list, &it, last); clist_append(&nl, last); continue; }
    size_t peek_i = it;
    uint32_t x1 = clist_decode(&sk->list, &peek_i, last), x2 = keys[i];
    if (x1 == x2) { it = peek_i; last = x1; clist_append(&nl, x1); i++; }
    else if (x1 > x2) { clist_append(&nl, x2); i++; }
    else { it = peek_i; last = x1; clist_append(&nl, x1); }
  }
  free(keys);
  clist_free(&sk->list);
  sk->list = nl;
  u32set_clear(&sk->tmp);
}

static void hll_insert_reg(or_hll* sk, uint32_t i, uint8_t r) { /* hyperloglog.go:168-183 */
  if ((uint8_t)(r - sk->b) >= HLL_CAPACITY) {
    uint8_t db = regs_min(sk);
    if (db > 0) { sk->b = (uint8_t)(sk->b + db); regs_rebase(sk, db); }
  }
  if (r > sk->b) {
    uint8_t d = (uint8_t)(r - sk->b);
    uint8_t val = d < HLL_CAPACITY - 1 ? d : (uint8_t)(HLL_CAPACITY - 1);
    if (val > regs_get(sk, i)) regs_set(sk, i, val);
  }
}

void or_hll_to_normal(or_hll* sk) { /* hyperloglog.go:152-166 */
  if (sk->tmp.len > 0) or_hll_merge_sparse(sk);
  regs_new(sk, sk->m);
  size_t it = 0;
  uint32_t last = 0;
  while (it < sk->list.len) {
    last = clist_decode(&sk->list, &it, last);
    uint32_t i; uint8_t r;
    or_hll_decode_hash(last, sk->p, HLL_PP, &i, &r);
    hll_insert_reg(sk, i, r);
  }
  sk->sparse = 0;
  u32set_free(&sk->tmp);
  clist_free(&sk->list);
  sk->has_list = 0;
}

static void hll_maybe_to_normal(or_hll* sk) { /* hyperloglog.go:80-87 */
  if ((uint32_t)sk->tmp.len * 100 > sk->m) {
    or_hll_merge_sparse(sk);
    if ((uint32_t)sk->list.len > sk->m) or_hll_to_normal(sk);
  }
}

void or_hll_insert_hash(or_hll* sk, uint64_t x) { /* hyperloglog.go:186-200 */
  if (sk->sparse) {
    u32set_add(&sk->tmp, or_hll_encode_hash(x, sk->p, HLL_PP));
    if ((uint32_t)sk->tmp.len * 100 > sk->m) {
      or_hll_merge_sparse(sk);
      if ((uint32_t)sk->list.len > sk->m) or_hll_to_normal(sk);
    }
  } else {
    uint64_t i; uint8_t r;
    or_hll_get_pos_val(x, sk->p, &i, &r);
    hll_insert_reg(sk, (uint32_t)i, r);
  }
}
void or_hll_insert(or_hll* sk, const uint8_t* e, size_t len) {
  or_hll_insert_hash(sk, or_metro_hash64(e, len, 1337)); /* utils.go:66-70 */
}

static double beta14(double ez) { /* utils.go:10-20 */
  double zl = or_go_log(ez + 1);
  return -0.370393911 * ez + 0.070471823 * zl + 0.17393686 * or_go_pow(zl, 2) +
         0.16339839 * or_go_pow(zl, 3) + -0.09237745 * or_go_pow(zl, 4) +
         0.03738027 * or_go_pow(zl, 5) + -0.005384159 * or_go_pow(zl, 6) +
         0.00042419 * or_go_pow(zl, 7);
}
static double beta16(double ez) { /* utils.go:22-32 */
  double zl = or_go_log(ez + 1);
  return -0.37331876643753059 * ez + -1.41704077448122989 * zl +
         0.40729184796612533 * or_go_pow(zl, 2) + 1.56152033906584164 * or_go_pow(zl, 3) +
         -0.99242233534286128 * or_go_pow(zl, 4) + 0.26064681399483092 * or_go_pow(zl, 5) +
         -0.03053811369682807 * or_go_pow(zl, 6) + 0.00155770210179105 * or_go_pow(zl, 7);
}
static double linear_count(uint32_t m, uint32_t v) { /* utils.go:53-56 */
  double fm = (double)m;
  return fm * or_go_log(fm / (double)v);
}
uint64_t or_hll_estimate(or_hll* sk) { /* hyperloglog.go:203-227 */
  if (sk->sparse) {
    or_hll_merge_sparse(sk);
    return or_go_f64_to_u64(linear_count(HLL_MP, HLL_MP - sk->list.count));
  }
  double sum, ez;
  regs_sum_and_zeros(sk, sk->b, &sum, &ez);
  double m = (double)sk->m;
  double est;
  double beta = sk->p < 16 ? beta14(ez) : beta16(ez);
  if (sk->b == 0) est = (sk->alpha * m * (m - ez) / (sum + beta)) + 0.5;
  else est = (sk->alpha * m * m / sum) + 0.5;
  return or_go_f64_to_u64(est + 0.5);
}

int or_hll_merge(or_hll* sk, const or_hll* other) { /* hyperloglog.go:92-149 */
  if (!other) return 0;
  or_hll* cp = or_hll_clone(other);
  if (sk->p != cp->p) { or_hll_free(cp); return -1; }
  if (sk->sparse && other->sparse) {
    uint32_t* keys = (uint32_t*)malloc((other->tmp.len + 1) * sizeof(uint32_t));
    size_t nk = u32set_sorted(&other->tmp, keys); /* Go iterates the map: order irrelevant here */
    for (size_t i = 0; i < nk; i++) u32set_add(&sk->tmp, keys[i]);
    free(keys);
    size_t it = 0;
    uint32_t last = 0;
    while (it < other->list.len) { last = clist_decode(&other->list, &it, last); u32set_add(&sk->tmp, last); }
    hll_maybe_to_normal(sk);
    or_hll_free(cp);
    return 0;
  }
  if (sk->sparse) or_hll_to_normal(sk);
  if (cp->sparse) {
    /* Go iterates cpOther.tmpSet in map order; the oracle uses ascending order. */
    uint32_t* keys = (uint32_t*)malloc((cp->tmp.len + 1) * sizeof(uint32_t));
    size_t nk = u32set_sorted(&cp->tmp, keys);
    for (size_t j = 0; j < nk; j++) {
      uint32_t i; uint8_t r;
      or_hll_decode_hash(keys[j], cp->p, HLL_PP, &i, &r);
      hll_insert_reg(sk, i, r);
    }
    free(keys);
    size_t it = 0;
    uint32_t last = 0;
    while (it < cp->list.len) {
      last = clist_decode(&cp->list, &it, last);
      uint32_t i; uint8_t r;
      or_hll_decode_hash(last, cp->p, HLL_PP, &i, &r);
      hll_insert_reg(sk, i, r);
    }
  } else {
    if (sk->b < cp->b) { regs_rebase(sk, (uint8_t)(cp->b - sk->b)); sk->b = cp->b; }
    else { regs_rebase(cp, (uint8_t)(sk->b - cp->b)); cp->b = sk->b; }
    for (uint32_t i = 0; i < cp->ntc; i++) {
      uint8_t v = cp->tc[i];
      uint8_t v1 = reg_get_nib(v, 0);
      if (v1 > regs_get(sk, i * 2)) regs_set(sk, i * 2, v1);
      uint8_t v2 = reg_get_nib(v, 1);
      if (v2 > regs_get(sk, 1 + i * 2)) regs_set(sk, 1 + i * 2, v2);
    }
  }
  or_hll_free(cp);
  return 0;
}

int or_hll_is_sparse(const or_hll* sk) { return sk->sparse; }
void or_hll_set_sparse_flag(or_hll* sk, int sparse) { sk->sparse = sparse; }
uint8_t or_hll_p(const or_hll* sk) { return sk->p; }
uint8_t or_hll_b(const or_hll* sk) { return sk->b; }
void or_hll_set_b(or_hll* sk, uint8_t b) { sk->b = b; }
uint32_t or_hll_nz(const or_hll* sk) { return sk->nz; }
uint32_t or_hll_m(const or_hll* sk) { return sk->m; }
uint8_t or_hll_reg_get(const or_hll* sk, uint32_t i) { return sk->has_regs ? regs_get(sk, i) : 0; }
void or_hll_reg_set(or_hll* sk, uint32_t i, uint8_t v) { if (sk->has_regs) regs_set(sk, i, v); }
void or_hll_reg_rebase(or_hll* sk, uint8_t delta) { if (sk->has_regs) regs_rebase(sk, delta); }
size_t or_hll_list_codes(const or_hll* sk, uint32_t* out, size_t cap) {
  size_t it = 0, n = 0;
  uint32_t last = 0;
  while (sk->has_list && it < sk->list.len) {
    last = clist_decode(&sk->list, &it, last);
    if (n < cap) out[n] = last;
    n++;
  }
  return n;
}
size_t or_hll_list_bytes(const or_hll* sk) { return sk->has_list ? sk->list.len : 0; }
uint32_t or_hll_list_count(const or_hll* sk) { return sk->has_list ? sk->list.count : 0; }
size_t or_hll_tmp_len(const or_hll* sk) { return sk->tmp.len; }
size_t or_hll_tmp_codes(const or_hll* sk, uint32_t* out, size_t cap) {
  if (sk->tmp.len == 0) return 0;
  uint32_t* keys = (uint32_t*)malloc(sk->tmp.len * sizeof(uint32_t));
  size_t n = u32set_sorted(&sk->tmp, keys);
  for (size_t i = 0; i < n && i < cap; i++) out[i] = keys[i];
  free(keys);
  return n;
}
void or_hll_tmp_add(or_hll* sk, uint32_t code) { u32set_add(&sk->tmp, code); }
void or_hll_list_append(or_hll* sk, uint32_t code) { if (sk->has_list) clist_append(&sk->list, code); }
size_t or_hll_tailcuts(const or_hll* sk, uint8_t* out, size_t cap) {
  if (!sk->has_regs) return 0;
  for (uint32_t i = 0; i < sk->ntc && i < cap; i++) out[i] = sk->tc[i];
  return sk->ntc;
}

/* MarshalBinary (hyperloglog.go:270-315) */
static size_t put_be32(uint8_t* out, size_t pos, size_t cap, uint32_t v) {
  if (pos + 4 <= cap) { out[pos] = (uint8_t)(v >> 24); out[pos + 1] = (uint8_t)(v >> 16); out[pos + 2] = (uint8_t)(v >> 8); out[pos + 3] = (uint8_t)v; }
  return pos + 4;
}
size_t or_hll_marshal(const or_hll* sk, uint8_t* out, size_t cap) {
  size_t pos = 0;
#define PUT(v) do { if (pos < cap) out[pos] = (uint8_t)(v); pos++; } while (0)
  PUT(HLL_VERSION); PUT(sk->p); PUT(sk->b);
  if (sk->sparse) {
    PUT(1);
    pos = put_be32(out, pos, cap, (uint32_t)sk->tmp.len);
    uint32_t* keys = (uint32_t*)malloc((sk->tmp.len + 1) * sizeof(uint32_t));
    size_t nk = u32set_sorted(&sk->tmp, keys);
    for (size_t i = 0; i < nk; i++) pos = put_be32(out, pos, cap, keys[i]);
    free(keys);
    pos = put_be32(out, pos, cap, sk->list.count);
    pos = put_be32(out, pos, cap, sk->list.last);
    pos = put_be32(out, pos, cap, (uint32_t)sk->list.len);
    for (size_t i = 0; i < sk->list.len; i++) PUT(sk->list.b[i]);
    return pos;
  }
  PUT(0);
  pos = put_be32(out, pos, cap, sk->ntc);
  for (uint32_t i = 0; i < sk->ntc; i++) PUT(sk->tc[i]);
  return pos;
#undef PUT
}
static uint32_t get_be32(const uint8_t* d) { return ((uint32_t)d[0] << 24) | ((uint32_t)d[1] << 16) | ((uint32_t)d[2] << 8) | d[3]; }
/* UnmarshalBinary (hyperloglog.go:318-376); -1 on truncated input (Go panics) */
int or_hll_unmarshal(or_hll* sk, const uint8_t* data, size_t len) {
  if (len < 4) return -1;
  or_hll* nh = or_hll_new(data[1]);
  if (!nh) return -2;
  /* *sk = *newh */
  u32set_free(&sk->tmp); clist_free(&sk->list); free(sk->tc);
  *sk = *nh;
  free(nh);
  sk->b = data[2];
  if (data[3] == 1) {
    sk->sparse = 1;
    if (len < 8) return -1;
    uint32_t tssz = get_be32(data + 4);
    size_t last_byte = (size_t)tssz * 4 + 8;
    if (len < last_byte + 12) return -1;
    for (size_t i = 8; i < last_byte; i += 4) u32set_add(&sk->tmp, get_be32(data + i));
    const uint8_t* d = data + last_byte;
    sk->list.count = get_be32(d);
    sk->list.last = get_be32(d + 4);
    uint32_t sz = get_be32(d + 8);
    if (len < last_byte + 12 + sz) return -1;
    sk->list.len = 0;
    for (uint32_t i = 0; i < sz; i++) clist_push(&sk->list, d[12 + i]);
    return 0;
  }
  sk->sparse = 0;
  clist_free(&sk->list); sk->has_list = 0;
  u32set_free(&sk->tmp);
  if (len < 8) return -1;
  uint32_t dsz = get_be32(data + 4);
  regs_new(sk, dsz * 2);
  size_t n = len - 8;
  for (size_t i = 0; i < n && i < sk->ntc; i++) {
    sk->tc[i] = data[8 + i];
    if ((uint8_t)((uint8_t)(sk->tc[i] << 4) >> 4) > 0) sk->nz--;
    if ((uint8_t)(sk->tc[i] >> 4) > 0) sk->nz--;
  }
  return 0;
}

/* math.Min / math.Max (Go): Min(-0,+0) = -0, Max(-0,+0) = +0 (NaN cannot reach here). */
static inline double go_min(double a, double b) {
  if (a == b) return signbit(a) ? a : b;
  return a < b ? a : b;
}
static inline double go_max(double a, double b) {
  if (a == b) return signbit(a) ? b : a;
  return a > b ? a : b;
}
/* =========================================================================
 * tdigest.MergingDigest (tdigest/merging_digest.go)
 * ========================================================================= */
typedef struct { double mean, weight; } centroid;
struct or_td {
  double compression;
  centroid* main; size_t nmain, capmain;
  double main_weight;
  centroid* temp; size_t ntemp, captemp;
  double temp_weight;
  double min, max;
};
static int estimate_temp_buffer(double compression) { /* merging_digest.go:87-93 */
  double tc = fmin(925, fmax(20, compression));
  return (int)(7.5 + 0.37 * tc - 2e-4 * tc * tc);
}
or_td* or_td_new(double compression) { /* merging_digest.go:72-85 */
  or_td* td = (or_td*)calloc(1, sizeof(or_td));
  td->compression = compression;
  td->capmain = (size_t)(int)((M_PI * compression / 2) + 0.5);
  if (td->capmain < 4) td->capmain = 4;
  td->main = (centroid*)malloc(td->capmain * sizeof(centroid));
  td->captemp = (size_t)estimate_temp_buffer(compression);
  td->temp = (centroid*)malloc((td->captemp + 1) * sizeof(centroid));
  td->min = INFINITY;
  td->max = -INFINITY;
  return td;
}
void or_td_free(or_td* td) { if (!td) return; free(td->main); free(td->temp); free(td); }

static double td_index_estimate(const or_td* td, double q) { /* merging_digest.go:240-243 */
  return td->compression * ((or_go_asin(2 * q - 1) / M_PI) + 0.5);
}
static void td_push_main(or_td* td, centroid c) {
  if (td->nmain == td->capmain) { td->capmain *= 2; td->main = (centroid*)realloc(td->main, td->capmain * sizeof(centroid)); }
  td->main[td->nmain++] = c;
}
/* mergeOne (merging_digest.go:210-236) */
static double td_merge_one(or_td* td, double before_weight, double total_weight, double before_index, centroid next) {
  double next_index = td_index_estimate(td, (before_weight + next.weight) / total_weight);
  if (next_index - before_index > 1 || td->nmain == 0) {
    td_push_main(td, next);
    return td_index_estimate(td, before_weight / total_weight);
  }
  centroid* c = &td->main[td->nmain - 1];
  c->weight += next.weight;
  c->mean += (next.mean - c->mean) * next.weight / c->weight;
  return before_index;
}
static int cl_less(void* d, int64_t i, int64_t j) { centroid* c = (centroid*)d; return c[i].mean < c[j].mean; }
static void cl_swap(void* d, int64_t i, int64_t j) { centroid* c = (centroid*)d; centroid t = c[i]; c[i] = c[j]; c[j] = t; }

/* mergeAllTemps (merging_digest.go:121-205): the in-place merge of the reference is a
 * two-way merge of main and the sorted temps (ties take the temp first). */
static void td_merge_all_temps(or_td* td) {
  if (td->ntemp == 0) return;
  go_sorter s = {cl_less, cl_swap, td->temp};
  go_sort(&s, (int64_t)td->ntemp);
  double total_weight = td->main_weight + td->temp_weight;
  double merged_weight = 0.0, last_merged_index = 0.0;
  centroid* old = td->main;
  size_t nold = td->nmain;
  size_t capold = td->capmain;
  td->capmain = capold;
  td->main = (centroid*)malloc(td->capmain * sizeof(centroid));
  td->nmain = 0;
  size_t mi = 0, ti = 0;
  while (mi < nold || ti < td->ntemp) {
    centroid next_temp = {INFINITY, 0};
    if (ti < td->ntemp) next_temp = td->temp[ti];
    centroid next_main = {INFINITY, 0};
    if (mi < nold) next_main = old[mi];
    if (next_main.mean < next_temp.mean) {
      mi++;
      last_merged_index = td_merge_one(td, merged_weight, total_weight, last_merged_index, next_main);
      merged_weight += next_main.weight;
    } else {
      ti++;
      last_merged_index = td_merge_one(td, merged_weight, total_weight, last_merged_index, next_temp);
      merged_weight += next_temp.weight;
    }
  }
  free(old);
  td->ntemp = 0;
  td->temp_weight = 0;
  td->main_weight = total_weight;
}

/* Study helper, not a reference function: merge n samples into the digest with ONE
 * mergeAllTemps (after merging whatever is pending), the way the engine's hot-key batch
 * path does.  Used by tools/tdigest_study.py to size the exact-replay threshold. */
int or_td_add_batch(or_td* td, const double* v, const double* w, size_t n) {
  td_merge_all_temps(td);
  if (n == 0) return 0;
  centroid* keep = td->temp;
  size_t keepcap = td->captemp;
  centroid* big = (centroid*)malloc(n * sizeof(centroid));
  if (!big) return -1;
  double tw = 0.0;
  for (size_t i = 0; i < n; i++) {
    big[i].mean = v[i];
    big[i].weight = w[i];
    tw += w[i];
    td->min = go_min(td->min, v[i]);
    td->max = go_max(td->max, v[i]);
  }
  td->temp = big;
  td->captemp = n;
  td->ntemp = n;
  td->temp_weight = tw;
  td_merge_all_temps(td);
  free(big);
  td->temp = keep;
  td->captemp = keepcap;
  return 0;
}

int or_td_add(or_td* td, double value, double weight) { /* merging_digest.go:97-118 */
  if (isnan(value) || isinf(value) || weight <= 0) return -1; /* Go: panic */
  if (td->ntemp == td->captemp) td_merge_all_temps(td);
  td->min = go_min(td->min, value);
  td->max = go_max(td->max, value);
  td->temp[td->ntemp].mean = value;
  td->temp[td->ntemp].weight = weight;
  td->ntemp++;
  td->temp_weight += weight;
  return 0;
}
/* convenience: Add() every sample in order; returns the index of the first rejected one, or -1 */
long or_td_add_many(or_td* td, const double* v, const double* w, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (or_td_add(td, v[i], w[i]) != 0) return (long)i;
  return -1;
}
double or_td_cdf(or_td* td, double value) { /* merging_digest.go:247-279 */
  td_merge_all_temps(td);
  if (td->nmain == 0) return NAN;
  if (value <= td->min) return 0;
  if (value >= td->max) return 1;
  double wsf = 0, lower = td->min;
  for (size_t i = 0; i < td->nmain; i++) {
    double upper = (i != td->nmain - 1) ? (td->main[i + 1].mean + td->main[i].mean) / 2 : td->max;
    if (value < upper) {
      wsf += td->main[i].weight * (value - lower) / (upper - lower);
      return wsf / td->main_weight;
    }
    wsf += td->main[i].weight;
    lower = upper;
  }
  return NAN;
}
double or_td_quantile(or_td* td, double quantile) { /* merging_digest.go:283-313 */
  if (quantile < 0 || quantile > 1) return NAN; /* Go: panic */
  td_merge_all_temps(td);
  double q = quantile * td->main_weight;
  double wsf = 0, lower = td->min;
  for (size_t i = 0; i < td->nmain; i++) {
    double upper = (i != td->nmain - 1) ? (td->main[i + 1].mean + td->main[i].mean) / 2 : td->max;
    double w = td->main[i].weight;
    if (q <= wsf + w) {
      double proportion = (q - wsf) / w;
      return lower + (proportion * (upper - lower));
    }
    wsf += w;
    lower = upper;
  }
  return NAN;
}
double or_td_min(const or_td* td) { return td->min; }
double or_td_max(const or_td* td) { return td->max; }
double or_td_count(const or_td* td) { return td->main_weight + td->temp_weight; }
size_t or_td_temp_len(const or_td* td) { return td->ntemp; }
void or_td_merge(or_td* td, or_td* other, const int64_t* perm) { /* merging_digest.go:344-356 */
  for (size_t k = 0; k < other->nmain; k++) {
    size_t i = perm ? (size_t)perm[k] : k;
    or_td_add(td, other->main[i].mean, other->main[i].weight);
  }
  for (size_t i = 0; i < other->ntemp; i++) or_td_add(td, other->temp[i].mean, other->temp[i].weight);
}
/* the main centroids as they are, pending temps not merged (diagnostics: a replay's state between
 * two ingest calls) */
size_t or_td_main(const or_td* td, double* means, double* weights, size_t cap) {
  for (size_t i = 0; i < td->nmain && i < cap; i++) { means[i] = td->main[i].mean; weights[i] = td->main[i].weight; }
  return td->nmain;
}
size_t or_td_centroids(or_td* td, double* means, double* weights, size_t cap) {
  td_merge_all_temps(td);
  for (size_t i = 0; i < td->nmain && i < cap; i++) { means[i] = td->main[i].mean; weights[i] = td->main[i].weight; }
  return td->nmain;
}
void or_td_set_state(or_td* td, const double* means, const double* weights, size_t n,
                     double compression, double mn, double mx) { /* GobDecode's effect (382-412) */
  td->nmain = 0;
  td->main_weight = 0;
  for (size_t i = 0; i < n; i++) {
    centroid c = {means[i], weights[i]};
    td_push_main(td, c);
  }
  td->compression = compression;
  td->min = mn;
  td->max = mx;
  for (size_t i = 0; i < n; i++) td->main_weight += weights[i];
  td->temp_weight = 0;
  size_t ts = (size_t)estimate_temp_buffer(compression);
  if (ts != td->captemp) { td->captemp = ts; td->temp = (centroid*)realloc(td->temp, (ts + 1) * sizeof(centroid)); }
  td->ntemp = 0;
}

/* ---- encoding/gob subset: the value stream MergingDigest.GobEncode writes
 * ([]Centroid, float64 compression, float64 min, float64 max), with the type
 * definitions Go emits for it (ids 66..68 as in fixtures/import.uncompressed). */
typedef struct { const uint8_t* d; size_t n, i; int err; } gobr;
static uint64_t gob_uint(gobr* r) {
  if (r->i >= r->n) { r->err = 1; return 0; }
  uint8_t b = r->d[r->i++];
  if (b < 0x80) return b;
  int cnt = -(int)(int8_t)b;
  if (cnt > 8 || r->i + (size_t)cnt > r->n) { r->err = 1; return 0; }
  uint64_t v = 0;
  for (int k = 0; k < cnt; k++) v = (v << 8) | r->d[r->i++];
  return v;
}
static int64_t gob_int(gobr* r) {
  uint64_t u = gob_uint(r);
  return (u & 1) ? ~(int64_t)(u >> 1) : (int64_t)(u >> 1);
}
static double gob_float(gobr* r) {
  uint64_t u = gob_uint(r), v = 0;
  for (int k = 0; k < 8; k++) { v = (v << 8) | (u & 0xff); u >>= 8; }
  double x;
  memcpy(&x, &v, 8);
  return x;
}
/* Minimal wire-type registry: slice(elem) / struct(fields) / builtin ids < 64. */
#define GOB_MAXT 32
typedef struct { int64_t id; int kind; int64_t elem; int nf; int64_t fid[8]; char fname[8][16]; } gobtype;
typedef struct { gobtype t[GOB_MAXT]; int n; } gobreg;
static gobtype* gob_find(gobreg* g, int64_t id) {
  for (int i = 0; i < g->n; i++) if (g->t[i].id == id) return &g->t[i];
  return NULL;
}
static void gob_skip_string(gobr* r) { uint64_t l = gob_uint(r); if (r->i + l > r->n) { r->err = 1; return; } r->i += l; }
static void gob_read_string(gobr* r, char* out, size_t cap) {
  uint64_t l = gob_uint(r);
  if (r->i + l > r->n) { r->err = 1; return; }
  size_t c = l < cap - 1 ? l : cap - 1;
  memcpy(out, r->d + r->i, c);
  out[c] = 0;
  r->i += l;
}
/* CommonType {Name string; Id typeId} -> returns Id */
static int64_t gob_common(gobr* r) {
  int64_t id = 0;
  int64_t f = -1;
  for (;;) {
    uint64_t delta = gob_uint(r);
    if (r->err || delta == 0) break;
    f += (int64_t)delta;
    if (f == 0) gob_skip_string(r);
    else if (f == 1) id = gob_int(r);
    else { r->err = 1; break; }
  }
  return id;
}
static void gob_wiretype(gobr* r, gobreg* g) {
  int64_t f = -1;
  for (;;) {
    uint64_t delta = gob_uint(r);
    if (r->err || delta == 0) break;
    f += (int64_t)delta;
    if (g->n >= GOB_MAXT) { r->err = 1; return; }
    gobtype* t = &g->t[g->n];
    memset(t, 0, sizeof(*t));
    if (f == 1 || f == 0) { /* SliceT / ArrayT {CommonType; Elem; [Len]} */
      int64_t sf = -1;
      t->kind = 1;
      for (;;) {
        uint64_t d2 = gob_uint(r);
        if (r->err || d2 == 0) break;
        sf += (int64_t)d2;
        if (sf == 0) t->id = gob_common(r);
        else if (sf == 1) t->elem = gob_int(r);
        else if (sf == 2) (void)gob_int(r);
        else { r->err = 1; return; }
      }
      g->n++;
    } else if (f == 2) { /* StructT {CommonType; Field []*fieldType} */
      int64_t sf = -1;
      t->kind = 2;
      for (;;) {
        uint64_t d2 = gob_uint(r);
        if (r->err || d2 == 0) break;
        sf += (int64_t)d2;
        if (sf == 0) t->id = gob_common(r);
        else if (sf == 1) {
          uint64_t nf = gob_uint(r);
          if (nf > 8) { r->err = 1; return; }
          t->nf = (int)nf;
          for (uint64_t k = 0; k < nf; k++) {
            int64_t ff = -1;
            for (;;) {
              uint64_t d3 = gob_uint(r);
              if (r->err || d3 == 0) break;
              ff += (int64_t)d3;
              if (ff == 0) gob_read_string(r, t->fname[k], 16);
              else if (ff == 1) t->fid[k] = gob_int(r);
              else { r->err = 1; return; }
            }
          }
        } else { r->err = 1; return; }
      }
      g->n++;
    } else { r->err = 1; return; }
  }
}
/* Decode one value of type id into a generic sink.  For []Centroid the sink is the digest. */
typedef struct { centroid* c; size_t n, cap; } cvec;
static void cvec_push(cvec* v, centroid c) {
  if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 16; v->c = (centroid*)realloc(v->c, v->cap * sizeof(centroid)); }
  v->c[v->n++] = c;
}
static void gob_skip_value(gobr* r, gobreg* g, int64_t id);
static void gob_skip_struct(gobr* r, gobreg* g, gobtype* t) {
  int64_t f = -1;
  for (;;) {
    uint64_t delta = gob_uint(r);
    if (r->err || delta == 0) break;
    f += (int64_t)delta;
    if (f >= t->nf) { r->err = 1; return; }
    gob_skip_value(r, g, t->fid[f]);
  }
}
static void gob_skip_value(gobr* r, gobreg* g, int64_t id) {
  if (id == 1 || id == 2 || id == 3 || id == 4) { (void)gob_uint(r); return; }
  if (id == 5 || id == 6) { gob_skip_string(r); return; }
  gobtype* t = gob_find(g, id);
  if (!t) { r->err = 1; return; }
  if (t->kind == 1) { uint64_t n = gob_uint(r); for (uint64_t k = 0; k < n && !r->err; k++) gob_skip_value(r, g, t->elem); }
  else gob_skip_struct(r, g, t);
}
static void gob_centroids(gobr* r, gobreg* g, gobtype* slice_t, cvec* out) {
  gobtype* st = gob_find(g, slice_t->elem);
  if (!st || st->kind != 2) { r->err = 1; return; }
  uint64_t n = gob_uint(r);
  for (uint64_t k = 0; k < n && !r->err; k++) {
    centroid c = {0, 0};
    int64_t f = -1;
    for (;;) {
      uint64_t delta = gob_uint(r);
      if (r->err || delta == 0) break;
      f += (int64_t)delta;
      if (f >= st->nf) { r->err = 1; return; }
      if (strcmp(st->fname[f], "Mean") == 0 && st->fid[f] == 4) c.mean = gob_float(r);
      else if (strcmp(st->fname[f], "Weight") == 0 && st->fid[f] == 4) c.weight = gob_float(r);
      else gob_skip_value(r, g, st->fid[f]);
    }
    cvec_push(out, c);
  }
}
int or_td_gob_decode(or_td* td, const uint8_t* data, size_t len) { /* merging_digest.go:382-412 */
  gobr r = {data, len, 0, 0};
  gobreg g;
  g.n = 0;
  cvec cs = {NULL, 0, 0};
  double vals[3];
  int nvals = 0, have_c = 0;
  while (r.i < r.n && !r.err && nvals < 3) {
    uint64_t mlen = gob_uint(&r);
    size_t end = r.i + mlen;
    if (r.err || end > r.n) { r.err = 1; break; }
    int64_t id = gob_int(&r);
    if (id < 0) { gob_wiretype(&r, &g); }
    else {
      if (gob_uint(&r) != 0) { r.err = 1; break; } /* singleton marker */
      if (!have_c) {
        gobtype* t = gob_find(&g, id);
        if (!t || t->kind != 1) { r.err = 1; break; }
        gob_centroids(&r, &g, t, &cs);
        have_c = 1;
      } else if (id == 4) vals[nvals++] = gob_float(&r);
      else { r.err = 1; break; }
    }
    if (r.i != end) { r.err = 1; break; }
  }
  if (r.err || !have_c || nvals != 3) { free(cs.c); return -1; }
  double* m = (double*)malloc((cs.n + 1) * sizeof(double));
  double* w = (double*)malloc((cs.n + 1) * sizeof(double));
  for (size_t i = 0; i < cs.n; i++) { m[i] = cs.c[i].mean; w[i] = cs.c[i].weight; }
  or_td_set_state(td, m, w, cs.n, vals[0], vals[1], vals[2]);
  free(m); free(w); free(cs.c);
  return 0;
}
typedef struct { uint8_t* d; size_t n, cap; } gobw;
static void gw_byte(gobw* w, uint8_t b) { if (w->n < w->cap) w->d[w->n] = b; w->n++; }
static void gw_uint(gobw* w, uint64_t u) {
  if (u < 0x80) { gw_byte(w, (uint8_t)u); return; }
  uint8_t buf[8]; int n = 0;
  while (u) { buf[n++] = (uint8_t)u; u >>= 8; }
  gw_byte(w, (uint8_t)(-n));
  for (int k = n - 1; k >= 0; k--) gw_byte(w, buf[k]);
}
static void gw_int(gobw* w, int64_t i) { gw_uint(w, i < 0 ? ((uint64_t)(~i) << 1) | 1 : (uint64_t)i << 1); }
static void gw_float(gobw* w, double x) {
  uint64_t v; memcpy(&v, &x, 8);
  uint64_t u = 0;
  for (int k = 0; k < 8; k++) { u = (u << 8) | (v & 0xff); v >>= 8; }
  gw_uint(w, u);
}
static void gw_str(gobw* w, const char* s) { size_t l = strlen(s); gw_uint(w, l); for (size_t i = 0; i < l; i++) gw_byte(w, (uint8_t)s[i]); }
/* message = uint(len) + body; body written into a scratch buffer first */
static void gw_msg(gobw* w, const gobw* body) { gw_uint(w, body->n); for (size_t i = 0; i < body->n; i++) gw_byte(w, body->d[i]); }
size_t or_td_gob_encode(or_td* td, uint8_t* out, size_t cap) { /* merging_digest.go:361-380 */
  td_merge_all_temps(td);
  gobw w = {out, 0, cap};
  size_t scap = 64 + td->nmain * 24;
  gobw b = {(uint8_t*)malloc(scap), 0, scap};
  /* type 68 = []Centroid (elem 66) */
  b.n = 0; gw_int(&b, -68); gw_uint(&b, 2); gw_uint(&b, 1); gw_uint(&b, 2); gw_int(&b, 68); gw_uint(&b, 0);
  gw_uint(&b, 1); gw_int(&b, 66); gw_uint(&b, 0); gw_uint(&b, 0); gw_msg(&w, &b);
  /* type 66 = struct Centroid {Mean float64; Weight float64; Samples []float64} */
  b.n = 0; gw_int(&b, -66); gw_uint(&b, 3); gw_uint(&b, 1); gw_uint(&b, 1); gw_str(&b, "Centroid");
  gw_uint(&b, 1); gw_int(&b, 66); gw_uint(&b, 0); gw_uint(&b, 1); gw_uint(&b, 3);
  gw_uint(&b, 1); gw_str(&b, "Mean"); gw_uint(&b, 1); gw_int(&b, 4); gw_uint(&b, 0);
  gw_uint(&b, 1); gw_str(&b, "Weight"); gw_uint(&b, 1); gw_int(&b, 4); gw_uint(&b, 0);
  gw_uint(&b, 1); gw_str(&b, "Samples"); gw_uint(&b, 1); gw_int(&b, 67); gw_uint(&b, 0);
  gw_uint(&b, 0); gw_uint(&b, 0); gw_msg(&w, &b);
  /* type 67 = []float64 */
  b.n = 0; gw_int(&b, -67); gw_uint(&b, 2); gw_uint(&b, 1); gw_uint(&b, 1); gw_str(&b, "[]float64");
  gw_uint(&b, 1); gw_int(&b, 67); gw_uint(&b, 0); gw_uint(&b, 1); gw_int(&b, 4); gw_uint(&b, 0); gw_uint(&b, 0);
  gw_msg(&w, &b);
  /* value: []Centroid */
  b.n = 0; gw_int(&b, 68); gw_uint(&b, 0); gw_uint(&b, td->nmain);
  for (size_t i = 0; i < td->nmain; i++) {
    /* zero fields are omitted by gob */
    int64_t last = -1;
    if (td->main[i].mean != 0) { gw_uint(&b, (uint64_t)(0 - last)); gw_float(&b, td->main[i].mean); last = 0; }
    if (td->main[i].weight != 0) { gw_uint(&b, (uint64_t)(1 - last)); gw_float(&b, td->main[i].weight); last = 1; }
    gw_uint(&b, 0);
  }
  gw_msg(&w, &b);
  double vals[3] = {td->compression, td->min, td->max};
  for (int k = 0; k < 3; k++) { b.n = 0; gw_int(&b, 4); gw_uint(&b, 0); gw_float(&b, vals[k]); gw_msg(&w, &b); }
  free(b.d);
  return w.n <= cap ? w.n : 0;
}

/* =========================================================================
 * samplers + Worker restatement (samplers/samplers.go, worker.go).  One slot
 * table per sampler class; the host's MetricKey interning picks the slot.
 * ========================================================================= */
typedef struct {
  double weight, min, max, sum, rsum;
  or_td* td;
} histo;
struct or_worker {
  uint32_t nc, ng, nh, ns;
  int64_t* cval; uint8_t* ctouch;
  double* gval; uint8_t* gtouch;
  histo* h; uint8_t* htouch;
  or_hll** s; uint8_t* stouch;
};
or_worker* or_worker_new(uint32_t nc, uint32_t ng, uint32_t nh, uint32_t ns) {
  or_worker* w = (or_worker*)calloc(1, sizeof(or_worker));
  w->nc = nc; w->ng = ng; w->nh = nh; w->ns = ns;
  w->cval = (int64_t*)calloc(nc + 1, 8); w->ctouch = (uint8_t*)calloc(nc + 1, 1);
  w->gval = (double*)calloc(ng + 1, 8); w->gtouch = (uint8_t*)calloc(ng + 1, 1);
  w->h = (histo*)calloc(nh + 1, sizeof(histo)); w->htouch = (uint8_t*)calloc(nh + 1, 1);
  w->s = (or_hll**)calloc(ns + 1, sizeof(or_hll*)); w->stouch = (uint8_t*)calloc(ns + 1, 1);
  return w;
}
void or_worker_free(or_worker* w) {
  if (!w) return;
  for (uint32_t i = 0; i < w->nh; i++) or_td_free(w->h[i].td);
  for (uint32_t i = 0; i < w->ns; i++) or_hll_free(w->s[i]);
  free(w->cval); free(w->ctouch); free(w->gval); free(w->gtouch);
  free(w->h); free(w->htouch); free(w->s); free(w->stouch);
  free(w);
}
static histo* worker_histo(or_worker* w, uint32_t slot) { /* Upsert -> NewHist (samplers.go:359-369) */
  histo* h = &w->h[slot];
  if (!w->htouch[slot]) {
    w->htouch[slot] = 1;
    h->td = or_td_new(100);
    h->weight = 0; h->min = INFINITY; h->max = -INFINITY; h->sum = 0; h->rsum = 0;
  }
  return h;
}
static or_hll* worker_set(or_worker* w, uint32_t slot) { /* Upsert -> NewSet (samplers.go:270-279) */
  if (!w->stouch[slot]) { w->stouch[slot] = 1; w->s[slot] = or_hll_new(14); }
  return w->s[slot];
}
void or_worker_counter(or_worker* w, const uint32_t* slot, const double* value, const float* rate, size_t n) {
  for (size_t i = 0; i < n; i++) { /* Counter.Sample, samplers.go:132-134 */
    uint32_t s = slot[i];
    w->ctouch[s] = 1;
    float inv = 1.0f / rate[i];
    uint64_t a = (uint64_t)or_go_f64_to_i64(value[i]);
    uint64_t b = (uint64_t)or_go_f64_to_i64((double)inv);
    w->cval[s] = (int64_t)((uint64_t)w->cval[s] + a * b);
  }
}
void or_worker_gauge(or_worker* w, const uint32_t* slot, const double* value, size_t n) {
  for (size_t i = 0; i < n; i++) { w->gtouch[slot[i]] = 1; w->gval[slot[i]] = value[i]; } /* Gauge.Sample */
}
void or_worker_histo(or_worker* w, const uint32_t* slot, const double* value, const float* rate, size_t n) {
  for (size_t i = 0; i < n; i++) { /* Histo.Sample, samplers.go:346-356 */
    histo* h = worker_histo(w, slot[i]);
    double sample = value[i];
    double weight = (double)(1.0f / rate[i]);
    or_td_add(h->td, sample, weight);
    h->weight += weight;
    h->min = go_min(h->min, sample);
    h->max = go_max(h->max, sample);
    h->sum += sample * weight;
    h->rsum += (1 / sample) * weight;
  }
}
void or_worker_set(or_worker* w, const uint32_t* slot, const uint32_t* off, const uint8_t* bytes, size_t n) {
  for (size_t i = 0; i < n; i++) or_hll_insert(worker_set(w, slot[i]), bytes + off[i], off[i + 1] - off[i]);
}
void or_worker_set_hashed(or_worker* w, const uint32_t* slot, const uint64_t* hashes, size_t n) {
  for (size_t i = 0; i < n; i++) or_hll_insert_hash(worker_set(w, slot[i]), hashes[i]);
}
void or_worker_import_counter(or_worker* w, uint32_t slot, int64_t v) { /* Counter.Combine */
  w->ctouch[slot] = 1;
  w->cval[slot] = (int64_t)((uint64_t)w->cval[slot] + (uint64_t)v);
}
void or_worker_import_gauge(or_worker* w, uint32_t slot, double v) { w->gtouch[slot] = 1; w->gval[slot] = v; }
int or_worker_import_set(or_worker* w, uint32_t slot, const uint8_t* data, size_t len) { /* Set.Combine */
  or_hll* sk = worker_set(w, slot);
  or_hll* other = or_hll_new(14);
  int rc = or_hll_unmarshal(other, data, len);
  if (rc == 0) rc = or_hll_merge(sk, other);
  or_hll_free(other);
  return rc;
}
int or_worker_import_histo(or_worker* w, uint32_t slot, const uint8_t* gob, size_t len, const int64_t* perm) {
  histo* h = worker_histo(w, slot); /* Histo.Combine, samplers.go:519-526 */
  or_td* other = or_td_new(100);
  int rc = or_td_gob_decode(other, gob, len);
  if (rc == 0) or_td_merge(h->td, other, perm);
  or_td_free(other);
  return rc;
}
int or_worker_touched(const or_worker* w, int cls, uint32_t slot) {
  switch (cls) {
    case 0: return w->ctouch[slot];
    case 1: return w->gtouch[slot];
    case 2: return w->htouch[slot];
    case 3: return w->stouch[slot];
  }
  return 0;
}
int64_t or_worker_counter_value(const or_worker* w, uint32_t slot) { return w->cval[slot]; }
double or_worker_gauge_value(const or_worker* w, uint32_t slot) { return w->gval[slot]; }
void or_worker_histo_stats(const or_worker* w, uint32_t slot, double* o) {
  const histo* h = &w->h[slot];
  o[0] = h->weight; o[1] = h->min; o[2] = h->max; o[3] = h->sum; o[4] = h->rsum;
  o[5] = h->td ? h->td->min : INFINITY;
  o[6] = h->td ? h->td->max : -INFINITY;
  o[7] = h->td ? or_td_count(h->td) : 0;
}
double or_worker_histo_quantile(or_worker* w, uint32_t slot, double q) {
  return w->h[slot].td ? or_td_quantile(w->h[slot].td, q) : NAN;
}
size_t or_worker_histo_centroids(or_worker* w, uint32_t slot, double* m, double* wt, size_t cap) {
  return w->h[slot].td ? or_td_centroids(w->h[slot].td, m, wt, cap) : 0;
}
uint64_t or_worker_set_estimate(or_worker* w, uint32_t slot) { return w->s[slot] ? or_hll_estimate(w->s[slot]) : 0; }
or_td* or_worker_histo_digest(or_worker* w, uint32_t slot) { return w->h[slot].td; }
or_hll* or_worker_set_sketch(or_worker* w, uint32_t slot) { return w->s[slot]; }

/* =========================================================================
 * Multi-threaded CPU baseline (veneur's worker pool: records routed by
 * slot hash % nthreads, each worker owns its keys; then the flush).
 * ========================================================================= */
typedef struct {
  int tid, nthreads;
  or_worker* w;
  const uint32_t *c_slot, *g_slot, *h_slot, *s_slot, *s_off;
  const double *c_val, *g_val, *h_val;
  const float *c_rate, *h_rate;
  const uint8_t* s_bytes;
  size_t n_c, n_g, n_h, n_s;
  const double* pct; int n_pct;
  uint32_t nc, ng, nh, ns;
  double checksum;
  const or_baseline_out* out;
} bl_arg;
static inline int owns(uint32_t slot, int cls, int tid, int n) {
  uint32_t h = (slot * 2654435761u) ^ (uint32_t)cls;
  return (int)(h % (uint32_t)n) == tid;
}
static void* bl_thread(void* p) {
  bl_arg* a = (bl_arg*)p;
  or_worker* w = a->w;
  for (size_t i = 0; i < a->n_c; i++)
    if (owns(a->c_slot[i], 0, a->tid, a->nthreads)) or_worker_counter(w, a->c_slot + i, a->c_val + i, a->c_rate + i, 1);
  for (size_t i = 0; i < a->n_g; i++)
    if (owns(a->g_slot[i], 1, a->tid, a->nthreads)) or_worker_gauge(w, a->g_slot + i, a->g_val + i, 1);
  for (size_t i = 0; i < a->n_h; i++)
    if (owns(a->h_slot[i], 2, a->tid, a->nthreads)) or_worker_histo(w, a->h_slot + i, a->h_val + i, a->h_rate + i, 1);
  for (size_t i = 0; i < a->n_s; i++)
    if (owns(a->s_slot[i], 3, a->tid, a->nthreads))
      or_hll_insert(worker_set(w, a->s_slot[i]), a->s_bytes + a->s_off[i], a->s_off[i + 1] - a->s_off[i]);
  /* flush (generateInterMetrics: Counter/Gauge value, Histo quantiles, Set Estimate) */
  const or_baseline_out* o = a->out;
  double cs = 0;
  for (uint32_t s = 0; s < a->nc; s++)
    if (w->ctouch[s]) {
      cs += (double)w->cval[s];
      if (o && o->counter) o->counter[s] = w->cval[s];
      if (o && o->touched[0]) o->touched[0][s] = 1;
    }
  for (uint32_t s = 0; s < a->ng; s++)
    if (w->gtouch[s]) {
      cs += w->gval[s];
      if (o && o->gauge) o->gauge[s] = w->gval[s];
      if (o && o->touched[1]) o->touched[1][s] = 1;
    }
  for (uint32_t s = 0; s < a->nh; s++)
    if (w->htouch[s]) {
      cs += w->h[s].weight;
      for (int k = 0; k < a->n_pct; k++) {
        double q = or_td_quantile(w->h[s].td, a->pct[k]);
        cs += q;
        if (o && o->histo_q) o->histo_q[(size_t)s * a->n_pct + k] = q;
      }
      if (o && o->histo_stats) or_worker_histo_stats(w, s, o->histo_stats + (size_t)s * 8);
      if (o && o->touched[2]) o->touched[2][s] = 1;
    }
  for (uint32_t s = 0; s < a->ns; s++)
    if (w->stouch[s]) {
      uint64_t est = or_hll_estimate(w->s[s]);
      cs += (double)est;
      if (o && o->set_est) o->set_est[s] = est;
      if (o && o->touched[3]) o->touched[3][s] = 1;
    }
  a->checksum = cs;
  return NULL;
}

static or_baseline_out g_bl_out;
static int g_bl_out_set = 0;
void or_baseline_set_output(const or_baseline_out* out) {
  if (out) { g_bl_out = *out; g_bl_out_set = 1; }
  else g_bl_out_set = 0;
}
double or_baseline_run(int nthreads, uint32_t nc, uint32_t ng, uint32_t nh, uint32_t ns,
                       const uint32_t* c_slot, const double* c_val, const float* c_rate, size_t n_c,
                       const uint32_t* g_slot, const double* g_val, size_t n_g,
                       const uint32_t* h_slot, const double* h_val, const float* h_rate, size_t n_h,
                       const uint32_t* s_slot, const uint32_t* s_off, const uint8_t* s_bytes, size_t n_s,
                       const double* pct, int n_pct, double* checksum_out) {
  if (nthreads < 1) nthreads = 1;
  bl_arg* args = (bl_arg*)calloc((size_t)nthreads, sizeof(bl_arg));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    bl_arg* a = &args[t];
    a->tid = t; a->nthreads = nthreads;
    a->w = or_worker_new(nc, ng, nh, ns);
    a->c_slot = c_slot; a->c_val = c_val; a->c_rate = c_rate; a->n_c = n_c;
    a->g_slot = g_slot; a->g_val = g_val; a->n_g = n_g;
    a->h_slot = h_slot; a->h_val = h_val; a->h_rate = h_rate; a->n_h = n_h;
    a->s_slot = s_slot; a->s_off = s_off; a->s_bytes = s_bytes; a->n_s = n_s;
    a->pct = pct; a->n_pct = n_pct;
    a->nc = nc; a->ng = ng; a->nh = nh; a->ns = ns;
    a->out = g_bl_out_set ? &g_bl_out : NULL;
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, bl_thread, &args[t]);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  double cs = 0;
  for (int t = 0; t < nthreads; t++) { cs += args[t].checksum; or_worker_free(args[t].w); }
  if (checksum_out) *checksum_out = cs;
  free(args); free(th);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

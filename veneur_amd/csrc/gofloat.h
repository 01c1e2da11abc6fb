// gofloat.h -- strconv.ParseFloat(s, 64 | 32) of Go 1.9, as samplers/parser.go:239,261 calls it,
// for one lane of the device DogStatsD parser (parse_device.hip).  Host + device code: the same
// functions run on the CPU through vn_go_parse_float (tests fuzz them against glibc strtod/strtof).
//
// Syntax (Go 1.9 atof.go special + readFloat): [+-]?(inf|infinity) and nan, case-insensitive (nan
// takes no sign); otherwise [+-]?(digits[.digits*] | .digits)([eE][+-]?digits)?, no underscores,
// no hex, no spaces.  The value is the correctly rounded binary64 / binary32 (round half to even),
// which every correct algorithm agrees on; out of range (rounds to +-Inf) is an error (ErrRange),
// underflow rounds to zero / a subnormal without error.  Three ways to the rounded value:
//   1. Go's atof64exact / atof32exact: a mantissa below 2^52 (2^23) scaled by an exact power of
//      ten with one IEEE multiply or divide (float32: done in binary64 and rounded once more,
//      which is exact-rounding safe for one operation since 53 >= 2*24 + 2);
//   2. an exact 128-bit integer: <= 19 significant digits times 10^e (0 <= e <= 19), or divided
//      by 5^k (1 <= k <= 27) with a 64-iteration long division and a sticky remainder -- then
//      rounded to 53 / 24 bits;
//   3. otherwise Go's decimal algorithm (decimal.go: an 800-digit decimal shifted by powers of
//      two, then floatBits), restated; slow but rare (more than 19 digits, |exponent| large).
#pragma once
#include <stdint.h>

namespace vn {
namespace gofloat {

#define VN_HD __host__ __device__ __forceinline__

VN_HD char lower(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }

VN_HD bool ieq(const char* p, uint32_t n, const char* w, uint32_t m) {
  if (n != m) return false;
  for (uint32_t i = 0; i < n; ++i)
    if (lower(p[i]) != w[i]) return false;
  return true;
}

VN_HD uint64_t bits_of(double d) {
  union { double d; uint64_t u; } x;
  x.d = d;
  return x.u;
}
VN_HD double from_bits(uint64_t u) {
  union { double d; uint64_t u; } x;
  x.u = u;
  return x.d;
}
VN_HD float f32_from_bits(uint32_t u) {
  union { float f; uint32_t u; } x;
  x.u = u;
  return x.f;
}

VN_HD int clz64(uint64_t x) {  // x != 0
  int n = 0;
  if (!(x >> 32)) { n += 32; x <<= 32; }
  if (!(x >> 48)) { n += 16; x <<= 16; }
  if (!(x >> 56)) { n += 8; x <<= 8; }
  if (!(x >> 60)) { n += 4; x <<= 4; }
  if (!(x >> 62)) { n += 2; x <<= 2; }
  if (!(x >> 63)) { n += 1; }
  return n;
}

VN_HD void mul64(uint64_t a, uint64_t b, uint64_t* hi, uint64_t* lo) {
  const uint64_t a0 = (uint32_t)a, a1 = a >> 32, b0 = (uint32_t)b, b1 = b >> 32;
  const uint64_t p00 = a0 * b0, p01 = a0 * b1, p10 = a1 * b0, p11 = a1 * b1;
  const uint64_t mid = (p00 >> 32) + (uint32_t)p01 + (uint32_t)p10;
  *lo = (mid << 32) | (uint32_t)p00;
  *hi = p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
}

struct FloatInfo {
  int mantbits, expbits, bias;
};
constexpr FloatInfo kF64{52, 11, -1023};
constexpr FloatInfo kF32{23, 8, -127};

// Round (hi:lo) * 2^E (+ a nonzero tail below it when sticky) to the format: returns the IEEE bit
// pattern (sign not set) and sets *ovf when it rounds past the largest finite value.
VN_HD uint64_t round_bits(uint64_t hi, uint64_t lo, bool sticky, int E, const FloatInfo& f, bool* ovf) {
  *ovf = false;
  if (!hi && !lo) return 0;
  const int L = hi ? 127 - clz64(hi) : 63 - clz64(lo);  // msb position
  const int p = f.mantbits + 1;
  const int emin = f.bias + 1;                          // exponent of the smallest normal
  int lsb = L + E - (p - 1);
  if (lsb < emin - (p - 1)) lsb = emin - (p - 1);
  const int shift = lsb - E;
  uint64_t mant;
  if (shift <= 0) {  // exact: at most p bits, shifted up
    mant = lo << -shift;  // L < p here, so the value sits in lo
  } else {
    // mant = Q >> shift, rest = Q mod 2^shift compared with half = 2^(shift-1)
    uint64_t m, rhi, rlo;  // m: quotient; (rhi:rlo): remainder bits
    if (shift >= 128) {
      m = 0; rhi = hi; rlo = lo;
    } else if (shift >= 64) {
      m = hi >> (shift - 64);
      rhi = shift == 64 ? 0 : hi & ((1ull << (shift - 64)) - 1);
      rlo = lo;
    } else {
      m = (lo >> shift) | (hi << (64 - shift));
      rhi = 0;
      rlo = lo & ((1ull << shift) - 1);
    }
    // compare remainder with half
    int cmp;  // -1 below half, 0 exactly half, 1 above
    if (shift > 128) {
      cmp = -1;  // remainder < 2^128 <= half
    } else {
      const int hb = shift - 1;  // half = 2^hb
      uint64_t hh = hb >= 64 ? 1ull << (hb - 64) : 0, hl = hb >= 64 ? 0 : 1ull << hb;
      if (rhi != hh) cmp = rhi > hh ? 1 : -1;
      else if (rlo != hl) cmp = rlo > hl ? 1 : -1;
      else cmp = 0;
    }
    const bool up = cmp > 0 || (cmp == 0 && (sticky || (m & 1)));
    mant = m + (up ? 1 : 0);
    if (mant >> p) {  // carried into a new bit
      mant >>= 1;
      lsb += 1;
    }
  }
  if (mant == 0) return 0;
  const int emax_field = (1 << f.expbits) - 1;
  uint64_t expf;
  if (mant >> (p - 1)) {
    expf = (uint64_t)(lsb + (p - 1) - f.bias);
    if ((int)expf >= emax_field) {
      *ovf = true;
      return (uint64_t)emax_field << f.mantbits;
    }
  } else {
    expf = 0;  // subnormal
  }
  return (expf << f.mantbits) | (mant & ((1ull << f.mantbits) - 1));
}

// ---- Go decimal.go restated: an 800-digit decimal, value = 0.d[0]d[1]... * 10^dp
constexpr int kDecDigits = 800;
struct Decimal {
  uint8_t d[kDecDigits];  // digit values 0..9
  int nd, dp;
  bool neg, trunc;
};

VN_HD void dec_trim(Decimal* a) {
  while (a->nd > 0 && a->d[a->nd - 1] == 0) a->nd--;
  if (a->nd == 0) a->dp = 0;
}

VN_HD void dec_right_shift(Decimal* a, unsigned k) {  // k <= 60
  int r = 0, w = 0;
  uint64_t n = 0;
  for (; (n >> k) == 0; r++) {
    if (r >= a->nd) {
      if (n == 0) {
        a->nd = 0;
        return;
      }
      while ((n >> k) == 0) {
        n = n * 10;
        r++;
      }
      break;
    }
    n = n * 10 + a->d[r];
  }
  a->dp -= r - 1;
  const uint64_t mask = (1ull << k) - 1;
  for (; r < a->nd; r++) {
    const uint64_t c = a->d[r];
    const uint64_t dig = n >> k;
    n &= mask;
    a->d[w++] = (uint8_t)dig;
    n = n * 10 + c;
  }
  while (n > 0) {
    const uint64_t dig = n >> k;
    n &= mask;
    if (w < kDecDigits) a->d[w++] = (uint8_t)dig;
    else if (dig > 0) a->trunc = true;
    n = n * 10;
  }
  a->nd = w;
  dec_trim(a);
}

// multiply by 2^k (k <= 60): digits from the right, carries out the left end
VN_HD void dec_left_shift(Decimal* a, unsigned k) {
  // pass 1: the final carry out of the left end -> count of new leading digits
  uint64_t n = 0;
  int extra = 0;
  for (int r = a->nd - 1; r >= 0; r--) {
    n = ((uint64_t)a->d[r] << k) + n;
    n /= 10;
  }
  for (uint64_t t = n; t > 0; t /= 10) extra++;
  // pass 2: write the digits right to left into their shifted positions
  const int total = a->nd + extra;
  n = 0;
  int w = total - 1;
  for (int r = a->nd - 1; r >= 0; r--, w--) {
    n = ((uint64_t)a->d[r] << k) + n;
    const uint8_t dig = (uint8_t)(n % 10);
    n /= 10;
    if (w < kDecDigits) a->d[w] = dig;
    else if (dig != 0) a->trunc = true;
  }
  for (; w >= 0; w--) {
    const uint8_t dig = (uint8_t)(n % 10);
    n /= 10;
    if (w < kDecDigits) a->d[w] = dig;
    else if (dig != 0) a->trunc = true;
  }
  a->nd = total < kDecDigits ? total : kDecDigits;
  a->dp += extra;
  dec_trim(a);
}

VN_HD void dec_shift(Decimal* a, int k) {
  constexpr int kMaxShift = 60;
  if (a->nd == 0) return;
  if (k > 0) {
    while (k > kMaxShift) { dec_left_shift(a, kMaxShift); k -= kMaxShift; }
    dec_left_shift(a, (unsigned)k);
  } else if (k < 0) {
    while (k < -kMaxShift) { dec_right_shift(a, kMaxShift); k += kMaxShift; }
    dec_right_shift(a, (unsigned)-k);
  }
}

VN_HD bool dec_should_round_up(const Decimal* a, int nd) {
  if (nd < 0 || nd >= a->nd) return false;
  if (a->d[nd] == 5 && nd + 1 == a->nd) {  // exactly halfway: round to even
    if (a->trunc) return true;
    return nd > 0 && (a->d[nd - 1] % 2) == 1;
  }
  return a->d[nd] >= 5;
}

VN_HD uint64_t dec_rounded_integer(const Decimal* a) {
  if (a->dp > 20) return 0xFFFFFFFFFFFFFFFFull;
  int i;
  uint64_t n = 0;
  for (i = 0; i < a->dp && i < a->nd; i++) n = n * 10 + a->d[i];
  for (; i < a->dp; i++) n *= 10;
  if (dec_should_round_up(a, a->dp)) n++;
  return n;
}

// decimal.floatBits: returns the IEEE bits with the sign; *ovf on overflow
VN_HD uint64_t dec_float_bits(Decimal* d, const FloatInfo& flt, bool* ovf) {
  const int powtab[9] = {1, 3, 6, 9, 13, 16, 19, 23, 26};
  int exp = 0;
  uint64_t mant = 0;
  *ovf = false;
  if (d->nd == 0) {
    mant = 0;
    exp = flt.bias;
    goto out;
  }
  if (d->dp > 310) goto overflow;
  if (d->dp < -330) {
    mant = 0;
    exp = flt.bias;
    goto out;
  }
  exp = 0;
  while (d->dp > 0) {
    const int n = d->dp >= 9 ? 27 : powtab[d->dp];
    dec_shift(d, -n);
    exp += n;
  }
  while (d->dp < 0 || (d->dp == 0 && d->d[0] < 5)) {
    const int n = -d->dp >= 9 ? 27 : powtab[-d->dp];
    dec_shift(d, n);
    exp -= n;
  }
  exp--;  // [0.5, 1) -> [1, 2)
  if (exp < flt.bias + 1) {
    const int n = flt.bias + 1 - exp;
    dec_shift(d, -n);
    exp += n;
  }
  if (exp - flt.bias >= (1 << flt.expbits) - 1) goto overflow;
  dec_shift(d, 1 + flt.mantbits);
  mant = dec_rounded_integer(d);
  if (mant == (2ull << flt.mantbits)) {
    mant >>= 1;
    exp++;
    if (exp - flt.bias >= (1 << flt.expbits) - 1) goto overflow;
  }
  if ((mant & (1ull << flt.mantbits)) == 0) exp = flt.bias;  // denormal
  goto out;
overflow:
  mant = 0;
  exp = (1 << flt.expbits) - 1 + flt.bias;
  *ovf = true;
out: {
  uint64_t bits = mant & ((1ull << flt.mantbits) - 1);
  bits |= (uint64_t)((exp - flt.bias) & ((1 << flt.expbits) - 1)) << flt.mantbits;
  if (d->neg) bits |= 1ull << flt.mantbits << flt.expbits;
  return bits;
}
}

// ---- ParseFloat
enum { kOk = 0, kSyntax = 1, kRange = 2, kDefer = 3 };

// Parses s[0, n) as Go 1.9 ParseFloat(s, bits) does; *out gets the value (as a double; for
// bits == 32 the float32 value widened).  scratch: a Decimal for the slow path, or null: then a
// number that needs it returns kDefer (syntax is checked first: kDefer means well-formed).
VN_HD int parse_float(const char* s, uint32_t n, int bits, double* out, Decimal* scratch) {
  // special(): [+-]inf, [+-]infinity, nan
  if (n) {
    const char c = s[0];
    if (c == '+' || c == '-') {
      if (ieq(s + 1, n - 1, "inf", 3) || ieq(s + 1, n - 1, "infinity", 8)) {
        *out = c == '-' ? -__builtin_huge_val() : __builtin_huge_val();
        return kOk;
      }
    } else if (c == 'n' || c == 'N') {
      if (ieq(s, n, "nan", 3)) {
        *out = __builtin_nan("");
        return kOk;
      }
    } else if (c == 'i' || c == 'I') {
      if (ieq(s, n, "inf", 3) || ieq(s, n, "infinity", 8)) {
        *out = __builtin_huge_val();
        return kOk;
      }
    }
  }
  // readFloat: mantissa (19 significant digits), decimal point, exponent
  uint32_t i = 0;
  bool neg = false;
  if (i < n && (s[i] == '+' || s[i] == '-')) {
    neg = s[i] == '-';
    i++;
  }
  bool sawdot = false, sawdigits = false, trunc = false;
  int nd = 0, ndm = 0, dp = 0;
  uint64_t mant = 0;
  const uint32_t digits_start = i;
  for (; i < n; i++) {
    const char c = s[i];
    if (c == '.') {
      if (sawdot) return kSyntax;
      sawdot = true;
      dp = nd;
      continue;
    }
    if (c >= '0' && c <= '9') {
      sawdigits = true;
      if (c == '0' && nd == 0) {  // leading zeros
        dp--;
        continue;
      }
      nd++;
      if (ndm < 19) {
        mant = mant * 10 + (uint64_t)(c - '0');
        ndm++;
      } else if (c != '0') {
        trunc = true;
      }
      continue;
    }
    break;
  }
  if (!sawdigits) return kSyntax;
  if (!sawdot) dp = nd;
  const uint32_t digits_end = i;
  int esum = 0;
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    i++;
    if (i >= n) return kSyntax;
    int esign = 1;
    if (s[i] == '+') i++;
    else if (s[i] == '-') { i++; esign = -1; }
    if (i >= n || s[i] < '0' || s[i] > '9') return kSyntax;
    int e = 0;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; i++)
      if (e < 10000) e = e * 10 + (s[i] - '0');
    esum = e * esign;
  }
  if (i != n) return kSyntax;
  dp += esum;
  const FloatInfo& f = bits == 32 ? kF32 : kF64;
  uint64_t b;  // IEEE bits of the magnitude (the sign is applied at the end)
  bool ovf = false;
  if (mant == 0) {  // every digit zero
    b = 0;
  } else {
    const int e10 = dp - ndm;  // value = mant * 10^e10 (+ a nonzero tail when trunc)
    bool done = false;
    if (!trunc) {
      // 1. atof64exact / atof32exact
      const double pow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
      if (bits == 64 && (mant >> 52) == 0) {
        double v = (double)mant;
        if (e10 == 0) { b = bits_of(v); done = true; }
        else if (e10 > 0 && e10 <= 15 + 22) {
          int e = e10;
          if (e > 22) { v *= pow10[e - 22]; e = 22; }
          if (!(v > 1e15)) { b = bits_of(v * pow10[e]); done = true; }
        } else if (e10 < 0 && e10 >= -22) {
          b = bits_of(v / pow10[-e10]);
          done = true;
        }
      } else if (bits == 32 && (mant >> 23) == 0) {
        // float32 arithmetic emulated in binary64: one rounding to 53 bits then to 24 bits is
        // the correctly rounded float32 for a single *, / (53 >= 2*24 + 2)
        double v = (double)mant;  // exact
        if (e10 == 0) { b = (uint64_t)__builtin_bit_cast(uint32_t, (float)v); done = true; }
        else if (e10 > 0 && e10 <= 7 + 10) {
          int e = e10;
          if (e > 10) { v = (double)(float)(v * pow10[e - 10]); e = 10; }  // exact: v*10^k < 2^24 checked next
          if (!(v > 1e7)) { b = (uint64_t)__builtin_bit_cast(uint32_t, (float)(v * pow10[e])); done = true; }
        } else if (e10 < 0 && e10 >= -10) {
          b = (uint64_t)__builtin_bit_cast(uint32_t, (float)(v / pow10[-e10]));
          done = true;
        }
      }
      // 2. exact 128-bit integer arithmetic
      if (!done && e10 >= 0 && e10 <= 19) {
        uint64_t p10 = 1;
        for (int k = 0; k < e10; k++) p10 *= 10;
        uint64_t hi, lo;
        mul64(mant, p10, &hi, &lo);
        b = round_bits(hi, lo, false, 0, f, &ovf);
        done = true;
      } else if (!done && e10 < 0 && e10 >= -27) {
        const int k = -e10;
        uint64_t p5 = 1;
        for (int j = 0; j < k; j++) p5 *= 5;  // < 2^63
        const int c = clz64(mant);
        const uint64_t m = mant << c;         // >= 2^63 > p5
        // (m : 0) / p5: high quotient word, then 64 bits of long division of the remainder
        const uint64_t qh = m / p5;
        uint64_t r = m % p5, ql = 0;
        for (int j = 63; j >= 0; j--) {
          r <<= 1;  // r < p5 < 2^63: no overflow
          if (r >= p5) {
            r -= p5;
            ql |= 1ull << j;
          }
        }
        b = round_bits(qh, ql, r != 0, -64 - c - k, f, &ovf);
        done = true;
      }
    }
    if (!done && !scratch) return kDefer;
    if (!done) {
      // 3. decimal.go: re-read the digits into an 800-digit decimal (decimal.set)
      Decimal* d = scratch;
      d->nd = 0;
      d->dp = 0;
      d->neg = false;
      d->trunc = false;
      bool sd = false;
      for (uint32_t j = digits_start; j < digits_end; j++) {
        const char c = s[j];
        if (c == '.') {
          sd = true;
          d->dp = d->nd;
          continue;
        }
        if (c == '0' && d->nd == 0) {
          d->dp--;
          continue;
        }
        if (d->nd < kDecDigits) d->d[d->nd++] = (uint8_t)(c - '0');
        else if (c != '0') d->trunc = true;
      }
      if (!sd) d->dp = d->nd;
      d->dp += esum;
      b = dec_float_bits(d, f, &ovf);
    }
  }
  if (ovf) return kRange;
  if (bits == 32) {
    const float v = f32_from_bits((uint32_t)b);
    *out = neg ? -(double)v : (double)v;
  } else {
    const double v = from_bits(b);
    *out = neg ? -v : v;
  }
  return kOk;
}

#undef VN_HD

}  // namespace gofloat
}  // namespace vn

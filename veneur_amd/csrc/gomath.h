// gomath.h -- device/host restatement of the Go 1.9 arithmetic the sketch path
// depends on bit-for-bit: math.Log (src/math/log.go; log_amd64.s evaluates the same
// expression tree), math.Pow's integer-exponent branch (src/math/pow.go), math.Asin
// (asin.go + atan.go, Cephes) for tdigest.indexEstimate (merging_digest.go:240-243),
// and Go's amd64 float->int conversions.
//
// Every floating-point operation is an explicit round-to-nearest intrinsic, so no
// multiply-add contraction can change a result whatever the -ffp-contract setting.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VN_HD __host__ __device__ __forceinline__

namespace vn {

#if defined(__HIP_DEVICE_COMPILE__)
VN_HD double dadd(double a, double b) { return __dadd_rn(a, b); }
VN_HD double dsub(double a, double b) { return __dsub_rn(a, b); }
VN_HD double dmul(double a, double b) { return __dmul_rn(a, b); }
VN_HD double ddiv(double a, double b) { return __ddiv_rn(a, b); }
VN_HD double dsqrt(double a) { return __dsqrt_rn(a); }
// a / b correctly rounded, as the hardware's division sequence (reciprocal, two Newton steps,
// quotient and residual correction) without v_div_scale and v_div_fixup, which change nothing when
// neither operand needs rescaling and the quotient is neither special nor subnormal (a zero or of
// magnitude within [2^-500, 2^500], b within [2^-300, 2^300]: the arguments of indexEstimate's
// divisions, whose q = P / T is 0 or at least 2^-53 away from every breakpoint)
VN_HD double ddiv_nr(double a, double b) {
  const double r0 = __builtin_amdgcn_rcp(b);
  const double e0 = __builtin_fma(-b, r0, 1.0);
  const double r1 = __builtin_fma(r0, e0, r0);
  const double e1 = __builtin_fma(-b, r1, 1.0);
  const double y = __builtin_fma(r1, e1, r1);
  const double q0 = __dmul_rn(a, y);
  const double rr = __builtin_fma(-b, q0, a);
  return __builtin_fma(rr, y, q0);
}
#else
// host build is compiled with -ffp-contract=off
VN_HD double dadd(double a, double b) { return a + b; }
VN_HD double dsub(double a, double b) { return a - b; }
VN_HD double dmul(double a, double b) { return a * b; }
VN_HD double ddiv(double a, double b) { return a / b; }
VN_HD double dsqrt(double a) { return __builtin_sqrt(a); }
VN_HD double ddiv_nr(double a, double b) { return a / b; }
#endif

VN_HD uint64_t dbits(double x) { return __builtin_bit_cast(uint64_t, x); }
VN_HD double bitsd(uint64_t u) { return __builtin_bit_cast(double, u); }
VN_HD bool d_isnan(double x) { return (dbits(x) & 0x7fffffffffffffffull) > 0x7ff0000000000000ull; }
VN_HD bool d_isinf(double x) { return (dbits(x) & 0x7fffffffffffffffull) == 0x7ff0000000000000ull; }
VN_HD bool d_signbit(double x) { return (dbits(x) >> 63) != 0; }
constexpr double kPi = 3.14159265358979323846264338327950288419716939937510582097494459;
constexpr double kSqrt2 = 1.41421356237309504880168872420969807856967187537694807317667974;
constexpr double kInf = __builtin_huge_val();

// math.Frexp for finite non-zero normal/subnormal x: frac in [0.5, 1).
VN_HD double frexp_go(double x, int* e) {
  uint64_t u = dbits(x);
  int ex = (int)((u >> 52) & 0x7ff);
  if (x == 0 || ex == 0x7ff) { *e = 0; return x; }
  int adj = 0;
  if (ex == 0) {  // subnormal: normalise (math.normalize)
    x = x * 4503599627370496.0;  // 2^52, exact
    u = dbits(x);
    ex = (int)((u >> 52) & 0x7ff);
    adj = -52;
  }
  *e = ex - 1022 + adj;
  u &= ~(0x7ffull << 52);
  u |= 1022ull << 52;
  return bitsd(u);
}

// math.Ldexp restricted to results in the normal range (all the sketch path produces).
VN_HD double ldexp_go(double frac, int e) {
  if (frac == 0 || d_isinf(frac) || d_isnan(frac)) return frac;
  int fe;
  double f = frexp_go(frac, &fe);
  int ex = fe + e;
  if (ex < -1021 || ex > 1024) {  // outside the range the path can reach: fall back to scaling
    double r = f;
    int k = ex - 1;
    while (k > 0) { r = dmul(r, 2.0); k--; }
    while (k < 0) { r = dmul(r, 0.5); k++; }
    return dmul(r, 2.0);
  }
  uint64_t u = dbits(f);
  u &= ~(0x7ffull << 52);
  u |= (uint64_t)(ex + 1022) << 52;
  return bitsd(u);
}

// math.Log (log.go)
VN_HD double log_go(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
               L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
               L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (d_isnan(x) || (d_isinf(x) && x > 0)) return x;
  if (x < 0) return __builtin_nan("");
  if (x == 0) return -kInf;
  int ki;
  double f1 = frexp_go(x, &ki);
  if (f1 < kSqrt2 / 2) { f1 = dmul(f1, 2.0); ki--; }
  double f = dsub(f1, 1.0);
  double k = (double)ki;
  double s = ddiv(f, dadd(2.0, f));
  double s2 = dmul(s, s);
  double s4 = dmul(s2, s2);
  double t1 = dmul(s2, dadd(L1, dmul(s4, dadd(L3, dmul(s4, dadd(L5, dmul(s4, L7)))))));
  double t2 = dmul(s4, dadd(L2, dmul(s4, dadd(L4, dmul(s4, L6)))));
  double R = dadd(t1, t2);
  double hfsq = dmul(dmul(0.5, f), f);
  return dsub(dmul(k, Ln2Hi), dsub(dsub(hfsq, dadd(dmul(s, dadd(hfsq, R)), dmul(k, Ln2Lo))), f));
}

// math.Pow(x, y) for finite x > 0 (or x == 0) and small non-negative integer y:
// the repeated-squaring branch of pow.go over Frexp's mantissa, then Ldexp.
VN_HD double powi_go(double x, int y) {
  if (y == 0 || x == 1) return 1;
  if (y == 1) return x;
  if (x == 0) return (y & 1) ? x : 0.0;
  double a1 = 1.0;
  int ae = 0;
  int xe;
  double x1 = frexp_go(x, &xe);
  for (int64_t i = y; i != 0; i >>= 1) {
    if (xe < -(1 << 12) || (1 << 12) < xe) { ae += xe; break; }
    if (i & 1) { a1 = dmul(a1, x1); ae += xe; }
    x1 = dmul(x1, x1);
    xe <<= 1;
    if (x1 < .5) { x1 = dadd(x1, x1); xe--; }
  }
  return ldexp_go(a1, ae);
}

// math.Asin (asin.go) with satan/xatan (atan.go)
VN_HD double xatan_go(double x) {
  const double P0 = -8.750608600031904122785e-01, P1 = -1.615753718733365076637e+01,
               P2 = -7.500855792314704667340e+01, P3 = -1.228866684490136173410e+02,
               P4 = -6.485021904942025371773e+01, Q0 = +2.485846490142306297962e+01,
               Q1 = +1.650270098316988542046e+02, Q2 = +4.328810604912902668951e+02,
               Q3 = +4.853903996359136964868e+02, Q4 = +1.945506571482613964425e+02;
  double z = dmul(x, x);
  double num = dadd(dmul(dadd(dmul(dadd(dmul(dadd(dmul(P0, z), P1), z), P2), z), P3), z), P4);
  double den = dadd(dmul(dadd(dmul(dadd(dmul(dadd(dmul(dadd(z, Q0), z), Q1), z), Q2), z), Q3), z), Q4);
  z = ddiv(dmul(z, num), den);
  return dadd(dmul(x, z), x);
}
VN_HD double satan_go(double x) {
  const double Morebits = 6.123233995736765886130e-17, Tan3pio8 = 2.41421356237309504880;
  if (x <= 0.66) return xatan_go(x);
  if (x > Tan3pio8) return dadd(dsub(kPi / 2, xatan_go(ddiv(1.0, x))), Morebits);
  return dadd(dadd(kPi / 4, xatan_go(ddiv(dsub(x, 1.0), dadd(x, 1.0)))), dmul(0.5, Morebits));
}
VN_HD double asin_go(double x) {
  if (x == 0) return x;
  bool sign = false;
  if (x < 0) { x = -x; sign = true; }
  if (x > 1) return __builtin_nan("");
  double temp = dsqrt(dsub(1.0, dmul(x, x)));
  if (x > 0.7) temp = dsub(kPi / 2, satan_go(ddiv(temp, x)));
  else temp = satan_go(ddiv(x, temp));
  return sign ? -temp : temp;
}

// The same function with every branch turned into a select, for wave-wide evaluation: each
// of asin's two and satan's three paths is one division feeding one xatan, so the paths
// share that code (x / 1.0 == x exactly) and a wave no longer runs each path in turn.
// Bit-identical to asin_go for every input in [-1, 1] (checked against the oracle).
#ifndef VN_INDEX_NR
#define VN_INDEX_NR false  // (build knob: true evaluates indexEstimate with ddiv_nr -- not kept)
#endif
template <bool NR = VN_INDEX_NR>  // NR: the divisions as ddiv_nr (indexEstimate's argument range); false: ddiv
VN_HD double asin_go_sel(double x) {
  const double Morebits = 6.123233995736765886130e-17, Tan3pio8 = 2.41421356237309504880;
  const double ax = x < 0 ? -x : x;
  const double temp = dsqrt(dsub(1.0, dmul(ax, ax)));
  const bool hi = ax > 0.7;
  const double y = NR ? ddiv_nr(hi ? temp : ax, hi ? ax : temp) : ddiv(hi ? temp : ax, hi ? ax : temp);  // (y >= 0)
  const bool s0 = y <= 0.66, s2 = y > Tan3pio8;
  const double an = s0 ? y : (s2 ? 1.0 : dsub(y, 1.0));
  const double ad = s0 ? 1.0 : (s2 ? y : dadd(y, 1.0));
  const double z = xatan_go(NR ? ddiv_nr(an, ad) : ddiv(an, ad));
  const double sat = s0 ? z : (s2 ? dadd(dsub(kPi / 2, z), Morebits) : dadd(dadd(kPi / 4, z), dmul(0.5, Morebits)));
  const double r = hi ? dsub(kPi / 2, sat) : sat;
  if (x == 0) return x;
  if (ax > 1) return __builtin_nan("");
  return x < 0 ? -r : r;
}

// int64(float64) on amd64 (CVTTSD2SQ): NaN / out of range -> 0x8000000000000000.
VN_HD int64_t f64_to_i64_go(double x) {
  if (d_isnan(x) || x >= 9.223372036854775808e18 || x <= -9.223372036854775808e18)
    return (int64_t)0x8000000000000000ull;
  return (int64_t)x;
}
VN_HD uint64_t f64_to_u64_go(double x) {
  if (x < 9.223372036854775808e18) return (uint64_t)f64_to_i64_go(x);
  return (uint64_t)f64_to_i64_go(dsub(x, 9.223372036854775808e18)) ^ 0x8000000000000000ull;
}

// math.Min / math.Max for non-NaN inputs: Min(-0,+0) = -0, Max(-0,+0) = +0.
VN_HD double min_go(double a, double b) {
  if (a == b) return d_signbit(a) ? a : b;
  return a < b ? a : b;
}
VN_HD double max_go(double a, double b) {
  if (a == b) return d_signbit(a) ? b : a;
  return a > b ? a : b;
}

// Order-preserving map of a non-NaN float64 onto uint64 (-0 sorts before +0).
VN_HD uint64_t ordered_bits(double x) {
  uint64_t u = dbits(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
VN_HD double from_ordered_bits(uint64_t k) {
  return bitsd((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k);
}

// tdigest indexEstimate (merging_digest.go:240-243): compression * (asin(2q-1)/pi + 0.5)
// indexEstimate (merging_digest.go:240-243) for q in [0, 1]; NR as asin_go_sel
template <bool NR = VN_INDEX_NR>
VN_HD double index_estimate(double compression, double q) {
  const double a = asin_go_sel<NR>(dsub(dmul(2.0, q), 1.0));
  return dmul(compression, dadd(NR ? ddiv_nr(a, kPi) : ddiv(a, kPi), 0.5));
}

}  // namespace vn

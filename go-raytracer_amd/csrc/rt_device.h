// rt_device.h -- device-side FP64 arithmetic of the render path (gfx950).
//
// Every operation follows the reference's Go op order with one rounding per
// operation (the library is compiled with -ffp-contract=off; Go on amd64
// fuses no multiply-adds), so the kernel reproduces the reference's pixels
// bit for bit. References are to timdestan/go-raytracer.
#pragma once
#pragma clang fp contract(off)

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

namespace rt {

struct d3 {
  double x, y, z;
};

__device__ __forceinline__ d3 mk(double x, double y, double z) { return d3{x, y, z}; }
__device__ __forceinline__ d3 add(d3 a, d3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }    // vec.go:23
__device__ __forceinline__ d3 sub(d3 a, d3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }    // vec.go:31
__device__ __forceinline__ d3 mul(d3 a, d3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }    // vec.go:40
__device__ __forceinline__ double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   // vec.go:48
__device__ __forceinline__ d3 scale(d3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }    // vec.go:70
// math.Sqrt (correctly rounded). hipcc expands an FP64 sqrt on gfx950 to
//   scale = x < 2^-767; x' = ldexp(x, scale ? 256 : 0); y = rsq(x');
//   g = x'y; h = y/2; r = fma(-h, g, 1/2); g = fma(g, r, g); h = fma(h, r, h);
//   2x { d = fma(-g, g, x'); g = fma(d, h, g) };  g = ldexp(g, scale ? -128 : 0);
//   result = class(x', +-0 | +inf) ? x' : g
// For 2^-767 <= x < inf the scaling steps are the identity and the class
// test is false, so the core below gives the same bits in 10 instead of 18
// VALU instructions.
#ifndef RT_FAST_SQRT
// 2: per-lane fix-up form (default; -2.6 % VALU, C3 -0.2..-1.2 %). 1:
// wave-uniform form (more scalar branch work, no faster). 0: full sequence.
#define RT_FAST_SQRT 2
#endif
__device__ __forceinline__ double sqrt_core(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}
// True when c holds on every active lane (compare mask == exec: no VALU
// beyond the compares).
__device__ __forceinline__ bool wave_all(bool c) {
  return __builtin_amdgcn_ballot_w64(c) == __builtin_amdgcn_read_exec();
}
__device__ __forceinline__ double gsqrt(double x) {
#if RT_FAST_SQRT == 2
  // every lane takes the core; lanes outside the range redo the full sequence
  double g = sqrt_core(x);
  if (__builtin_expect((uint32_t)__double2hiint(x) - 0x10000000u >= 0x6ff00000u, 0)) g = __builtin_sqrt(x);
  return g;
#elif RT_FAST_SQRT
  // 2^-767 <= x < inf  <=>  high word in [0x10000000, 0x7ff00000) (sign clear; one compare)
  if (wave_all((uint32_t)__double2hiint(x) - 0x10000000u < 0x6ff00000u)) return sqrt_core(x);
#endif
  return __builtin_sqrt(x);
}
__device__ __forceinline__ double len(d3 v) { return gsqrt(v.x * v.x + v.y * v.y + v.z * v.z); }  // vec.go:95
// Shared-denominator division, bit-identical to `/`. hipcc lowers an FP64
// division on gfx950 to
//   d' = div_scale(d); y = rcp(d'); 2x { e = fma(-d', y, 1); y = fma(y, e, y) }
//   n' = div_scale(n); q = n' * y; r = fma(-d', q, n'); div_fmas(r, y, q); div_fixup
// div_scale rescales by a power of two only to keep y, q and the residual r
// out of the subnormal range, div_fmas undoes it, and div_fixup handles zero /
// inf / NaN operands. For d in [2^-100, 2^100) and n = +-0 or |n| >= 2^-800,
// y, q = n*y and r (zero, or a multiple of ulp(d)*ulp(q) >= 2^-904) are all
// normal or zero, so the unscaled sequence rounds exactly as the scaled one
// (round-to-nearest commutes with power-of-two scaling in the normal range),
// and the reciprocal depends on d alone: the three quotients of a
// normalisation share it. A zero numerator gives r = +0 and a +0 quotient
// where div_fixup returns the numerator's sign: copysign restores it.
__device__ __forceinline__ double rcp_refined(double d) {
  double y = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-d, y, 1.0);
  return __builtin_fma(y, e, y);
}
__device__ __forceinline__ double div_rcp(double n, double d, double y) {
  const double q = n * y;
  return __builtin_copysign(__builtin_fma(__builtin_fma(-d, q, n), y, q), n);
}
__device__ __forceinline__ uint64_t num_ok(double n) {
  return __builtin_amdgcn_ballot_w64(__builtin_fabs(n) >= 0x1p-800) | __builtin_amdgcn_ballot_w64(n == 0.0);
}
#ifndef RT_FAST_NORM
// 2: per-lane fix-up form (default; C3 -2.3 % wave cycles). 1: wave-uniform
// form (more scalar branch work). 0: hardware divisions.
#define RT_FAST_NORM 2
#endif
#if RT_FAST_NORM == 2
// The branch-free half of norm_len: core sqrt and shared-reciprocal quotients,
// ok = false where a lane must redo them with the hardware sequences
// (norm_len_fix), so that several normalisations can share one fix-up branch.
__device__ __forceinline__ d3 norm_len_core(d3 v, double& m, bool& ok) {
  const double x = v.x * v.x + v.y * v.y + v.z * v.z;
  m = sqrt_core(x);
  const double y = rcp_refined(m);
  const int en = min(min(__builtin_amdgcn_frexp_exp(v.x), __builtin_amdgcn_frexp_exp(v.y)),
                     __builtin_amdgcn_frexp_exp(v.z));
  ok = ((uint32_t)__double2hiint(x) - 0x33700000u < 0x18E00000u) & (en > -800);
  return mk(div_rcp(v.x, m, y), div_rcp(v.y, m, y), div_rcp(v.z, m, y));
}
__device__ __forceinline__ d3 norm_len_fix(d3 v, double& m) {
  m = __builtin_sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
  return mk(v.x / m, v.y / m, v.z / m);
}
#endif
// norm(v) that also hands back |v| (the same bits as len(v)).
__device__ __forceinline__ d3 norm_len(d3 v, double& m) {                                        // vec.go:78,95
#if RT_FAST_NORM == 2
  // Every lane takes the core square root and the shared-reciprocal
  // quotients; lanes outside their ranges redo both with the full hardware
  // sequences under one (rarely entered) branch. x = m^2 in [2^-200, 2^198)
  // puts x in the core sqrt range and m in [2^-100, 2^100) (sqrt is
  // correctly rounded and monotone; 2^198 keeps a round-up to 2^100 out).
  // Numerators: +-0 or |n| >= 2^-800 <=> frexp exponent >= -799 (a zero's
  // exponent is 0, a denormal's < -1021; inf/NaN components fail on x).
  bool ok;
  d3 r = norm_len_core(v, m, ok);
  if (__builtin_expect(!ok, 0)) r = norm_len_fix(v, m);
  return r;
#else
  m = gsqrt(v.x * v.x + v.y * v.y + v.z * v.z);
#endif
#if RT_FAST_NORM == 1
  // d in [2^-100, 2^100): high word in [0x39B00000, 0x46300000) (one compare)
  const uint64_t ok = __builtin_amdgcn_ballot_w64((uint32_t)__double2hiint(m) - 0x39B00000u < 0x0C800000u) &
                      num_ok(v.x) & num_ok(v.y) & num_ok(v.z);
  if (ok == __builtin_amdgcn_read_exec()) {
    const double y = rcp_refined(m);
    return mk(div_rcp(v.x, m, y), div_rcp(v.y, m, y), div_rcp(v.z, m, y));
  }
#endif
#if RT_FAST_NORM != 2
  return mk(v.x / m, v.y / m, v.z / m);
#endif
}
__device__ __forceinline__ d3 norm(d3 v) {  // vec.go:78
  double m;
  return norm_len(v, m);
}
__device__ __forceinline__ d3 neg(d3 v) { return mk(-v.x, -v.y, -v.z); }                          // vec.go:87
__device__ __forceinline__ d3 lerp(d3 a, d3 b, double t) {                                        // vec.go:56
  return mk(a.x + (b.x - a.x) * t, a.y + (b.y - a.y) * t, a.z + (b.z - a.z) * t);
}
__device__ __forceinline__ bool iszero(d3 v) { return v.x == 0.0 && v.y == 0.0 && v.z == 0.0; }   // vec.go:99

__device__ __forceinline__ bool signbit64(double x) { return (__double_as_longlong(x) >> 63) != 0; }

// math.Max / math.Min (Go dim.go): +-Inf first, then NaN, then signed zeros.
__device__ __forceinline__ double go_max(double x, double y) {
  if (__builtin_isinf(x) && x > 0) return x;
  if (__builtin_isinf(y) && y > 0) return y;
  if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nan("");
  if (x == 0 && x == y) return signbit64(x) ? y : x;
  return x > y ? x : y;
}
__device__ __forceinline__ double go_min(double x, double y) {
  if (__builtin_isinf(x) && x < 0) return x;
  if (__builtin_isinf(y) && y < 0) return y;
  if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nan("");
  if (x == 0 && x == y) return signbit64(x) ? x : y;
  return x < y ? x : y;
}
// The two shapes the path uses, reduced from the rules above with one operand
// constant: Max(0, v) is v when v > 0 or NaN, else +0 (v = -0 gives +0: the
// signed-zero rule returns the +0 operand; -Inf gives +0); Min(Max(v, 0), 1)
// is v in (0, 1), 1 from 1 up to +Inf, +0 at or below 0, NaN for NaN. (A NaN
// result keeps v's payload where Go returns its canonical NaN; no output of
// the path depends on a NaN's payload.)
__device__ __forceinline__ double go_max0(double v) { return (v > 0.0 || v != v) ? v : 0.0; }
__device__ __forceinline__ double clamp01(double x) {                                         // vec.go:218
  return x != x ? x : (x > 0.0 ? (x < 1.0 ? x : 1.0) : 0.0);
}
__device__ __forceinline__ d3 clamp(d3 c) { return mk(clamp01(c.x), clamp01(c.y), clamp01(c.z)); } // vec.go:110

// math.Modf for f >= 0 (Pow only passes Abs(y)).
__device__ __forceinline__ double go_modf_pos(double f, double* frac) {
  if (f < 1) {
    *frac = f;
    return f == 0 ? f : 0.0;
  }
  double ip = __builtin_trunc(f);
  *frac = f - ip;
  return ip;
}

__device__ __forceinline__ bool go_is_odd_int(double x) {
  if (__builtin_fabs(x) >= 9007199254740992.0) return false;
  double xf;
  double xi = (x < 0) ? -go_modf_pos(-x, &xf) : go_modf_pos(x, &xf);
  return xf == 0 && ((long long)xi & 1) == 1;
}

// math.Exp: Go exp.go `exp` + `expmulti` (the portable FreeBSD-derived
// algorithm): k = int(Log2e*x +- 0.5), r = hi - lo with hi = x - k*Ln2Hi,
// lo = k*Ln2Lo, a degree-5 rational for e^r, Ldexp. Op for op the oracle's
// go_exp (oracle/go_math.h), so a fractional Pow is bit-identical on both
// sides. (Go on amd64 runs exp_amd64.s instead, a CPU-dependent FMA/no-FMA
// series: the reference's own fractional Pow is not reproducible across
// CPUs, and no reference fixture exercises it)
__device__ __noinline__ double go_exp(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double Log2e = 1.44269504088896338700e+00;
  const double P1 = 1.66666666666666657415e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  if (__builtin_isnan(x) || x == __builtin_inf()) return x;
  if (x == -__builtin_inf()) return 0;
  if (x > 7.09782712893383973096e+02) return __builtin_inf();
  if (x < -7.45133219101941108420e+02) return 0;
  if (-3.725290298461914e-09 < x && x < 3.725290298461914e-09) return 1 + x;  // |x| < 2^-28
  long long k = 0;
  if (x < 0)
    k = (long long)(Log2e * x - 0.5);
  else if (x > 0)
    k = (long long)(Log2e * x + 0.5);
  const double hi = x - (double)k * Ln2Hi;
  const double lo = (double)k * Ln2Lo;
  const double r = hi - lo;
  const double t = r * r;
  const double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  const double y = 1 - ((lo - (r * c) / (2 - c)) - hi);
  return ldexp(y, (int)k);
}

// math.Log: Go log.go `log` (FreeBSD e_log.c), op for op the oracle's go_log.
__device__ __noinline__ double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (__builtin_isnan(x) || x == __builtin_inf()) return x;
  if (x < 0) return __builtin_nan("");
  if (x == 0) return -__builtin_inf();
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 0.70710678118654752440) {  // Sqrt2/2
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1;
  const double k = (double)ki;
  const double s = f / (2 + f);
  const double s2 = s * s;
  const double s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2;
  const double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

// math.Exp / math.Log as Go runs them on amd64 (exp_amd64.s, log_amd64.s),
// op for op the oracle's go_exp_amd64 / go_log_amd64 (oracle/go_math.h has
// the algorithm notes; recalled from the Go sources, parity unpinned by any
// reference fixture). fma: the AVX2+FMA branch (fused reduction and series).
__device__ __noinline__ double go_exp_amd64(double x, bool fma) {
  const double LOG2E = 1.4426950408889634073599246810018920;
  const double LN2U = 0.69314718055966295651160180568695068359375;
  const double LN2L = 0.28235290563031577122588448175013436025525412068e-12;
  const double T0 = 0.5, T1 = 1.0, T2 = 2.0, T3 = 1.6666666666666666667e-1, T4 = 4.1666666666666666667e-2,
               T5 = 8.3333333333333333333e-3, T6 = 1.3888888888888888889e-3, T7 = 1.9841269841269841270e-4,
               T8 = 2.4801587301587301587e-5;
  const uint64_t bx = (uint64_t)__double_as_longlong(x);
  if ((bx & ~(1ull << 63)) >= 0x7FF0000000000000ull) return bx == 0xFFF0000000000000ull ? 0.0 : x;
  if (x > 7.09782712893384e+02) return __builtin_inf();
  const double t = LOG2E * x;
  const int e = (t > -2147483649.0 && t < 2147483648.0) ? (int)t : (int)0x80000000;  // CVTTSD2SL
  const double fe = (double)e;
  double r, p = T8;
  if (fma) {
    r = __builtin_fma(-fe, LN2U, x);
    r = __builtin_fma(-fe, LN2L, r);
    r = r * 0.0625;
    p = __builtin_fma(r, p, T7);
    p = __builtin_fma(r, p, T6);
    p = __builtin_fma(r, p, T5);
    p = __builtin_fma(r, p, T4);
    p = __builtin_fma(r, p, T3);
    p = __builtin_fma(r, p, T0);
    p = __builtin_fma(r, p, T1);
  } else {
    r = x - LN2U * fe;
    r = r - LN2L * fe;
    r = r * 0.0625;
    p = p * r + T7;
    p = p * r + T6;
    p = p * r + T5;
    p = p * r + T4;
    p = p * r + T3;
    p = p * r + T0;
    p = p * r + T1;
  }
  double y = r * p;
  for (int i = 0; i < 4; i++) y = y * (y + T2);
  y = y + T1;
  int b = e + 0x3FF;
  if (b <= 0) {  // denormal (exp_amd64.s: JLE after the bias add)
    if (b < -52) return 0.0;
    b += 0x3FE;
    y = y * __longlong_as_double((long long)((uint64_t)(uint32_t)b << 52));
    return y * __longlong_as_double((long long)(1ull << 52));
  }
  if ((uint32_t)b > 0x7FFu) return __builtin_inf();
  return y * __longlong_as_double((long long)((uint64_t)(uint32_t)b << 52));
}
__device__ __noinline__ double go_log_amd64(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  const uint64_t bx = (uint64_t)__double_as_longlong(x);
  if ((bx & ~(1ull << 63)) == 0) return -__builtin_inf();
  if ((long long)bx < 0) return __builtin_nan("");
  if (bx >= 0x7FF0000000000000ull) return x;
  double f1 = __longlong_as_double((long long)((bx & 0x000FFFFFFFFFFFFFull) | 0x3FE0000000000000ull));
  double k = (double)((int)((bx >> 52) & 0x7FF) - 0x3FE);
  if (f1 < 0.70710678118654752440) {
    f1 *= 2;
    k -= 1;
  }
  const double f = f1 - 1;
  const double s = f / (2 + f);
  const double s2 = s * s;
  const double s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2;
  const double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}
// RT_EXP_* (include/rt_abi.h): 0 amd64 with FMA, 1 amd64, 2 portable.
__device__ __forceinline__ double go_exp_mode(double x, int mode) {
  return mode == 2 ? go_exp(x) : go_exp_amd64(x, mode == 0);
}
__device__ __forceinline__ double go_log_mode(double x, int mode) { return mode == 2 ? go_log(x) : go_log_amd64(x); }

// math.Pow (Go pow.go): special cases, then Frexp + repeated squaring with
// mantissa renormalisation and a final Ldexp. Integer exponents (the
// reference's specular n and Schlick's 5) are reproduced exactly; the
// fractional part is Exp(yf * Log(x)) of the platform `mode` selects
// (go_exp_mode), restated identically here and in the oracle.
__device__ __noinline__ double go_pow_general(double x, double y, int mode) {
  if (y == 0 || x == 1) return 1;
  if (y == 1) return x;
  if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nan("");
  if (x == 0) {
    if (y < 0) return (signbit64(x) && go_is_odd_int(y)) ? -__builtin_inf() : __builtin_inf();
    if (y > 0) return (signbit64(x) && go_is_odd_int(y)) ? x : 0.0;
  }
  if (__builtin_isinf(y)) {
    if (x == -1) return 1;
    if ((__builtin_fabs(x) < 1) == (y > 0)) return 0;
    return __builtin_inf();
  }
  if (__builtin_isinf(x)) {
    if (x < 0) {  // Pow(1/x, -y) with 1/x = -0
      double nx = -0.0, ny = -y;
      if (ny < 0) return (go_is_odd_int(ny)) ? -__builtin_inf() : __builtin_inf();
      return go_is_odd_int(ny) ? nx : 0.0;
    }
    if (y < 0) return 0;
    if (y > 0) return __builtin_inf();
  }
  if (y == 0.5) return __builtin_sqrt(x);
  if (y == -0.5) return 1 / __builtin_sqrt(x);

  double yf;
  double yi = go_modf_pos(__builtin_fabs(y), &yf);
  if (yf != 0 && x < 0) return __builtin_nan("");
  if (yi >= 9223372036854775808.0) {
    if (x == -1) return 1;
    if ((__builtin_fabs(x) < 1) == (y > 0)) return 0;
    return __builtin_inf();
  }
  double a1 = 1.0;
  int ae = 0;
  if (yf != 0) {
    if (yf > 0.5) {
      yf--;
      yi++;
    }
    a1 = go_exp_mode(yf * go_log_mode(x, mode), mode);
  }
  int xe;
  double x1 = frexp(x, &xe);
  for (long long i = (long long)yi; i != 0; i >>= 1) {
    if (xe < -(1 << 12) || (1 << 12) < xe) {
      ae += xe;
      break;
    }
    if ((i & 1) == 1) {
      a1 *= x1;
      ae += xe;
    }
    x1 *= x1;
    xe <<= 1;
    if (x1 < .5) {
      x1 += x1;
      xe--;
    }
  }
  if (y < 0) {
    a1 = 1 / a1;
    ae = -ae;
  }
  return ldexp(a1, ae);
}

// math.Pow as computeLighting calls it: Pow(max(0, N.H), n) with a finite
// positive base and, in practice, an integer exponent. For 0 < x < inf,
// x != 1 and integer 2 <= y < 2^31 every special case of go_pow_general is
// false, yf == 0 and y > 0, so it reduces to the Frexp / repeated-squaring /
// Ldexp loop below (same ops, same order); x == 0 takes its zero case. The
// general routine (with the exp/log fraction path) stays out of line: inlined
// it doubled the kernel's register spills.
#ifndef RT_POW_DIRECT
#define RT_POW_DIRECT 1  // exact direct binary powering for small integer exponents (see go_pow)
#endif
__device__ __forceinline__ double go_pow(double x, double y, int mode = 2) {
#if RT_POW_DIRECT
  // Integer 2 <= y <= 64 and 2^-15 <= x <= 2^15: every power the loop below
  // forms (x^(2^k) for 2^k <= y, and the partial products, all between x^y and
  // 1) is a normal number, where round-to-nearest commutes with scaling by
  // powers of two. Go's mantissa renormalisation (x1 += x1, xe--) and the final
  // Ldexp therefore only move exponents: the same multiplications on x itself
  // round identically, and the result is a1 (its xe guard cannot trigger:
  // |xe| <= 16 * 64). The square after the last bit is unused in Go, so it is
  // skipped here (it could leave the normal range).
  if (x >= 0x1p-15 && x <= 0x1p15 && y >= 2 && y <= 64 && __builtin_floor(y) == y) {
    double a1 = 1.0, x1 = x;
    for (int i = (int)y;;) {
      if (i & 1) a1 *= x1;
      i >>= 1;
      if (i == 0) break;
      x1 *= x1;
    }
    return a1;
  }
#endif
  if (x > 0 && x < __builtin_inf() && x != 1 && y >= 2 && y < 2147483648.0 && __builtin_floor(y) == y) {
    int xe;
    double x1 = frexp(x, &xe);
    double a1 = 1.0;
    int ae = 0;
    for (int i = (int)y; i != 0; i >>= 1) {
      if (xe < -(1 << 12) || (1 << 12) < xe) {
        ae += xe;
        break;
      }
      if ((i & 1) == 1) {
        a1 *= x1;
        ae += xe;
      }
      x1 *= x1;
      xe <<= 1;
      if (x1 < .5) {
        x1 += x1;
        xe--;
      }
    }
    return ldexp(a1, ae);
  }
  if (x == 0 && y > 0) return (signbit64(x) && go_is_odd_int(y)) ? x : 0.0;
  return go_pow_general(x, y, mode);
}

// go_pow's direct path without branches, for interleaving several powers:
// ok reports whether (x, y) is in that path's domain (then the result equals
// go_pow(x, y) bit for bit), extended to x = +0, where every power is +0 as
// in Go's Pow(+0, y > 0). Squares past the exponent's top bit may leave the
// normal range; they are never multiplied in. RT_SPEC_POWBITS (host: bit
// length of the scene's largest integer exponent) bounds the unrolled steps.
#ifndef RT_SPEC_POWBITS
#define RT_SPEC_POWBITS 7
#endif
__device__ __forceinline__ double pow_small_int(double x, double y, bool& ok) {
  ok = (x == 0.0 || (x >= 0x1p-15 && x <= 0x1p15)) && y >= 2 && y <= (double)((1 << RT_SPEC_POWBITS) - 1) &&
       y <= 64 && __builtin_floor(y) == y && !signbit64(x);
  const int n = ok ? (int)y : 0;
  double a1 = 1.0, x1 = x;
#pragma unroll
  for (int k = 0; k < RT_SPEC_POWBITS; k++) {
    if ((n >> k) & 1) a1 = a1 * x1;
    if (k + 1 < RT_SPEC_POWBITS) x1 = x1 * x1;
  }
  return a1;
}

// math/rand/v2 PCG (pcg.go): 128-bit LCG, DXSM output; Rand.Float64.
struct Pcg {
  uint64_t hi, lo;
};

__device__ __forceinline__ uint64_t pcg_uint64(Pcg& p) {
  const uint64_t mulHi = 2549297995355413924ULL, mulLo = 4865540595714422341ULL;
  const uint64_t incHi = 6364136223846793005ULL, incLo = 1442695040888963407ULL;
  uint64_t lo = p.lo * mulLo;
  uint64_t hi = __umul64hi(p.lo, mulLo);
  hi += p.hi * mulLo + p.lo * mulHi;
  uint64_t lo2 = lo + incLo;
  uint64_t c = lo2 < lo ? 1ULL : 0ULL;
  hi = hi + incHi + c;
  p.lo = lo2;
  p.hi = hi;
  hi ^= hi >> 32;
  hi *= 0xda942042e4dd58b5ULL;
  hi ^= hi >> 48;
  hi *= (lo2 | 1ULL);
  return hi;
}

__device__ __forceinline__ double pcg_float64(Pcg& p) {
  return (double)(pcg_uint64(p) << 11 >> 11) / 9007199254740992.0;
}

// state' = A*state + C (mod 2^128): k LCG steps at once.
__device__ __forceinline__ Pcg pcg_jump(Pcg s, uint64_t ahi, uint64_t alo, uint64_t chi, uint64_t clo) {
  uint64_t lo = alo * s.lo;
  uint64_t hi = __umul64hi(alo, s.lo) + ahi * s.lo + alo * s.hi;
  uint64_t lo2 = lo + clo;
  hi = hi + chi + (lo2 < lo ? 1ULL : 0ULL);
  return Pcg{hi, lo2};
}

// int64(v) for float64 v on amd64 (CVTTSD2SQ): MinInt64 on NaN/overflow.
__device__ __forceinline__ long long go_f2i(double v) {
  if (!(v >= -9223372036854775808.0 && v < 9223372036854775808.0)) return (long long)0x8000000000000000ULL;
  return (long long)v;
}

// math.Sin / math.Cos (Go sin.go, Cephes; |x| < 2^29, larger -> NaN here,
// where Go would use Payne-Hanek: flagged by the caller as unpinned).
__device__ __forceinline__ double go_trig(double x, bool want_cos) {
  const double S0 = 1.58962301576546568060e-10, S1 = -2.50507477628578072866e-8, S2 = 2.75573136213857245213e-6,
               S3 = -1.98412698295895385996e-4, S4 = 8.33333333332211858878e-3, S5 = -1.66666666666666307295e-1;
  const double C0 = -1.13585365213876817300e-11, C1 = 2.08757008419747316778e-9, C2 = -2.75573141792967388112e-7,
               C3 = 2.48015872888517045348e-5, C4 = -1.38888888888730564116e-3, C5 = 4.16666666666665929218e-2;
  const double PI4A = 7.85398125648498535156e-1, PI4B = 3.77489470793079817668e-8, PI4C = 2.69515142907905952645e-15;
  if (__builtin_isnan(x) || __builtin_isinf(x)) return __builtin_nan("");
  if (!want_cos && x == 0) return x;
  bool sign = false;
  if (want_cos) {
    x = __builtin_fabs(x);
  } else if (x < 0) {
    x = -x;
    sign = true;
  }
  if (x >= 536870912.0) return __builtin_nan("");
  unsigned long long j = (unsigned long long)(x * 1.2732395447351628);
  double y = (double)j;
  if (j & 1) {
    j++;
    y++;
  }
  j &= 7;
  double z = ((x - y * PI4A) - y * PI4B) - y * PI4C;
  if (j > 3) {
    j -= 4;
    sign = !sign;
  }
  if (want_cos && j > 1) sign = !sign;
  double zz = z * z;
  bool use_cos_poly = want_cos ? !(j == 1 || j == 2) : (j == 1 || j == 2);
  if (use_cos_poly)
    y = 1.0 - 0.5 * zz + zz * zz * ((((((C0 * zz) + C1) * zz + C2) * zz + C3) * zz + C4) * zz + C5);
  else
    y = z + z * zz * ((((((S0 * zz) + S1) * zz + S2) * zz + S3) * zz + S4) * zz + S5);
  return sign ? -y : y;
}
__device__ __forceinline__ double go_sin(double x) { return go_trig(x, false); }
__device__ __forceinline__ double go_cos(double x) { return go_trig(x, true); }

// math.Atan / Asin / Acos / Atan2 (Go atan.go, asin.go, atan2.go).
__device__ __forceinline__ double go_xatan(double x) {
  const double P0 = -8.750608600031904122785e-01, P1 = -1.615753718733365076637e+01,
               P2 = -7.500855792314704667340e+01, P3 = -1.228866684490136173410e+02,
               P4 = -6.485021904942025371773e+01, Q0 = +2.485846490142306297962e+01,
               Q1 = +1.650270098316988542046e+02, Q2 = +4.328810604912902668951e+02,
               Q3 = +4.853903996359136964868e+02, Q4 = +1.945506571482613964425e+02;
  double z = x * x;
  z = z * ((((P0 * z + P1) * z + P2) * z + P3) * z + P4) / (((((z + Q0) * z + Q1) * z + Q2) * z + Q3) * z + Q4);
  return x * z + x;
}
__device__ __forceinline__ double go_satan(double x) {
  const double Morebits = 6.123233995736765886130e-17, Tan3pio8 = 2.41421356237309504880;
  if (x <= 0.66) return go_xatan(x);
  if (x > Tan3pio8) return 1.5707963267948966 - go_xatan(1 / x) + Morebits;
  return 0.7853981633974483 + go_xatan((x - 1) / (x + 1)) + 0.5 * Morebits;
}
__device__ __forceinline__ double go_acos(double x) {
  double a;  // Asin(x)
  if (x == 0) {
    a = x;
  } else {
    bool sign = x < 0;
    double ax = sign ? -x : x;
    if (ax > 1) return __builtin_nan("");
    double temp = __builtin_sqrt(1 - ax * ax);
    temp = (ax > 0.7) ? 1.5707963267948966 - go_satan(temp / ax) : go_satan(ax / temp);
    a = sign ? -temp : temp;
  }
  return 1.5707963267948966 - a;
}
__device__ __forceinline__ double go_atan2(double y, double x) {
  const double PI = 3.141592653589793;
  if (__builtin_isnan(y) || __builtin_isnan(x)) return __builtin_nan("");
  if (y == 0) {
    if (x >= 0 && !signbit64(x)) return __builtin_copysign(0.0, y);
    return __builtin_copysign(PI, y);
  }
  if (x == 0) return __builtin_copysign(1.5707963267948966, y);
  if (__builtin_isinf(x)) {
    if (x > 0) return __builtin_isinf(y) ? __builtin_copysign(0.7853981633974483, y) : __builtin_copysign(0.0, y);
    return __builtin_isinf(y) ? __builtin_copysign(2.356194490192345, y) : __builtin_copysign(PI, y);
  }
  if (__builtin_isinf(y)) return __builtin_copysign(1.5707963267948966, y);
  double r = y / x;
  double q = (r == 0) ? r : (r > 0 ? go_satan(r) : -go_satan(-r));
  if (x < 0) return q <= 0 ? q + PI : q - PI;
  return q;
}

// uint32(v) for float64 v as Go compiles it on amd64 (CVTTSD2SQ, low 32 bits).
__device__ __forceinline__ uint32_t go_f64_to_u32(double v) {
  if (!(v > -9223372036854775808.0 && v < 9223372036854775808.0)) return 0u;
  return (uint32_t)(uint64_t)(long long)v;
}

}  // namespace rt

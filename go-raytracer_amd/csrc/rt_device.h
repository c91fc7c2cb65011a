// rt_device.h -- device-side FP64 arithmetic of the render path (gfx950).
//
// Every operation follows the reference's Go op order with one rounding per
// operation (the library is compiled with -ffp-contract=off; Go on amd64
// fuses no multiply-adds), so the kernel reproduces the reference's pixels
// bit for bit. References are to timdestan/go-raytracer.
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
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
__device__ __forceinline__ double len(d3 v) { return __builtin_sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }  // vec.go:95
__device__ __forceinline__ d3 norm(d3 v) {                                                        // vec.go:78
  double m = __builtin_sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
  return mk(v.x / m, v.y / m, v.z / m);
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
__device__ __forceinline__ double clamp01(double x) { return go_min(go_max(x, 0.0), 1.0); }      // vec.go:218
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

// math.Pow (Go pow.go): special cases, then Frexp + repeated squaring with
// mantissa renormalisation and a final Ldexp. Integer exponents (the
// reference's specular n and Schlick's 5) are reproduced exactly; the
// fractional part goes through exp/log, whose Go amd64 assembly is not
// restated (parity for fractional specular exponents is unpinned).
__device__ __forceinline__ double go_pow(double x, double y) {
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
    a1 = exp(yf * log(x));
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

// uint32(v) for float64 v as Go compiles it on amd64 (CVTTSD2SQ, low 32 bits).
__device__ __forceinline__ uint32_t go_f64_to_u32(double v) {
  if (!(v > -9223372036854775808.0 && v < 9223372036854775808.0)) return 0u;
  return (uint32_t)(uint64_t)(long long)v;
}

}  // namespace rt

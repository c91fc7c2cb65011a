/*
 * go_math.h -- TEST INFRASTRUCTURE (oracle). Plain-C restatement of the Go
 * standard-library arithmetic the reference's render path calls. Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
 * anything under oracle/.
 *
 * Third-party source (absent from /root/reference): the Go standard library
 * at the reference's `go 1.24.5` directive (go.mod:3). Restated here from the
 * published algorithms:
 *   math.Max / math.Min        (dim.go; amd64 assembly has the same semantics)
 *   math.Pow                   (pow.go: Frexp + repeated squaring, Ldexp)
 *   math.Exp / math.Log        (exp.go, log.go: the portable FreeBSD-derived
 *                               algorithms; used by Pow's fractional part)
 *   math.Tan / math.Sin / Cos  (tan.go, sin.go: Cephes, Cody-Waite reduction)
 *   math/rand/v2 PCG + Float64 (pcg.go: 128-bit LCG, DXSM output;
 *                               rand.go: Float64 = (u<<11>>11) / 2^53)
 *   float64 -> uint32 conversion on amd64 (CVTTSD2SQ then truncate)
 * Compiled with -ffp-contract=off: Go on amd64 (GOAMD64=v1) fuses no
 * multiply-adds.
 */
#ifndef GO_MATH_H
#define GO_MATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint64_t go_f64bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double go_f64frombits(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }
static inline int go_signbit(double x) { return (int)(go_f64bits(x) >> 63); }

/* math.Max (dim.go): +Inf wins, then NaN, then max(+0,-0) = +0. */
static inline double go_max(double x, double y) {
    if (isinf(x) && x > 0) return x;
    if (isinf(y) && y > 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return go_signbit(x) ? y : x;
    return x > y ? x : y;
}

/* math.Min (dim.go): -Inf wins, then NaN, then min(+0,-0) = -0. */
static inline double go_min(double x, double y) {
    if (isinf(x) && x < 0) return x;
    if (isinf(y) && y < 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return go_signbit(x) ? x : y;
    return x < y ? x : y;
}

/* math.Frexp: frac in [0.5,1), normalises subnormals. */
static inline double go_frexp(double f, int *e) {
    *e = 0;
    if (f == 0 || isinf(f) || isnan(f)) return f;
    return frexp(f, e);
}

/* math.Modf for f >= 0 (Pow only calls it on Abs(y)). */
static inline double go_modf(double f, double *frac) {
    double ip;
    if (f < 1) {
        if (f < 0) { double fr; ip = -go_modf(-f, &fr); *frac = -fr; return ip; }
        if (f == 0) { *frac = f; return f; }
        *frac = f; return 0;
    }
    ip = trunc(f);
    *frac = f - ip;
    return ip;
}

static inline int go_is_odd_int(double x) {
    if (fabs(x) >= (double)(1ULL << 53)) return 0;
    double xf;
    double xi = go_modf(x, &xf);
    return xf == 0 && ((int64_t)xi & 1) == 1;
}

/* math.Ldexp: exact scaling with a single rounding for subnormal results --
 * identical to C ldexp for every finite input. */
static inline double go_ldexp(double frac, int e) { return ldexp(frac, e); }

/* math.Exp, Go exp.go `exp` (the portable algorithm): argument reduction
 * x = k*ln2 + r with r = hi - lo, a degree-5 minimax rational for e^r
 * (expmulti), then Ldexp. The same restatement is rt_device.h go_exp, so HIP
 * and oracle agree bit for bit. NOTE: on amd64 Go dispatches Exp to assembly
 * (exp_amd64.s, a different series that uses FMA when the CPU has it), so
 * the reference's own Exp is CPU-dependent; no reference fixture exercises a
 * fractional Pow (parity for it is pinned to this restatement only). */
static inline double go_exp(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01; /* 3fe62e42 fee00000 */
    const double Ln2Lo = 1.90821492927058770002e-10; /* 3dea39ef 35793c76 */
    const double Log2e = 1.44269504088896338700e+00;
    const double Overflow = 7.09782712893383973096e+02;
    const double Underflow = -7.45133219101941108420e+02;
    const double NearZero = 1.0 / (1 << 28);
    const double P1 = 1.66666666666666657415e-01;  /* 3FC55555 55555555 */
    const double P2 = -2.77777777770155933842e-03; /* BF66C16C 16BEBD93 */
    const double P3 = 6.61375632143793436117e-05;  /* 3F11566A AF25DE2C */
    const double P4 = -1.65339022054652515390e-06; /* BEBBBD41 C5D26BF1 */
    const double P5 = 4.13813679705723846039e-08;  /* 3E663769 72BEA4D0 */
    if (isnan(x) || (isinf(x) && x > 0)) return x;
    if (isinf(x)) return 0;
    if (x > Overflow) return INFINITY;
    if (x < Underflow) return 0;
    if (-NearZero < x && x < NearZero) return 1 + x;
    int64_t k = 0;
    if (x < 0) k = (int64_t)(Log2e * x - 0.5);
    else if (x > 0) k = (int64_t)(Log2e * x + 0.5);
    double hi = x - (double)k * Ln2Hi;
    double lo = (double)k * Ln2Lo;
    /* expmulti(hi, lo, k) */
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1 - ((lo - (r * c) / (2 - c)) - hi);
    return ldexp(y, (int)k);
}

/* math.Log, Go log.go `log` (FreeBSD e_log.c): Frexp reduction to
 * f1 in [sqrt(2)/2, sqrt(2)), s = f/(2+f), Remez polynomial in s^2. amd64 Go
 * has log_amd64.s for the same algorithm; restated from log.go. */
static inline double go_log(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01; /* 3fe62e42 fee00000 */
    const double Ln2Lo = 1.90821492927058770002e-10; /* 3dea39ef 35793c76 */
    const double L1 = 6.666666666666735130e-01;      /* 3FE55555 55555593 */
    const double L2 = 3.999999999940941908e-01;      /* 3FD99999 9997FA04 */
    const double L3 = 2.857142874366239149e-01;      /* 3FD24924 94229359 */
    const double L4 = 2.222219843214978396e-01;      /* 3FCC71C5 1D8E78AF */
    const double L5 = 1.818357216161805012e-01;      /* 3FC74664 96CB03DE */
    const double L6 = 1.531383769920937332e-01;      /* 3FC39A09 D078C69F */
    const double L7 = 1.479819860511658591e-01;      /* 3FC2F112 DF3E5244 */
    if (isnan(x) || (isinf(x) && x > 0)) return x;
    if (x < 0) return NAN;
    if (x == 0) return -INFINITY;
    int ki;
    double f1 = go_frexp(x, &ki);
    if (f1 < 0.70710678118654752440 /* Sqrt2/2 */) { f1 *= 2; ki--; }
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

/* math.Exp and math.Log as Go runs them on amd64 (math/exp_asm.go:
 * haveArchExp, haveArchLog), restated from exp_amd64.s / log_amd64.s of the Go
 * release go.mod:3 names (1.24.5). Those sources are not in /root/reference
 * and there is no network: the restatement follows the published algorithm
 * as recalled, and no reference fixture pins it (parity unpinned).
 *
 * exp_amd64.s (N. Shibata's method, from SLEEF): e = int32(trunc(x*log2(e)));
 * r = (x - e*LN2U) - e*LN2L; r /= 16; y = e^r - 1 by a degree-8 Taylor series
 * in Horner form; four doublings y = y*(y + 2) give e^(16r) - 1; + 1; times
 * 2^e built from the exponent bits (two factors below the normal range).
 * With AVX2+FMA (useFMA, i.e. any x86 server CPU of the last decade) the
 * reduction and the series are fused multiply-adds: fma != 0. */
static inline double go_bits_f64(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static inline double go_exp_amd64(double x, int fma_) {
    const double LOG2E = 1.4426950408889634073599246810018920;
    const double LN2U = 0.69314718055966295651160180568695068359375;
    const double LN2L = 0.28235290563031577122588448175013436025525412068e-12;
    const double Overflow = 7.09782712893384e+02;
    /* exprodata: 1/2, 1, 2, 1/3!, 1/4!, ..., 1/8! */
    static const double T[9] = {0.5, 1.0, 2.0, 1.6666666666666666667e-1, 4.1666666666666666667e-2,
                                8.3333333333333333333e-3, 1.3888888888888888889e-3, 1.9841269841269841270e-4,
                                2.4801587301587301587e-5};
    uint64_t bx;
    memcpy(&bx, &x, 8);
    if ((bx & ~(1ull << 63)) >= 0x7FF0000000000000ull)  /* not finite: -Inf -> 0, NaN / +Inf -> x */
        return bx == 0xFFF0000000000000ull ? 0.0 : x;
    if (x > Overflow) return INFINITY;
    const double t = LOG2E * x;
    /* CVTTSD2SL: truncation; out of int32 range -> 0x80000000 */
    const int32_t e = (t > -2147483649.0 && t < 2147483648.0) ? (int32_t)t : INT32_MIN;
    const double fe = (double)e;
    double r, p;
    if (fma_) {
        r = fma(-fe, LN2U, x); /* VFNMADD231SD */
        r = fma(-fe, LN2L, r);
    } else {
        r = x - LN2U * fe;
        r = r - LN2L * fe;
    }
    r = r * 0.0625;
    p = T[8];
    if (fma_) {
        p = fma(r, p, T[7]); /* VFMADD213SD */
        p = fma(r, p, T[6]);
        p = fma(r, p, T[5]);
        p = fma(r, p, T[4]);
        p = fma(r, p, T[3]);
        p = fma(r, p, T[0]);
        p = fma(r, p, T[1]);
    } else {
        p = p * r + T[7];
        p = p * r + T[6];
        p = p * r + T[5];
        p = p * r + T[4];
        p = p * r + T[3];
        p = p * r + T[0];
        p = p * r + T[1];
    }
    double y = r * p;
    for (int i = 0; i < 4; i++) y = y * (y + T[2]);
    y = y + T[1];
    /* return y * 2**e: biased exponent e + 1023 as bits */
    int32_t b = e + 0x3FF;
    if (b <= 0) { /* denormal (exp_amd64.s: JLE after the bias add) */
        if (b < -52) return 0.0;
        b += 0x3FE;
        y = y * go_bits_f64((uint64_t)(uint32_t)b << 52);
        return y * go_bits_f64(1ull << 52);
    }
    if ((uint32_t)b > 0x7FF) return INFINITY;
    return y * go_bits_f64((uint64_t)(uint32_t)b << 52);
}

/* log_amd64.s: log.go's algorithm; Frexp is done on the bits without
 * normalising a subnormal argument (exponent field 0 reads as 2^-1022 times
 * 0.5 + mantissa) -- the only difference from go_log. */
static inline double go_log_amd64(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
    const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
                 L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                 L7 = 1.479819860511658591e-01;
    uint64_t bx;
    memcpy(&bx, &x, 8);
    if ((bx & ~(1ull << 63)) == 0) return -INFINITY;           /* +-0 */
    if ((int64_t)bx < 0) return NAN;                             /* negative (or -NaN) */
    if (bx >= 0x7FF0000000000000ull) return x;                   /* +Inf, NaN */
    double f1 = go_bits_f64((bx & 0x000FFFFFFFFFFFFFull) | 0x3FE0000000000000ull);
    double k = (double)((int)((bx >> 52) & 0x7FF) - 0x3FE);
    if (f1 < 0.70710678118654752440) { f1 *= 2; k -= 1; }
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

/* Which Exp/Log a fractional Pow runs (rt_scene.exp_mode, include/rt_abi.h):
 * 0 = amd64 with FMA (the reference's deployment), 1 = amd64 without FMA,
 * 2 = the portable exp.go / log.go. */
static inline double go_exp_mode(double x, int mode) {
    return mode == 2 ? go_exp(x) : go_exp_amd64(x, mode == 0);
}
static inline double go_log_mode(double x, int mode) { return mode == 2 ? go_log(x) : go_log_amd64(x); }

/* math.Pow (pow.go). Integer exponents (specular n, Schlick 5) run the
 * Frexp/squaring loop; a fractional part goes through Exp(yf*Log(x)) of the
 * platform `mode` selects (go_exp_mode). */
static inline double go_pow_m(double x, double y, int mode) {
    if (y == 0 || x == 1) return 1;
    if (y == 1) return x;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0) {
        if (y < 0) {
            if (go_signbit(x) && go_is_odd_int(y)) return -INFINITY;
            return INFINITY;
        }
        if (y > 0) {
            if (go_signbit(x) && go_is_odd_int(y)) return x;
            return 0;
        }
    }
    if (isinf(y)) {
        if (x == -1) return 1;
        if ((fabs(x) < 1) == (y > 0)) return 0;
        return INFINITY;
    }
    if (isinf(x)) {
        if (x < 0) return go_pow_m(1 / x, -y, mode);
        if (y < 0) return 0;
        if (y > 0) return INFINITY;
    }
    if (y == 0.5) return sqrt(x);
    if (y == -0.5) return 1 / sqrt(x);

    double yf;
    double yi = go_modf(fabs(y), &yf);
    if (yf != 0 && x < 0) return NAN;
    if (yi >= 9223372036854775808.0) {
        if (x == -1) return 1;
        if ((fabs(x) < 1) == (y > 0)) return 0;
        return INFINITY;
    }
    double a1 = 1.0;
    int ae = 0;
    if (yf != 0) {
        if (yf > 0.5) { yf--; yi++; }
        a1 = go_exp_mode(yf * go_log_mode(x, mode), mode);
    }
    int xe;
    double x1 = go_frexp(x, &xe);
    for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
        if (xe < -(1 << 12) || (1 << 12) < xe) {
            ae += xe;
            break;
        }
        if ((i & 1) == 1) { a1 *= x1; ae += xe; }
        x1 *= x1;
        xe <<= 1;
        if (x1 < .5) { x1 += x1; xe--; }
    }
    if (y < 0) { a1 = 1 / a1; ae = -ae; }
    return go_ldexp(a1, ae);
}
static inline double go_pow(double x, double y) { return go_pow_m(x, y, 2); }

/* Cephes coefficients as in Go's sin.go / tan.go. */
static const double go_sin_c[6] = {
    1.58962301576546568060e-10, -2.50507477628578072866e-8,
    2.75573136213857245213e-6,  -1.98412698295895385996e-4,
    8.33333333332211858878e-3,  -1.66666666666666307295e-1,
};
static const double go_cos_c[6] = {
    -1.13585365213876817300e-11, 2.08757008419747316778e-9,
    -2.75573141792967388112e-7,  2.48015872888517045348e-5,
    -1.38888888888730564116e-3,  4.16666666666665929218e-2,
};
static const double go_tanP[3] = {
    -1.30936939181383777646e4, 1.15351664838587416140e6, -1.79565251976484877988e7,
};
static const double go_tanQ[5] = {
    1.0, 1.36812963470692954678e4, -1.32089234440210967447e6,
    2.50083801823357915839e7, -5.38695755929454629881e7,
};
#define GO_PI4A 7.85398125648498535156e-1
#define GO_PI4B 3.77489470793079817668e-8
#define GO_PI4C 2.69515142907905952645e-15
#define GO_4_OVER_PI 1.2732395447351628 /* const 4/Pi rounded once: 0x3ff45f306dc9c883 */
#define GO_REDUCE_THRESHOLD ((double)(1 << 29))

/* Arguments >= 2^29 need Payne-Hanek (trigReduce); the render path only uses
 * fov/2 and fuzz values, far below it. Callers check. */
static inline double go_sin(double x) {
    if (x == 0 || isnan(x)) return x;
    if (isinf(x)) return NAN;
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    uint64_t j = (uint64_t)(x * GO_4_OVER_PI);
    double y = (double)j;
    if ((j & 1) == 1) { j++; y++; }
    j &= 7;
    double z = ((x - y * GO_PI4A) - y * GO_PI4B) - y * GO_PI4C;
    if (j > 3) { sign = !sign; j -= 4; }
    double zz = z * z;
    if (j == 1 || j == 2)
        y = 1.0 - 0.5 * zz + zz * zz * ((((((go_cos_c[0] * zz) + go_cos_c[1]) * zz + go_cos_c[2]) * zz + go_cos_c[3]) * zz + go_cos_c[4]) * zz + go_cos_c[5]);
    else
        y = z + z * zz * ((((((go_sin_c[0] * zz) + go_sin_c[1]) * zz + go_sin_c[2]) * zz + go_sin_c[3]) * zz + go_sin_c[4]) * zz + go_sin_c[5]);
    return sign ? -y : y;
}

static inline double go_cos(double x) {
    if (isnan(x) || isinf(x)) return NAN;
    int sign = 0;
    x = fabs(x);
    uint64_t j = (uint64_t)(x * GO_4_OVER_PI);
    double y = (double)j;
    if ((j & 1) == 1) { j++; y++; }
    j &= 7;
    double z = ((x - y * GO_PI4A) - y * GO_PI4B) - y * GO_PI4C;
    if (j > 3) { j -= 4; sign = !sign; }
    if (j > 1) sign = !sign;
    double zz = z * z;
    if (j == 1 || j == 2)
        y = z + z * zz * ((((((go_sin_c[0] * zz) + go_sin_c[1]) * zz + go_sin_c[2]) * zz + go_sin_c[3]) * zz + go_sin_c[4]) * zz + go_sin_c[5]);
    else
        y = 1.0 - 0.5 * zz + zz * zz * ((((((go_cos_c[0] * zz) + go_cos_c[1]) * zz + go_cos_c[2]) * zz + go_cos_c[3]) * zz + go_cos_c[4]) * zz + go_cos_c[5]);
    return sign ? -y : y;
}

static inline double go_tan(double x) {
    if (x == 0 || isnan(x)) return x;
    if (isinf(x)) return NAN;
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    uint64_t j = (uint64_t)(x * GO_4_OVER_PI);
    double y = (double)j;
    if ((j & 1) == 1) { j++; y++; }
    double z = ((x - y * GO_PI4A) - y * GO_PI4B) - y * GO_PI4C;
    double zz = z * z;
    if (zz > 1e-14)
        y = z + z * (zz * (((go_tanP[0] * zz) + go_tanP[1]) * zz + go_tanP[2]) /
                     ((((zz + go_tanQ[1]) * zz + go_tanQ[2]) * zz + go_tanQ[3]) * zz + go_tanQ[4]));
    else
        y = z;
    if ((j & 2) == 2) y = -1 / y;
    return sign ? -y : y;
}

/* math.Atan / Asin / Acos / Atan2 (atan.go, asin.go, atan2.go): Cephes
 * rational approximation with argument reduction. Used for closure-surface
 * u coordinates (raytracer.go:147, :345). */
#define GO_PI_2 1.5707963267948966  /* const Pi/2 */
#define GO_PI_4 0.7853981633974483  /* const Pi/4 */
static inline double go_xatan(double x) {
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
static inline double go_satan(double x) {
    const double Morebits = 6.123233995736765886130e-17, Tan3pio8 = 2.41421356237309504880;
    if (x <= 0.66) return go_xatan(x);
    if (x > Tan3pio8) return GO_PI_2 - go_xatan(1 / x) + Morebits;
    return GO_PI_4 + go_xatan((x - 1) / (x + 1)) + 0.5 * Morebits;
}
static inline double go_atan(double x) {
    if (x == 0) return x;
    if (x > 0) return go_satan(x);
    return -go_satan(-x);
}
static inline double go_asin(double x) {
    if (x == 0) return x;
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    if (x > 1) return NAN;
    double temp = sqrt(1 - x * x);
    if (x > 0.7) temp = GO_PI_2 - go_satan(temp / x);
    else temp = go_satan(x / temp);
    return sign ? -temp : temp;
}
static inline double go_acos(double x) { return GO_PI_2 - go_asin(x); }
static inline double go_atan2(double y, double x) {
    if (isnan(y) || isnan(x)) return NAN;
    if (y == 0) {
        if (x >= 0 && !go_signbit(x)) return copysign(0, y);
        return copysign(M_PI, y);
    }
    if (x == 0) return copysign(GO_PI_2, y);
    if (isinf(x)) {
        if (x > 0) return isinf(y) ? copysign(GO_PI_4, y) : copysign(0, y);
        return isinf(y) ? copysign(2.356194490192345, y) : copysign(M_PI, y);
    }
    if (isinf(y)) return copysign(GO_PI_2, y);
    double q = go_atan(y / x);
    if (x < 0) {
        if (q <= 0) return q + M_PI;
        return q - M_PI;
    }
    return q;
}

/* math/rand/v2 PCG (pcg.go): state = state*mul + inc mod 2^128; DXSM. */
typedef struct go_pcg { uint64_t hi, lo; } go_pcg;

static inline uint64_t go_pcg_uint64(go_pcg *p) {
    const uint64_t mulHi = 2549297995355413924ULL, mulLo = 4865540595714422341ULL;
    const uint64_t incHi = 6364136223846793005ULL, incLo = 1442695040888963407ULL;
    unsigned __int128 m = (unsigned __int128)p->lo * mulLo;
    uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    hi += p->hi * mulLo + p->lo * mulHi;
    uint64_t lo2 = lo + incLo;
    uint64_t c = lo2 < lo;
    hi = hi + incHi + c;
    p->lo = lo2;
    p->hi = hi;
    hi ^= hi >> 32;
    hi *= 0xda942042e4dd58b5ULL;
    hi ^= hi >> 48;
    hi *= (lo2 | 1);
    return hi;
}

/* rand.go: Float64 = float64(Uint64()<<11>>11) / (1<<53). */
static inline double go_rand_float64(go_pcg *p) {
    return (double)(go_pcg_uint64(p) << 11 >> 11) / 9007199254740992.0;
}

/* uint32(v) for float64 v on amd64: CVTTSD2SQ (int64, "indefinite"
 * 0x8000000000000000 on NaN/overflow), then the low 32 bits. */
static inline uint32_t go_f64_to_u32(double v) {
    if (!(v > -9223372036854775808.0 && v < 9223372036854775808.0)) return 0u;
    return (uint32_t)(uint64_t)(int64_t)v;
}

#endif /* GO_MATH_H */

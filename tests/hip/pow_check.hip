// Device check (test infrastructure): rt_device.h go_exp / go_log / go_pow
// (the kernel's math.Exp, math.Log, math.Pow restatements) in each RT_EXP_*
// mode (amd64 assembly with / without FMA, portable Go) against the
// oracle's host restatements (oracle/go_math.h) bit for bit, on random and
// edge inputs: specular-style bases in (0, 1], wide-range bases, fractional
// and integer exponents, spot-light falloff exponents, specials.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (tests/hip/Makefile)
#include "rt_device.h"
extern "C" {
#include "go_math.h"
}
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// mode: RT_EXP_AMD64_FMA 0 / RT_EXP_AMD64 1 / RT_EXP_PORTABLE 2 (include/rt_abi.h)
__global__ void run(int n, int mode, const double* x, const double* y, double* pw, double* ex, double* lg) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  pw[i] = rt::go_pow(x[i], y[i], mode);
  ex[i] = rt::go_exp_mode(y[i] * (x[i] > 0.5 ? -1.0 : 1.0) * 7.0, mode);
  lg[i] = rt::go_log_mode(x[i], mode);
}

static uint64_t s_state = 0x243F6A8885A308D3ULL;
static uint64_t next() {
  s_state += 0x9E3779B97F4A7C15ULL;
  uint64_t z = s_state;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static double uni() { return (double)(next() >> 11) / 9007199254740992.0; }
static bool same(double a, double b) {
  if (a != a && b != b) return true;
  uint64_t ua, ub;
  memcpy(&ua, &a, 8);
  memcpy(&ub, &b, 8);
  return ua == ub;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : (1 << 22);
  std::vector<double> x(n), y(n);
  const double spec[] = {0.5, 2.5, 7.3, 33.3, 1.5, 0.25, 12.75, 99.99, 3.0, 50.0, 5.0, -2.5, 0.0, 1.0, 64.0, 65.5};
  const double xs[] = {0.0, -0.0, 1.0, 1e-300, 4.9e-324, 0.999999999, 1e300, __builtin_inf(), -2.0, __builtin_nan("")};
  for (int i = 0; i < n; i++) {
    const int m = (int)(next() % 8);
    if (m < 3) {  // specular: base in (0, 1], listed exponents
      x[i] = uni();
      y[i] = spec[next() % 16];
    } else if (m < 5) {  // random fractional exponent up to 200
      x[i] = uni();
      y[i] = uni() * 200.0;
    } else if (m < 6) {  // wide-range base
      x[i] = ldexp(0.5 + uni() * 0.5, (int)(next() % 400) - 200);
      y[i] = (uni() - 0.5) * 40.0;
    } else if (m < 7) {  // bases near 1 (log cancellation), spot falloff style
      x[i] = 1.0 - uni() * 1e-3;
      y[i] = uni() * 10.0;
    } else {  // specials
      x[i] = xs[next() % 10];
      y[i] = spec[next() % 16];
    }
  }
  double *dx, *dy, *dp, *de, *dl;
  const size_t b = sizeof(double) * n;
  if (hipMalloc(&dx, b) || hipMalloc(&dy, b) || hipMalloc(&dp, b) || hipMalloc(&de, b) || hipMalloc(&dl, b)) return 2;
  if (hipMemcpy(dx, x.data(), b, hipMemcpyHostToDevice) || hipMemcpy(dy, y.data(), b, hipMemcpyHostToDevice)) return 2;
  std::vector<double> p(n), e(n), l(n);
  long bad_all = 0;
  printf("{\"cases\": %d, \"modes\": [", n);
  for (int mode = 0; mode < 3; mode++) {
    run<<<(n + 255) / 256, 256>>>(n, mode, dx, dy, dp, de, dl);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    if (hipMemcpy(p.data(), dp, b, hipMemcpyDeviceToHost) || hipMemcpy(e.data(), de, b, hipMemcpyDeviceToHost) ||
        hipMemcpy(l.data(), dl, b, hipMemcpyDeviceToHost))
      return 2;
    long bad_p = 0, bad_e = 0, bad_l = 0, frac = 0;
    for (int i = 0; i < n; i++) {
      double yf;
      go_modf(fabs(y[i]), &yf);
      frac += yf != 0;
      const double want = go_pow_m(x[i], y[i], mode);
      if (!same(p[i], want)) {
        if (bad_p++ < 5) fprintf(stderr, "mode %d pow(%.17g, %.17g): gpu %.17g oracle %.17g\n", mode, x[i], y[i], p[i], want);
      }
      if (!same(e[i], go_exp_mode(y[i] * (x[i] > 0.5 ? -1.0 : 1.0) * 7.0, mode))) bad_e++;
      if (!same(l[i], go_log_mode(x[i], mode))) bad_l++;
    }
    printf("%s{\"mode\": %d, \"fractional\": %ld, \"pow_mismatches\": %ld, \"exp_mismatches\": %ld, "
           "\"log_mismatches\": %ld}", mode ? ", " : "", mode, frac, bad_p, bad_e, bad_l);
    bad_all += bad_p + bad_e + bad_l;
  }
  printf("]}\n");
  return bad_all ? 1 : 0;
}

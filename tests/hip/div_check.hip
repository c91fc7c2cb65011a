// Device check (test infrastructure): rt::norm's core square root and
// shared-reciprocal division equal IEEE sqrt and three `/` bit for bit, on
// random vectors spanning the safe exponent range, its edges and beyond
// (fix-up path), plus zeros, signed zeros, denormals, infinities and NaN
// components.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../go-raytracer_amd/csrc div_check.hip
#include "rt_device.h"
#include <cstdio>
#include <cstdlib>

using namespace rt;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb93fe53a85b3ULL; x ^= x >> 33;
  return x;
}
__device__ double gen(uint64_t& s, int mode) {
  s = mix(s + 0x9E3779B97F4A7C15ULL);
  const uint64_t r = s;
  switch (mode) {
    case 0: {  // |x| in roughly [2^-60, 2^60], random mantissa
      const uint64_t e = 1023 - 60 + (r >> 52) % 121;
      return __longlong_as_double((long long)(((r & 1) << 63) | (e << 52) | (mix(r) & 0xFFFFFFFFFFFFFULL)));
    }
    case 1: {  // any finite exponent, incl. denormals and the fallback range
      const uint64_t e = (r >> 52) % 2047;
      return __longlong_as_double((long long)(((r & 1) << 63) | (e << 52) | (mix(r) & 0xFFFFFFFFFFFFFULL)));
    }
    case 2: {  // around the safe-range edges (numerators 2^-800, m 2^-100 / 2^99, far out)
      const int64_t edge[4] = {223, 923, 1122, 1423};
      const int64_t e = edge[(r >> 1) & 3] + (int64_t)((r >> 8) % 5) - 2;
      return __longlong_as_double((long long)(((r & 1) << 63) | ((uint64_t)e << 52) | (mix(r) & 0xFFFFFFFFFFFFFULL)));
    }
    default: {  // specials
      const double sp[8] = {0.0, -0.0, 1.0, -1.0, __builtin_inf(), -__builtin_inf(), __builtin_nan(""), 4.9e-324};
      return (r & 8) ? sp[(r >> 4) & 7] : (double)((int64_t)(r >> 40) - (1LL << 23));
    }
  }
}

__global__ void check(uint64_t seed, int iters, unsigned long long* bad, unsigned long long* fast) {
  uint64_t s = seed ^ ((uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) << 20);
  for (int it = 0; it < iters; it++) {
    // wave-uniform mode, so whole waves meet the fast-path preconditions
    const uint64_t wave = (uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int mode = (int)(mix(seed ^ (wave << 24) ^ (uint64_t)it) % 16);
    const int m = mode < 11 ? 0 : (mode < 13 ? 1 : (mode < 15 ? 2 : 3));
    d3 v = mk(gen(s, m), gen(s, m), gen(s, mode == 10 ? 3 : m));
    d3 a = norm(v);
    double mm = __builtin_sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    d3 b = mk(v.x / mm, v.y / mm, v.z / mm);
    bool same = __double_as_longlong(a.x) == __double_as_longlong(b.x) &&
                __double_as_longlong(a.y) == __double_as_longlong(b.y) &&
                __double_as_longlong(a.z) == __double_as_longlong(b.z);
    if (!same) {
      // NaN payloads may legitimately differ in sign/payload only if both NaN
      bool nan_ok = (a.x != a.x) == (b.x != b.x) && (a.y != a.y) == (b.y != b.y) && (a.z != a.z) == (b.z != b.z) &&
                    (a.x == b.x || a.x != a.x) && (a.y == b.y || a.y != a.y) && (a.z == b.z || a.z != a.z);
      if (!nan_ok) {
        unsigned long long k = atomicAdd(bad, 1ULL);
        if (k < 8)
          printf("MISMATCH v=(%a,%a,%a) fast=(%a,%a,%a) div=(%a,%a,%a)\n", v.x, v.y, v.z, a.x, a.y, a.z, b.x, b.y,
                 b.z);
      }
    }
    // lanes meeting the fast-path preconditions (the others take the fix-up)
    const bool num = (__builtin_fabs(v.x) >= 0x1p-800 || v.x == 0.0) &&
                     (__builtin_fabs(v.y) >= 0x1p-800 || v.y == 0.0) &&
                     (__builtin_fabs(v.z) >= 0x1p-800 || v.z == 0.0);
    if (num && mm >= 0x1p-100 && mm < 0x1p100) atomicAdd(fast, 1ULL);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 256;
  unsigned long long *bad, *fast;
  if (hipMallocManaged(&bad, 8) != hipSuccess || hipMallocManaged(&fast, 8) != hipSuccess) return 2;
  *bad = 0;
  *fast = 0;
  const int blocks = 4096, threads = 256;
  hipLaunchKernelGGL(check, dim3(blocks), dim3(threads), 0, 0, 12345ULL, iters, bad, fast);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  const unsigned long long n = (unsigned long long)blocks * threads * iters;
  printf("{\"vectors\": %llu, \"fast_path\": %llu, \"mismatches\": %llu}\n", n, *fast, *bad);
  return *bad == 0 ? 0 : 1;
}

// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the render kernel's
// own access widths (MI355X_MICROARCH.md §HBM: only 16-B/lane streams are
// calibrated there). Each kernel moves a known number of bytes through HBM
// (512 MiB, twice the Infinity Cache), with the widths the render kernel uses:
//   read8  : 8 B/lane coalesced loads   (frame-stack fields, lane-interleaved)
//   write8 : 8 B/lane coalesced stores  (frame-stack fields)
//   write4 : 4 B/lane coalesced stores  (RGBA8 framebuffer)
// Run each under its own `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
// pass and divide the counter (KB) by the bytes printed here.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void read8(const double* __restrict__ a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 12345.678) out[0] = s;  // keeps the loads alive; never true for zeros
}
__global__ void write8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}
__global__ void write4(unsigned* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (unsigned)i;
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  const size_t bytes = (size_t)512 << 20;
  void* buf = nullptr;
  double* out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc((void**)&out, sizeof(double)));
  CK(hipMemset(buf, 0, bytes));
  CK(hipDeviceSynchronize());
  const int grid = 256 * 16, block = 256;
  hipLaunchKernelGGL(read8, dim3(grid), dim3(block), 0, 0, (const double*)buf, bytes / 8, out);
  hipLaunchKernelGGL(write8, dim3(grid), dim3(block), 0, 0, (double*)buf, bytes / 8);
  hipLaunchKernelGGL(write4, dim3(grid), dim3(block), 0, 0, (unsigned*)buf, bytes / 4);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("{\"bytes_per_kernel\": %zu}\n", bytes);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}

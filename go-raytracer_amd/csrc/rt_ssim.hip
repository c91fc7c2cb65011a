// rt_ssim.hip -- SSIM of two RGBA8 frames on the device (parity harness, SURVEY
// §8 f3). Restates prim.SSIM (internal/prim/ssim.go:27-182): 11x11 Gaussian
// window (sigma 1.5, weights normalised by their sum, ssim.go:147-164), the
// 16-bit RGBA() channel values (v8 * 257), two-pass weighted means and
// (co)variances per channel in the reference's loop order, formula (13) with
// c1 = (0.01 * 65535)^2 and c2 = (0.03 * 65535)^2, the mean of R, G, B, and
// the average over windows at x < W - 11, y < H - 11 (ssim.go:53-58: the last
// row and column of windows are not visited, so W == 11 gives 0/0 = NaN).
// Per-window values use the same op order as Go (no contraction); only the
// final sum over windows is ordered differently (the reference's goroutines
// sum columns in completion order, i.e. its own order is not fixed either).
// Included by rt_kernel.hip (shares rt_context and the error plumbing).

namespace {

enum { SSIM_K = 11, SSIM_T = 16, SSIM_TILE = SSIM_T + SSIM_K - 1 };

__global__ __launch_bounds__(SSIM_T* SSIM_T) void rt_ssim_kernel(const uint32_t* __restrict__ a,
                                                                 const uint32_t* __restrict__ b, int width, int height,
                                                                 int nx, int ny, const double* __restrict__ kern,
                                                                 double* __restrict__ partial) {
  __shared__ uint32_t ta[SSIM_TILE][SSIM_TILE + 1], tb[SSIM_TILE][SSIM_TILE + 1];
  __shared__ double kw[SSIM_K * SSIM_K];
  __shared__ double red[SSIM_T * SSIM_T];
  const int tx = threadIdx.x, ty = threadIdx.y, tid = ty * SSIM_T + tx;
  const int x0 = blockIdx.x * SSIM_T, y0 = blockIdx.y * SSIM_T;  // window origins: x column, y row
  for (int i = tid; i < SSIM_K * SSIM_K; i += SSIM_T * SSIM_T) kw[i] = kern[i];
  for (int i = tid; i < SSIM_TILE * SSIM_TILE; i += SSIM_T * SSIM_T) {
    const int r = i / SSIM_TILE, c = i % SSIM_TILE;
    const int gy = min(y0 + r, height - 1), gx = min(x0 + c, width - 1);
    ta[r][c] = a[(size_t)gy * width + gx];
    tb[r][c] = b[(size_t)gy * width + gx];
  }
  __syncthreads();
  double s = 0.0;
  if (x0 + tx < nx && y0 + ty < ny) {
    double m1[3] = {0, 0, 0}, m2[3] = {0, 0, 0};
    for (int k1 = 0; k1 < SSIM_K; k1++)    // x offset (ssim.go:86)
      for (int k2 = 0; k2 < SSIM_K; k2++) {  // y offset
        const double w = kw[k1 * SSIM_K + k2];
        const uint32_t p = ta[ty + k2][tx + k1], q = tb[ty + k2][tx + k1];
        for (int ch = 0; ch < 3; ch++) {
          m1[ch] += (double)(((p >> (8 * ch)) & 0xffu) * 257u) * w;
          m2[ch] += (double)(((q >> (8 * ch)) & 0xffu) * 257u) * w;
        }
      }
    double v1[3] = {0, 0, 0}, v2[3] = {0, 0, 0}, v12[3] = {0, 0, 0};
    for (int k1 = 0; k1 < SSIM_K; k1++)
      for (int k2 = 0; k2 < SSIM_K; k2++) {
        const double w = kw[k1 * SSIM_K + k2];
        const uint32_t p = ta[ty + k2][tx + k1], q = tb[ty + k2][tx + k1];
        for (int ch = 0; ch < 3; ch++) {
          const double d1 = (double)(((p >> (8 * ch)) & 0xffu) * 257u) - m1[ch];
          const double d2 = (double)(((q >> (8 * ch)) & 0xffu) * 257u) - m2[ch];
          v1[ch] += w * (d1 * d1);
          v2[ch] += w * (d2 * d2);
          v12[ch] += w * d1 * d2;
        }
      }
    const double c1 = 429483.6225, c2 = 3865352.6025;  // (0.01*65535)^2, (0.03*65535)^2
    double ch_ssim[3];
    for (int ch = 0; ch < 3; ch++) {
      const double num = (2 * m1[ch] * m2[ch] + c1) * (2 * v12[ch] + c2);
      const double den = (m1[ch] * m1[ch] + m2[ch] * m2[ch] + c1) * (v1[ch] + v2[ch] + c2);
      ch_ssim[ch] = num / den;
    }
    s = (ch_ssim[0] + ch_ssim[1] + ch_ssim[2]) / 3.0;
  }
  red[tid] = s;
  __syncthreads();
  for (int w = SSIM_T * SSIM_T / 2; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) partial[blockIdx.y * gridDim.x + blockIdx.x] = red[0];
}

}  // namespace

extern "C" int rt_ssim_rgba8(rt_context* c, const uint8_t* d_a, const uint8_t* d_b, int width, int height,
                             double* out, void* stream) {
  if (!c || !d_a || !d_b || !out) return fail(RT_E_INVALID, "rt_ssim_rgba8: NULL argument");
  if (width < SSIM_K || height < SSIM_K) return fail(RT_E_INVALID, "images are too small");  // ssim.go:32-34
  const int nx = width - SSIM_K, ny = height - SSIM_K;
  if (nx == 0 || ny == 0) {  // no window visited: sum / n = 0 / 0
    *out = std::numeric_limits<double>::quiet_NaN();
    return RT_OK;
  }
  DeviceGuard guard(c->device);
  hipStream_t st = (hipStream_t)stream;
  // makeGaussianKernel (ssim.go:147-164)
  double kern[SSIM_K * SSIM_K], total = 0.0;
  const double center = (double)(SSIM_K - 1) / 2, sd = 1.5;
  for (int i = 0; i < SSIM_K; i++)
    for (int j = 0; j < SSIM_K; j++) {
      const double x = (double)i - center, y = (double)j - center;
      const double v = std::exp(-(x * x + y * y) / (2 * sd * sd));
      kern[i * SSIM_K + j] = v;
      total += v;
    }
  for (int i = 0; i < SSIM_K * SSIM_K; i++) kern[i] /= total;
  const dim3 grid((nx + SSIM_T - 1) / SSIM_T, (ny + SSIM_T - 1) / SSIM_T);
  const size_t nblk = (size_t)grid.x * grid.y;
  const size_t need = sizeof kern + nblk * sizeof(double);
  if (need > c->ssim_bytes) {
    (void)hipFree(c->ssim_buf);
    c->ssim_buf = nullptr;
    c->ssim_bytes = 0;
    HIP_TRY(hipMalloc((void**)&c->ssim_buf, need));
    c->ssim_bytes = need;
  }
  double* dk = reinterpret_cast<double*>(c->ssim_buf);
  double* dpart = dk + SSIM_K * SSIM_K;
  HIP_TRY(hipMemcpyAsync(dk, kern, sizeof kern, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(rt_ssim_kernel, grid, dim3(SSIM_T, SSIM_T), 0, st, reinterpret_cast<const uint32_t*>(d_a),
                     reinterpret_cast<const uint32_t*>(d_b), width, height, nx, ny, dk, dpart);
  HIP_TRY(hipGetLastError());
  std::vector<double> part(nblk);
  HIP_TRY(hipMemcpyAsync(part.data(), dpart, nblk * sizeof(double), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  double sum = 0.0;
  for (double p : part) sum += p;
  *out = sum / ((double)nx * (double)ny);
  return RT_OK;
}

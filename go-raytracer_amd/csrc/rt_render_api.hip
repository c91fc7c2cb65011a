// rt_render_api.hip -- the synchronous Render() seam (include/rt_abi.h
// rt_render): the replacement of func Render(*Scene) image.Image
// (raytracer.go:589-682), which the reference's GML interpreter calls through
// EvalState.Render (evaluator.go:48, installed at raytracer.go:700-708).
// Included by rt_kernel.hip (shares rt_context and the error plumbing); host
// code only, so it is not part of the kernel source id the PMC summaries are
// keyed on.
//
// One call = scene conversion + upload, one whole frame, the image in the
// caller's (pageable) host buffer, the counters. What keeps it close to the
// kernel's own frame time:
//   * the scene is kept between calls: its bytes (every array the rt_scene
//     points at, serialised) are compared with the last scene set, and an
//     unchanged scene skips the conversion, the upload and the tile-cost
//     estimate launch (exact: a byte compare, no hash);
//   * two contexts with the scene, launched alternately on two streams (frames
//     in flight, rt_set_frames_in_flight): the frame is rendered as row bands,
//     band k on context k mod 2, so one band's last waves share the chip with
//     the next band's first;
//   * each finished band is copied by DMA into a library-owned pinned buffer
//     (a copy stream waits on the band's event) while later bands render, and
//     the host copies it on to the caller's buffer with several threads --
//     a pageable device-to-host copy ran at ~5.7 GB/s (round 4: 5.8 ms for the
//     33 MB 4K frame), the pinned DMA runs at PCIe rate;
//   * the counters are read (and reset) once per call at the end.
// rt_render_last_timing reports the parts of the calling thread's last call
// on one host timeline, so they add up to its total.

#include <thread>

namespace {

// Serialised scene: the rt_scene's scalars and every array it points at, as
// rt_set_scene reads them. Two scenes with equal bytes convert to the same
// device scene.
void scene_bytes(const rt_scene* s, std::vector<char>& out) {
  out.clear();
  auto put = [&](const void* p, size_t n) {
    if (!p || n == 0) return;
    const char* c = static_cast<const char*>(p);
    out.insert(out.end(), c, c + n);
  };
  auto cnt = [](int32_t n) { return (size_t)std::max(0, (int)n); };
  // scalars (the pointers themselves are not compared, their contents are)
  put(&s->width, sizeof(int32_t) * 4);
  put(&s->fov, sizeof(double) * 10);
  put(&s->num_objects, sizeof(int32_t) * 2);
  put(&s->num_programs, sizeof(int32_t) * 3);
  put(&s->exp_mode, sizeof(int32_t));
  put(&s->num_ext_lights, sizeof(int32_t));
  put(&s->num_csg_leaves, sizeof(int32_t) * 2);
  put(s->lights, cnt(s->num_lights) * sizeof(rt_point_light));
  put(s->objects, cnt(s->num_objects) * sizeof(rt_object));
  put(s->materials, cnt(s->num_materials) * sizeof(rt_material));
  put(s->program_code, cnt(s->program_code_words) * sizeof(uint32_t));
  put(s->program_consts, cnt(s->program_const_count) * sizeof(uint64_t));
  put(s->program_entry, cnt(s->num_programs) * sizeof(int32_t));
  put(s->ext_lights, cnt(s->num_ext_lights) * sizeof(rt_light));
  put(s->csg_leaves, cnt(s->num_csg_leaves) * sizeof(rt_object));
  put(s->csg_code, cnt(s->csg_code_words) * sizeof(int32_t));
}

enum { API_CTX = 2, API_MAX_BANDS = 16 };

struct ApiSlot {
  rt_context* c[API_CTX] = {nullptr, nullptr};
  hipStream_t st[API_CTX] = {nullptr, nullptr};
  hipStream_t copy = nullptr;
  hipEvent_t ev_start = nullptr, ev_end = nullptr;
  hipEvent_t band_done[API_MAX_BANDS] = {}, copy_done[API_MAX_BANDS] = {};
  void* buf = nullptr;  // device frame
  size_t bytes = 0;
  uint8_t* pinned = nullptr;  // host bounce buffer (hipHostMalloc)
  size_t pinned_bytes = 0;
  std::vector<char> scene;  // bytes of the scene both contexts hold (empty: none)
  bool dirty = true;        // counters may hold a failed call's work: reset before the next
  bool spec = false;        // contexts specialise (hipRTC)
};

thread_local rt_render_timing g_api_timing;

int env_int(const char* name, int def) {
  const char* e = getenv(name);
  return e ? atoi(e) : def;
}

// Row bands of one frame: RT_RENDER_BANDS (environment) or one band per
// ~2 M pixels, at most 4 (a 4K frame: 4 bands of 540 rows); bands start on
// 8-row tile rows. Measured on C3 4K (scripts/api_seam.py,
// profiles/r05/seam/): 1 / 2 / 4 / 8 bands 4.65 / 4.16 / 3.89 / 4.10 ms per
// call with 4-8 copy threads (more bands: a shorter exposed copy of the last
// band, but each band launch has its own tail).
int api_bands(int width, int height, int* rows) {
  const long long px = (long long)width * height;
  int nb = env_int("RT_RENDER_BANDS", 0);
  if (nb <= 0) nb = (int)std::min<long long>(4, std::max<long long>(1, (px + (1 << 20)) / (2 << 20)));
  nb = std::max(1, std::min(nb, (int)API_MAX_BANDS));
  const int trows = (height + TILE - 1) / TILE;
  nb = std::min(nb, trows);
  for (int k = 0; k <= nb; k++) rows[k] = std::min(height, (int)((long long)trows * k / nb) * TILE);
  rows[nb] = height;
  return nb;
}

// Host copy pinned -> caller memory with up to `threads` threads.
void par_copy(uint8_t* dst, const uint8_t* src, size_t n, int threads) {
  const size_t min_part = (size_t)1 << 20;
  const int t = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), n / min_part));
  if (t <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> pool;
  const size_t part = (n + t - 1) / t;
  for (int i = 1; i < t; i++) {
    const size_t a = (size_t)i * part, b = std::min(n, a + part);
    if (a < b) pool.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
  }
  std::memcpy(dst, src, std::min(n, part));
  for (auto& th : pool) th.join();
}

int api_slot_init(ApiSlot& sl, int dev) {
  DeviceGuard guard(dev);
  for (int i = 0; i < API_CTX; i++) {
    int rc = rt_create(dev, &sl.c[i]);
    if (rc != RT_OK) return rc;
    rt_set_frames_in_flight(sl.c[i], API_CTX);
    HIP_TRY(hipStreamCreateWithFlags(&sl.st[i], hipStreamNonBlocking));
  }
  HIP_TRY(hipStreamCreateWithFlags(&sl.copy, hipStreamNonBlocking));
  HIP_TRY(hipEventCreate(&sl.ev_start));
  HIP_TRY(hipEventCreate(&sl.ev_end));
  for (int k = 0; k < API_MAX_BANDS; k++) {
    HIP_TRY(hipEventCreateWithFlags(&sl.band_done[k], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&sl.copy_done[k], hipEventDisableTiming));
  }
  // scene specialisation (hipRTC, cached per process by scene shape): the
  // first call with a new shape pays the compile; RT_RENDER_SPECIALIZE=0 keeps
  // the generic kernel (hipRTC runs in its own link-map namespace with its own
  // libc, so it is only ever called on the caller's thread)
  sl.spec = env_int("RT_RENDER_SPECIALIZE", 1) != 0;
  for (int i = 0; i < API_CTX && sl.spec; i++) {
    int rc = rt_set_specialize(sl.c[i], 1);
    if (rc != RT_OK) return rc;  // (no scene yet: cannot fail on a compile)
  }
  return RT_OK;
}

// rt_set_scene on every context of the slot; a failed specialisation (no
// hipRTC, or the compile fails) falls back to the generic kernel, which
// renders the same pixels: logged once per process.
int api_set_scene(ApiSlot& sl, const rt_scene* scene) {
  for (int i = 0; i < API_CTX; i++) {
    int rc = rt_set_scene(sl.c[i], scene);
    // (an invalid or singular scene fails before specialisation, with its own code)
    if (rc == RT_E_DEVICE && sl.spec) {
      static bool logged = false;
      if (!logged) {
        logged = true;
        fprintf(stderr, "rt_render: scene specialisation failed, using the generic kernel (%s)\n", rt_last_error());
      }
      for (int j = 0; j < API_CTX; j++) rt_set_specialize(sl.c[j], 0);
      sl.spec = false;
      rc = RT_OK;
      for (int j = 0; j < API_CTX && rc == RT_OK; j++) rc = rt_set_scene(sl.c[j], scene);
      return rc;
    }
    if (rc != RT_OK) return rc;
  }
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_render_last_timing(rt_render_timing* out) {
  if (!out) return fail(RT_E_INVALID, "rt_render_last_timing: NULL argument");
  *out = g_api_timing;
  return RT_OK;
}

int rt_render(const rt_scene* scene, uint8_t* rgba_out, rt_stats* stats) {
  typedef std::chrono::steady_clock clk;
  const auto t0 = clk::now();
  auto ms_since = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  g_api_timing = rt_render_timing();
  if (!scene || !rgba_out) return fail(RT_E_INVALID, "rt_render: NULL argument");
  if (scene->width <= 1 || scene->height <= 1) return fail(RT_E_INVALID, "rt_set_scene: width/height must be > 1");
  // one slot (two contexts, streams, device frame, pinned bounce buffer) per
  // device, kept between calls (the reference's Render allocates its image per
  // call, raytracer.go:590)
  static std::mutex mu;
  static std::vector<ApiSlot> cache;
  std::lock_guard<std::mutex> lock(mu);
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if ((int)cache.size() <= dev) cache.resize(dev + 1);
  ApiSlot& sl = cache[dev];
  if (!sl.c[0]) {
    int rc = api_slot_init(sl, dev);
    if (rc != RT_OK) {
      for (int i = 0; i < API_CTX; i++) {
        rt_destroy(sl.c[i]);
        sl.c[i] = nullptr;
      }
      return rc;
    }
  }
  DeviceGuard guard(dev);
  const size_t bytes = (size_t)scene->width * scene->height * 4;
  if (bytes > sl.bytes) {
    (void)hipFree(sl.buf);
    (void)hipHostFree(sl.pinned);
    sl.buf = nullptr;
    sl.pinned = nullptr;
    sl.bytes = 0;
    if (hipMalloc(&sl.buf, bytes) != hipSuccess) return fail(RT_E_NOMEM, "rt_render: frame buffer");
    if (hipHostMalloc((void**)&sl.pinned, bytes, hipHostMallocDefault) != hipSuccess) {
      (void)hipFree(sl.buf);
      sl.buf = nullptr;
      return fail(RT_E_NOMEM, "rt_render: pinned bounce buffer");
    }
    sl.bytes = bytes;
  }
  // scene: converted and uploaded only when its bytes changed
  std::vector<char> sb;
  scene_bytes(scene, sb);
  const bool reuse = !sl.scene.empty() && sb == sl.scene;
  if (!reuse) {
    sl.scene.clear();
    int rc = api_set_scene(sl, scene);
    if (rc != RT_OK) return rc;
    sl.scene.swap(sb);
  }
  if (sl.dirty) {
    rt_stats tmp;
    for (int i = 0; i < API_CTX; i++) {
      int rc = rt_read_stats(sl.c[i], sl.st[i], 1, &tmp);
      if (rc != RT_OK) return rc;
    }
    sl.dirty = false;
  }
  sl.dirty = true;  // until this call's counters are read
  // bands, alternating contexts/streams; each band's DMA into the pinned
  // buffer on the copy stream once the band is done
  int rows[API_MAX_BANDS + 1];
  const int nb = api_bands(scene->width, scene->height, rows);
  const int W = scene->width;
  HIP_TRY(hipEventRecord(sl.ev_start, sl.st[0]));
  HIP_TRY(hipStreamWaitEvent(sl.st[1], sl.ev_start, 0));
  for (int k = 0; k < nb; k++) {
    const int i = k % API_CTX;
    const size_t off = (size_t)rows[k] * W * 4, n = (size_t)(rows[k + 1] - rows[k]) * W * 4;
    int rc = rt_render_rows_async(sl.c[i], rows[k], rows[k + 1], (char*)sl.buf + off, sl.st[i]);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipEventRecord(sl.band_done[k], sl.st[i]));
    HIP_TRY(hipStreamWaitEvent(sl.copy, sl.band_done[k], 0));
    HIP_TRY(hipMemcpyAsync(sl.pinned + off, (char*)sl.buf + off, n, hipMemcpyDeviceToHost, sl.copy));
    HIP_TRY(hipEventRecord(sl.copy_done[k], sl.copy));
  }
  // GPU span: first band's start to the last band's end (both streams)
  HIP_TRY(hipStreamWaitEvent(sl.st[0], sl.band_done[nb - 1], 0));
  if (nb > 1) HIP_TRY(hipStreamWaitEvent(sl.st[0], sl.band_done[nb - 2], 0));
  HIP_TRY(hipEventRecord(sl.ev_end, sl.st[0]));
  const auto t_launched = clk::now();
  const int threads = std::max(1, env_int("RT_RENDER_COPY_THREADS", 4));
  for (int k = 0; k + 1 < nb; k++) {  // bands before the last, while later bands render
    HIP_TRY(hipEventSynchronize(sl.copy_done[k]));
    const size_t off = (size_t)rows[k] * W * 4, n = (size_t)(rows[k + 1] - rows[k]) * W * 4;
    par_copy(rgba_out + off, sl.pinned + off, n, threads);
  }
  HIP_TRY(hipEventSynchronize(sl.ev_end));
  const auto t_rendered = clk::now();
  {
    const int k = nb - 1;
    HIP_TRY(hipEventSynchronize(sl.copy_done[k]));
    const size_t off = (size_t)rows[k] * W * 4, n = (size_t)(rows[k + 1] - rows[k]) * W * 4;
    par_copy(rgba_out + off, sl.pinned + off, n, threads);
  }
  // counters of both contexts, read and reset
  rt_stats sum;
  std::memset(&sum, 0, sizeof sum);
  for (int i = 0; i < API_CTX; i++) {
    rt_stats s;
    int rc = rt_read_stats(sl.c[i], sl.st[i], 1, &s);
    if (rc != RT_OK) return rc;
    sum.primary_rays += s.primary_rays;
    sum.secondary_rays += s.secondary_rays;
    sum.shadow_rays += s.shadow_rays;
    for (int q = 0; q < RT_NUM_KINDS; q++) {
      sum.tests[q] += s.tests[q];
      sum.shadow_tests[q] += s.shadow_tests[q];
    }
    sum.shaded_hits += s.shaded_hits;
    sum.surface_errors += s.surface_errors;
  }
  sl.dirty = false;
  float gms = 0.f;
  HIP_TRY(hipEventElapsedTime(&gms, sl.ev_start, sl.ev_end));
  sum.kernel_ms = gms;
  if (stats) *stats = sum;
  const auto t_end = clk::now();
  rt_render_timing& tm = g_api_timing;
  tm.total_ms = ms_since(t0, t_end);
  tm.setup_ms = ms_since(t0, t_launched);
  tm.render_wait_ms = ms_since(t_launched, t_rendered);
  tm.copy_tail_ms = ms_since(t_rendered, t_end);
  tm.gpu_ms = gms;
  tm.bands = nb;
  tm.scene_reused = reuse ? 1 : 0;
  tm.specialized = sl.spec ? 1 : 0;
  return RT_OK;
}

}  // extern "C"

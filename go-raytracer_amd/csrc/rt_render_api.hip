// rt_render_api.hip -- the synchronous Render() seam (include/rt_abi.h
// rt_render / rt_render_ex): the replacement of func Render(*Scene)
// image.Image (raytracer.go:589-682), which the reference's GML interpreter
// calls through EvalState.Render (evaluator.go:48, installed at
// raytracer.go:700-708). The reference's Render uses all its workers
// (raytracer.go:611-677, 8 of them, :725) from its one entry point; this one
// uses one or several GPUs of the process the same way.
// Included by rt_kernel.hip (shares rt_context and the error plumbing); host
// code plus a small de-interleave kernel, not part of the kernel source id
// the PMC summaries are keyed on.
//
// One call = one whole frame into the caller's buffer, the counters. Per
// device (a "slot": a device of the call's list, a repeated ordinal getting a
// slot of its own) the library keeps between calls:
//   * two contexts with the last scene. A call compares the scene's bytes
//     (every array the rt_scene points at, serialised) with the last one; a
//     changed scene is converted once (rt_set_scene on the first slot's first
//     context, with its tile-cost estimate) and cloned to every other context
//     of every device (scene_clone: upload of the converted bytes, the same
//     tile costs) -- no second conversion, BVH build or estimate;
//   * the share buffer: the slot's 8-row tile rows (t = slot, slot + N, ...),
//     packed, rendered as row bands alternating over the two contexts and
//     their streams (frames in flight, rt_set_frames_in_flight), so one band's
//     last waves share the chip with the next band's first;
//   * a copy stream and events.
// The gather (RT_GATHER_HOST): each finished band is DMAed by its own device,
// over its own PCIe link, straight to its final rows of one pinned frame
// (strided 2-D copies: a tile row is 8 contiguous image rows), and the host
// copies finished bands on to the caller's pageable buffer with several
// threads while later bands render (a pageable device-to-host copy ran at
// ~5.7 GB/s: round 4, 5.8 ms for the 33 MB 4K frame). RT_GATHER_PEER copies
// every share to the first device over xGMI (hipMemcpyPeerAsync) where a
// kernel de-interleaves it into one frame: the caller's device buffer
// (RT_RENDER_OUT_DEVICE), or a frame that one DMA brings to the host.
// Specialised kernels compile in the background (rt_kernel.hip spec_build):
// a new scene shape renders with the generic kernel until its own is ready.
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

int env_int(const char* name, int def) {
  const char* e = rt_getenv(name);  // (the load-time copy: rt_kernel.hip env_snap)
  return e ? atoi(e) : def;
}

// ---------------------------------------------------------------------------
// The frame plan: who renders which tile rows, in which bands, and where each
// byte of a share lands in the frame. Pure host arithmetic, shared by the
// device path and rt_debug_assemble (the CPU test of the assembly).
// ---------------------------------------------------------------------------

// One copy run: `height` rows of `width` bytes, row r from src + r*spitch to
// dst + r*dpitch (offsets: dst in the frame, src in the slot's share buffer).
struct CopyOp {
  size_t dst, src, width, height, dpitch, spitch;
};

struct ApiPlan {
  int W = 0, H = 0, N = 1, trows = 0;
  std::vector<int> ntr;                  // tile rows of each slot's share
  std::vector<std::vector<int>> bounds;  // per slot: band k = share tile rows [bounds[k], bounds[k+1])
  size_t row_bytes() const { return (size_t)W * 4; }
  size_t trow_bytes() const { return (size_t)TILE * W * 4; }
  // image rows of share tile row j of slot d
  int row0(int d, int j) const { return (d + j * N) * TILE; }
  int nrows(int d, int j) const { return std::min((int)TILE, H - row0(d, j)); }
  int bands() const {
    int n = 0;
    for (const auto& b : bounds) n += (int)b.size() - 1;
    return n;
  }
  // bytes of band k of slot d in its (packed) share buffer, from its first row
  size_t band_bytes(int d, int k) const {
    const int j0 = bounds[d][k], j1 = bounds[d][k + 1];
    return (size_t)(j1 - 1 - j0) * trow_bytes() + (size_t)nrows(d, j1 - 1) * row_bytes();
  }
};

// Tile rows dealt round-robin: slot d of N gets tile rows d, d+N, ... (SURVEY
// 8(e): every device the same mix of sky, floor and glass). Bands per slot:
// `forced` (> 0), else RT_RENDER_BANDS, else one per ~2 M pixels of the share,
// at most 4 -- measured on C3 4K with one device (scripts/api_seam.py,
// profiles/r05/seam/): 1 / 2 / 4 / 8 equal bands 4.65 / 4.16 / 3.89 / 4.10 ms
// per call (more bands: a shorter exposed copy of the last band, but each band
// launch has its own tail). Band sizes decrease (weights 4:3:2:1 for 4 bands;
// RT_RENDER_BAND_SHAPE=0: equal), so the exposed copy is that of the smallest
// band: C3 3.83-3.84 -> 3.61-3.72 ms per call, c4csg 12.44 -> 11.45 ms
// (scripts/gpu/r6_bands.sh, profiles/r06/bands/).
ApiPlan api_plan(int W, int H, int N, int forced) {
  ApiPlan p;
  p.W = W;
  p.H = H;
  p.N = N;
  p.trows = (H + TILE - 1) / TILE;
  const int env = env_int("RT_RENDER_BANDS", 0);
  const int shape = env_int("RT_RENDER_BAND_SHAPE", 1);
  for (int d = 0; d < N; d++) {
    const int n = d < p.trows ? (p.trows - 1 - d) / N + 1 : 0;
    p.ntr.push_back(n);
    std::vector<int> b;
    if (n > 0) {
      const long long px = (long long)n * TILE * W;
      int nb = forced > 0 ? forced : env > 0 ? env : (int)std::min<long long>(4, std::max<long long>(1, (px + (1 << 20)) / (2 << 20)));
      nb = std::max(1, std::min({nb, (int)API_MAX_BANDS, n}));
      if (shape == 1 && nb > 1) {
        // decreasing bands (weights nb, nb-1, ..., 1): the last band, whose
        // copy is the exposed tail, is the smallest
        const long long tot = (long long)nb * (nb + 1) / 2;
        long long acc = 0;
        b.push_back(0);
        for (int k = 0; k < nb; k++) {
          acc += nb - k;
          const int e = (int)(n * acc / tot);
          b.push_back(std::max(e, b.back() + 1));
        }
        b.back() = n;
        bool ok = true;  // (tiny shares: equal bands)
        for (size_t k = 1; k < b.size(); k++) ok = ok && b[k] > b[k - 1];
        if (!ok) {
          b.clear();
          for (int k = 0; k <= nb; k++) b.push_back((int)((long long)n * k / nb));
        }
      } else {
        for (int k = 0; k <= nb; k++) b.push_back((int)((long long)n * k / nb));
      }
    }
    p.bounds.push_back(b);
  }
  return p;
}

// The DMA runs of band k of slot d: one per tile row, merged into strided runs
// (equal widths at constant pitches) -- with one device a band is one
// contiguous run plus, when the image height is not a multiple of 8, the
// clipped last tile row.
std::vector<CopyOp> band_ops(const ApiPlan& p, int d, int k) {
  std::vector<CopyOp> ops;
  for (int j = p.bounds[d][k]; j < p.bounds[d][k + 1]; j++) {
    const size_t dst = (size_t)p.row0(d, j) * p.row_bytes(), src = (size_t)j * p.trow_bytes();
    const size_t len = (size_t)p.nrows(d, j) * p.row_bytes();
    if (!ops.empty()) {
      CopyOp& o = ops.back();
      if (len == o.width && o.height == 1 && dst > o.dst && src > o.src && dst - o.dst >= len && src - o.src >= len) {
        o.dpitch = dst - o.dst;
        o.spitch = src - o.src;
        o.height = 2;
        continue;
      }
      if (len == o.width && o.height > 1 && dst == o.dst + o.height * o.dpitch && src == o.src + o.height * o.spitch) {
        o.height++;
        continue;
      }
    }
    ops.push_back(CopyOp{dst, src, len, 1, len, len});
  }
  // a run whose rows are contiguous on both sides is one plain copy
  for (CopyOp& o : ops)
    if (o.height > 1 && o.dpitch == o.width && o.spitch == o.width) {
      o.width *= o.height;
      o.height = 1;
      o.dpitch = o.spitch = o.width;
    }
  return ops;
}

// Frame byte ranges [first, second) band k of slot d fills (merged).
std::vector<std::pair<size_t, size_t>> band_ranges(const ApiPlan& p, int d, int k) {
  std::vector<std::pair<size_t, size_t>> r;
  for (const CopyOp& o : band_ops(p, d, k))
    for (size_t h = 0; h < o.height; h++) {
      const size_t a = o.dst + h * o.dpitch, b = a + o.width;
      if (!r.empty() && r.back().second == a) r.back().second = b;
      else r.push_back({a, b});
    }
  return r;
}

// Host copy of frame ranges (pinned -> caller memory) with up to `threads`
// threads, the bytes split evenly.
void par_copy_ranges(uint8_t* dst, const uint8_t* src, const std::vector<std::pair<size_t, size_t>>& ranges,
                     int threads) {
  size_t total = 0;
  for (const auto& r : ranges) total += r.second - r.first;
  const size_t min_part = (size_t)1 << 20;
  const int t = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), total / min_part));
  auto run = [&](size_t lo, size_t hi) {  // bytes [lo, hi) of the concatenated ranges
    size_t at = 0;
    for (const auto& r : ranges) {
      const size_t n = r.second - r.first, a = std::max(lo, at), b = std::min(hi, at + n);
      if (a < b) std::memcpy(dst + r.first + (a - at), src + r.first + (a - at), b - a);
      at += n;
    }
  };
  if (t <= 1) {
    run(0, total);
    return;
  }
  std::vector<std::thread> pool;
  const size_t part = (total + t - 1) / t;
  for (int i = 1; i < t; i++) {
    const size_t a = (size_t)i * part, b = std::min(total, a + part);
    if (a < b) pool.emplace_back([=, &run] { run(a, b); });
  }
  run(0, std::min(total, part));
  for (auto& th : pool) th.join();
}

// ---------------------------------------------------------------------------
// Device resources
// ---------------------------------------------------------------------------

// xGMI gather, the de-interleave on the first device: `ntrows` packed tile
// rows of slot d's share (src, from share tile row j0) to their image rows of
// the frame dst (4-byte pixels). One block row per tile row.
__global__ void rt_scatter_tile_rows(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, int W, int H, int d,
                                     int N, int j0) {
  const int j = j0 + (int)blockIdx.y;
  const int r0 = (d + j * N) * TILE;
  const int rows = min((int)TILE, H - r0);
  const size_t words = (size_t)rows * W;
  const uint32_t* s = src + (size_t)blockIdx.y * TILE * W;
  uint32_t* o = dst + (size_t)r0 * W;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x)
    o[i] = s[i];
}

// One device of rt_render_ex frames: two contexts with the scene, their
// streams, a copy stream, events, the share buffer.
struct ApiSlot {
  int device = -1;
  rt_context* c[API_CTX] = {nullptr, nullptr};
  hipStream_t st[API_CTX] = {nullptr, nullptr};
  hipStream_t copy = nullptr;
  hipEvent_t ev_start = nullptr, ev_end = nullptr;
  hipEvent_t band_done[API_MAX_BANDS] = {}, copy_done[API_MAX_BANDS] = {};
  void* buf = nullptr;  // the share: its tile rows, packed (device)
  size_t bytes = 0;
  std::vector<char> scene;  // bytes of the scene both contexts hold (empty: none)
  bool dirty = true;        // counters may hold a failed call's work: reset before the next
  int spec = -1;            // contexts specialise (1) or not (0); -1 not set yet
};

// The first device's gather resources (RT_GATHER_PEER) and the pinned frame.
struct ApiFrame {
  uint8_t* pinned = nullptr;  // host frame (hipHostMalloc, portable)
  size_t pinned_bytes = 0;
  int root = -1;               // device of frame / staging
  void* frame = nullptr;       // device frame on root (host output, peer gather)
  size_t frame_bytes = 0;
  void* staging = nullptr;     // other devices' shares copied over xGMI
  size_t staging_bytes = 0;
  hipStream_t gather = nullptr;  // root: de-interleave and the frame's DMA
  hipEvent_t gather_done = nullptr;
};

thread_local rt_render_timing g_api_timing;

void api_slot_free(ApiSlot& sl) {
  if (sl.device >= 0) {
    DeviceGuard guard(sl.device);
    for (int i = 0; i < API_CTX; i++) {
      rt_destroy(sl.c[i]);
      if (sl.st[i]) (void)hipStreamDestroy(sl.st[i]);
    }
    if (sl.copy) (void)hipStreamDestroy(sl.copy);
    if (sl.ev_start) (void)hipEventDestroy(sl.ev_start);
    if (sl.ev_end) (void)hipEventDestroy(sl.ev_end);
    for (int k = 0; k < API_MAX_BANDS; k++) {
      if (sl.band_done[k]) (void)hipEventDestroy(sl.band_done[k]);
      if (sl.copy_done[k]) (void)hipEventDestroy(sl.copy_done[k]);
    }
    (void)hipFree(sl.buf);
  }
  sl = ApiSlot();
}

int api_slot_init(ApiSlot& sl, int dev) {
  sl = ApiSlot();
  sl.device = dev;
  DeviceGuard guard(dev);
  int rc = RT_OK;
  auto hip = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && rc == RT_OK) rc = fail(RT_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
  };
  for (int i = 0; i < API_CTX && rc == RT_OK; i++) {
    rc = rt_create(dev, &sl.c[i]);
    if (rc != RT_OK) break;
    rt_set_frames_in_flight(sl.c[i], API_CTX);
    sl.c[i]->spec_fallback = true;  // a failed compile renders with the generic kernel
    hip(hipStreamCreateWithFlags(&sl.st[i], hipStreamNonBlocking), "stream");
  }
  hip(hipStreamCreateWithFlags(&sl.copy, hipStreamNonBlocking), "copy stream");
  hip(hipEventCreate(&sl.ev_start), "event");
  hip(hipEventCreate(&sl.ev_end), "event");
  for (int k = 0; k < API_MAX_BANDS; k++) {
    hip(hipEventCreateWithFlags(&sl.band_done[k], hipEventDisableTiming), "event");
    hip(hipEventCreateWithFlags(&sl.copy_done[k], hipEventDisableTiming), "event");
  }
  if (rc != RT_OK) api_slot_free(sl);  // (everything created so far)
  return rc;
}

// Log a failed specialisation once per process (the generic kernel renders).
void api_log_spec_failure(const std::string& msg) {
  static bool logged = false;
  if (logged) return;
  logged = true;
  fprintf(stderr, "rt_render: scene specialisation failed, using the generic kernel (%s)\n", msg.c_str());
}

// The rt_render_opts device list.
int api_devices(const rt_render_opts* o, std::vector<int>& devs) {
  devs.clear();
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (o && o->device_mask) {
    for (int d = 0; d < 32; d++)
      if (o->device_mask & (1u << d)) devs.push_back(d);
  } else if (o && o->device_count > 0) {
    if (o->device_count > RT_MAX_DEVICES) return fail(RT_E_INVALID, "rt_render_ex: more than RT_MAX_DEVICES devices");
    for (int i = 0; i < o->device_count; i++)
      devs.push_back((o->flags & RT_RENDER_DEVICE_LIST) ? o->devices[i] : i);
  } else {
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    devs.push_back(cur);
  }
  if ((int)devs.size() > RT_MAX_DEVICES) return fail(RT_E_INVALID, "rt_render_ex: more than RT_MAX_DEVICES devices");
  for (int d : devs)
    if (d < 0 || d >= ndev) return fail(RT_E_INVALID, "rt_render_ex: device ordinal out of range");
  return RT_OK;
}

// Peer access from `a` to `b` (once per pair; devices that cannot still copy
// through hipMemcpyPeerAsync's staged path).
void api_peer(int a, int b) {
  static std::vector<std::pair<int, int>> done;
  if (a == b || std::find(done.begin(), done.end(), std::make_pair(a, b)) != done.end()) return;
  done.push_back({a, b});
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) return;
  DeviceGuard guard(a);
  if (hipDeviceEnablePeerAccess(b, 0) != hipSuccess) (void)hipGetLastError();  // (already enabled)
}

int api_alloc_pinned(ApiFrame& fr, size_t bytes) {
  if (bytes <= fr.pinned_bytes) return RT_OK;
  (void)hipHostFree(fr.pinned);
  fr.pinned = nullptr;
  fr.pinned_bytes = 0;
  if (hipHostMalloc((void**)&fr.pinned, bytes, hipHostMallocPortable) != hipSuccess) {
    fr.pinned = nullptr;
    return fail(RT_E_NOMEM, "rt_render: pinned frame");
  }
  fr.pinned_bytes = bytes;
  return RT_OK;
}

int api_alloc_dev(int dev, void** p, size_t* have, size_t bytes, const char* what) {
  if (bytes <= *have) return RT_OK;
  DeviceGuard guard(dev);
  (void)hipFree(*p);
  *p = nullptr;
  *have = 0;
  if (hipMalloc(p, std::max<size_t>(1, bytes)) != hipSuccess) {
    *p = nullptr;
    return fail(RT_E_NOMEM, std::string("rt_render: ") + what);
  }
  *have = bytes;
  return RT_OK;
}

// Enqueue one DMA run (device -> pinned host frame) on `st`.
int api_dma(const CopyOp& o, uint8_t* dst_base, const uint8_t* src_base, hipStream_t st) {
  if (o.height == 1)
    HIP_TRY(hipMemcpyAsync(dst_base + o.dst, src_base + o.src, o.width, hipMemcpyDeviceToHost, st));
  else
    HIP_TRY(hipMemcpy2DAsync(dst_base + o.dst, o.dpitch, src_base + o.src, o.spitch, o.width, o.height,
                             hipMemcpyDeviceToHost, st));
  return RT_OK;
}

void add_stats(rt_stats& sum, const rt_stats& s) {
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

}  // namespace

extern "C" {

int rt_render_last_timing(rt_render_timing* out) {
  if (!out) return fail(RT_E_INVALID, "rt_render_last_timing: NULL argument");
  *out = g_api_timing;
  return RT_OK;
}

int rt_render(const rt_scene* scene, uint8_t* rgba_out, rt_stats* stats) {
  return rt_render_ex(scene, nullptr, rgba_out, stats);
}

int rt_render_ex(const rt_scene* scene, const rt_render_opts* opts, uint8_t* rgba_out, rt_stats* stats) {
  typedef std::chrono::steady_clock clk;
  const auto t0 = clk::now();
  auto ms_since = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  g_api_timing = rt_render_timing();
  // RT_DEBUG_SEAM=1 (diagnostics): the setup steps of each call on stderr
  static const bool dbg_seam = env_int("RT_DEBUG_SEAM", 0) != 0;
  auto t_mark = t0;
  auto mark = [&](const char* what) {
    if (!dbg_seam) return;
    const auto t = clk::now();
    fprintf(stderr, "[seam] %-22s %8.3f ms\n", what, ms_since(t_mark, t));
    t_mark = t;
  };
  if (!scene || !rgba_out) return fail(RT_E_INVALID, "rt_render: NULL argument");
  if (scene->width <= 1 || scene->height <= 1) return fail(RT_E_INVALID, "rt_set_scene: width/height must be > 1");
  const int flags = opts ? opts->flags : 0;
  if (flags & ~(RT_RENDER_DEVICE_LIST | RT_RENDER_OUT_DEVICE | RT_RENDER_GENERIC | RT_RENDER_SPEC_SYNC))
    return fail(RT_E_INVALID, "rt_render_ex: unknown flags");
  const bool out_dev = (flags & RT_RENDER_OUT_DEVICE) != 0;
  int gather = opts ? opts->gather : RT_GATHER_AUTO;
  if (gather == RT_GATHER_AUTO) gather = out_dev ? RT_GATHER_PEER : RT_GATHER_HOST;
  if (gather != RT_GATHER_HOST && gather != RT_GATHER_PEER) return fail(RT_E_INVALID, "rt_render_ex: unknown gather");
  if (out_dev && gather != RT_GATHER_PEER)
    return fail(RT_E_INVALID, "rt_render_ex: device output is gathered on the first device (RT_GATHER_PEER)");
  if (opts && (opts->bands < 0 || opts->bands > API_MAX_BANDS)) return fail(RT_E_INVALID, "rt_render_ex: bands");
  std::vector<int> devs;
  {
    int rc = api_devices(opts, devs);
    if (rc != RT_OK) return rc;
  }
  const int N = (int)devs.size();
  const bool want_spec = !(flags & RT_RENDER_GENERIC) && env_int("RT_RENDER_SPECIALIZE", 1) != 0;
  const bool async_spec = !(flags & RT_RENDER_SPEC_SYNC) && env_int("RT_RENDER_SPEC_SYNC", 0) == 0;

  // slots (kept per (device, repeat) for the process), calls serialised
  static std::mutex mu;
  static std::map<std::pair<int, int>, ApiSlot*> cache;
  static ApiFrame fr;
  std::lock_guard<std::mutex> lock(mu);
  std::vector<ApiSlot*> slots;
  {
    std::map<int, int> seen;
    for (int d : devs) {
      const std::pair<int, int> key(d, seen[d]++);
      ApiSlot*& sl = cache[key];
      if (!sl) {
        sl = new ApiSlot();
        int rc = api_slot_init(*sl, d);
        if (rc != RT_OK) {
          delete sl;
          sl = nullptr;
          return rc;
        }
      }
      slots.push_back(sl);
    }
  }
  mark("slots");
  const int W = scene->width, H = scene->height;
  const ApiPlan plan = api_plan(W, H, N, opts ? opts->bands : 0);
  const size_t frame_bytes = (size_t)W * H * 4;
  // buffers: each share, packed; the pinned frame (host output); the first
  // device's frame and staging (peer gather)
  const int root = devs[0];
  for (int d = 0; d < N; d++) {
    const bool direct = out_dev && N == 1;  // (one device, device output: rows straight into rgba_out)
    if (direct || plan.ntr[d] == 0) continue;
    int rc = api_alloc_dev(slots[d]->device, &slots[d]->buf, &slots[d]->bytes, (size_t)plan.ntr[d] * plan.trow_bytes(),
                           "share buffer");
    if (rc != RT_OK) return rc;
  }
  if (!out_dev) {
    int rc = api_alloc_pinned(fr, frame_bytes);
    if (rc != RT_OK) return rc;
  }
  mark("buffers");
  size_t stage_bytes = 0;
  std::vector<size_t> stage_off(N, 0);
  if (gather == RT_GATHER_PEER) {
    if (fr.root != root) {  // (resources of another first device: released)
      if (fr.root >= 0) {
        DeviceGuard g(fr.root);
        (void)hipFree(fr.frame);
        (void)hipFree(fr.staging);
        if (fr.gather) (void)hipStreamDestroy(fr.gather);
        if (fr.gather_done) (void)hipEventDestroy(fr.gather_done);
      }
      fr.frame = fr.staging = nullptr;
      fr.frame_bytes = fr.staging_bytes = 0;
      fr.gather = nullptr;
      fr.gather_done = nullptr;
      fr.root = root;
      DeviceGuard g(root);
      HIP_TRY(hipStreamCreateWithFlags(&fr.gather, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&fr.gather_done, hipEventDisableTiming));
    }
    for (int d = 1; d < N; d++) {
      stage_off[d] = stage_bytes;
      stage_bytes += (size_t)plan.ntr[d] * plan.trow_bytes();
      api_peer(root, devs[d]);
      api_peer(devs[d], root);
    }
    int rc = api_alloc_dev(root, &fr.staging, &fr.staging_bytes, stage_bytes, "xGMI staging buffer");
    if (rc == RT_OK && !out_dev) rc = api_alloc_dev(root, &fr.frame, &fr.frame_bytes, frame_bytes, "gather frame");
    if (rc != RT_OK) return rc;
  }

  mark("peer gather setup");
  // scene: converted once when its bytes changed, cloned to every context
  std::vector<char> sb;
  scene_bytes(scene, sb);
  bool reuse = true;
  {
    std::vector<char> stale(N, 0);
    for (int d = 0; d < N; d++) {
      stale[d] = slots[d]->scene.empty() || slots[d]->scene != sb || slots[d]->spec != (int)want_spec;
      reuse = reuse && !stale[d];
    }
    rt_context* src = nullptr;
    for (ApiSlot* sl : slots)
      for (int i = 0; i < API_CTX; i++) sl->c[i]->spec_async = async_spec;
    auto set = [&](rt_context* c, bool convert) {
      c->specialize = want_spec;
      c->spec_failed = false;
      int rc = convert ? rt_set_scene(c, scene) : scene_clone(c, src);
      if (rc == RT_E_DEVICE && c->spec_failed && c->has_scene) {  // (a complete scene, generic kernel)
        api_log_spec_failure(c->spec_err);
        rc = RT_OK;
      }
      return rc;
    };
    for (int d = 0; d < N; d++) {
      if (!stale[d]) {
        if (!src) src = slots[d]->c[0];
        continue;
      }
      slots[d]->scene.clear();
    }
    for (int d = 0; d < N; d++) {
      if (!stale[d]) continue;
      for (int i = 0; i < API_CTX; i++) {
        rt_context* c = slots[d]->c[i];
        int rc = set(c, src == nullptr);
        if (rc != RT_OK) return rc;
        if (!src) src = c;
      }
      slots[d]->scene = sb;
      slots[d]->spec = want_spec;
    }
  }
  mark("scene set / clone");
  // reset counters a failed call may have left; the specialised variants the
  // bands will launch queued now (async compiles)
  for (int d = 0; d < N; d++) {
    ApiSlot& sl = *slots[d];
    if (sl.dirty) {
      rt_stats tmp;
      for (int i = 0; i < API_CTX; i++) {
        int rc = rt_read_stats(sl.c[i], sl.st[i], 1, &tmp);
        if (rc != RT_OK) return rc;
      }
      sl.dirty = false;
    }
    sl.dirty = true;  // until this call's counters are read
    for (int k = 0; k + 1 < (int)plan.bounds[d].size(); k++) {  // (the launch's pixel count, as launch() sees it)
      const int j0 = plan.bounds[d][k], j1 = plan.bounds[d][k + 1];
      const uint64_t rows = N == 1 ? (uint64_t)(std::min(H, j1 * TILE) - j0 * TILE) : (uint64_t)(j1 - j0) * TILE;
      spec_prefetch(sl.c[k % API_CTX], (uint64_t)W * rows);
    }
  }

  mark("counters + prefetch");
  // launches: per slot its bands alternating over the two contexts / streams;
  // each band's copy queued behind it
  bool all_spec = true;
  for (int d = 0; d < N; d++) {
    ApiSlot& sl = *slots[d];
    const int nb = (int)plan.bounds[d].size() - 1;
    if (nb <= 0) continue;
    DeviceGuard guard(sl.device);
    HIP_TRY(hipEventRecord(sl.ev_start, sl.st[0]));
    HIP_TRY(hipStreamWaitEvent(sl.st[1], sl.ev_start, 0));
    for (int k = 0; k < nb; k++) {
      const int i = k % API_CTX;
      const int j0 = plan.bounds[d][k], j1 = plan.bounds[d][k + 1];
      int rc;
      if (N == 1) {  // one device: the band's rows (the same pixels as its tile rows)
        const int y0 = j0 * TILE, y1 = std::min(H, j1 * TILE);
        char* dst = out_dev ? (char*)rgba_out + (size_t)y0 * W * 4 : (char*)sl.buf + (size_t)y0 * W * 4;
        rc = rt_render_rows_async(sl.c[i], y0, y1, dst, sl.st[i]);
      } else {
        rc = rt_render_tile_rows_async(sl.c[i], d + j0 * N, N, j1 - j0, (char*)sl.buf + (size_t)j0 * plan.trow_bytes(),
                                       sl.st[i]);
      }
      if (rc != RT_OK) return rc;
      all_spec = all_spec && sl.c[i]->last_spec;
      HIP_TRY(hipEventRecord(sl.band_done[k], sl.st[i]));
      if (gather == RT_GATHER_HOST) {
        HIP_TRY(hipStreamWaitEvent(sl.copy, sl.band_done[k], 0));
        for (const CopyOp& o : band_ops(plan, d, k)) {
          int rc2 = api_dma(o, fr.pinned, (const uint8_t*)sl.buf, sl.copy);
          if (rc2 != RT_OK) return rc2;
        }
        HIP_TRY(hipEventRecord(sl.copy_done[k], sl.copy));
      } else if (d > 0) {  // xGMI: the band's packed bytes to the first device's staging buffer
        HIP_TRY(hipStreamWaitEvent(sl.copy, sl.band_done[k], 0));
        const size_t off = (size_t)j0 * plan.trow_bytes();
        HIP_TRY(hipMemcpyPeerAsync((char*)fr.staging + stage_off[d] + off, root, (char*)sl.buf + off, sl.device,
                                   plan.band_bytes(d, k), sl.copy));
        HIP_TRY(hipEventRecord(sl.copy_done[k], sl.copy));
      }
    }
    // the slot's GPU span: its first band's start to its last band's end
    for (int k = std::max(0, nb - 2); k < nb; k++) HIP_TRY(hipStreamWaitEvent(sl.st[0], sl.band_done[k], 0));
    HIP_TRY(hipEventRecord(sl.ev_end, sl.st[0]));
  }
  if (gather == RT_GATHER_PEER && !(out_dev && N == 1)) {
    // the first device de-interleaves every band into the frame as it arrives
    DeviceGuard guard(root);
    uint8_t* frame = out_dev ? rgba_out : (uint8_t*)fr.frame;
    for (int k = 0; k < API_MAX_BANDS; k++)
      for (int d = 0; d < N; d++) {
        if (k + 1 >= (int)plan.bounds[d].size()) continue;
        ApiSlot& sl = *slots[d];
        const int j0 = plan.bounds[d][k], j1 = plan.bounds[d][k + 1];
        HIP_TRY(hipStreamWaitEvent(fr.gather, d == 0 ? sl.band_done[k] : sl.copy_done[k], 0));
        const char* src = d == 0 ? (const char*)sl.buf + (size_t)j0 * plan.trow_bytes()
                                 : (const char*)fr.staging + stage_off[d] + (size_t)j0 * plan.trow_bytes();
        hipLaunchKernelGGL(rt_scatter_tile_rows, dim3(32, j1 - j0), dim3(256), 0, fr.gather, (uint32_t*)frame,
                           (const uint32_t*)src, W, H, d, N, j0);
        HIP_TRY(hipGetLastError());
      }
    if (!out_dev) HIP_TRY(hipMemcpyAsync(fr.pinned, fr.frame, frame_bytes, hipMemcpyDeviceToHost, fr.gather));
    HIP_TRY(hipEventRecord(fr.gather_done, fr.gather));
  }
  mark("launches");
  const auto t_launched = clk::now();

  // host side: finished bands copied on to rgba_out while later ones render
  const int threads = std::max(1, env_int("RT_RENDER_COPY_THREADS", 4));
  auto copy_band = [&](int d, int k) -> int {
    HIP_TRY(hipEventSynchronize(slots[d]->copy_done[k]));
    par_copy_ranges(rgba_out, fr.pinned, band_ranges(plan, d, k), threads);
    return RT_OK;
  };
  if (gather == RT_GATHER_HOST)
    for (int k = 0; k < API_MAX_BANDS; k++)
      for (int d = 0; d < N; d++)
        if (k + 2 < (int)plan.bounds[d].size()) {  // (every band but each slot's last)
          int rc = copy_band(d, k);
          if (rc != RT_OK) return rc;
        }
  for (int d = 0; d < N; d++)
    if (plan.bounds[d].size() > 1) HIP_TRY(hipEventSynchronize(slots[d]->ev_end));
  const auto t_rendered = clk::now();
  if (gather == RT_GATHER_HOST) {
    for (int d = 0; d < N; d++)
      if (plan.bounds[d].size() > 1) {
        int rc = copy_band(d, (int)plan.bounds[d].size() - 2);
        if (rc != RT_OK) return rc;
      }
  } else if (!(out_dev && N == 1)) {
    HIP_TRY(hipEventSynchronize(fr.gather_done));
    if (!out_dev) par_copy_ranges(rgba_out, fr.pinned, {{0, frame_bytes}}, threads);
  }

  // counters of every context, read and reset; per-device spans
  rt_stats sum;
  std::memset(&sum, 0, sizeof sum);
  sum.devices = N;
  double gmax = 0;
  for (int d = 0; d < N; d++) {
    ApiSlot& sl = *slots[d];
    for (int i = 0; i < API_CTX; i++) {
      rt_stats s;
      int rc = rt_read_stats(sl.c[i], sl.st[i], 1, &s);
      if (rc != RT_OK) return rc;
      add_stats(sum, s);
    }
    sl.dirty = false;
    float gms = 0.f;
    if (plan.bounds[d].size() > 1) {
      DeviceGuard guard(sl.device);
      HIP_TRY(hipEventElapsedTime(&gms, sl.ev_start, sl.ev_end));
    }
    sum.device_kernel_ms[d] = gms;
    gmax = std::max(gmax, (double)gms);
  }
  const auto t_end = clk::now();
  sum.kernel_ms = gmax;
  sum.gather_ms = ms_since(t_rendered, t_end);
  if (stats) *stats = sum;
  for (int d = 0; d < N; d++)
    for (int i = 0; i < API_CTX; i++)
      if (slots[d]->c[i]->spec_failed) api_log_spec_failure(slots[d]->c[i]->spec_err);
  rt_render_timing& tm = g_api_timing;
  tm.total_ms = ms_since(t0, t_end);
  tm.setup_ms = ms_since(t0, t_launched);
  tm.render_wait_ms = ms_since(t_launched, t_rendered);
  tm.copy_tail_ms = ms_since(t_rendered, t_end);
  tm.gpu_ms = gmax;
  tm.bands = plan.bands();
  tm.scene_reused = reuse ? 1 : 0;
  tm.specialized = (want_spec && all_spec) ? 1 : 0;
  tm.devices = N;
  tm.pending_compiles = want_spec ? spec_jobs_pending() : 0;
  return RT_OK;
}

int rt_debug_assemble(int width, int height, int ndev, int bands, const uint8_t* const* shares, uint8_t* out) {
  if (width <= 0 || height <= 0 || ndev <= 0 || ndev > RT_MAX_DEVICES || bands < 0 || bands > API_MAX_BANDS || !shares || !out)
    return fail(RT_E_INVALID, "rt_debug_assemble: bad arguments");
  const ApiPlan plan = api_plan(width, height, ndev, bands);
  std::vector<uint8_t> pinned((size_t)width * height * 4, 0);
  // the device path's DMA runs (here memcpy per row) into the frame, then its
  // host copies band by band: every band but each slot's last, then the last
  for (int d = 0; d < ndev; d++)
    for (int k = 0; k + 1 < (int)plan.bounds[d].size(); k++)
      for (const CopyOp& o : band_ops(plan, d, k))
        for (size_t h = 0; h < o.height; h++)
          std::memcpy(pinned.data() + o.dst + h * o.dpitch, shares[d] + o.src + h * o.spitch, o.width);
  for (int k = 0; k < API_MAX_BANDS; k++)
    for (int d = 0; d < ndev; d++)
      if (k + 1 < (int)plan.bounds[d].size()) par_copy_ranges(out, pinned.data(), band_ranges(plan, d, k), 2);
  return RT_OK;
}

}  // extern "C"

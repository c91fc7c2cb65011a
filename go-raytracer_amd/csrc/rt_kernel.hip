// rt_kernel.hip -- MI355X (gfx950) megakernel for the GML raytracer hot path
// plus the C ABI of include/rt_abi.h.
//
// Replaces (timdestan/go-raytracer):
//   raytracer.go:589-682  Render: camera, PCG jitter, 4-sample AA, quantise
//   raytracer.go:469-562  closestHit / traceRay (recursion -> explicit stack)
//   raytracer.go:372-467  computeLighting / inShadow / refract / fresnel
//   raytracer.go:51-370   Sphere/Plane/Cube/Cylinder Intersect + surface props
//   raytracer.go:724-830  scene conversion (host side, below)
//
// Execution model
//   * Persistent 256-thread workgroups = 4 independent wave64s sharing one
//     LDS copy of the scene (staged once per workgroup; large scenes stay in
//     HBM/L2 and are read with wave-uniform scalar loads).
//   * Each LANE owns one pixel at a time and runs the reference's recursion
//     as a state machine over an explicit per-lane frame stack
//     (lane-interleaved in HBM, so pushes/pops are coalesced rows).
//   * Lanes alternate between a TRACE pass (closestHit of the lane's current
//     ray against every object) and a SHADE pass (surface props, lighting with
//     shadow rays, reflection/refraction set-up). A wave only runs the SHADE
//     pass once enough of its lanes hold a hit, so shading -- the expensive
//     part -- runs with mostly-full lanes; lanes whose ray missed resolve
//     their background colour and immediately trace their next ray.
//   * Idle lanes are refilled from a per-wave pool of 64 contiguous pixels
//     (one 8x8 tile) taken from a global atomic queue: the analogue of the
//     reference's channel of (column, 20-row) work items
//     (raytracer.go:611-677), with per-lane granularity.
//   * Object loops are wave-uniform (brute force over the flattened object
//     list, exactly like closestHit), so object records are broadcast reads
//     and the primitive-kind switch never diverges.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <hip/hiprtc.h>
#include <sys/syscall.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <thread>
#include <cmath>
#include <array>
#include <cstdio>
#include <utility>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/rt_abi.h"
#include "rt_device.h"

// The generic kernels run at 3 waves/SIMD like the specialised ones
// (RT_MIN_WAVES from rt_render.h). Round 3 had dropped them to 2 after a
// build rendered 14 deep-glass tiles of a reduced C4 frame wrong in the
// serial-sample schedule; rebuilding that tree at 3 waves with each of its two
// candidate fixes (profiles/r04/generic/) reproduced the failure exactly
// without the fixes and with the t0/t1 initialisation alone, and removed it
// with the BVH stack push from every active lane (WaveStack::push) alone: a
// push written by lane 0 only was lost whenever lane 0 was inactive there.
// At 3 waves the generic C3 kernel takes 4.61 ms instead of 5.51 (C2 0.44
// instead of 0.49), GPU suite green.
#include "rt_render.h"
#include "rt_jit_src.inc"

// Diagnostic: run surface program `prog` of the current scene on n inputs.
__global__ void rt_debug_vm_kernel(const char* __restrict__ blob, int off_code, int off_consts, int off_entry, int prog,
                                   const long long* face, const double* u, const double* v, double* out, int* err,
                                   int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* code = reinterpret_cast<const uint32_t*>(blob + off_code);
  const uint64_t* consts = reinterpret_cast<const uint64_t*>(blob + off_consts);
  const int* entry = reinterpret_cast<const int*>(blob + off_entry);
  err[i] = run_vm(code, consts, entry[prog], face[i], u[i], v[i], out + (size_t)i * 10) ? 1 : 0;
}

// The ahead-of-time flavours: <scene in LDS, BVH, CSG, pixel quads>, indexed
// by kernel_index(); launch() picks one per scene.
constexpr int kernel_index(bool lds, bool bvh, bool csg, bool quads) {
  return (lds ? 1 : 0) | (bvh ? 2 : 0) | (csg ? 4 : 0) | (quads ? 8 : 0);
}
template <int I>
constexpr const void* kernel_at() {
  return (const void*)rt_render_kernel<(I & 1) != 0, (I & 2) != 0, (I & 4) != 0, (I & 8) != 0>;
}
template <int... I>
constexpr std::array<const void*, sizeof...(I)> kernel_table(std::integer_sequence<int, I...>) {
  return {kernel_at<I>()...};
}
const std::array<const void*, 16> k_kernels = kernel_table(std::make_integer_sequence<int, 16>{});
// ===========================================================================
// Host side: scene conversion (raytracer.go:724-830) and the C ABI
// ===========================================================================
namespace {

// The process environment as it was when this library loaded. Python's
// os.environ (putenv / unsetenv) reallocates the environment array and frees
// the strings it replaces while this library's calls run without the GIL
// (ctypes releases it), and glibc's getenv takes no lock, so reading
// `environ` or calling getenv during a call can touch freed memory: the
// environment-race GPU test (tests/test_gpu_render_ex.py) segfaulted that way
// once in round 6, in the per-call band-plan lookup. The library reads its
// knobs (rt_getenv), and gives the compile helper and the in-process
// compiler's namespace, this load-time copy only; environment changes made
// after the library is loaded do not reach it (set RT_* knobs before loading).
struct EnvSnap {
  std::vector<std::string> s;
  std::vector<char*> p;  // execve-style array into s
};
EnvSnap* env_snap() {
  static EnvSnap* e = [] {
    EnvSnap* x = new EnvSnap;  // (never freed: pointers into it are handed out)
    for (char** v = environ; v && *v; ++v) x->s.emplace_back(*v);
    for (auto& t : x->s) x->p.push_back(&t[0]);
    x->p.push_back(nullptr);
    return x;
  }();
  return e;
}
__attribute__((constructor)) void env_snap_at_load() { (void)env_snap(); }
const char* rt_getenv(const char* name) {
  const size_t n = strlen(name);
  for (const std::string& t : env_snap()->s)
    if (t.size() > n && t[n] == '=' && t.compare(0, n, name) == 0) return t.c_str() + n + 1;
  return nullptr;
}

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(RT_E_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

struct M4 {
  double m[4][4];
};

M4 ident() {
  M4 r;
  std::memset(&r, 0, sizeof r);
  r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1.0;
  return r;
}

// prim.Mat4.Inverse (vec.go:319-365)
bool inverse(const M4& M, M4& inv) {
  const double(*m)[4] = M.m;
  double a = m[0][0], b = m[0][1], c = m[0][2];
  double d = m[1][0], e = m[1][1], f = m[1][2];
  double g = m[2][0], h = m[2][1], i = m[2][2];
  double det = a * (e * i - f * h) - b * (d * i - f * g) + c * (d * h - e * g);
  if (det == 0.0) return false;
  inv.m[0][0] = (e * i - f * h) / det;
  inv.m[0][1] = (c * h - b * i) / det;
  inv.m[0][2] = (b * f - c * e) / det;
  inv.m[1][0] = (f * g - d * i) / det;
  inv.m[1][1] = (a * i - c * g) / det;
  inv.m[1][2] = (c * d - a * f) / det;
  inv.m[2][0] = (d * h - e * g) / det;
  inv.m[2][1] = (b * g - a * h) / det;
  inv.m[2][2] = (a * e - b * d) / det;
  inv.m[3][0] = inv.m[3][1] = inv.m[3][2] = 0.0;
  inv.m[3][3] = 1.0;
  inv.m[0][3] = -(inv.m[0][0] * m[0][3] + inv.m[0][1] * m[1][3] + inv.m[0][2] * m[2][3]);
  inv.m[1][3] = -(inv.m[1][0] * m[0][3] + inv.m[1][1] * m[1][3] + inv.m[1][2] * m[2][3]);
  inv.m[2][3] = -(inv.m[2][0] * m[0][3] + inv.m[2][1] * m[1][3] + inv.m[2][2] * m[2][3]);
  return true;
}

// createPlane's NormalWorld = WorldToObject^T.MulDir(normal).Normalize() and
// D = -normal.Dot(point) (raytracer.go:764-774).
void plane_consts(const M4& w2o, const double pt[3], const double n[3], double nw[3], double* dval) {
  // Transpose then MulDir: row i of W2O^T is column i of W2O.
  double x = w2o.m[0][0] * n[0] + w2o.m[1][0] * n[1] + w2o.m[2][0] * n[2];
  double y = w2o.m[0][1] * n[0] + w2o.m[1][1] * n[1] + w2o.m[2][1] * n[2];
  double z = w2o.m[0][2] * n[0] + w2o.m[1][2] * n[1] + w2o.m[2][2] * n[2];
  double mag = std::sqrt(x * x + y * y + z * z);
  nw[0] = x / mag;
  nw[1] = y / mag;
  nw[2] = z / mag;
  *dval = -(n[0] * pt[0] + n[1] * pt[1] + n[2] * pt[2]);
}

// prim.PlanesForUnitCube (internal/prim/plane.go:29-38)
const double kCubePt[6][3] = {{0, 0, 0}, {0, 0, 1}, {0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 0}};
const double kCubeN[6][3] = {{0, 0, -1}, {0, 0, 1}, {-1, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, -1, 0}};

// Go math.Tan (tan.go), Sin/Cos (sin.go): Cephes, Cody-Waite reduction.
const double kSin[6] = {1.58962301576546568060e-10, -2.50507477628578072866e-8, 2.75573136213857245213e-6,
                        -1.98412698295895385996e-4, 8.33333333332211858878e-3, -1.66666666666666307295e-1};
const double kCos[6] = {-1.13585365213876817300e-11, 2.08757008419747316778e-9, -2.75573141792967388112e-7,
                        2.48015872888517045348e-5,   -1.38888888888730564116e-3, 4.16666666666665929218e-2};
const double kPI4A = 7.85398125648498535156e-1, kPI4B = 3.77489470793079817668e-8,
             kPI4C = 2.69515142907905952645e-15, k4OverPi = 1.2732395447351628;

double poly_sin(double z, double zz) {
  return z + z * zz * ((((((kSin[0] * zz) + kSin[1]) * zz + kSin[2]) * zz + kSin[3]) * zz + kSin[4]) * zz + kSin[5]);
}
double poly_cos(double zz) {
  return 1.0 - 0.5 * zz + zz * zz * ((((((kCos[0] * zz) + kCos[1]) * zz + kCos[2]) * zz + kCos[3]) * zz + kCos[4]) * zz + kCos[5]);
}
bool reduce(double x, uint64_t& j, double& z) {  // x >= 0
  if (x >= (double)(1 << 29)) return false;        // Payne-Hanek range: not restated
  j = (uint64_t)(x * k4OverPi);
  double y = (double)j;
  if (j & 1) {
    j++;
    y++;
  }
  z = ((x - y * kPI4A) - y * kPI4B) - y * kPI4C;
  return true;
}
bool go_sin(double x, double& out) {
  if (x == 0 || std::isnan(x)) { out = x; return true; }
  if (std::isinf(x)) { out = NAN; return true; }
  bool sign = false;
  if (x < 0) { x = -x; sign = true; }
  uint64_t j;
  double z;
  if (!reduce(x, j, z)) return false;
  j &= 7;
  if (j > 3) { sign = !sign; j -= 4; }
  double zz = z * z;
  double y = (j == 1 || j == 2) ? poly_cos(zz) : poly_sin(z, zz);
  out = sign ? -y : y;
  return true;
}
bool go_cos(double x, double& out) {
  if (std::isnan(x) || std::isinf(x)) { out = NAN; return true; }
  bool sign = false;
  x = std::fabs(x);
  uint64_t j;
  double z;
  if (!reduce(x, j, z)) return false;
  j &= 7;
  if (j > 3) { j -= 4; sign = !sign; }
  if (j > 1) sign = !sign;
  double zz = z * z;
  double y = (j == 1 || j == 2) ? poly_sin(z, zz) : poly_cos(zz);
  out = sign ? -y : y;
  return true;
}
bool go_tan(double x, double& out) {
  static const double P[3] = {-1.30936939181383777646e4, 1.15351664838587416140e6, -1.79565251976484877988e7};
  static const double Q[5] = {1.0, 1.36812963470692954678e4, -1.32089234440210967447e6, 2.50083801823357915839e7,
                              -5.38695755929454629881e7};
  if (x == 0 || std::isnan(x)) { out = x; return true; }
  if (std::isinf(x)) { out = NAN; return true; }
  bool sign = false;
  if (x < 0) { x = -x; sign = true; }
  uint64_t j;
  double z;
  if (!reduce(x, j, z)) return false;
  double zz = z * z;
  double y;
  if (zz > 1e-14)
    y = z + z * (zz * (((P[0] * zz) + P[1]) * zz + P[2]) / ((((zz + Q[1]) * zz + Q[2]) * zz + Q[3]) * zz + Q[4]));
  else
    y = z;
  if (j & 2) y = -1 / y;
  out = sign ? -y : y;
  return true;
}

struct DevScene {
  int width = 0, height = 0, depth = 0, nobj = 0, nlights = 0, nmats = 0;
  int pow_bits = 7;  // bit length of the largest integer specular exponent in 2..64 (7 with surface programs)
  double vw = 0, vh = 0;
  double amb[3] = {0, 0, 0}, bg0[3] = {0, 0, 0}, bg1[3] = {0, 0, 0};
  char* blob = nullptr;
  int blob_bytes = 0;
  int off_geo = 0, off_shade = 0, off_mats = 0, off_lights = 0, off_kind = 0, off_objmat = 0, off_prefb = 0,
      off_csg = 0;
  bool has_csg = false;
  std::vector<int> kinds;  // host copy for the per-kind test counts
  int off_code = 0, off_consts = 0, off_entry = 0, num_programs = 0;
  // BVH flavour: one device buffer nodes | leaf objects | planes | prefix counts
  char* accel = nullptr;
  bool use_bvh = false;
  int nplanes = 0, nnodes = 0, kind_mask = 0;
  int light_mask = 0;  // bit k: the scene has lights of kind k (RT_LIGHT_*)
  bool branching = false;  // some material is reflective and transparent, or a surface program may make one
  int leaf_kind_mask = 0;  // bit k: some CSG leaf has kind k
  size_t off_nodes = 0, off_bobj = 0, off_planes = 0, off_runs = 0, off_arec = 0, off_urec = 0;
  double bvh_lo[3] = {0, 0, 0}, bvh_hi[3] = {0, 0, 0};  // padded box of the BVH objects (far_shift)
  int nruns = 0;
  // host copies of what blob and accel hold: another context (the rt_render
  // seam's second context, another device) takes the converted scene from
  // here instead of converting it again (scene_clone)
  std::vector<char> h_blob, h_accel;
};

// A sphere whose WorldToObject is a scale + translation (rt_render.h
// AXIS_REC): off-diagonal entries +-0, diagonal magnitudes in [2^-100, 2^100],
// translations finite and non-zero. Its rayToObjectSpace (vec.go:298-313) then
// equals the diagonal form bit for bit on rays that axis_ray_ok accepts.
bool axis_sphere(const double* m) {
  for (int q : {1, 2, 4, 6, 8, 9})
    if (m[q] != 0.0) return false;
  for (int q : {0, 5, 10}) {
    const double a = std::fabs(m[q]);
    if (!(a >= 0x1p-100 && a <= 0x1p100)) return false;
  }
  for (int q : {3, 7, 11})
    if (!std::isfinite(m[q]) || m[q] == 0.0) return false;
  return true;
}

#ifndef RT_BVH_SAH
#define RT_BVH_SAH 1  // binned-SAH splits (median split when degenerate)
#endif
// Scenes with at least this many bounded objects use the BVH flavour.
#ifndef RT_FAR_MIN_OBJ
#define RT_FAR_MIN_OBJ 1024  // BVH scenes from this many objects keep the far-origin shift when specialised
#endif
#ifndef RT_BVH_LEAF
#define RT_BVH_LEAF 4  // objects per BVH leaf (<= 7: the leaf ref holds the count in 3 bits)
#endif
#ifndef RT_BVH_MIN
#define RT_BVH_MIN 12
#endif

float f_down(double x) {
  float f = (float)x;
  return (double)f > x ? std::nextafter(f, -std::numeric_limits<float>::infinity()) : f;
}
float f_up(double x) {
  float f = (float)x;
  return (double)f < x ? std::nextafter(f, std::numeric_limits<float>::infinity()) : f;
}

// Median-split BVH over the bounded objects' padded bounding spheres (boxes
// rounded outwards to FP32). Median splits keep the depth at ~log2(n / 4), far
// below the device stack (BVH_STACK entries); leaves hold <= 4 objects in
// ascending index order, copied (geo record + index + kind) into leaf order.
struct BvhBuild {
  const std::vector<double>* c;  // [n][3] centres
  const std::vector<double>* r;  // [n] radii
  const std::vector<double>* geo;
  const std::vector<int>* kind;
  std::vector<int> ord;          // object indices
  std::vector<float> nodes;      // [m][BN]
  std::vector<double> leaf_geo;  // [n][GEO] in leaf order
  int max_depth = 0;

  struct Sub {
    int ref;
    float box[6];
    int minidx;
  };
  Sub build(int lo, int hi, int depth) {
    max_depth = std::max(max_depth, depth);
    Sub out;
    double bl[3] = {1e300, 1e300, 1e300}, bh[3] = {-1e300, -1e300, -1e300};
    double cl[3] = {1e300, 1e300, 1e300}, ch[3] = {-1e300, -1e300, -1e300};
    out.minidx = 0x7fffffff;
    for (int j = lo; j < hi; j++) {
      const int i = ord[j];
      out.minidx = std::min(out.minidx, i);
      for (int k = 0; k < 3; k++) {
        const double cc = (*c)[(size_t)i * 3 + k], rr = (*r)[i];
        bl[k] = std::min(bl[k], cc - rr);
        bh[k] = std::max(bh[k], cc + rr);
        cl[k] = std::min(cl[k], cc);
        ch[k] = std::max(ch[k], cc);
      }
    }
    for (int k = 0; k < 3; k++) {
      out.box[k] = f_down(bl[k]);
      out.box[3 + k] = f_up(bh[k]);
    }
    if (hi - lo <= RT_BVH_LEAF) {
      std::sort(ord.begin() + lo, ord.begin() + hi);
      const int first = (int)(leaf_geo.size() / GEO);
      for (int j = lo; j < hi; j++) {
        const int i = ord[j];
        leaf_geo.insert(leaf_geo.end(), geo->begin() + (size_t)i * GEO, geo->begin() + (size_t)(i + 1) * GEO);
        int* gi = reinterpret_cast<int*>(&leaf_geo[leaf_geo.size() - GEO + 14]);
        gi[0] = i;
        // scale + translation sphere: the kernel may take the diagonal transform (rt_render.h axis_o)
        gi[1] = (*kind)[i] == RT_SPHERE && axis_sphere(&(*geo)[(size_t)i * GEO]) ? 1 : 0;
        gi[2] = (*kind)[i];
        gi[3] = 0;
      }
      out.ref = (first << 3) | (hi - lo);
      return out;
    }
    int axis = 0;
    for (int k = 1; k < 3; k++)
      if (ch[k] - cl[k] > ch[axis] - cl[axis]) axis = k;
    int mid = -1;
#if RT_BVH_SAH
    // Binned SAH over the centroids (16 bins per axis): minimise
    // area(left) * n(left) + area(right) * n(right); down to the median split
    // when every centroid lands in one bin or below depth 40 (keeps the depth,
    // hence the device stack, bounded).
    if (depth < 40) {
      enum { NB = 16 };
      double best = 1e300;
      int bax = -1, bbin = -1;
      for (int ax = 0; ax < 3; ax++) {
        const double ext = ch[ax] - cl[ax];
        if (!(ext > 0.0)) continue;
        double blo[NB][3], bhi[NB][3];
        int bn[NB] = {0};
        for (int q = 0; q < NB; q++)
          for (int k = 0; k < 3; k++) {
            blo[q][k] = 1e300;
            bhi[q][k] = -1e300;
          }
        for (int j = lo; j < hi; j++) {
          const int i = ord[j];
          int q = (int)((((*c)[(size_t)i * 3 + ax]) - cl[ax]) / ext * NB);
          q = q < 0 ? 0 : (q >= NB ? NB - 1 : q);
          bn[q]++;
          for (int k = 0; k < 3; k++) {
            blo[q][k] = std::min(blo[q][k], (*c)[(size_t)i * 3 + k] - (*r)[i]);
            bhi[q][k] = std::max(bhi[q][k], (*c)[(size_t)i * 3 + k] + (*r)[i]);
          }
        }
        auto area = [](const double* l, const double* h) {
          const double dx = h[0] - l[0], dy = h[1] - l[1], dz = h[2] - l[2];
          return dx < 0 ? 0.0 : dx * dy + dy * dz + dz * dx;
        };
        double rl[NB][3], rh[NB][3];
        int rn[NB];
        double al[3] = {1e300, 1e300, 1e300}, ah[3] = {-1e300, -1e300, -1e300};
        int an = 0;
        for (int q = NB - 1; q >= 0; q--) {
          for (int k = 0; k < 3; k++) {
            al[k] = std::min(al[k], blo[q][k]);
            ah[k] = std::max(ah[k], bhi[q][k]);
            rl[q][k] = al[k];
            rh[q][k] = ah[k];
          }
          an += bn[q];
          rn[q] = an;
        }
        double ll[3] = {1e300, 1e300, 1e300}, lh[3] = {-1e300, -1e300, -1e300};
        int ln = 0;
        for (int q = 0; q < NB - 1; q++) {
          for (int k = 0; k < 3; k++) {
            ll[k] = std::min(ll[k], blo[q][k]);
            lh[k] = std::max(lh[k], bhi[q][k]);
          }
          ln += bn[q];
          if (ln == 0 || rn[q + 1] == 0) continue;
          const double cost = area(ll, lh) * ln + area(rl[q + 1], rh[q + 1]) * rn[q + 1];
          if (cost < best) {
            best = cost;
            bax = ax;
            bbin = q;
          }
        }
      }
      if (bax >= 0) {
        const double ext = ch[bax] - cl[bax];
        auto it = std::partition(ord.begin() + lo, ord.begin() + hi, [&](int i) {
          int q = (int)((((*c)[(size_t)i * 3 + bax]) - cl[bax]) / ext * NB);
          q = q < 0 ? 0 : (q >= NB ? NB - 1 : q);
          return q <= bbin;
        });
        mid = (int)(it - ord.begin());
        if (mid <= lo || mid >= hi) mid = -1;
      }
    }
#endif
    if (mid < 0) {
      mid = (lo + hi) / 2;
      std::nth_element(ord.begin() + lo, ord.begin() + mid, ord.begin() + hi, [&](int a, int b) {
        const double ca = (*c)[(size_t)a * 3 + axis], cb = (*c)[(size_t)b * 3 + axis];
        return ca < cb || (ca == cb && a < b);
      });
    }
    const int node = (int)(nodes.size() / BN);
    nodes.resize(nodes.size() + BN, 0.0f);
    const Sub l = build(lo, mid, depth + 1);
    const Sub rr = build(mid, hi, depth + 1);
    float* nb = &nodes[(size_t)node * BN];
    for (int k = 0; k < 6; k++) {
      nb[k] = l.box[k];
      nb[6 + k] = rr.box[k];
    }
    int* ni = reinterpret_cast<int*>(nb + 12);
    ni[0] = l.ref;
    ni[1] = rr.ref;
    ni[2] = l.minidx;
    ni[3] = rr.minidx;
    out.ref = node << 3;
    return out;
  }
};

int align16(int v) { return (v + 15) & ~15; }

}  // namespace

// What a specialised kernel is compiled for. Serialised as the cache key
// "lds:bvh:csg:nobj:kinds:kmask:feat"; nobj > 0 (kinds = "k0,k1,...") unrolls the
// object loops of a small linear LDS scene, nobj = 0 only fixes the kind mask
// and the feature bits (BVH, global-memory and larger linear scenes).
struct SpecKey {
  int lds = 1, bvh = 0, csg = 0, nobj = 0;
  std::string kinds;
  int kmask = 0, feat = 0, nlights = 0;  // nlights > 0: light loop unrolled for that count
  int pow_bits = 7;                      // unrolled specular powering steps
  int nocull = 0;                        // rt_set_accel without RT_ACCEL_CULL: -DRT_CULL=0
  int quads = 0;                         // pixel schedule: SCH_SERIAL / SCH_QUADS / SCH_PAIRS (pick_schedule)
  int share = 0;                         // work sharing at the tail (rt_set_work_sharing): -DRT_SHARE=<mode>
  int far = 1;                           // 0: -DRT_FAR_SHIFT=0 (BVH scenes below RT_FAR_MIN_OBJ objects)
  std::string str() const {
    return std::to_string(lds) + ":" + std::to_string(bvh) + ":" + std::to_string(csg) + ":" + std::to_string(nobj) + ":" + kinds + ":" +
           std::to_string(kmask) + ":" + std::to_string(feat) + ":" + std::to_string(nlights) + ":" + std::to_string(pow_bits) +
           ":" + std::to_string(nocull) + ":" + std::to_string(quads) + ":" + std::to_string(share) + ":" + std::to_string(far);
  }
};

// Launch configuration of one (kernel, fixed LDS, frames) combination.
struct LaunchPlan {
  const void* fn = nullptr;
  int shmem_fixed = -1, frames = 0, per_cu = 0, lds_levels = 0, lds_full = 0;
};

struct rt_context {
  int device = 0;
  int last_waves = 0, launches = 0;  // diagnostics (RT_PHASE_TIMING wave lifetimes)
  int sched = RT_SCHED_AUTO;         // rt_set_schedule
  int inflight = 1;                  // rt_set_frames_in_flight: launches overlap other contexts' launches
  LaunchPlan plan;                   // last launch's occupancy / LDS plan
  unsigned long long* wdiag = nullptr;  // diagnostic build: per-wave lifetimes (RT_PHASE_TIMING)
  int cus = 0;
  int lds_per_cu = 0, lds_per_block = 0;  // bytes (device properties)
  int grid_lds = 0, grid_glb = 0;  // persistent grids (workgroups) per kernel flavour
  DevScene sc;
  bool has_scene = false;
  uint64_t* jump = nullptr;
  unsigned int* queue = nullptr;  // two sets of QHEADS queue heads (launches alternate)
  int qset = 0;                    // the set the next launch dequeues from
  unsigned long long* stats = nullptr;
  unsigned long long* stats_part = nullptr;  // [workgroup slot][STATS_PART] frame counters (Params::stats_part)
  int stats_parts = 0;                       // workgroup slots (cus * 8: any persistent grid)
  double* stack = nullptr;
  double* vm_global = nullptr;  // per-lane VM material records (global flavour)
  size_t vm_global_bytes = 0;
  size_t stack_bytes = 0;
  int stack_waves = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  char* ssim_buf = nullptr;  // SSIM kernel weights + per-block partial sums
  size_t ssim_bytes = 0;
  uint64_t primary_pending = 0;  // host-side count of launched primary rays
  hipStream_t last_stream = nullptr;  // stream of the previous launch (queue-set ordering)
  bool launched = false;
  // Tile order (rt_set_tile_order): at scene setup one centre sample per frame
  // tile is traced (estimate launch); launches then deal their tiles most
  // expensive first, so the end of a launch is made of cheap tiles.
  bool order_on = true;
  int share_mode = RT_SHARE_AUTO;  // rt_set_work_sharing (specialised kernels only)
  // device-wide sharing (RT_SHARE_DEVICE): slots per (wave slot, lane, level),
  // the ring of posted slot ids and its head / tail tickets (rt_render.h gs_*)
  uint64_t* gboard = nullptr;
  uint64_t* gring = nullptr;
  uint64_t* gctl = nullptr;
  size_t gslots = 0;  // slots gboard holds (stack_waves * 64 * frames of its layout)
  int gframes = 0;    // frames per lane of that layout
  unsigned int* est = nullptr;              // device: rays traced per frame tile
  size_t est_cap = 0;                       // tiles est can hold
  unsigned long long* est_stats = nullptr;  // the estimate launch's counters (discarded)
  std::vector<uint32_t> tile_cost;          // host copy (empty: no order)
  double order_ms = 0;                      // the estimate's wall time at scene setup
  std::map<std::array<int, 5>, unsigned int*> orders;  // device tile order per launch shape
  // scene specialisation (rt_set_specialize)
  bool specialize = false;
  int accel = RT_ACCEL_BVH | RT_ACCEL_CULL;  // rt_set_accel
  hipFunction_t spec_fn = nullptr;  // specialised kernel of the current scene, if any
  std::map<int, hipFunction_t> spec_alt;  // ... for other (schedule, work sharing) pairs (spec_for)
  SpecKey spec_key;                     // what spec_fn was compiled for
  double spec_ms = 0;               // hipRTC compile time of spec_fn (0 = cache hit)
  // The rt_render seam's contexts compile in the background (spec_build
  // async): until the scene's kernel is ready, launches run the generic one.
  bool spec_async = false;
  bool spec_fallback = false;  // a failed compile leaves the generic kernel instead of failing the launch
  bool spec_pending = false;   // the scene's specialised kernel is still compiling
  bool spec_failed = false;    // its compile (or one of a launch's schedule variants) failed
  std::string spec_err;        // ... with this message
  bool last_spec = false;      // the last render launch ran a specialised kernel
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

void free_scene(DevScene& s) {
  (void)hipFree(s.blob);
  (void)hipFree(s.accel);
  s = DevScene();
}

void clear_orders(rt_context* c) {
  for (auto& kv : c->orders) (void)hipFree(kv.second);
  c->orders.clear();
  c->tile_cost.clear();
  c->order_ms = 0;
}

template <typename T>
int upload(T** dst, const std::vector<T>& src) {
  size_t bytes = std::max<size_t>(1, src.size()) * sizeof(T);
  HIP_TRY(hipMalloc((void**)dst, bytes));
  if (!src.empty()) HIP_TRY(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return RT_OK;
}

// ---------------------------------------------------------------------------
// Scene specialisation: the render kernel recompiled through hipRTC with the
// object count and primitive kinds of a small linear scene as compile-time
// constants (RT_SPEC_NOBJ / RT_SPEC_KINDS in rt_render.h), so closestHit's and
// inShadow's object loops unroll with no kind switch. Identical operations in
// identical order: the images and counters are bit-identical to the generic
// kernel (tests/test_gpu_parity.py checks both).
//
// hipRTC is loaded from the ROCm installation into a private link-map
// namespace (dlmopen), so it drives the same compiler as the ahead-of-time
// build even when the host process (PyTorch) already mapped another comgr.
// Compiled code objects are cached per process by specialisation key, loaded
// modules per (device, key).
// ---------------------------------------------------------------------------
enum { SPEC_MAX_OBJ = 8, SPEC_MAX_LIGHTS = 8 };
static_assert(SF_VM == RT_SPEC_SURFACES && SF_LDIR == RT_SPEC_DIRECTIONAL && SF_LSPOT == RT_SPEC_SPOT,
              "feature bits of rt_render.h and include/rt_abi.h");

struct Rtc {
  bool tried = false;
  std::string err;
  decltype(&hiprtcCreateProgram) create = nullptr;
  decltype(&hiprtcAddNameExpression) add_name = nullptr;
  decltype(&hiprtcCompileProgram) compile = nullptr;
  decltype(&hiprtcGetLoweredName) lowered = nullptr;
  decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
  decltype(&hiprtcGetProgramLog) log = nullptr;
  decltype(&hiprtcGetCodeSize) code_size = nullptr;
  decltype(&hiprtcGetCode) code = nullptr;
  decltype(&hiprtcDestroyProgram) destroy = nullptr;
  decltype(&hiprtcGetErrorString) errstr = nullptr;
  // the private namespace's copy of libc's environment pointer (see rtc_sync_env)
  char*** env = nullptr;
};

struct SpecCode {
  std::vector<char> code;
  std::string lowered;
};

// Two locks: g_rtc_mu serialises every use of the hipRTC namespace (its
// loading, the environment copy, a compile: seconds); g_spec_mu guards the
// caches and the background-compile queue below (held for map lookups only,
// so a render never waits for a compile it did not ask to wait for).
std::mutex g_rtc_mu;
std::mutex g_spec_mu;
Rtc g_rtc;
std::map<std::string, SpecCode> g_spec_code;  // entries are never erased (references stay valid)
std::map<std::pair<int, std::string>, hipFunction_t> g_spec_fn;

// Compile state by key (background queue and failures; guarded by g_spec_mu):
// a key that failed once fails again at once, in either mode.
struct SpecJob {
  int state = 0;    // 0 queued or compiling, 1 compiled, -1 failed
  std::string err;  // (failed: the compiler's message)
};
std::map<std::string, SpecJob> g_jobs;

// Caller holds g_rtc_mu.
bool rtc_load() {
  if (g_rtc.tried) return g_rtc.create != nullptr;
  g_rtc.tried = true;
  std::string path;
  if (const char* e = rt_getenv("RT_HIPRTC_LIB")) path = e;
  else path = std::string(rt_getenv("ROCM_PATH") ? rt_getenv("ROCM_PATH") : "/opt/rocm") + "/lib/libhiprtc.so.7";
  void* h = dlmopen(LM_ID_NEWLM, path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    const char* de = dlerror();
    g_rtc.err = "cannot load hipRTC (" + path + "): " + (de ? de : "?");
    return false;
  }
  Rtc r;
  r.tried = true;
#define RTC_SYM(f, n)                                                    \
  r.f = reinterpret_cast<decltype(r.f)>(dlsym(h, n));                    \
  if (!r.f) {                                                            \
    g_rtc.err = std::string("hipRTC symbol missing: ") + n;              \
    return false;                                                        \
  }
  RTC_SYM(create, "hiprtcCreateProgram")
  RTC_SYM(add_name, "hiprtcAddNameExpression")
  RTC_SYM(compile, "hiprtcCompileProgram")
  RTC_SYM(lowered, "hiprtcGetLoweredName")
  RTC_SYM(log_size, "hiprtcGetProgramLogSize")
  RTC_SYM(log, "hiprtcGetProgramLog")
  RTC_SYM(code_size, "hiprtcGetCodeSize")
  RTC_SYM(code, "hiprtcGetCode")
  RTC_SYM(destroy, "hiprtcDestroyProgram")
  RTC_SYM(errstr, "hiprtcGetErrorString")
#undef RTC_SYM
  // The namespace has its own libc, whose environment pointer was set once,
  // when the namespace was created. The host process's setenv / unsetenv
  // (Python's os.environ, pytest's PYTEST_CURRENT_TEST) reallocate the
  // environment array and free the old one, so the private copy can dangle,
  // and the compiler reading its environment then crashed the process (a
  // segfault inside rt_set_scene, seen once in a full GPU test run).
  // rtc_sync_env points it at the library's load-time copy before every
  // compile.
  Lmid_t lm;
  if (dlinfo(h, RTLD_DI_LMID, &lm) == 0) {
    if (void* lc = dlmopen(lm, "libc.so.6", RTLD_NOW | RTLD_NOLOAD)) {
      r.env = reinterpret_cast<char***>(dlsym(lc, "__environ"));
      if (!r.env) r.env = reinterpret_cast<char***>(dlsym(lc, "environ"));
    }
  }
  g_rtc = r;
  return true;
}

// The namespace's environment: the library's load-time copy (env_snap),
// owned by the library and never freed or changed, so neither a host thread's
// setenv nor a compile that keeps pointers getenv gave it can see it move.
// Caller holds g_rtc_mu.
void rtc_sync_env() {
  if (g_rtc.env) *g_rtc.env = env_snap()->p.data();
}


// CSG membership program for the device (csg_eval): the composite's postfix
// program (include/rt_abi.h RT_CSG) with every maximal union-only or
// intersect-only group of leaf operands collapsed into one test of the
// leaves' inside mask -- RT_CSG_ANY (some bit set) / RT_CSG_ALL (all set),
// each followed by four 32-bit words of leaf bits -- and other operands kept
// as they are. Union and intersection are associative and commutative, so the
// boolean result is the original program's; "cube minus a union of 64
// spheres" becomes three steps instead of 129.
void csg_mask_program(const int* code, int len, std::vector<int>& out) {
  struct Node {
    int op, l, r;
  };
  std::vector<Node> nodes;
  std::vector<int> st;
  for (int k = 0; k < len; k++) {
    const int op = code[k];
    if (op >= 0) {
      nodes.push_back({op, -1, -1});
    } else {
      const int r = st.back();
      st.pop_back();
      const int l = st.back();
      st.pop_back();
      nodes.push_back({op, l, r});
    }
    st.push_back((int)nodes.size() - 1);
  }
  std::function<void(int)> emit = [&](int n) {
    const Node& nd = nodes[n];
    if (nd.op >= 0) {
      out.push_back(nd.op);
      return;
    }
    if (nd.op == RT_CSG_DIFFERENCE) {
      emit(nd.l);
      emit(nd.r);
      out.push_back(RT_CSG_DIFFERENCE);
      return;
    }
    std::vector<int> leaves, others;
    std::function<void(int)> flat = [&](int x) {
      if (nodes[x].op == nd.op) {
        flat(nodes[x].l);
        flat(nodes[x].r);
      } else if (nodes[x].op >= 0) {
        leaves.push_back(nodes[x].op);
      } else {
        others.push_back(x);
      }
    };
    flat(n);
    bool first = true;
    if (leaves.size() == 1) {
      out.push_back(leaves[0]);
      first = false;
    } else if (leaves.size() > 1) {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int j : leaves) w[j >> 5] |= 1u << (j & 31);
      out.push_back(nd.op == RT_CSG_UNION ? RT_CSG_ANY : RT_CSG_ALL);
      for (int q = 0; q < 4; q++) out.push_back((int)w[q]);
      first = false;
    }
    for (int x : others) {
      emit(x);
      if (!first) out.push_back(nd.op);
      first = false;
    }
  };
  emit(st.back());
}

// Scene blob staged in LDS (small scenes) or read from global memory with
// wave-uniform scalar loads. RT_SCENE_GLOBAL=1 forces the global flavour
// (tuning experiments only).
// Pixel quads (rt_render.h QUADS): a pixel's 4 samples in 4 lanes at once.
// They pay where the longest pixels, not the total work, set the frame time:
// recursion depth >= 7 (C4, C5, canned, c4csg: the glass trees of the last
// pixels otherwise keep a few waves running long after the rest), and scenes
// with branching materials (reflective and transparent: binary ray trees)
// when a launch gives each lane fewer than 16 pixels -- a strong-scaling
// share of a frame (C3 over 4 / 8 ranks: 1.65 / 1.63 ms serial vs 0.99 /
// 0.55 ms with quads: serially a deep glass pixel's 4 samples alone take
// ~1.6 ms; over 2 ranks, 21 pixels per lane, serial wins: 1.98 vs 2.10 ms,
// c3cone 2.26 vs 2.22, profiles/r03/strong) -- and any scene below 4 pixels
// per lane (C2 over 4 / 8 ranks: 0.22 / 0.19 vs 0.18 / 0.14 ms). Otherwise the
// idle siblings cost more than the balance gains (C3 whole frame 3.44 vs
// 4.39 ms, C2 0.38 vs 0.45 ms).
// With frames in flight (rt_set_frames_in_flight >= 2) the next frame's
// workgroups fill the CUs a launch's tail leaves idle, so for a launch with
// many pixels per lane the cheaper serial schedule wins even at depth >= 7 on
// LDS scenes without CSG when a launch gives each lane >= 32 pixels (C4 whole
// frame, 42 px/lane, two in flight: 4.23 ms serial vs 5.09 ms quads); CSG
// keeps quads (c4csg 23.5 vs 12.8 ms), and so do scenes read from HBM (not
// measured) and launches with fewer pixels per lane.
// rt_set_schedule overrides the choice; so does RT_PIXEL_QUADS=0/1 in the
// environment at process start (experiments).
bool scene_in_lds(const DevScene& s);
bool use_quads(int sched, const DevScene& s, uint64_t pixels, int cus, int inflight) {
  static const int env = rt_getenv("RT_PIXEL_QUADS") ? atoi(rt_getenv("RT_PIXEL_QUADS")) : -1;
  if (env >= 0) return env != 0;
  if (sched == RT_SCHED_PIXEL) return false;
  if (sched == RT_SCHED_QUADS) return true;
  const double lanes = (double)std::max(1, cus) * 4 * 3 * 64;  // 3 waves per SIMD
  if (s.depth >= 7 && inflight > 1 && scene_in_lds(s) && !s.has_csg)
    return (double)pixels < 32.0 * lanes;  // C4 over 2 ranks (21 px/lane): 2.87 ms serial vs 2.44 quads
  return s.depth >= 7 || (double)pixels < (s.branching ? 16.0 : 4.0) * lanes;
}

// Pixel schedules of a launch (SpecKey.quads): serial samples, pixel quads,
// or pixel pairs -- a pixel's samples 0-1 in one lane and 2-3 in its
// neighbour, summed in sample order by the first (specialised kernels only,
// -DRT_PAIRS=1; the generic kernels run quads instead). Pairs are chosen by
// rt_set_schedule(RT_SCHED_PAIRS) or RT_PIXEL_PAIRS=1 in the environment
// (experiments), and by RT_SCHED_AUTO with frames in flight for branching LDS
// scenes without CSG (two in flight, ms per slowest rank's share,
// profiles/r03/pairs/): depth < 7 from 8 to 16 pixels per lane (C3 over 4
// ranks: 0.849 pairs vs 0.937 quads; over 8, 5 px/lane, 0.447 vs 0.451;
// over 2, 21 px/lane, serial 1.575 vs 1.706), depth >= 7 from 16 (C4 whole
// frame 4.15 vs 4.25 serial, over 2 ranks 2.08 vs 2.46 quads; over 4,
// 10 px/lane, quads 1.16 vs 1.39).
enum { SCH_SERIAL = 0, SCH_QUADS = 1, SCH_PAIRS = 2 };
// Work sharing of a launch (SpecKey.share; specialised kernels only).
// RT_SHARE_AUTO (the default) takes the device-wide board (rt_render.h gs_*)
// for CSG scenes of depth >= 7 on launches that leave deep glass trees alone
// at the end: strong-scaling shares (< 16 pixels per lane) and launches
// without frames in flight. c4csg (cube - 64 spheres, 4K, depth 8; ms,
// profiles/r05/gshare/): 8-rank share (two in flight) 4.52 -> 2.24, whole
// frame serially 14.07 -> 11.5, but two whole frames in flight 10.63 ->
// 11.00 (the board's polling and posting cost more than the overlapped tail
// gains), so those keep it off.
int pick_share(int mode, const DevScene& s, uint64_t pixels, int cus, int inflight) {
  if (mode != RT_SHARE_AUTO) return mode;
  const double ppl = (double)pixels / ((double)std::max(1, cus) * 4 * 3 * 64);  // pixels per lane
  return (s.has_csg && s.depth >= 7 && (inflight <= 1 || ppl < 16.0)) ? RT_SHARE_DEVICE : RT_SHARE_OFF;
}

int pick_schedule(int sched, const DevScene& s, uint64_t pixels, int cus, int inflight, bool spec) {
  static const int env = rt_getenv("RT_PIXEL_PAIRS") ? atoi(rt_getenv("RT_PIXEL_PAIRS")) : -1;
  if (env > 0 || sched == RT_SCHED_PAIRS) return SCH_PAIRS;
  static const int qenv = rt_getenv("RT_PIXEL_QUADS") ? atoi(rt_getenv("RT_PIXEL_QUADS")) : -1;
  if (sched == RT_SCHED_AUTO && qenv < 0 && env < 0 && spec && inflight > 1 && scene_in_lds(s) && !s.has_csg &&
      s.branching) {
    const double ppl = (double)pixels / ((double)std::max(1, cus) * 4 * 3 * 64);  // pixels per lane
    if (s.depth >= 7) return ppl >= 16.0 ? SCH_PAIRS : SCH_QUADS;
    if (ppl >= 8.0 && ppl < 16.0) return SCH_PAIRS;
  }
  return use_quads(sched, s, pixels, cus, inflight) ? SCH_QUADS : SCH_SERIAL;
}

bool scene_in_lds(const DevScene& s) {
  static const bool force_global = rt_getenv("RT_SCENE_GLOBAL") && atoi(rt_getenv("RT_SCENE_GLOBAL")) != 0;
  return !force_global && s.blob_bytes <= (int)LDS_MAX_BYTES;
}

// Specialisation of a scene; false when it runs the generic kernel (no
// objects).
bool spec_key(const DevScene& s, SpecKey* k) {
  if (s.nobj < 1) return false;
  k->lds = scene_in_lds(s);
  k->bvh = s.use_bvh;
  k->csg = s.has_csg;
  k->nobj = (!s.use_bvh && !s.has_csg && s.nobj <= SPEC_MAX_OBJ) ? s.nobj : 0;
  k->kinds.clear();
  for (int i = 0; i < k->nobj; i++) k->kinds += (i ? "," : "") + std::to_string(s.kinds[i]);
  k->kmask = s.kind_mask | s.leaf_kind_mask;  // CSG leaves are shaded by their own kind
  k->feat = (s.num_programs ? SF_VM : 0) | ((s.light_mask >> RT_LIGHT_DIRECTIONAL) & 1 ? SF_LDIR : 0) |
            ((s.light_mask >> RT_LIGHT_SPOT) & 1 ? SF_LSPOT : 0);
  k->nlights = (s.nlights >= 1 && s.nlights <= SPEC_MAX_LIGHTS) ? s.nlights : 0;
  k->pow_bits = s.num_programs ? 7 : s.pow_bits;  // surface programs set exponents at run time
  // the BVH culls' far-origin shift (rt_render.h far_shift) pays where a
  // far ray would otherwise sweep many leaves (C5 serial 347 -> 120 ms); a
  // small BVH only carries its registers (C4 +3 %)
  k->far = (!s.use_bvh || s.nobj >= RT_FAR_MIN_OBJ) ? 1 : 0;
  return true;
}

// The compile helper next to this library (csrc/rt_spec_cc, built with it):
// every hipRTC compile runs in a child process, so a compiler abort cannot
// take the renderer's process down and the host's environment changes cannot
// reach the compiler. "" when it is missing, unusable (a failed start, then
// for the rest of the process) or RT_SPEC_INPROC=1 asks for the in-process
// compiler (hipRTC in a private dlmopen namespace, below).
std::atomic<int> g_helper_off{0};

std::string spec_helper() {
  static std::string path;
  static std::once_flag once;
  std::call_once(once, [] {
    Dl_info info;
    if (dladdr((void*)&rt_abi_version, &info) && info.dli_fname) {
      std::string lib = info.dli_fname;
      const size_t k = lib.rfind('/');
      const std::string p = (k == std::string::npos ? std::string(".") : lib.substr(0, k)) + "/rt_spec_cc";
      if (access(p.c_str(), X_OK) == 0) path = p;
    }
  });
  const char* e = rt_getenv("RT_SPEC_INPROC");
  if ((e && atoi(e) != 0) || g_helper_off.load()) return std::string();
  return path;
}

// Run the helper for one variant: "" on success (sc filled), else the
// compiler's message. *unavailable: the helper could not be started at all
// (the caller then compiles in process). fork + exec like Python's
// subprocess: the child makes only async-signal-safe calls before execve.
std::string spec_compile_child(const std::string& helper, const std::vector<const char*>& opts, const std::string& name,
                               SpecCode* sc, bool* unavailable) {
  *unavailable = false;
  const char* td = rt_getenv("TMPDIR");
  std::string tmpl = std::string(td && *td ? td : "/tmp") + "/rt_spec_XXXXXX";
  std::vector<char> dbuf(tmpl.begin(), tmpl.end());
  dbuf.push_back(0);
  if (!mkdtemp(dbuf.data())) {
    *unavailable = true;
    return "mkdtemp failed";
  }
  const std::string dir = dbuf.data(), out = dir + "/code", outname = out + ".name", log = dir + "/log";
  std::vector<const char*> argv = {helper.c_str(), out.c_str(), name.c_str()};
  argv.insert(argv.end(), opts.begin(), opts.end());
  argv.push_back(nullptr);
  char* const* envp = env_snap()->p.data();  // the child's environment: the load-time copy
  auto cleanup = [&] {
    unlink(out.c_str());
    unlink(outname.c_str());
    unlink(log.c_str());
    rmdir(dir.c_str());
  };
  const int lfd = open(log.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
  const int nfd = open("/dev/null", O_RDONLY | O_CLOEXEC);
  const pid_t pid = fork();
  if (pid == 0) {
    if (nfd >= 0) dup2(nfd, 0);
    if (lfd >= 0) {
      dup2(lfd, 1);
      dup2(lfd, 2);
    }
#ifdef SYS_close_range
    if (syscall(SYS_close_range, 3u, ~0u, 0u) != 0)
#endif
      for (int fd = 3; fd < 4096; fd++) close(fd);
    execve(helper.c_str(), (char* const*)argv.data(), envp);
    _exit(127);
  }
  if (lfd >= 0) close(lfd);
  if (nfd >= 0) close(nfd);
  if (pid < 0) {
    cleanup();
    *unavailable = true;
    return "fork failed";
  }
  int status = 0;
  pid_t w;
  do {
    w = waitpid(pid, &status, 0);
  } while (w < 0 && errno == EINTR);
  auto slurp = [](const std::string& path, size_t cap) {
    std::string t;
    if (FILE* f = fopen(path.c_str(), "rb")) {
      char b[65536];
      size_t n;
      while (t.size() < cap && (n = fread(b, 1, sizeof b, f)) > 0) t.append(b, n);
      fclose(f);
    }
    return t;
  };
  const std::string logtxt = slurp(log, 1 << 16);
  std::string code = slurp(out, (size_t)1 << 30), lowered = slurp(outname, 4096);
  cleanup();
  const bool exited = w == pid && WIFEXITED(status);
  if (exited && WEXITSTATUS(status) == 127) {  // (execve failed: no helper in this environment)
    *unavailable = true;
    return "cannot start " + helper;
  }
  // (w < 0, ECHILD: a host that ignores SIGCHLD reaped it; the files decide)
  const bool ok = (exited && WEXITSTATUS(status) == 0) || (w < 0 && errno == ECHILD && !lowered.empty());
  if (!ok || code.empty() || lowered.empty()) {
    std::string why = exited ? "exit " + std::to_string(WEXITSTATUS(status))
                             : (w == pid && WIFSIGNALED(status) ? "signal " + std::to_string(WTERMSIG(status)) : "lost");
    return "compile process " + why + ": " + logtxt;
  }
  sc->code.assign(code.begin(), code.end());
  sc->lowered = lowered;
  return std::string();
}

// Keys being compiled right now (one compile per key; other threads wait).
std::set<std::string> g_compiling;
std::condition_variable g_compile_cv;

// Compile the code object for `key` into g_spec_code (no device needed): in
// the helper process, or in process under g_rtc_mu. Takes g_spec_mu for the
// cache; the caller holds no lock.
int spec_compile(const SpecKey& sk, double* ms) {
  *ms = 0;
  const std::string key = sk.str();
  // a key that failed to compile fails again at once (no second compile)
  auto failed = [&](std::string* err) {
    auto it = g_jobs.find(key);
    if (it == g_jobs.end() || it->second.state >= 0) return false;
    *err = it->second.err;
    return true;
  };
  // every failure is recorded under the key (g_jobs) and reported the same way
  auto bad = [&](const std::string& msg) {
    {
      std::lock_guard<std::mutex> l(g_spec_mu);
      SpecJob& j = g_jobs[key];
      j.state = -1;
      j.err = msg;
    }
    return fail(RT_E_DEVICE, "scene specialisation: " + msg);
  };
  std::string err;
  {
    std::unique_lock<std::mutex> l(g_spec_mu);
    for (;;) {
      if (g_spec_code.count(key)) return RT_OK;
      if (failed(&err)) return fail(RT_E_DEVICE, "scene specialisation: " + err);
      if (!g_compiling.count(key)) break;
      g_compile_cv.wait(l);  // (another thread compiles it)
    }
    g_compiling.insert(key);
  }
  struct Done {
    const std::string& k;
    ~Done() {
      {
        std::lock_guard<std::mutex> l(g_spec_mu);
        g_compiling.erase(k);
      }
      g_compile_cv.notify_all();
    }
  } done{key};
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::string> defs = {"-DRT_SPEC_KMASK=" + std::to_string(sk.kmask),
                                   "-DRT_SPEC_FEAT=" + std::to_string(sk.feat)};
  if (sk.nobj > 0) {
    defs.push_back("-DRT_SPEC_NOBJ=" + std::to_string(sk.nobj));
    defs.push_back("-DRT_SPEC_KINDS=" + sk.kinds);
  }
  if (sk.nlights > 0) defs.push_back("-DRT_SPEC_NLIGHTS=" + std::to_string(sk.nlights));
  defs.push_back("-DRT_SPEC_POWBITS=" + std::to_string(sk.pow_bits));
  if (sk.nocull) defs.push_back("-DRT_CULL=0");
  if (sk.share) defs.push_back("-DRT_SHARE=" + std::to_string(sk.share));
  if (sk.quads == SCH_PAIRS) defs.push_back("-DRT_PAIRS=1");
  if (!sk.far) defs.push_back("-DRT_FAR_SHIFT=0");
  std::vector<const char*> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off"};
  for (const auto& d : defs) opts.push_back(d.c_str());
  // RT_SPEC_EXTRA_FLAGS: extra compiler options (tuning experiments only);
  // RT_JIT_DEFS: the same, baked into an A/B build of the library
  std::vector<std::string> extra;
#ifdef RT_JIT_DEFS
  const char* baked = RT_JIT_DEFS;
#else
  const char* baked = nullptr;
#endif
  for (const char* e : {baked, (const char*)rt_getenv("RT_SPEC_EXTRA_FLAGS")}) {
    if (!e) continue;
    std::string cur;
    for (const char* q = e;; q++) {
      if (*q == ' ' || *q == 0) {
        if (!cur.empty()) extra.push_back(cur);
        cur.clear();
        if (!*q) break;
      } else {
        cur += *q;
      }
    }
  }
  for (const auto& x : extra) opts.push_back(x.c_str());
  const std::string name = std::string("rt_render_kernel<") + (sk.lds ? "true" : "false") + ", " +
                           (sk.bvh ? "true" : "false") + ", " + (sk.csg ? "true" : "false") + ", " +
                           (sk.quads == SCH_QUADS ? "true" : "false") + ">";
  SpecCode sc;
  std::string msg;
  bool compiled = false;
  const std::string helper = spec_helper();
  if (!helper.empty()) {
    bool unavailable = false;
    msg = spec_compile_child(helper, opts, name, &sc, &unavailable);
    if (unavailable) {  // the in-process compiler from now on
      if (!g_helper_off.exchange(1)) fprintf(stderr, "librtamd: compile helper unusable (%s): compiling in process\n", msg.c_str());
      msg.clear();
    } else {
      compiled = true;
    }
  }
  if (!compiled) {
    std::lock_guard<std::mutex> rl(g_rtc_mu);
    if (!rtc_load()) return bad(g_rtc.err);
    const char* name_expr = name.c_str();
    hiprtcProgram prog;
    rtc_sync_env();
    hiprtcResult r = g_rtc.create(&prog, "#include \"rt_render.h\"\n", "rt_spec.hip", k_jit_nsrc, k_jit_srcs,
                                  k_jit_names);
    if (r != HIPRTC_SUCCESS) return bad(std::string("hiprtcCreateProgram: ") + g_rtc.errstr(r));
    r = g_rtc.add_name(prog, name_expr);
    if (r == HIPRTC_SUCCESS) r = g_rtc.compile(prog, (int)opts.size(), opts.data());
    if (r != HIPRTC_SUCCESS) {
      size_t n = 0;
      std::string log;
      if (g_rtc.log_size(prog, &n) == HIPRTC_SUCCESS && n > 1) {
        log.resize(n);
        (void)g_rtc.log(prog, &log[0]);
      }
      msg = std::string("hiprtcCompileProgram: ") + g_rtc.errstr(r) + "\n" + log;
    } else {
      const char* low = nullptr;
      size_t n = 0;
      if (g_rtc.lowered(prog, name_expr, &low) != HIPRTC_SUCCESS || !low) msg = "hiprtcGetLoweredName failed";
      else if (g_rtc.code_size(prog, &n) != HIPRTC_SUCCESS || n == 0) msg = "hiprtcGetCodeSize failed";
      else {
        sc.lowered = low;
        sc.code.resize(n);
        if (g_rtc.code(prog, sc.code.data()) != HIPRTC_SUCCESS) msg = "hiprtcGetCode failed";
      }
    }
    (void)g_rtc.destroy(&prog);
  }
  if (!msg.empty()) return bad(msg);
  {
    std::lock_guard<std::mutex> l(g_spec_mu);
    g_spec_code.emplace(key, std::move(sc));
    auto it = g_jobs.find(key);
    if (it != g_jobs.end()) it->second.state = 1;
  }
  *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return RT_OK;
}

// ---------------------------------------------------------------------------
// Background compiles (the rt_render seam: a first Render() of a new scene
// shape must not wait for hipRTC). A context in async mode (rt_context
// spec_async) never compiles on the caller's thread: a missing code object is
// queued here, the launch renders with the ahead-of-time generic kernel
// (same pixels and counters), and a later launch switches once the code is
// ready. One worker thread, started on first use; an atexit handler lets the
// compile in progress finish before the process tears down the hipRTC
// namespace under it (at most one compile, ~0.5-2 s).
// ---------------------------------------------------------------------------
enum { SPEC_PENDING = 1 };  // internal status of spec_build: queued or compiling

std::vector<SpecKey> g_job_q;  // FIFO of keys to compile; guarded by g_spec_mu
std::condition_variable g_job_cv;
std::vector<std::thread*> g_workers;  // up to 3 (compiles run in helper processes, so they can overlap)
bool g_worker_stop = false;

void spec_worker() {
  std::unique_lock<std::mutex> lk(g_spec_mu);
  for (;;) {
    g_job_cv.wait(lk, [] { return g_worker_stop || !g_job_q.empty(); });
    if (g_worker_stop) return;  // (queued jobs are dropped at exit)
    const SpecKey sk = g_job_q.front();
    g_job_q.erase(g_job_q.begin());
    lk.unlock();
    double ms = 0;
    (void)spec_compile(sk, &ms);  // records the key's state, compiled or failed, in g_jobs
    lk.lock();
  }
}

// Specialised kernels queued or compiling in the background.
int spec_jobs_pending() {
  std::lock_guard<std::mutex> l(g_spec_mu);
  int n = 0;
  for (const auto& kv : g_jobs) n += kv.second.state == 0;
  return n;
}

void spec_worker_exit() {
  {
    std::lock_guard<std::mutex> l(g_spec_mu);
    g_worker_stop = true;
  }
  g_job_cv.notify_all();
  for (std::thread* t : g_workers)
    if (t->joinable()) t->join();
}

// Queue `sk` (caller holds g_spec_mu; the key is not compiled and not queued).
void spec_enqueue(const SpecKey& sk) {
  g_jobs[sk.str()] = SpecJob();
  g_job_q.push_back(sk);
  if (g_workers.size() < 3) {
    if (g_workers.empty()) std::atexit(spec_worker_exit);
    g_workers.push_back(new std::thread(spec_worker));
  }
  g_job_cv.notify_one();
}

// Compile (or fetch) the specialised kernel for `sk` and load it on `device`.
// async: a code object not compiled yet is queued for the worker and
// SPEC_PENDING returned (no wait); a failed background compile returns its
// error. Takes the locks it needs; the caller holds none.
int spec_build(int device, const SpecKey& sk, hipFunction_t* fn, double* ms, bool async = false) {
  *ms = 0;
  *fn = nullptr;
  const std::string key = sk.str();
  {
    std::lock_guard<std::mutex> l(g_spec_mu);
    auto fit = g_spec_fn.find({device, key});
    if (fit != g_spec_fn.end()) {
      *fn = fit->second;
      return RT_OK;
    }
    if (async && !g_spec_code.count(key)) {
      auto jit = g_jobs.find(key);
      if (jit == g_jobs.end()) {
        spec_enqueue(sk);
        return SPEC_PENDING;
      }
      if (jit->second.state == 0) return SPEC_PENDING;
      // (state -1: spec_compile reports the recorded failure)
    }
  }
  int rc = spec_compile(sk, ms);  // (a cache hit when the worker compiled it)
  if (rc != RT_OK) return rc;
  const SpecCode* sc;
  {
    std::lock_guard<std::mutex> l(g_spec_mu);
    sc = &g_spec_code.at(key);
  }
  DeviceGuard guard(device);
  hipModule_t mod;
  HIP_TRY(hipModuleLoadData(&mod, sc->code.data()));
  hipFunction_t f;
  HIP_TRY(hipModuleGetFunction(&f, mod, sc->lowered.c_str()));
  std::lock_guard<std::mutex> l(g_spec_mu);
  *fn = g_spec_fn.emplace(std::make_pair(device, key), f).first->second;
  return RT_OK;
}

// Point c->spec_fn at the specialised kernel of the current scene (or clear
// it). In async mode a kernel still compiling leaves spec_fn clear and
// spec_pending set (launch() retries), and a failed compile sets spec_failed.
int spec_prepare(rt_context* c) {
  c->spec_fn = nullptr;
  c->spec_ms = 0;
  c->spec_pending = false;
  c->spec_failed = false;
  if (!c->specialize || !c->has_scene) return RT_OK;
  SpecKey sk;
  if (!spec_key(c->sc, &sk)) return RT_OK;
  sk.nocull = (c->accel & RT_ACCEL_CULL) ? 0 : 1;
  sk.quads = pick_schedule(c->sched, c->sc, (uint64_t)c->sc.width * c->sc.height, c->cus, c->inflight, true);
  sk.share = pick_share(c->share_mode, c->sc, (uint64_t)c->sc.width * c->sc.height, c->cus, c->inflight);
  if (sk.share == RT_SHARE_GROUP && sk.quads == SCH_PAIRS) sk.quads = SCH_QUADS;  // the LDS board assumes one owner lane per pixel
  c->spec_key = sk;
  c->spec_alt.clear();
  const int rc = spec_build(c->device, sk, &c->spec_fn, &c->spec_ms, c->spec_async);
  if (rc == SPEC_PENDING) {
    c->spec_pending = true;
    return RT_OK;
  }
  if (rc != RT_OK) {
    c->spec_failed = true;
    c->spec_err = g_err;
  }
  return rc;
}

// Queue (async contexts) the specialised variant a launch of `pixels` pixels
// will ask for when it differs from the scene's own (schedule or sharing), so
// that it compiles alongside the scene's kernel rather than after it.
void spec_prefetch(rt_context* c, uint64_t pixels) {
  if (!c->spec_async || !c->has_scene || !(c->spec_pending || c->spec_fn)) return;
  int sch = pick_schedule(c->sched, c->sc, pixels, c->cus, c->inflight, true);
  const int share = pick_share(c->share_mode, c->sc, pixels, c->cus, c->inflight);
  if (share == RT_SHARE_GROUP && sch == SCH_PAIRS) sch = SCH_QUADS;
  if (sch == c->spec_key.quads && share == c->spec_key.share) return;
  SpecKey sk = c->spec_key;
  sk.quads = sch;
  sk.share = share;
  hipFunction_t f = nullptr;
  double ms = 0;
  (void)spec_build(c->device, sk, &f, &ms, true);  // queued, or loaded if already compiled
}

// The specialised kernel for schedule `sch` and work-sharing mode `share`
// (another pair than the scene's is compiled on first use: a launch covering
// a small share of the frame). In async mode a pair still compiling (or
// failed) gives *fn = nullptr: this launch runs the generic kernel.
int spec_for(rt_context* c, int sch, int share, hipFunction_t* fn) {
  if (share == RT_SHARE_GROUP && sch == SCH_PAIRS) sch = SCH_QUADS;
  if (!c->spec_fn || (c->spec_key.quads == sch && c->spec_key.share == share)) {
    *fn = c->spec_fn;
    return RT_OK;
  }
  const int k = sch * 4 + share;
  auto it = c->spec_alt.find(k);
  if (it == c->spec_alt.end()) {
    SpecKey sk = c->spec_key;
    sk.quads = sch;
    sk.share = share;
    double ms = 0;
    hipFunction_t f = nullptr;
    int rc = spec_build(c->device, sk, &f, &ms, c->spec_async);
    if (rc == SPEC_PENDING) {
      *fn = nullptr;
      return RT_OK;
    }
    if (rc != RT_OK && !c->spec_fallback) return rc;
    if (rc != RT_OK) {  // (the generic kernel from now on for this pair)
      c->spec_failed = true;
      c->spec_err = g_err;
    }
    it = c->spec_alt.emplace(k, f).first;
  }
  *fn = it->second;
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_set_accel(rt_context* c, int flags) {
  if (!c) return fail(RT_E_INVALID, "rt_set_accel: NULL context");
  if (flags & ~(RT_ACCEL_BVH | RT_ACCEL_CULL)) return fail(RT_E_INVALID, "rt_set_accel: unknown flags");
  c->accel = flags;
  return spec_prepare(c);
}

int rt_set_schedule(rt_context* c, int mode) {
  if (!c) return fail(RT_E_INVALID, "rt_set_schedule: NULL context");
  if (mode != RT_SCHED_AUTO && mode != RT_SCHED_PIXEL && mode != RT_SCHED_QUADS && mode != RT_SCHED_PAIRS)
    return fail(RT_E_INVALID, "rt_set_schedule: unknown mode");
  c->sched = mode;
  return RT_OK;
}

int rt_set_frames_in_flight(rt_context* c, int n) {
  if (!c) return fail(RT_E_INVALID, "rt_set_frames_in_flight: NULL context");
  if (n < 1) return fail(RT_E_INVALID, "rt_set_frames_in_flight: n < 1");
  c->inflight = n;
  return c->has_scene ? spec_prepare(c) : RT_OK;
}

int rt_set_specialize(rt_context* c, int enable) {
  if (!c) return fail(RT_E_INVALID, "rt_set_specialize: NULL context");
  c->specialize = enable != 0;
  return spec_prepare(c);
}

int rt_spec_precompile(int nobj, const int* kinds, int features, double* compile_ms) {
  if (compile_ms) *compile_ms = 0;
  if (features & ~(SF_VM | SF_LDIR | SF_LSPOT | (0xF << 8))) return fail(RT_E_INVALID, "rt_spec_precompile: unknown feature bits");
  const int nlights = (features >> 8) & 0xF;
  if (nlights > SPEC_MAX_LIGHTS) return fail(RT_E_INVALID, "rt_spec_precompile: 0..8 lights");
  if (nobj < 1 || nobj > SPEC_MAX_OBJ || !kinds) return fail(RT_E_INVALID, "rt_spec_precompile: 1..8 objects");
  SpecKey sk;
  sk.nobj = nobj;
  for (int i = 0; i < nobj; i++) {
    if (kinds[i] < 0 || kinds[i] >= RT_NUM_KINDS || kinds[i] == RT_CSG)
      return fail(RT_E_INVALID, "rt_spec_precompile: bad primitive kind");
    sk.kinds += (i ? "," : "") + std::to_string(kinds[i]);
    sk.kmask |= 1 << kinds[i];
  }
  sk.feat = features & (SF_VM | SF_LDIR | SF_LSPOT);
  sk.nlights = nlights;
  double ms = 0;
  int rc = spec_compile(sk, &ms);
  if (compile_ms) *compile_ms = ms;
  return rc;
}

const char* rt_debug_getenv(const char* name) { return name ? rt_getenv(name) : nullptr; }

int rt_debug_spec_compile(const char* key, double* compile_ms) {
  if (compile_ms) *compile_ms = 0;
  if (!key) return fail(RT_E_INVALID, "rt_debug_spec_compile: NULL key");
  std::vector<std::string> f;
  std::string cur;
  for (const char* q = key;; q++) {
    if (*q == ':' || *q == 0) {
      f.push_back(cur);
      cur.clear();
      if (!*q) break;
    } else {
      cur += *q;
    }
  }
  if (f.size() != 13) return fail(RT_E_INVALID, "rt_debug_spec_compile: 13 fields expected");
  SpecKey sk;
  try {
    sk.lds = std::stoi(f[0]);
    sk.bvh = std::stoi(f[1]);
    sk.csg = std::stoi(f[2]);
    sk.nobj = std::stoi(f[3]);
    sk.kinds = f[4];
    sk.kmask = std::stoi(f[5]);
    sk.feat = std::stoi(f[6]);
    sk.nlights = std::stoi(f[7]);
    sk.pow_bits = std::stoi(f[8]);
    sk.nocull = std::stoi(f[9]);
    sk.quads = std::stoi(f[10]);
    sk.share = std::stoi(f[11]);
    sk.far = std::stoi(f[12]);
  } catch (...) {
    return fail(RT_E_INVALID, "rt_debug_spec_compile: malformed key");
  }
  if (sk.quads < SCH_SERIAL || sk.quads > SCH_PAIRS || sk.share < RT_SHARE_OFF || sk.share > RT_SHARE_DEVICE ||
      sk.nlights < 0 || sk.nlights > SPEC_MAX_LIGHTS || sk.nobj < 0 || sk.nobj > SPEC_MAX_OBJ)
    return fail(RT_E_INVALID, "rt_debug_spec_compile: field out of range");
  double ms = 0;
  const int rc = spec_compile(sk, &ms);
  if (compile_ms) *compile_ms = ms;
  return rc;
}

int rt_scene_info(rt_context* c, int* flags) {
  if (!c || !flags) return fail(RT_E_INVALID, "rt_scene_info: NULL argument");
  if (!c->has_scene) return fail(RT_E_INVALID, "rt_scene_info: no scene set");
  const DevScene& s = c->sc;
  const bool lds = scene_in_lds(s);
  *flags = (lds ? RT_INFO_LDS : 0) | (s.use_bvh ? RT_INFO_BVH : 0) | (s.has_csg ? RT_INFO_CSG : 0) |
           ((!lds && !s.use_bvh && !s.has_csg) ? RT_INFO_STREAM : 0) |
           ((c->spec_fn && c->spec_key.share) ? RT_INFO_WAVEFRONT : 0) |
           ((c->spec_fn && c->spec_key.share == RT_SHARE_DEVICE) ? RT_INFO_SHARE_DEVICE : 0) |
           (c->tile_cost.empty() ? 0 : RT_INFO_ORDERED);
  return RT_OK;
}

int rt_specialized(rt_context* c, int* active, double* compile_ms) {
  if (!c) return fail(RT_E_INVALID, "rt_specialized: NULL context");
  if (active) *active = c->spec_fn != nullptr;
  if (compile_ms) *compile_ms = c->spec_ms;
  return RT_OK;
}

const char* rt_last_error(void) { return g_err.c_str(); }

int rt_create(int device, rt_context** out) {
  if (!out) return fail(RT_E_INVALID, "rt_create: out is NULL");
  *out = nullptr;
  if (device < 0) HIP_TRY(hipGetDevice(&device));
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device >= ndev) return fail(RT_E_INVALID, "rt_create: device index out of range");
  DeviceGuard guard(device);
  rt_context* c = new rt_context();
  c->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    delete c;
    return fail(RT_E_DEVICE, "hipGetDeviceProperties failed");
  }
  c->cus = prop.multiProcessorCount;
  c->lds_per_cu = (int)prop.maxSharedMemoryPerMultiProcessor;
  c->lds_per_block = (int)prop.sharedMemPerBlock;
  // Persistent grids: as many workgroups as are resident (any extra block just
  // finds the queue drained). The LDS flavour is sized for the LDS budget.
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_kernels[kernel_index(true, false, false, false)], WG, LDS_MAX_BYTES) !=
          hipSuccess || per_cu <= 0)
    per_cu = 2;
  c->grid_lds = c->cus * std::min(per_cu, 8);
  per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_kernels[kernel_index(false, false, false, false)], WG, 0) != hipSuccess ||
      per_cu <= 0)
    per_cu = 2;
  c->grid_glb = c->cus * std::min(per_cu, 8);
  // PCG jump table: entry (r, k) = 8*r + 2*k LCG steps (pcg.go: mul/inc
  // constants), r = 0..19 the row within its 20-row strip, k = 0..3 the
  // sample (its first draw, raytracer.go:642-643) -- one jump per sample.
  std::vector<uint64_t> jump(JUMP_ENTRIES * 4);
  {
    typedef unsigned __int128 u128;
    const u128 mul = ((u128)2549297995355413924ULL << 64) | 4865540595714422341ULL;
    const u128 inc = ((u128)6364136223846793005ULL << 64) | 1442695040888963407ULL;
    u128 A = 1, Cc = 0;
    for (int step = 0; step < 2 * JUMP_ENTRIES; step++) {
      if (step % 2 == 0) {
        const int e = step / 2;  // = 4*r + k
        jump[e * 4 + 0] = (uint64_t)(A >> 64);
        jump[e * 4 + 1] = (uint64_t)A;
        jump[e * 4 + 2] = (uint64_t)(Cc >> 64);
        jump[e * 4 + 3] = (uint64_t)Cc;
      }
      A = A * mul;
      Cc = Cc * mul + inc;
    }
  }
  int rc = upload(&c->jump, jump);
  if (rc == RT_OK && hipMalloc((void**)&c->queue, 2 * QSET_ALLOC * sizeof(unsigned int)) != hipSuccess)
    rc = fail(RT_E_NOMEM, "queue alloc");
  if (rc == RT_OK && hipMemset(c->queue, 0, 2 * QSET_ALLOC * sizeof(unsigned int)) != hipSuccess)
    rc = fail(RT_E_DEVICE, "queue memset");
  if (rc == RT_OK && hipMalloc((void**)&c->stats, sizeof(unsigned long long) * 64) != hipSuccess)
    rc = fail(RT_E_NOMEM, "stats alloc");
  if (rc == RT_OK && hipMemset(c->stats, 0, sizeof(unsigned long long) * 64) != hipSuccess)
    rc = fail(RT_E_DEVICE, "stats memset");
  c->stats_parts = c->cus * 8;
  if (rc == RT_OK && hipMalloc((void**)&c->stats_part, sizeof(unsigned long long) * STATS_PART * c->stats_parts) != hipSuccess)
    rc = fail(RT_E_NOMEM, "stats alloc");
  if (rc == RT_OK && hipMemset(c->stats_part, 0, sizeof(unsigned long long) * STATS_PART * c->stats_parts) != hipSuccess)
    rc = fail(RT_E_DEVICE, "stats memset");
  if (rc == RT_OK && (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess))
    rc = fail(RT_E_DEVICE, "event create");
  if (rc != RT_OK) {
    rt_destroy(c);
    return rc;
  }
  *out = c;
  return RT_OK;
}

void rt_destroy(rt_context* c) {
  if (!c) return;
  DeviceGuard guard(c->device);
  free_scene(c->sc);
  (void)hipFree(c->ssim_buf);
  (void)hipFree(c->jump);
  (void)hipFree(c->queue);
  (void)hipFree(c->stats);
  (void)hipFree(c->stats_part);
  (void)hipFree(c->stack);
  (void)hipFree(c->vm_global);
  clear_orders(c);
  (void)hipFree(c->est);
  (void)hipFree(c->est_stats);
  (void)hipFree(c->gboard);
  (void)hipFree(c->gring);
  (void)hipFree(c->gctl);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  delete c;
}

static int launch(rt_context* c, int y0, int y1, int trow0, int stride, int ntrows, void* d_rgba, void* stream,
                  bool est);
static int estimate_costs(rt_context* c);
static bool want_order(const rt_context* c);
static int scene_install(rt_context* c, DevScene& s, const std::vector<uint32_t>* costs);

int rt_set_scene(rt_context* c, const rt_scene* in) {
  if (!c || !in) return fail(RT_E_INVALID, "rt_set_scene: NULL argument");
  if (in->width <= 1 || in->height <= 1) return fail(RT_E_INVALID, "rt_set_scene: width/height must be > 1");
  if (in->exp_mode < RT_EXP_AMD64_FMA || in->exp_mode > RT_EXP_PORTABLE)
    return fail(RT_E_INVALID, "rt_set_scene: unknown exp_mode");
  if (in->num_objects < 0 || in->num_lights < 0 || in->num_materials <= 0)
    return fail(RT_E_INVALID, "rt_set_scene: negative counts or no materials");
  if ((in->num_objects > 0 && !in->objects) || (in->num_lights > 0 && !in->lights) || !in->materials)
    return fail(RT_E_INVALID, "rt_set_scene: NULL array");
  DeviceGuard guard(c->device);
  DevScene s;
  s.width = in->width;
  s.height = in->height;
  s.depth = in->depth <= 0 ? 3 : in->depth;                  // raytracer.go:592-595
  double fov = in->fov <= 0.0 ? 90.0 : in->fov;              // raytracer.go:597-600
  double fovr = fov * M_PI / 180.0;                          // :601
  double tn;
  if (!go_tan(fovr / 2.0, tn)) return fail(RT_E_INVALID, "fov outside the restated math.Tan range");
  s.vw = 2.0 / tn;                                           // :602
  s.vh = s.vw * ((double)in->height / (double)in->width);    // :603
  for (int k = 0; k < 3; k++) {
    s.amb[k] = in->ambient[k];
    s.bg0[k] = in->bg_start[k];
    s.bg1[k] = in->bg_end[k];
  }
  s.nobj = in->num_objects;
  const bool ext_lights = in->num_ext_lights > 0;
  if (ext_lights && !in->ext_lights) return fail(RT_E_INVALID, "ext_lights is NULL");
  s.nlights = ext_lights ? in->num_ext_lights : in->num_lights;
  s.nmats = in->num_materials;

  // CSG composites (extension): their leaves follow the top-level objects in
  // every per-object array (index nobj + leaf).
  const int nleaves = std::max(0, in->num_csg_leaves), ncsg = std::max(0, in->csg_code_words);
  if ((nleaves && !in->csg_leaves) || (ncsg && !in->csg_code)) return fail(RT_E_INVALID, "CSG arrays are NULL");
  const int ntot = s.nobj + nleaves;
  std::vector<double> geo((size_t)ntot * GEO, 0.0), shade((size_t)ntot * SHD, 0.0);
  std::vector<int> kind(ntot), objmat((size_t)ntot * OMAT, 0);
  std::vector<double> bcen((size_t)ntot * 3, 0.0), brad((size_t)ntot, 0.0);  // padded bounding spheres
  for (int i = 0; i < ntot; i++) {
    const bool leaf = i >= s.nobj;
    const rt_object& o = leaf ? in->csg_leaves[i - s.nobj] : in->objects[i];
    if (o.kind < 0 || o.kind >= RT_NUM_KINDS) return fail(RT_E_INVALID, "unknown scene object type");
    if (leaf && o.kind != RT_SPHERE && o.kind != RT_CUBE && o.kind != RT_CYLINDER && o.kind != RT_PLANE)
      return fail(RT_E_INVALID, "CSG leaves are spheres, cubes, cylinders or planes");
    kind[i] = o.kind;
    if (o.kind == RT_CSG) {  // validated program; geometry filled in below
      if (o.csg_count <= 0 || o.csg_count > RT_CSG_MAX_LEAVES || o.csg_first < 0 ||
          o.csg_first + o.csg_count > nleaves || o.csg_code < 0 || o.csg_code_len <= 0 ||
          o.csg_code + o.csg_code_len > ncsg)
        return fail(RT_E_INVALID, "CSG composite: leaf / program range");
      int depth = 0;
      for (int k = 0; k < o.csg_code_len; k++) {
        const int op = in->csg_code[o.csg_code + k];
        if (op >= 0) {
          if (op >= o.csg_count) return fail(RT_E_INVALID, "CSG program: leaf index");
          depth++;
        } else {
          if (op < RT_CSG_DIFFERENCE || depth < 2) return fail(RT_E_INVALID, "CSG program: operator");
          depth--;
        }
        if (depth > RT_CSG_MAX_LEAVES) return fail(RT_E_INVALID, "CSG program: depth");
      }
      if (depth != 1) return fail(RT_E_INVALID, "CSG program: does not reduce to one solid");
      continue;
    }
    for (int f = 0; f < RT_MAX_FACES; f++) {
      if (o.material[f] >= in->num_materials || o.material[f] < -std::max(0, in->num_programs))
        return fail(RT_E_INVALID, "material / surface program index out of range");
      objmat[(size_t)i * OMAT + f] = o.material[f];
    }
    M4 o2w = ident(), w2o = ident();  // raytracer.go:757-762
    if (o.has_transform) {
      std::memcpy(o2w.m, o.transform, sizeof(double) * 16);
      if (!inverse(o2w, w2o)) return fail(RT_E_SINGULAR, "object transform is singular (det == 0)");
    }
    double* g = &geo[(size_t)i * GEO];
    double* sh = &shade[(size_t)i * SHD];
    for (int r = 0; r < 3; r++)
      for (int k = 0; k < 4; k++) {
        g[r * 4 + k] = w2o.m[r][k];
        sh[r * 4 + k] = o2w.m[r][k];
      }
    if (o.kind != RT_PLANE) {
      // World-space bounding sphere of the unit primitive: centre = O2W(local
      // centre), radius <= ||L||_F * local radius (spectral <= Frobenius),
      // padded for FP32 culling (see may_hit). Stored as 4 floats in 12..13.
      const double lc[RT_NUM_KINDS][3] = {{0, 0, 0}, {0, 0, 0}, {0.5, 0.5, 0.5}, {0, 0.5, 0}, {0, 0.5, 0}};
      const double lr[RT_NUM_KINDS] = {1.0, 0.0, 0.8660254037844387, 1.118033988749895, 1.118033988749895};
      double fro = 0.0;
      for (int r = 0; r < 3; r++)
        for (int k = 0; k < 3; k++) fro += o2w.m[r][k] * o2w.m[r][k];
      fro = std::sqrt(fro);
      double cc[3], cmax = 0.0;
      for (int r = 0; r < 3; r++) {
        cc[r] = o2w.m[r][0] * lc[o.kind][0] + o2w.m[r][1] * lc[o.kind][1] + o2w.m[r][2] * lc[o.kind][2] + o2w.m[r][3];
        cmax = std::max(cmax, std::fabs(cc[r]));
      }
      double rad = fro * lr[o.kind] * 1.0001 + 1e-4 * (1.0 + cmax + fro);
      float* b = reinterpret_cast<float*>(&g[12]);
      b[0] = (float)cc[0];
      b[1] = (float)cc[1];
      b[2] = (float)cc[2];
      b[3] = f_up(rad);
      for (int k = 0; k < 3; k++) bcen[(size_t)i * 3 + k] = cc[k];
      brad[i] = rad;
    }
    if (o.kind == RT_PLANE) {
      double nw[3], dv;
      plane_consts(w2o, o.plane_point, o.plane_normal, nw, &dv);

      g[12] = o.plane_normal[0];
      g[13] = o.plane_normal[1];
      g[14] = o.plane_normal[2];
      g[15] = dv;
      for (int k = 0; k < 3; k++) sh[12 + k] = nw[k];
      // world-space plane + term scale for may_hit_plane (shade 16..19)
      const double* n = o.plane_normal;
      float* c = reinterpret_cast<float*>(&sh[16]);
      double dabs = std::fabs(dv), dw = dv;
      for (int k = 0; k < 3; k++) {
        double wk = 0.0, ak = 0.0;
        for (int r = 0; r < 3; r++) {
          wk += n[r] * w2o.m[r][k];
          ak += std::fabs(n[r]) * std::fabs(w2o.m[r][k]);
        }
        c[k] = (float)wk;
        c[4 + k] = (float)(ak * 1.001);
      }
      for (int r = 0; r < 3; r++) {
        dw += n[r] * w2o.m[r][3];
        dabs += std::fabs(n[r]) * std::fabs(w2o.m[r][3]);
      }
      c[3] = (float)dw;
      c[7] = (float)(dabs * 1.001);
      if (!std::isfinite(c[0] + c[1] + c[2] + c[3] + c[4] + c[5] + c[6] + c[7]))
        for (int k = 0; k < 8; k++) c[k] = std::numeric_limits<float>::quiet_NaN();  // never culls
    } else if (o.kind == RT_CUBE) {
      for (int f = 0; f < 6; f++) {
        double nw[3], dv;
        plane_consts(w2o, kCubePt[f], kCubeN[f], nw, &dv);
        for (int k = 0; k < 3; k++) sh[12 + f * 3 + k] = nw[k];
      }
    }
  }
  std::vector<int> mcode;  // device membership programs (csg_mask_program)
  // CSG composites: bounding sphere from the leaves (union: enclosing sphere,
  // intersect: the smaller operand, difference: the left operand; a plane leaf
  // is unbounded), leaf range and program in geo slots 14..15.
  for (int i = 0; i < s.nobj; i++) {
    if (kind[i] != RT_CSG) continue;
    const rt_object& o = in->objects[i];
    struct Bd {
      double c[3], r;
      bool fin;
    };
    std::vector<Bd> st;
    for (int k = 0; k < o.csg_code_len; k++) {
      const int op = in->csg_code[o.csg_code + k];
      if (op >= 0) {
        const int li = s.nobj + o.csg_first + op;
        Bd b;
        b.fin = kind[li] != RT_PLANE;
        for (int q = 0; q < 3; q++) b.c[q] = bcen[(size_t)li * 3 + q];
        b.r = brad[li];
        st.push_back(b);
        continue;
      }
      const Bd y = st.back();
      st.pop_back();
      const Bd x = st.back();
      st.pop_back();
      Bd r = x;
      if (op == RT_CSG_UNION) {
        if (!x.fin || !y.fin) {
          r.fin = false;
        } else {
          const double d = std::sqrt((y.c[0] - x.c[0]) * (y.c[0] - x.c[0]) + (y.c[1] - x.c[1]) * (y.c[1] - x.c[1]) +
                                     (y.c[2] - x.c[2]) * (y.c[2] - x.c[2]));
          if (d + y.r <= x.r) {
            r = x;
          } else if (d + x.r <= y.r) {
            r = y;
          } else {
            r.r = (d + x.r + y.r) / 2.0;
            for (int q = 0; q < 3; q++) r.c[q] = x.c[q] + (y.c[q] - x.c[q]) * ((r.r - x.r) / d);
            r.r = r.r * 1.0001 + 1e-9;
          }
        }
      } else if (op == RT_CSG_INTERSECT) {
        r = !x.fin ? y : (!y.fin ? x : (y.r < x.r ? y : x));
      }  // difference: the left operand's bound
      st.push_back(r);
    }
    double* g = &geo[(size_t)i * GEO];
    float* b = reinterpret_cast<float*>(&g[12]);
    if (st.back().fin) {
      for (int q = 0; q < 3; q++) b[q] = (float)st.back().c[q];
      b[3] = f_up(st.back().r + 1e-4 * (1.0 + std::fabs(st.back().c[0]) + std::fabs(st.back().c[1]) +
                                         std::fabs(st.back().c[2])));
    } else {
      b[0] = b[1] = b[2] = 0.0f;
      b[3] = std::numeric_limits<float>::infinity();  // never culled
    }
    int* ci = reinterpret_cast<int*>(&g[14]);
    ci[0] = o.csg_first;
    ci[1] = o.csg_count;
    ci[2] = (int)mcode.size();
    // leaf groups (rt_render.h csg_hit): header [ngroups, ngroups x (FP32
    // bounding sphere of the members' padded spheres, 8 leaf indices as
    // bytes)], then the membership program. Groups are spatial (median splits
    // of the bounded leaves' centres, <= 8 leaves each; planes in groups of
    // their own, never culled); small composites get none.
    {
      std::vector<std::vector<int>> groups;
      std::vector<int> bounded_l, plane_l;
      for (int j = 0; j < o.csg_count; j++)
        (kind[s.nobj + o.csg_first + j] == RT_PLANE ? plane_l : bounded_l).push_back(j);
      if (o.csg_count >= CSG_GROUP_MIN) {
        std::function<void(std::vector<int>)> split = [&](std::vector<int> v) {
          if (v.size() <= 8) {
            groups.push_back(v);
            return;
          }
          double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
          for (int j : v)
            for (int q = 0; q < 3; q++) {
              lo[q] = std::min(lo[q], bcen[(size_t)(s.nobj + o.csg_first + j) * 3 + q]);
              hi[q] = std::max(hi[q], bcen[(size_t)(s.nobj + o.csg_first + j) * 3 + q]);
            }
          int ax = 0;
          for (int q = 1; q < 3; q++)
            if (hi[q] - lo[q] > hi[ax] - lo[ax]) ax = q;
          std::sort(v.begin(), v.end(), [&](int a, int b) {
            const double ca = bcen[(size_t)(s.nobj + o.csg_first + a) * 3 + ax],
                         cb = bcen[(size_t)(s.nobj + o.csg_first + b) * 3 + ax];
            return ca < cb || (ca == cb && a < b);
          });
          const size_t half = (v.size() + 1) / 2;
          split(std::vector<int>(v.begin(), v.begin() + half));
          split(std::vector<int>(v.begin() + half, v.end()));
        };
        if (!bounded_l.empty()) split(bounded_l);
        for (size_t q = 0; q < plane_l.size(); q += 8)
          groups.push_back(std::vector<int>(plane_l.begin() + q, plane_l.begin() + std::min(plane_l.size(), q + 8)));
      }
      mcode.push_back((int)groups.size());
      for (const auto& gv : groups) {
        bool fin = true;
        double c[3] = {0, 0, 0}, lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (int j : gv) {
          const int li = s.nobj + o.csg_first + j;
          if (kind[li] == RT_PLANE) fin = false;
          for (int q = 0; q < 3; q++) {
            lo[q] = std::min(lo[q], bcen[(size_t)li * 3 + q] - brad[li]);
            hi[q] = std::max(hi[q], bcen[(size_t)li * 3 + q] + brad[li]);
          }
        }
        for (int q = 0; q < 3; q++) c[q] = 0.5 * (lo[q] + hi[q]);
        double rr = 0.0;
        for (int j : gv) {
          const int li = s.nobj + o.csg_first + j;
          const double d = std::sqrt((bcen[(size_t)li * 3] - c[0]) * (bcen[(size_t)li * 3] - c[0]) +
                                     (bcen[(size_t)li * 3 + 1] - c[1]) * (bcen[(size_t)li * 3 + 1] - c[1]) +
                                     (bcen[(size_t)li * 3 + 2] - c[2]) * (bcen[(size_t)li * 3 + 2] - c[2]));
          rr = std::max(rr, d + brad[li]);
        }
        float gf[4] = {(float)c[0], (float)c[1], (float)c[2],
                       fin ? f_up(rr * 1.0001 + 1e-6 * (1.0 + std::fabs(c[0]) + std::fabs(c[1]) + std::fabs(c[2])))
                           : std::numeric_limits<float>::infinity()};
        int w[6];
        std::memcpy(w, gf, sizeof gf);
        // leaf numbers as bytes, 0xff = end of list (csg_hit): leaf numbers must stay below 255
        static_assert(RT_CSG_MAX_LEAVES < 255, "CSG leaf groups pack leaf numbers in bytes (0xff ends a list)");
        uint32_t lb[2] = {0xffffffffu, 0xffffffffu};
        for (size_t q = 0; q < gv.size(); q++) {
          lb[q >> 2] &= ~(0xffu << (8 * (q & 3)));
          lb[q >> 2] |= (uint32_t)gv[q] << (8 * (q & 3));
        }
        w[4] = (int)lb[0];
        w[5] = (int)lb[1];
        mcode.insert(mcode.end(), w, w + 6);
      }
    }
    const int prog0 = (int)mcode.size();
    csg_mask_program(in->csg_code + o.csg_code, o.csg_code_len, mcode);
    ci[3] = (int)mcode.size() - prog0;
    s.has_csg = true;
  }
  std::vector<double> mats((size_t)s.nmats * MAT, 0.0);
  for (int m = 0; m < s.nmats; m++) {
    const rt_material& mm = in->materials[m];
    if (mm.reflectivity > 0 && mm.transparency > 0) s.branching = true;
    double* d = &mats[(size_t)m * MAT];
    d[0] = mm.color[0];
    d[1] = mm.color[1];
    d[2] = mm.color[2];
    d[3] = mm.reflectivity;
    double fuzz = mm.fuzziness;
    if (fuzz >= 0) {  // raytracer.go:516-522: constant offset, not random
      double cf, sf;
      if (!go_cos(fuzz, cf) || !go_sin(fuzz, sf)) return fail(RT_E_INVALID, "fuzziness outside restated range");
      d[4] = fuzz * cf * cf;
      d[5] = fuzz * sf * sf;
      d[6] = 1.0;
    }
    d[7] = mm.transparency;
    d[8] = mm.refractive_index;
    d[9] = mm.kd;
    d[10] = mm.ks;
    d[11] = mm.specular_exponent;
    // per-material terms of refract / fresnel, formed here with the device's
    // operations (correctly rounded either way): 1 / ior (n1 / n2 outside the
    // object, raytracer.go:438) and ((1 - ior) / (1 + ior))^2 (r0,
    // raytracer.go:460-461)
    d[12] = 1.0 / mm.refractive_index;
    const double r0 = (1.0 - mm.refractive_index) / (1.0 + mm.refractive_index);
    d[13] = r0 * r0;
  }
  {  // unrolled steps of the device's branch-free specular powering (pow_small_int)
    int maxn = 1;
    for (int m = 0; m < s.nmats; m++) {
      const double n = in->materials[m].specular_exponent;
      if (n >= 2 && n <= 64 && std::floor(n) == n) maxn = std::max(maxn, (int)n);
    }
    int bits = 0;
    while ((1 << bits) <= maxn) bits++;
    s.pow_bits = std::max(1, bits);
  }
  std::vector<double> lights(GLOB + (size_t)std::max(1, s.nlights) * LGT, 0.0);
  for (int k = 0; k < 3; k++) {
    lights[k] = s.amb[k];
    lights[3 + k] = s.bg0[k];
    lights[6 + k] = s.bg1[k];
  }
  lights[9] = s.vw;
  lights[10] = s.vh;
  lights[11] = (double)in->exp_mode;  // RT_EXP_*: the Exp/Log of a fractional Pow
  for (int l = 0; l < s.nlights; l++) {
    double* L = &lights[GLOB + (size_t)l * LGT];
    if (!ext_lights) {
      for (int k = 0; k < 3; k++) {
        L[k] = in->lights[l].position[k];
        L[3 + k] = in->lights[l].color[k];
      }
      s.light_mask |= 1 << RT_LIGHT_POINT;
      continue;
    }
    // contest-extension lights (oracle/rt_oracle.c convert_scene)
    const rt_light& e = in->ext_lights[l];
    if (e.kind < RT_LIGHT_POINT || e.kind > RT_LIGHT_SPOT) return fail(RT_E_INVALID, "unknown light kind");
    s.light_mask |= 1 << e.kind;
    for (int k = 0; k < 3; k++) {
      L[k] = e.position[k];
      L[3 + k] = e.color[k];
    }
    L[9] = (double)e.kind;
    double d[3] = {e.direction[0], e.direction[1], e.direction[2]};
    if (e.kind == RT_LIGHT_DIRECTIONAL)
      for (int k = 0; k < 3; k++) d[k] = -d[k];
    if (e.kind == RT_LIGHT_SPOT)
      for (int k = 0; k < 3; k++) d[k] = d[k] - e.position[k];
    if (e.kind != RT_LIGHT_POINT) {  // vec.go:78 Normalize
      const double m = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
      for (int k = 0; k < 3; k++) L[6 + k] = d[k] / m;
    }
    if (e.kind == RT_LIGHT_SPOT) {
      double cc;
      if (!go_cos(e.cutoff * 0.017453292519943295, cc)) return fail(RT_E_INVALID, "spot cutoff outside restated range");
      L[10] = cc;
      L[11] = e.exponent;
    }
  }
  // One blob: geo | shade | mats | lights | kind | objmat (16-B aligned sections).
  s.off_geo = 0;
  s.off_shade = align16(s.off_geo + (int)(geo.size() * sizeof(double)));
  s.off_mats = align16(s.off_shade + (int)(shade.size() * sizeof(double)));
  s.off_lights = align16(s.off_mats + (int)(mats.size() * sizeof(double)));
  s.off_kind = align16(s.off_lights + (int)(lights.size() * sizeof(double)));
  s.off_objmat = align16(s.off_kind + (int)(kind.size() * sizeof(int)));
  // Surface programs: validated so the device never reads outside them.
  const int nprog = std::max(0, in->num_programs);
  const int ncode = nprog ? in->program_code_words : 0, nconst = nprog ? in->program_const_count : 0;
  if (nprog) {
    if (!in->program_code || !in->program_consts || !in->program_entry || ncode <= 0 || nconst < 0)
      return fail(RT_E_INVALID, "surface programs: NULL array or empty code");
    for (int pi = 0; pi < nprog; pi++) {
      int pc = in->program_entry[pi];
      if (pc < 0 || (pc & 1)) return fail(RT_E_INVALID, "surface program entry out of range");
      bool ret = false;
      for (int steps = 0; steps < VM_MAX_STEPS && pc + 1 < ncode; steps++, pc += 2) {
        uint32_t w0 = in->program_code[pc], cc = in->program_code[pc + 1];
        int op = (int)(w0 & 0xff);
        if (op > VM_RET || ((w0 >> 8) & 0xff) >= VM_REGS || ((w0 >> 16) & 0xff) >= VM_REGS ||
            (w0 >> 24) >= VM_REGS)
          return fail(RT_E_INVALID, "surface program: bad opcode or register");
        if (op == VM_CONST && cc >= (uint32_t)nconst) return fail(RT_E_INVALID, "surface program: bad constant");
        if (op == VM_TBL) {
          if (cc >= (uint32_t)nconst) return fail(RT_E_INVALID, "surface program: bad table");
          uint64_t n = in->program_consts[cc];
          if (n == 0 || n > (uint64_t)nconst || cc + 1 + n > (uint64_t)nconst)
            return fail(RT_E_INVALID, "surface program: bad table length");
        }
        if (op == VM_SEL && cc >= VM_REGS) return fail(RT_E_INVALID, "surface program: bad register");
        if (op == VM_RET) {
          ret = true;
          break;
        }
      }
      if (!ret) return fail(RT_E_INVALID, "surface program does not end in RET");
    }
  }
  s.num_programs = nprog;
  if (nprog > 0) s.branching = true;  // a surface program may return a reflective, transparent material
  // per-kind prefix counts (shadow-test counters)
  std::vector<uint32_t> prefb((size_t)(s.nobj + 1) * PREF, 0u);
  for (int i = 0; i < s.nobj; i++) {
    for (int k = 0; k < RT_NUM_KINDS; k++) prefb[(size_t)(i + 1) * PREF + k] = prefb[(size_t)i * PREF + k];
    prefb[(size_t)(i + 1) * PREF + kind[i]]++;
  }
  s.off_prefb = align16(s.off_objmat + (int)(objmat.size() * sizeof(int)));
  s.off_csg = align16(s.off_prefb + (int)(prefb.size() * sizeof(uint32_t)));
  s.off_code = align16(s.off_csg + (int)(mcode.size() * sizeof(int)));
  s.off_consts = align16(s.off_code + ncode * (int)sizeof(uint32_t));
  s.off_entry = align16(s.off_consts + nconst * (int)sizeof(uint64_t));
  s.blob_bytes = align16(s.off_entry + nprog * (int)sizeof(int));
  {
    std::vector<char> blob((size_t)s.blob_bytes, 0);
    std::memcpy(blob.data() + s.off_geo, geo.data(), geo.size() * sizeof(double));
    std::memcpy(blob.data() + s.off_shade, shade.data(), shade.size() * sizeof(double));
    std::memcpy(blob.data() + s.off_mats, mats.data(), mats.size() * sizeof(double));
    std::memcpy(blob.data() + s.off_lights, lights.data(), lights.size() * sizeof(double));
    std::memcpy(blob.data() + s.off_kind, kind.data(), kind.size() * sizeof(int));
    std::memcpy(blob.data() + s.off_objmat, objmat.data(), objmat.size() * sizeof(int));
    std::memcpy(blob.data() + s.off_prefb, prefb.data(), prefb.size() * sizeof(uint32_t));
    if (!mcode.empty()) std::memcpy(blob.data() + s.off_csg, mcode.data(), mcode.size() * sizeof(int));
    if (nprog) {
      std::memcpy(blob.data() + s.off_code, in->program_code, (size_t)ncode * sizeof(uint32_t));
      std::memcpy(blob.data() + s.off_consts, in->program_consts, (size_t)nconst * sizeof(uint64_t));
      std::memcpy(blob.data() + s.off_entry, in->program_entry, (size_t)nprog * sizeof(int));
    }
    int rc = upload(&s.blob, blob);
    if (rc != RT_OK) {
      free_scene(s);
      return rc;
    }
    s.h_blob.swap(blob);
  }
  s.kinds.assign(kind.begin(), kind.begin() + s.nobj);  // top-level objects (test counts)
  {
    // Acceleration buffer: [BVH nodes | leaf objects] | planes.
    std::vector<int> bounded, planes;
    for (int i = 0; i < s.nobj; i++) (kind[i] == RT_PLANE || kind[i] == RT_CSG ? planes : bounded).push_back(i);
    BvhBuild b;
    if ((c->accel & RT_ACCEL_BVH) && (int)bounded.size() >= RT_BVH_MIN) {
      b.c = &bcen;
      b.r = &brad;
      b.geo = &geo;
      b.kind = &kind;
      b.ord = bounded;
      b.build(0, (int)bounded.size(), 0);  // root: node 0 (> 4 objects)
      s.use_bvh = b.max_depth + 2 < BVH_STACK;
    }
    if (!s.use_bvh) {
      b.nodes.clear();
      b.leaf_geo.clear();
    }
    for (int i = 0; i < s.nobj; i++) s.kind_mask |= 1 << kind[i];
    for (int i = s.nobj; i < ntot; i++) s.leaf_kind_mask |= 1 << kind[i];
    s.off_nodes = 0;
    s.off_bobj = (b.nodes.size() * sizeof(float) + 15) & ~(size_t)15;
    s.off_planes = s.off_bobj + ((b.leaf_geo.size() * sizeof(double) + 15) & ~(size_t)15);
    // maximal runs of consecutive top-level objects of one kind (brute-force
    // loops over global linear scenes: first, count, kind, axis), spheres split
    // further into scale + translation runs (axis = 1: their compact records
    // AXIS_REC doubles each, m0 m3 m5 m7 m10 m11, at off_arec by object index)
    // and of those the runs of one uniform scale (axis = 2: m0 == m5 == m10,
    // equal over the run; records m3 m7 m11 m0 at off_urec, rt_render.h UNI_REC)
    std::vector<int> runs;
    std::vector<double> arec, urec;
    double run_scale = 0.0;
    for (int i = 0; i < s.nobj; i++) {
      int ax = kind[i] == RT_SPHERE && axis_sphere(&geo[(size_t)i * GEO]) ? 1 : 0;
      if (ax) {
        const double* m = &geo[(size_t)i * GEO];
        if (m[0] == m[5] && m[0] == m[10]) {
          ax = 2;
          if (urec.empty()) urec.assign((size_t)s.nobj * UNI_REC, 0.0);
          double* u = &urec[(size_t)i * UNI_REC];
          u[0] = m[3];
          u[1] = m[7];
          u[2] = m[11];
          u[3] = m[0];
        }
      }
      if (ax && arec.empty()) arec.assign((size_t)s.nobj * AXIS_REC, 0.0);
      if (ax) {
        const double* m = &geo[(size_t)i * GEO];
        double* a = &arec[(size_t)i * AXIS_REC];
        a[0] = m[0];
        a[1] = m[3];
        a[2] = m[5];
        a[3] = m[7];
        a[4] = m[10];
        a[5] = m[11];
      }
      const double sc = ax == 2 ? geo[(size_t)i * GEO] : 0.0;
      if (runs.empty() || runs[runs.size() - 2] != kind[i] || runs[runs.size() - 1] != ax ||
          (ax == 2 && sc != run_scale))
        runs.insert(runs.end(), {i, 0, kind[i], ax});
      run_scale = sc;
      runs[runs.size() - 3]++;
    }
    s.nruns = (int)runs.size() / 4;
    s.off_runs = s.off_planes + ((std::max<size_t>(1, planes.size()) * sizeof(int) + 15) & ~(size_t)15);
    s.off_arec = (s.off_runs + std::max<size_t>(1, runs.size()) * sizeof(int) + 63) & ~(size_t)63;
    s.off_urec = (s.off_arec + std::max<size_t>(1, arec.size()) * sizeof(double) + 63) & ~(size_t)63;
    if (!urec.empty()) urec.resize(urec.size() + 8 * UNI_REC, 0.0);  // scan_uni may load records past a run
    std::vector<char> acc(s.off_urec + std::max<size_t>(1, urec.size()) * sizeof(double), 0);
    if (!runs.empty()) std::memcpy(acc.data() + s.off_runs, runs.data(), runs.size() * sizeof(int));
    if (!arec.empty()) std::memcpy(acc.data() + s.off_arec, arec.data(), arec.size() * sizeof(double));
    if (!urec.empty()) std::memcpy(acc.data() + s.off_urec, urec.data(), urec.size() * sizeof(double));
    if (!b.nodes.empty()) std::memcpy(acc.data() + s.off_nodes, b.nodes.data(), b.nodes.size() * sizeof(float));
    if (s.use_bvh && !b.nodes.empty()) {
      // the box of the BVH objects' padded bounding spheres, and a generous
      // pad: every BVH object lies inside
      double ext = 0.0;
      for (int k = 0; k < 3; k++) {
        s.bvh_lo[k] = 1e300;
        s.bvh_hi[k] = -1e300;
      }
      for (int i : b.ord)
        for (int k = 0; k < 3; k++) {
          s.bvh_lo[k] = std::min(s.bvh_lo[k], bcen[(size_t)i * 3 + k] - brad[i]);
          s.bvh_hi[k] = std::max(s.bvh_hi[k], bcen[(size_t)i * 3 + k] + brad[i]);
        }
      for (int k = 0; k < 3; k++) ext = std::max(ext, s.bvh_hi[k] - s.bvh_lo[k]);
      const double pad = 1e-3 * (1.0 + ext);
      for (int k = 0; k < 3; k++) {
        s.bvh_lo[k] -= pad;
        s.bvh_hi[k] += pad;
      }
    }
    if (!b.leaf_geo.empty())
      std::memcpy(acc.data() + s.off_bobj, b.leaf_geo.data(), b.leaf_geo.size() * sizeof(double));
    if (!planes.empty()) std::memcpy(acc.data() + s.off_planes, planes.data(), planes.size() * sizeof(int));
    int rc = upload(&s.accel, acc);
    if (rc != RT_OK) {
      free_scene(s);
      return rc;
    }
    s.h_accel.swap(acc);
    s.nplanes = (int)planes.size();
    s.nnodes = (int)(b.nodes.size() / BN);
  }
  return scene_install(c, s, nullptr);
}

// Make the converted scene `s` (blob and accel already on c's device) the
// context's scene: frame stack and VM records sized for it, the specialised
// kernel prepared, and the tile costs either estimated (costs == nullptr) or
// taken from a context holding the same scene (the estimate counts rays,
// which do not depend on the device or the kernel). On failure s is freed.
static int scene_install(rt_context* c, DevScene& s, const std::vector<uint32_t>* costs) {
  const int nprog = s.num_programs;
  // Frame stack: (depth - 1) frames per lane, lane-interleaved per wave slot.
  int frames = std::max(1, s.depth - 1);
  const int waves = c->cus * 8 * WAVES_PER_WG;  // upper bound of any persistent grid
  size_t need = (size_t)waves * frames * FRAME_FIELDS * 64 * sizeof(double);
  if (need > c->stack_bytes) {
    (void)hipFree(c->stack);
    c->stack = nullptr;
    c->stack_bytes = 0;
    if (hipMalloc((void**)&c->stack, need) != hipSuccess) {
      free_scene(s);
      return fail(RT_E_NOMEM, "frame stack allocation failed");
    }
    c->stack_bytes = need;
  }
  c->stack_waves = (int)(c->stack_bytes / ((size_t)frames * FRAME_FIELDS * 64 * sizeof(double)));
  if (nprog) {  // per-lane VM material records for the global-scene flavour
    size_t vneed = (size_t)c->stack_waves * 64 * MAT * sizeof(double);
    if (vneed > c->vm_global_bytes) {
      (void)hipFree(c->vm_global);
      c->vm_global = nullptr;
      c->vm_global_bytes = 0;
      if (hipMalloc((void**)&c->vm_global, vneed) != hipSuccess) {
        free_scene(s);
        return fail(RT_E_NOMEM, "surface VM record allocation failed");
      }
      c->vm_global_bytes = vneed;
    }
  }
  free_scene(c->sc);
  c->sc = std::move(s);
  c->has_scene = true;
  clear_orders(c);
  // a failed specialisation still leaves a complete scene (generic kernel,
  // tile order): the caller may render it (the rt_render seam falls back)
  const int spec_rc = spec_prepare(c);
  const std::string spec_msg = g_err;
  int rc = RT_OK;
  if (!costs) rc = estimate_costs(c);
  else if (want_order(c)) c->tile_cost = *costs;
  if (rc != RT_OK) return rc;
  if (spec_rc != RT_OK) return fail(spec_rc, spec_msg);
  return RT_OK;
}

// Give context c the scene `src` holds (same device or another one): the
// host copies of src's converted scene uploaded to c's device, src's tile
// costs reused -- no conversion, BVH build or estimate launch again. Used by
// the rt_render seam for its second context and for every further device.
static int scene_clone(rt_context* c, const rt_context* src) {
  if (!src->has_scene) return fail(RT_E_INVALID, "scene_clone: no scene");
  DeviceGuard guard(c->device);
  DevScene s = src->sc;  // (host fields and copies; device pointers replaced below)
  s.blob = nullptr;
  s.accel = nullptr;
  if (hipMalloc((void**)&s.blob, std::max<size_t>(1, s.h_blob.size())) != hipSuccess) {
    s.blob = nullptr;
    free_scene(s);
    return fail(RT_E_NOMEM, "scene_clone: scene blob");
  }
  if (hipMalloc((void**)&s.accel, std::max<size_t>(1, s.h_accel.size())) != hipSuccess) {
    s.accel = nullptr;
    free_scene(s);
    return fail(RT_E_NOMEM, "scene_clone: acceleration buffer");
  }
  if ((!s.h_blob.empty() && hipMemcpy(s.blob, s.h_blob.data(), s.h_blob.size(), hipMemcpyHostToDevice) != hipSuccess) ||
      (!s.h_accel.empty() && hipMemcpy(s.accel, s.h_accel.data(), s.h_accel.size(), hipMemcpyHostToDevice) != hipSuccess)) {
    free_scene(s);
    return fail(RT_E_DEVICE, "scene_clone: upload");
  }
  return scene_install(c, s, &src->tile_cost);
}

// Tile order for a launch of `tiles_x` x `tiles_y` tiles (rows [y0, y1), or
// tile rows trow0 + j*stride): the costliest quarter by descending estimated
// cost (the frame tile holding each one's centre), then the rest in tile
// order. Cached per launch shape; nullptr without an estimate.
static int order_for(rt_context* c, int y0, int trow0, int stride, int tiles_x, int tiles_y, const unsigned int** out) {
  *out = nullptr;
  if (c->tile_cost.empty()) return RT_OK;
  const std::array<int, 5> key = {y0, trow0, stride, tiles_x, tiles_y};
  auto it = c->orders.find(key);
  if (it != c->orders.end()) {
    *out = it->second;
    return RT_OK;
  }
  const DevScene& s = c->sc;
  const int ftx = (s.width + TILE - 1) / TILE, fty = (s.height + TILE - 1) / TILE;
  const int n = tiles_x * tiles_y;
  std::vector<uint32_t> cost(n), ord(n);
  for (int v = 0; v < n; v++) {
    const int tr = v / tiles_x, tc = v % tiles_x;
    int fr = stride > 0 ? trow0 + tr * stride : (y0 + tr * TILE + TILE / 2) / TILE;
    fr = std::min(fr, fty - 1);
    cost[v] = tc < ftx ? c->tile_cost[(size_t)fr * ftx + tc] : 0u;
    ord[v] = (uint32_t)v;
  }
  std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
  // Only the costliest quarter of the tiles is dealt first (in cost order);
  // the rest keep tile order. Sorting every tile (LPT proper) loses the
  // locality of neighbouring tiles -- similar rays, the same BVH nodes and
  // frame-stack lines -- and starts every SIMD on deep glass trees at once:
  // C3 4.14 vs 3.89 ms with the quarter, 3.95-4.04 ms unordered; C4 5.66 /
  // 5.35 / 6.07 ms; quarters of 1/8 and 1/2, and the quarter kept in tile
  // order, measured no better (profiles/r03/order). Round 5 (two frames in
  // flight): the costliest sixth instead of the quarter, c4csg 10.01-10.06 ->
  // 9.96-9.99 ms, C3 3.013-3.016 -> 2.991-3.010 ms (an eighth: c4csg 9.94-9.98,
  // C3 3.021-3.026; profiles/r05/order_ab/). RT_ORDER_TOP=d (environment,
  // experiments): the costliest 1/d first, d = 1 sorts all.
  static const int topd = rt_getenv("RT_ORDER_TOP") ? std::max(1, atoi(rt_getenv("RT_ORDER_TOP"))) : 6;
  // RT_ORDER_TAIL=d (experiments): the cheapest 1/d of the tiles go last, in
  // tile order, so waves that run out of work early finish on short tiles.
  // Measured slower: C3 3.53-3.56 vs 3.43 ms, C4 5.25-5.29 vs 5.16 (d = 4, 8,
  // 16), 8-rank shares within 2 % (profiles/r03/order/tail.log): off.
  static const int taild = rt_getenv("RT_ORDER_TAIL") ? std::max(0, atoi(rt_getenv("RT_ORDER_TAIL"))) : 0;
  {
    const int top = n / topd;
    const int tail = taild > 0 ? std::min(n - top, n / taild) : 0;
    std::vector<char> cls(n, 1);  // 0 costliest (first, cost order), 1 middle, 2 cheapest (last)
    for (int i = 0; i < top; i++) cls[ord[i]] = 0;
    for (int i = n - tail; i < n; i++) cls[ord[i]] = 2;
    int k = top;
    for (int v = 0; v < n; v++)
      if (cls[v] == 1) ord[k++] = (uint32_t)v;
    for (int v = 0; v < n; v++)
      if (cls[v] == 2) ord[k++] = (uint32_t)v;
  }
  unsigned int* d = nullptr;
  HIP_TRY(hipMalloc((void**)&d, (size_t)n * sizeof(unsigned int)));
  if (hipMemcpy(d, ord.data(), (size_t)n * sizeof(unsigned int), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return fail(RT_E_DEVICE, "tile order upload failed");
  }
  c->orders[key] = d;
  *out = d;
  return RT_OK;
}

// Shared launch: contiguous rows [y0, y1) (stride == 0) or `ntrows` 8-row tile
// rows starting at tile row trow0 with stride `stride` (y0 = 0, y1 = height).
// est: the scene-setup cost estimate (estimate_costs) instead of a render.
static int launch(rt_context* c, int y0, int y1, int trow0, int stride, int ntrows, void* d_rgba, void* stream,
                  bool est) {
  const DevScene& s = c->sc;
  DeviceGuard guard(c->device);
  hipStream_t st = (hipStream_t)stream;
  // async contexts (the rt_render seam): switch to the specialised kernel as
  // soon as its background compile has finished (a failed compile leaves the
  // generic kernel, spec_failed set)
  if (c->spec_pending && !est) (void)spec_prepare(c);
  const bool lds = scene_in_lds(s);
  // Dynamic LDS: [scene blob (LDS flavour)] [VM records] [BVH stack]
  // [counters] [drained-head mask] [PCG jump rows] [frame cores of the first lds_levels levels]
  const int vm_off = lds ? s.blob_bytes : 0;
  const int stack_off = vm_off + ((lds && s.num_programs) ? WG * MAT * (int)sizeof(double) : 0);
  const int cnt_off = stack_off + (s.use_bvh ? WAVES_PER_WG * BVH_STACK * 12 : 0);
  const int qmask_off = cnt_off + CNT_BYTES;
  // per-wave object-record stream buffers (global linear scenes, RT_STREAM)
  const int jump_off = qmask_off + 16;  // after the drained-head mask: the sample-0 jump rows
  const int board_off = jump_off + 20 * 4 * (int)sizeof(uint64_t);  // work-sharing board (RT_SHARE)
  const uint64_t launch_pixels = (uint64_t)s.width * (uint64_t)(stride > 0 ? ntrows * TILE : y1 - y0);
  const int sch =
      est ? (int)SCH_SERIAL : pick_schedule(c->sched, s, launch_pixels, c->cus, c->inflight, c->spec_fn != nullptr);
  const int share_m = (c->spec_fn && !est) ? pick_share(c->share_mode, s, launch_pixels, c->cus, c->inflight) : 0;
  // The tile-cost estimate runs the ahead-of-time generic kernel (serial
  // samples, no sharing): its rays per tile do not depend on the kernel, and
  // a specialised variant of the estimate's schedule would be one more hipRTC
  // compile at scene setup (C1 / C4 / c4csg / canned render with quads: 0.4 -
  // 1.8 s in round 5).
  hipFunction_t spec = nullptr;  // built for this scene's flavour (spec_key), this schedule and sharing
  if (!est) {
    int rc = spec_for(c, sch, share_m, &spec);
    if (rc != RT_OK) return rc;
  }
  // (the brute-force specialised kernel, RT_CULL=0, reads records with scalar
  // loads instead: no stream buffers; tuning builds with RT_SPEC_EXTRA_FLAGS
  // keep the buffers: they may select the LDS stream)
  static const bool spec_extra = rt_getenv("RT_SPEC_EXTRA_FLAGS") != nullptr;
  const bool use_stream = !lds && !s.use_bvh && !s.has_csg && (spec_extra || !(spec && !(c->accel & RT_ACCEL_CULL)));
  // the generic kernels have no pairs flavour: quads instead (same pixels)
  const bool quads = sch == SCH_QUADS || (sch == SCH_PAIRS && !spec);
  const void* kfn = k_kernels[kernel_index(lds, s.use_bvh, s.has_csg, quads)];
  // the board is in LDS only for a kernel compiled with work sharing
  const bool share = spec && share_m == RT_SHARE_GROUP;  // (the device-wide board is in HBM)
  const int stream_off = board_off + (share ? BOARD_BYTES : 0);
  const int frames_off = stream_off + (use_stream ? WAVES_PER_WG * SCH * (GEO * (int)sizeof(double) + (int)sizeof(int)) : 0);
  int shmem = frames_off;
  auto occupancy = [&](int bytes) {
    int n = 0;
    if (spec) {
      if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, spec, WG, bytes) != hipSuccess) n = 0;
    } else if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kfn, WG, bytes) != hipSuccess) {
      n = 0;
    }
    return n;
  };
  // The occupancy queries take host time comparable to a small launch (a
  // strong-scaling share of a frame), so the plan is kept per (kernel, LDS).
  const void* plan_fn = spec ? (const void*)spec : kfn;
  const int frames = std::max(1, s.depth - 1);
  LaunchPlan& pl = c->plan;
  const bool plan_hit = pl.fn == plan_fn && pl.shmem_fixed == shmem && pl.frames == frames;
  int per_cu = plan_hit ? pl.per_cu : occupancy(shmem);
  if (per_cu <= 0) per_cu = 1;
  // The frame cores of the shallowest recursion levels live in the LDS that
  // is left over at this occupancy (never lowering it); deeper levels stay in
  // the HBM frame stack. RT_LDS_LEVELS=n caps the count (experiments).
  // RT_LDS_FULL=n (experiments) also moves the other frame fields (first
  // child's colour, pending refraction ray) of the first n levels to LDS.
  const int level_bytes = WAVES_PER_WG * CORE * 64 * (int)sizeof(double);
  const int ext_bytes = WAVES_PER_WG * EXT_ROWS * 64 * (int)sizeof(double);
  int lds_levels = plan_hit ? pl.lds_levels : 0, lds_full = plan_hit ? pl.lds_full : 0;
  if (!plan_hit && c->lds_per_cu > 0 && c->lds_per_block > 0) {
    const int avail = std::min(c->lds_per_block, c->lds_per_cu / std::min(per_cu, 8)) - shmem;
    if (const char* e = rt_getenv("RT_LDS_FULL")) lds_full = std::max(0, std::min(frames, atoi(e)));
    while (lds_full > 0 && lds_full * (ext_bytes + level_bytes) > avail) lds_full--;
    lds_levels = std::max(lds_full, std::min(frames, (avail - lds_full * ext_bytes) / level_bytes));
    if (const char* e = rt_getenv("RT_LDS_LEVELS")) lds_levels = std::max(lds_full, std::min(lds_levels, atoi(e)));
    while (lds_levels > 0 && occupancy(shmem + lds_levels * level_bytes + lds_full * ext_bytes) < per_cu) {
      lds_levels--;
      lds_full = std::min(lds_full, lds_levels);
    }
  }
  if (!plan_hit) pl = LaunchPlan{plan_fn, shmem, frames, per_cu, lds_levels, lds_full};
  const int ext_off = shmem + lds_levels * level_bytes;
  shmem = ext_off + lds_full * ext_bytes;
  static const bool dbg = rt_getenv("RT_DEBUG_LAUNCH") != nullptr;
  if (dbg)
    fprintf(stderr, "[launch] blocks/CU %d, LDS/block %d B (fixed %d, frame cores %d levels, full frames %d levels), frames %d\n",
            per_cu, shmem, frames_off, lds_levels, lds_full, frames);
  const int grid = c->cus * std::min(per_cu, 8);
  c->last_waves = grid * WAVES_PER_WG;
  c->launches++;
  if (grid * WAVES_PER_WG > c->stack_waves) return fail(RT_E_INVALID, "frame stack smaller than the grid");
  if (spec && share_m == RT_SHARE_DEVICE) {
    // device-wide board: zeroed (slots FREE, ring tickets 0) whenever its
    // layout changes, so a stale ticket can only name a slot of this layout
    const size_t need = (size_t)c->stack_waves * 64 * frames;
    if (need != c->gslots || frames != c->gframes) {
      (void)hipFree(c->gboard);
      c->gboard = nullptr;
      c->gslots = 0;
      // uncached (no XCD's L2 may hold a stale copy: rt_render.h gs_*)
      if (hipExtMallocWithFlags((void**)&c->gboard, need * GS_REC * sizeof(uint64_t), hipDeviceMallocUncached) !=
          hipSuccess)
        return fail(RT_E_NOMEM, "device-wide work-sharing slots");
      if (!c->gring && hipExtMallocWithFlags((void**)&c->gring, (size_t)GS_RING * sizeof(uint64_t),
                                             hipDeviceMallocUncached) != hipSuccess)
        return fail(RT_E_NOMEM, "device-wide work-sharing ring");
      if (!c->gctl && hipExtMallocWithFlags((void**)&c->gctl, GS_CTL_U64 * sizeof(uint64_t), hipDeviceMallocUncached) !=
                          hipSuccess)
        return fail(RT_E_NOMEM, "device-wide work-sharing control");
      HIP_TRY(hipMemsetAsync(c->gboard, 0, need * GS_REC * sizeof(uint64_t), st));
      HIP_TRY(hipMemsetAsync(c->gring, 0, (size_t)GS_RING * sizeof(uint64_t), st));
      HIP_TRY(hipMemsetAsync(c->gctl, 0, GS_CTL_U64 * sizeof(uint64_t), st));
      c->gslots = need;
      c->gframes = frames;
    }
  }
  Params P;
  std::memset(&P, 0, sizeof P);
  P.lds_frames_off = frames_off;
  P.lds_levels = lds_levels;
  P.lds_full = lds_full;
  P.stream_off = stream_off;
  P.lds_ext_off = ext_off;
  P.qmask_off = qmask_off;
  P.jump_off = jump_off;
  P.board_off = board_off;
  P.gboard = c->gboard;
  P.gring = c->gring;
  P.gctl = c->gctl;
  P.gslots = c->gslots;
  P.gset = c->qset;  // (alternates with the queue sets)
  P.off_geo = s.off_geo;
  P.off_shade = s.off_shade;
  P.off_mats = s.off_mats;
  P.off_lights = s.off_lights;
  P.off_kind = s.off_kind;
  P.off_objmat = s.off_objmat;
  P.off_pref = s.off_prefb;
  P.off_csg = s.off_csg;
  P.off_code = s.off_code;
  P.off_consts = s.off_consts;
  P.off_entry = s.off_entry;
  P.lds_vm_off = vm_off;
  P.vm_global = c->vm_global;
  P.blob_bytes = s.blob_bytes;
  P.jump = c->jump;
  // this launch dequeues from set qset and zeroes the other set for the next
  // one (launches on a context are stream-ordered): no memset per launch
  P.queue = c->queue + c->qset * QSET_ALLOC;
  P.queue_next = c->queue + (1 - c->qset) * QSET_ALLOC;
  P.stats = est ? c->est_stats : c->stats;
  P.stats_part = est ? nullptr : c->stats_part;  // the estimate's counts are not the frame's
  P.est_out = est ? c->est : nullptr;
#ifdef RT_PHASE_TIMING
  if (!c->wdiag && hipMalloc((void**)&c->wdiag, sizeof(unsigned long long) * 4 * 8192) != hipSuccess) c->wdiag = nullptr;
  if (c->wdiag) HIP_TRY(hipMemsetAsync(c->wdiag, 0, sizeof(unsigned long long) * 4 * 8192, st));
  P.wdiag = c->wdiag;
#endif
  P.stack = c->stack;
  P.out = (uint32_t*)d_rgba;
  P.width = s.width;
  P.height = s.height;
  P.depth = s.depth;
  P.nobj = s.nobj;
  P.nlights = s.nlights;
  P.y0 = y0;
  P.y1 = y1;
  P.trow0 = trow0;
  P.trow_stride = stride;
  P.tiles_x = (s.width + TILE - 1) / TILE;
  int tiles_y = stride > 0 ? ntrows : (y1 - y0 + TILE - 1) / TILE;
  // estimate: one unit per frame tile; a render: the launch's pixels, its
  // tiles dealt in order of estimated cost
  // (estimate points per tile: RT_EST_PTS=1 in the environment, experiments)
  static const int est_pts = rt_getenv("RT_EST_PTS") && atoi(rt_getenv("RT_EST_PTS")) == 1 ? 1 : 4;
  P.est_pts = est_pts;
  size_t slots = est ? (size_t)P.tiles_x * tiles_y * est_pts : (size_t)P.tiles_x * tiles_y * TILE * TILE;
  if (!est) {
    int rc = order_for(c, y0, trow0, stride, P.tiles_x, tiles_y, &P.order);
    if (rc != RT_OK) return rc;
  }
  if (slots >= 0xFFFFFFFFull - 2u * CHUNK * (size_t)grid * WAVES_PER_WG)
    return fail(RT_E_INVALID, "image too large for one launch");
  P.total_slots = (unsigned int)slots;
  P.frames = std::max(1, s.depth - 1);
  P.kind_mask = s.kind_mask;
  P.cnt_off = cnt_off;
  P.runs = reinterpret_cast<const int*>(s.accel + s.off_runs);
  P.nruns = s.nruns;
  P.arec = reinterpret_cast<const double*>(s.accel + s.off_arec);
  P.urec = reinterpret_cast<const double*>(s.accel + s.off_urec);
  if (s.use_bvh) {
    P.bvh_nodes = reinterpret_cast<const float*>(s.accel + s.off_nodes);
    P.bvh_geo = reinterpret_cast<const double*>(s.accel + s.off_bobj);
    P.planes = reinterpret_cast<const int*>(s.accel + s.off_planes);
    P.nplanes = s.nplanes;
    P.bvh_stack_off = stack_off;
    for (int k = 0; k < 3; k++) {
      P.bvh_lo[k] = s.bvh_lo[k];
      P.bvh_hi[k] = s.bvh_hi[k];
    }
  }

  // Launches on a context alternate between two sets of queue heads, each
  // launch zeroing the other set: a launch on another stream than the
  // previous one first waits for that launch to end.
  if (c->launched && st != c->last_stream) HIP_TRY(hipStreamWaitEvent(st, c->ev1, 0));
  c->last_stream = st;
  c->launched = true;
  if (!est) HIP_TRY(hipEventRecord(c->ev0, st));
  const char* blob = s.blob;
  void* args[] = {(void*)&blob, (void*)&P};
  if (spec)
    HIP_TRY(hipModuleLaunchKernel(spec, grid, 1, 1, WG, 1, 1, shmem, st, args, nullptr));
  else
    HIP_TRY(hipLaunchKernel(kfn, dim3(grid), dim3(WG), args, shmem, st));
  HIP_TRY(hipGetLastError());
  c->qset ^= 1;
  HIP_TRY(hipEventRecord(c->ev1, st));
  if (est) return RT_OK;
  c->timed = true;
  c->last_spec = spec != nullptr;
  uint64_t rows = 0;
  if (stride > 0) {
    for (int j = 0; j < ntrows; j++) {
      int r0 = (trow0 + j * stride) * TILE;
      rows += (uint64_t)std::max(0, std::min((int)TILE, s.height - r0));
    }
  } else {
    rows = (uint64_t)(y1 - y0);
  }
  c->primary_pending += (uint64_t)4 * (uint64_t)s.width * rows;
  return RT_OK;
}

// Which scenes get a tile order: scenes in LDS (C2, C3, C4's BVH, c4csg).
// Scenes read from HBM lose by it: the BVH of C5 (100 k spheres) runs from the
// L2, and tiles dealt out of neighbourhood order thrash it (C5 517-527 vs
// 459-479 ms unordered); the brute-force search over a large scene would pay
// a costly estimate. RT_TILE_ORDER=0 / 2 (environment, experiments): never /
// also for HBM scenes with a BVH.
static bool want_order(const rt_context* c) {
  static const int env = rt_getenv("RT_TILE_ORDER") ? atoi(rt_getenv("RT_TILE_ORDER")) : 1;
  const DevScene& s = c->sc;
  return env != 0 && c->order_on && s.nobj > 0 && (scene_in_lds(s) || (env == 2 && s.use_bvh));
}

// Scene setup: the estimate launch (one centre sample per frame tile, traced
// rays counted per tile), synchronous, its wall time kept in order_ms.
static int estimate_costs(rt_context* c) {
  clear_orders(c);
  if (!want_order(c)) return RT_OK;
  const DevScene& s = c->sc;
  DeviceGuard guard(c->device);
  const size_t n = (size_t)((s.width + TILE - 1) / TILE) * ((s.height + TILE - 1) / TILE);
  if (n > c->est_cap) {
    (void)hipFree(c->est);
    c->est = nullptr;
    c->est_cap = 0;
    HIP_TRY(hipMalloc((void**)&c->est, n * sizeof(unsigned int)));
    c->est_cap = n;
  }
  if (!c->est_stats) {
    HIP_TRY(hipMalloc((void**)&c->est_stats, sizeof(unsigned long long) * 64));
    HIP_TRY(hipMemset(c->est_stats, 0, sizeof(unsigned long long) * 64));
  }
  const auto t0 = std::chrono::steady_clock::now();
  HIP_TRY(hipMemset(c->est, 0, n * sizeof(unsigned int)));
  int rc = launch(c, 0, s.height, 0, 0, 0, nullptr, nullptr, true);
  if (rc != RT_OK) return rc;
  std::vector<uint32_t> cost(n);
  HIP_TRY(hipMemcpy(cost.data(), c->est, n * sizeof(unsigned int), hipMemcpyDeviceToHost));  // (synchronises)
  unsigned long long wd = 0;
  HIP_TRY(hipMemcpy(&wd, c->est_stats + ST_WATCHDOG, sizeof wd, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemset(c->est_stats, 0, sizeof(unsigned long long) * 64));
  if (wd) return fail(RT_E_DEVICE, "render watchdog in the tile-cost estimate (kernel bug)");
  c->tile_cost.swap(cost);
  c->order_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  c->timed = false;
  return RT_OK;
}

int rt_set_work_sharing(rt_context* c, int enable) {
  if (!c) return fail(RT_E_INVALID, "rt_set_work_sharing: NULL context");
  if (enable < 0 || enable > RT_SHARE_AUTO) return fail(RT_E_INVALID, "rt_set_work_sharing: unknown mode");
  c->share_mode = enable;
  return c->has_scene ? spec_prepare(c) : RT_OK;
}

int rt_set_tile_order(rt_context* c, int enable) {
  if (!c) return fail(RT_E_INVALID, "rt_set_tile_order: NULL context");
  c->order_on = enable != 0;
  if (!c->has_scene) return RT_OK;
  if (!c->order_on) {
    clear_orders(c);
    return RT_OK;
  }
  return c->tile_cost.empty() ? estimate_costs(c) : RT_OK;
}

int rt_tile_order_info(rt_context* c, int* active, double* estimate_ms) {
  if (!c || !active || !estimate_ms) return fail(RT_E_INVALID, "rt_tile_order_info: NULL argument");
  *active = c->tile_cost.empty() ? 0 : 1;
  *estimate_ms = c->order_ms;
  return RT_OK;
}

int rt_render_rows_async(rt_context* c, int y0, int y1, void* d_rgba, void* stream) {
  if (!c || !c->has_scene) return fail(RT_E_INVALID, "rt_render_rows_async: no scene set");
  if (!d_rgba) return fail(RT_E_INVALID, "rt_render_rows_async: NULL output");
  if (y0 < 0 || y1 > c->sc.height || y1 <= y0) return fail(RT_E_INVALID, "rt_render_rows_async: bad row range");
  return launch(c, y0, y1, 0, 0, 0, d_rgba, stream, false);
}

int rt_render_tile_rows_async(rt_context* c, int trow0, int trow_stride, int ntrows, void* d_rgba, void* stream) {
  if (!c || !c->has_scene) return fail(RT_E_INVALID, "rt_render_tile_rows_async: no scene set");
  if (!d_rgba) return fail(RT_E_INVALID, "rt_render_tile_rows_async: NULL output");
  if (trow0 < 0 || trow_stride <= 0 || ntrows <= 0) return fail(RT_E_INVALID, "rt_render_tile_rows_async: bad tile rows");
  return launch(c, 0, c->sc.height, trow0, trow_stride, ntrows, d_rgba, stream, false);
}


int rt_read_stats(rt_context* c, void* stream, int reset, rt_stats* out) {
  if (!c || !out) return fail(RT_E_INVALID, "rt_read_stats: NULL argument");
  DeviceGuard guard(c->device);
  hipStream_t st = (hipStream_t)stream;
  unsigned long long h[ST_COUNT] = {}, wd = 0;
  // frame counters: one record per workgroup slot, summed here
  std::vector<unsigned long long> part((size_t)STATS_PART * c->stats_parts);
  HIP_TRY(hipMemcpyAsync(part.data(), c->stats_part, part.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&wd, c->stats + ST_WATCHDOG, sizeof wd, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  for (int b = 0; b < c->stats_parts; b++)
    for (int k = 0; k < ST_COUNT; k++) h[k] += part[(size_t)b * STATS_PART + k];
  if (wd) {
    // the frames since the last reset are incomplete: clear everything (as a
    // reset would) so that later reads report later launches, then fail
    HIP_TRY(hipMemsetAsync(c->stats, 0, sizeof(unsigned long long) * 64, st));
    HIP_TRY(hipMemsetAsync(c->stats_part, 0, part.size() * sizeof(unsigned long long), st));
    c->gslots = 0;  // a stopped launch may leave device-wide board slots claimed: rebuilt at the next launch
    HIP_TRY(hipStreamSynchronize(st));
    c->primary_pending = 0;
    c->launches = 0;
    return fail(RT_E_DEVICE, "render watchdog: " + std::to_string(wd) + " waves stopped unfinished (kernel bug)");
  }
  std::memset(out, 0, sizeof *out);
  // Intersect calls from closestHit: every traced ray tests every object.
  uint64_t per_kind[RT_NUM_KINDS] = {0, 0, 0, 0, 0};
  if (c->has_scene)
    for (int k : c->sc.kinds) per_kind[k]++;
  out->primary_rays = c->primary_pending;
  out->secondary_rays = h[ST_TRACED] - c->primary_pending;
  out->shadow_rays = h[ST_SHADOW];
  for (int k = 0; k < RT_NUM_KINDS; k++) {
    out->tests[k] = h[ST_TRACED] * per_kind[k];
    out->shadow_tests[k] = h[ST_STESTS + k];
  }
  out->shaded_hits = h[ST_SHADED];
  out->surface_errors = h[ST_SURFERR];
#ifdef RT_PHASE_TIMING
  {
    unsigned long long ph[N_PHASE];
    HIP_TRY(hipMemcpy(ph, c->stats + ST_PHASE, sizeof ph, hipMemcpyDeviceToHost));
    unsigned long long tot = 0;
    for (int k = 0; k < N_PHASE; k++) tot += ph[k];
    if (tot) {
      static const char* nm[N_PHASE] = {"refill", "gen", "trace_loop", "trace_unwind", "shade_surface",
                                        "light_dirs", "shadow_loops", "lighting", "material", "shade_unwind"};
      fprintf(stderr, "[phase]");
      for (int k = 0; k < N_PHASE; k++) fprintf(stderr, " %s=%.3f", nm[k], (double)ph[k] / (double)tot);
      fprintf(stderr, " total_wave_cycles=%.4g\n", (double)tot);
      unsigned long long bd[8];
      HIP_TRY(hipMemcpy(bd, c->stats + ST_BVHDIAG, sizeof bd, hipMemcpyDeviceToHost));
      if (c->wdiag && c->last_waves > 0) {
        // last launch: lifetime percentiles, and the longest waves' last chunk
        std::vector<unsigned long long> w((size_t)c->last_waves * 4);
        HIP_TRY(hipMemcpy(w.data(), c->wdiag, w.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        std::vector<std::pair<unsigned long long, int>> life;
        for (int i = 0; i < c->last_waves; i++) life.push_back({w[(size_t)i * 4], i});
        std::sort(life.begin(), life.end());
        auto pct = [&](double q) { return (double)life[std::min(life.size() - 1, (size_t)(q * life.size()))].first; };
        fprintf(stderr, "[tail] lifetime p10 %.4g p50 %.4g p90 %.4g p99 %.4g max %.4g;", pct(0.1), pct(0.5), pct(0.9),
                pct(0.99), (double)life.back().first);
        for (int k = 1; k <= 4 && k <= (int)life.size(); k++) {
          const int i = life[life.size() - k].second;
          fprintf(stderr, " [life %.4g chunks %llu last-chunk %.4g]", (double)w[(size_t)i * 4], w[(size_t)i * 4 + 1],
                  (double)w[(size_t)i * 4 + 2]);
        }
        double lc = 0;
        for (int i = 0; i < c->last_waves; i++) lc += (double)w[(size_t)i * 4 + 2];
        fprintf(stderr, " mean last-chunk %.4g\n", lc / c->last_waves);
      }
#ifdef RT_CSG_DIAG
      {
        unsigned long long cd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyFromSymbol(cd, HIP_SYMBOL(g_csg_diag), sizeof cd) == hipSuccess && cd[0]) {
          fprintf(stderr, "[csg] searches %llu, register-list overflows %llu (%.2f%%), mean live leaves %.2f\n", cd[0],
                  cd[1], 100.0 * cd[1] / cd[0], (double)cd[2] / cd[0]);
          if (cd[6])
            fprintf(stderr,
                    "[csg] group visits %llu: leaf-major iterations %llu (lanes %.1f of 64), lane-major %llu (lanes "
                    "%.1f), lane-leaf candidates %llu\n",
                    cd[6], cd[3], cd[3] ? (double)cd[5] / cd[3] : 0.0, cd[4], cd[4] ? (double)cd[5] / cd[4] : 0.0, cd[5]);
        }
      }
#endif
      {
        unsigned long long sh[6];
        HIP_TRY(hipMemcpy(sh, c->stats + ST_SHDIAG, sizeof sh, hipMemcpyDeviceToHost));
        fprintf(stderr, "[share] posted samples %llu subtrees %llu, claims %llu, reclaims %llu, waits %llu, idle polls %llu\n",
                sh[0], sh[1], sh[2], sh[3], sh[4], sh[5]);
      }
      {
        unsigned long long pd[6];
        HIP_TRY(hipMemcpy(pd, c->stats + ST_PASSDIAG, sizeof pd, hipMemcpyDeviceToHost));
        fprintf(stderr, "[passes] trace %llu (%.1f lanes), shade %llu (%.1f lanes), gen %llu (%.1f lanes)\n", pd[0],
                (double)pd[1] / std::max(1ull, pd[0]), pd[2], (double)pd[3] / std::max(1ull, pd[2]), pd[4],
                (double)pd[5] / std::max(1ull, pd[4]));
        unsigned long long ld[2];
        HIP_TRY(hipMemcpy(ld, c->stats + ST_LANEDIAG, sizeof ld, hipMemcpyDeviceToHost));
        fprintf(stderr, "[lanes] rounds %llu, lanes waiting in S_DONE (finished quad / pair samples) %.2f per round\n", ld[1],
                (double)ld[0] / (double)std::max(1ull, ld[1]));
      }
      unsigned long long steps = 0;
      HIP_TRY(hipMemcpy(&steps, c->stats + ST_CLOCKSTEP, sizeof steps, hipMemcpyDeviceToHost));
      const double nw = std::max(1.0, (double)c->last_waves * c->launches - (double)steps);
      fprintf(stderr, "[waves] lifetime mean %.4g cycles, max %.4g cycles (mean/max %.3f; %llu waves with a clock step left out)\n",
              (double)bd[6] / nw, (double)bd[7], (double)bd[6] / nw / (double)std::max(1ull, bd[7]), steps);
      if (bd[4] + bd[5])
        fprintf(stderr, "[bvh] wave traversals trace=%llu shadow=%llu; nodes/traversal trace=%.1f shadow=%.1f; "
                        "leaves/traversal trace=%.1f shadow=%.1f\n", bd[4], bd[5], (double)bd[0] / (double)std::max(1ull, bd[4]),
                (double)bd[1] / (double)std::max(1ull, bd[5]), (double)bd[2] / (double)std::max(1ull, bd[4]),
                (double)bd[3] / (double)std::max(1ull, bd[5]));
#ifdef RT_EXACT_DIAG
      unsigned long long ex[2 * RT_NUM_KINDS + 2];
      HIP_TRY(hipMemcpy(ex, c->stats + ST_EXDIAG, sizeof ex, hipMemcpyDeviceToHost));
      fprintf(stderr, "[exact] lane tests after culling per kind (trace/shadow):");
      for (int k = 0; k < RT_NUM_KINDS; k++) fprintf(stderr, " k%d=%llu/%llu", k, ex[2 * k], ex[2 * k + 1]);
      fprintf(stderr, "; wave batches trace=%llu shadow=%llu\n", ex[2 * RT_NUM_KINDS], ex[2 * RT_NUM_KINDS + 1]);
#endif
    }
  }
#endif
  float ms = 0.f;
  if (c->timed && hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) out->kernel_ms = ms;
  out->devices = 1;
  out->device_kernel_ms[0] = out->kernel_ms;
  if (reset) {
    HIP_TRY(hipMemsetAsync(c->stats, 0, sizeof(unsigned long long) * 64, st));
    HIP_TRY(hipMemsetAsync(c->stats_part, 0, part.size() * sizeof(unsigned long long), st));
    HIP_TRY(hipStreamSynchronize(st));
    c->primary_pending = 0;
    c->launches = 0;
  }
  return RT_OK;
}

int rt_last_kernel_ms(rt_context* c, double* ms_out) {
  if (!c || !ms_out) return fail(RT_E_INVALID, "rt_last_kernel_ms: NULL argument");
  if (!c->timed) return fail(RT_E_INVALID, "rt_last_kernel_ms: nothing rendered yet");
  DeviceGuard guard(c->device);
  HIP_TRY(hipEventSynchronize(c->ev1));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  *ms_out = ms;
  return RT_OK;
}

int rt_debug_run_surface(rt_context* c, int program, int n, const long long* face, const double* u,
                         const double* v, double* out10, int* err) {
  if (!c || !c->has_scene || n <= 0 || !face || !u || !v || !out10 || !err)
    return fail(RT_E_INVALID, "rt_debug_run_surface: bad arguments");
  if (program < 0 || program >= c->sc.num_programs) return fail(RT_E_INVALID, "rt_debug_run_surface: no such program");
  DeviceGuard guard(c->device);
  long long* df = nullptr;
  double *du = nullptr, *dv = nullptr, *dout = nullptr;
  int* derr = nullptr;
  int rc = RT_OK;
  if (hipMalloc((void**)&df, n * sizeof(long long)) != hipSuccess || hipMalloc((void**)&du, n * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&dv, n * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&dout, (size_t)n * 10 * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&derr, n * sizeof(int)) != hipSuccess)
    rc = fail(RT_E_NOMEM, "rt_debug_run_surface: alloc");
  if (rc == RT_OK && (hipMemcpy(df, face, n * sizeof(long long), hipMemcpyHostToDevice) != hipSuccess ||
                      hipMemcpy(du, u, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
                      hipMemcpy(dv, v, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess))
    rc = fail(RT_E_DEVICE, "rt_debug_run_surface: copy");
  if (rc == RT_OK) {
    hipLaunchKernelGGL(rt_debug_vm_kernel, dim3((n + 63) / 64), dim3(64), 0, nullptr, (const char*)c->sc.blob,
                       c->sc.off_code, c->sc.off_consts, c->sc.off_entry, program, df, du, dv, dout, derr, n);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      rc = fail(RT_E_DEVICE, "rt_debug_run_surface: launch");
  }
  if (rc == RT_OK && (hipMemcpy(out10, dout, (size_t)n * 10 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
                      hipMemcpy(err, derr, n * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess))
    rc = fail(RT_E_DEVICE, "rt_debug_run_surface: copy back");
  (void)hipFree(df);
  (void)hipFree(du);
  (void)hipFree(dv);
  (void)hipFree(dout);
  (void)hipFree(derr);
  return rc;
}

}  // extern "C"

#include "rt_ssim.hip"
#include "rt_render_api.hip"

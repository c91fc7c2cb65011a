// rt_render.h -- device side of the render megakernel (see rt_kernel.hip for
// the execution model and the scene blob layout notes at the top of this file).
//
// Compiled twice:
//   * ahead of time into librtamd.so by rt_kernel.hip (generic flavours:
//     object count and kinds read from the scene blob at run time);
//   * at run time through hipRTC when a context enables scene specialisation
//     (rt_set_specialize): the same source with RT_SPEC_NOBJ / RT_SPEC_KINDS
//     defined, so the closestHit and inShadow object loops of a small linear
//     scene are fully unrolled with compile-time primitive kinds. Same
//     operations in the same order -> bit-identical images and counters.
#pragma once
#pragma clang fp contract(off)

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

#include "rt_abi.h"
#include "rt_device.h"

#ifndef RT_SHADE_NUM
#define RT_SHADE_NUM 3  // shade when >= NUM/DEN of the wave's busy lanes hold a hit
#endif
#ifndef RT_SHADE_DEN
#define RT_SHADE_DEN 4
#endif
#ifndef RT_DIV_SKIP
#define RT_DIV_SKIP 0  // skip divisions whose sign proves t <= 0 (exact, see t_nonpos): measured
                       // slower -- a skip pays only when the whole wave skips, the tests and
                       // branches are paid always
#endif
// Framebuffer stores (raytracer.go:656): a lane holds its finished pixel and
// the wave stores all held pixels with one instruction when a holder is about
// to finish another pixel, and at exit -- instead of one store per scheduling
// round in which some lane finished (0: store at once, A/B).
#ifndef RT_PIX_BATCH
#define RT_PIX_BATCH 1
#endif
// Pixel pairs (specialised kernels, the host's RT_SCHED_PAIRS): with the
// serial-sample flavour (QUADS = false), a pixel's samples 0-1 run in an even
// lane and 2-3 in the odd lane after it; the even lane adds the four colours
// in sample order.
#ifndef RT_PAIRS
#define RT_PAIRS 0
#endif
#ifndef RT_FRAME_PREFETCH
#define RT_FRAME_PREFETCH 1  // load the parent frame during the TRACE pass
#endif
#ifndef RT_CULL
#define RT_CULL 1  // wave-uniform conservative bounding-sphere culling (exact, see may_hit)
#endif
#ifndef RT_STMAX_F32
#define RT_STMAX_F32 1  // shadow-ray cull bound dist/|d| from an FP32 reciprocal (exact: bound only; C3 -1..-1.7 %)
#endif
#ifndef RT_STREAM_PREFETCH
#define RT_STREAM_PREFETCH 0  // next record in registers while the current one is tested: measured slower
                              // (brute-force C5 480x270: 2.98 vs 2.51 s; 2x / 4x unrolling also slower)
#endif
#ifndef RT_STREAM
#define RT_STREAM 1  // global linear scenes: object records stream through per-wave LDS buffers
#endif
#ifndef RT_STREAM_SMEM
#define RT_STREAM_SMEM 1  // ... or, in the brute-force build (RT_CULL=0), through scalar loads in kind runs
#endif
#ifndef RT_SHADOW_JOINT
#define RT_SHADOW_JOINT 1  // brute force, specialised light count: one sweep for all shadow rays of a hit
#endif
#ifndef RT_SHADOW_CHECK
#define RT_SHADOW_CHECK 8  // brute-force shadow runs: wave-level "any ray open?" test every N objects
#endif
#ifndef RT_CULL_NOBRANCH
#define RT_CULL_NOBRANCH 1  // cull tests combined without short-circuit branches (see CULL_AND)
#endif
// a && b for the pure, cheap lane predicates of the culls: evaluated on every
// lane without a branch (no exec-mask save/restore, and the result stays a
// lane mask for the wave's any-lane test instead of being rematerialised)
#if RT_CULL_NOBRANCH
#define CULL_AND(a, b) (bool)((int)(bool)(a) & (int)(bool)(b))
#else
#define CULL_AND(a, b) ((a) && (b))
#endif
#ifndef RT_AXIS_LEAF
#define RT_AXIS_LEAF 0  // BVH leaves' scale + translation spheres take the diagonal transform (exact, see axis_o);
                        // measured: C4 +3 % (a branch per leaf object, more spills), C5 within noise: off
#endif
#ifndef RT_CUBE_FAST
#define RT_CUBE_FAST 1  // axis-aligned cube faces (bit-identical, see cube_hit)
#endif

using namespace rt;

// Scene specialisation (hipRTC build, see rt_kernel.hip spec_compile): the
// object kinds and the scene features below are compile-time constants, so
// branches for kinds, surface programs and light kinds the scene lacks fold
// away. The generic build keeps every branch (all bits set).
enum { SF_VM = 1, SF_LDIR = 2, SF_LSPOT = 4 };  // closure surfaces, directional / spot lights
#ifdef RT_SPEC_NOBJ
constexpr int spec_kinds[RT_SPEC_NOBJ] = {RT_SPEC_KINDS};
constexpr int spec_kind_mask() {
  int m = 0;
  for (int i = 0; i < RT_SPEC_NOBJ; i++) m |= 1 << spec_kinds[i];
  return m;
}
constexpr int SPEC_KMASK = spec_kind_mask();
constexpr int SPEC_FEAT = RT_SPEC_FEAT;
static_assert(SPEC_KMASK == RT_SPEC_KMASK, "RT_SPEC_KINDS and RT_SPEC_KMASK disagree");
#elif defined(RT_SPEC_KMASK)
constexpr int SPEC_KMASK = RT_SPEC_KMASK;
constexpr int SPEC_FEAT = RT_SPEC_FEAT;
#else
constexpr int SPEC_KMASK = -1;
constexpr int SPEC_FEAT = -1;
#endif
// May the scene hold objects of kind k / use feature f?
__device__ constexpr bool spec_kind(int k) { return ((SPEC_KMASK >> k) & 1) != 0; }
__device__ constexpr bool spec_feat(int f) { return (SPEC_FEAT & f) != 0; }

// ---------------------------------------------------------------------------
// Scene blob (built by rt_set_scene), one contiguous allocation, 16-B aligned
// sections; strides in doubles:
// geo    [nobj][GEO]  0..11 WorldToObject rows 0-2; planes: 12..14 normal, 15 D;
//                     bounded kinds: 12..13 = 4 floats (centre xyz, padded
//                     radius^2) of a world-space bounding sphere (culling only)
// shade  [nobj][SHD]  0..11 ObjectToWorld rows 0-2, 12..29 NormalWorld per face;
//                     planes: 16..19 = 8 floats of the world-space plane for
//                     culling (see may_hit_plane)
// mats   [nmat][MAT]  0..2 colour, 3 reflectivity, 4..5 baked fuzz offset
//                     (fuzz*cos^2, fuzz*sin^2; raytracer.go:517-521), 6 fuzz>=0,
//                     7 transparency, 8 ior, 9 kd, 10 ks, 11 specular exponent
// lights [nl][LGT]    0..2 position, 3..5 colour, 6..8 directional: normalize(-dir),
//                     spot: normalize(at - pos); 9 kind, 10 spot cos(cutoff),
//                     11 spot exponent (kinds: include/rt_abi.h RT_LIGHT_*)
// kind   [nobj] int32;  objmat [nobj][OMAT] int32 per-face material index
// ---------------------------------------------------------------------------
enum { GEO = 16, SHD = 32, MAT = 16, LGT = 16, OMAT = 8, GLOB = 16 };
// GLOB record (head of the lights section): 0..2 ambient, 3..5 bg start,
// 6..8 bg end, 9 viewport width, 10 viewport height, 11 exp mode (RT_EXP_*,
// the Exp/Log of a fractional Pow) (read where used, so they
// do not occupy scalar registers across the whole kernel)
// Frame of one traceRay activation that has children (post-order combine).
// Global layout, lane-interleaved rows: Lw[3] ext[6] kr packed colour[3]
// reflectivity (the last four for VM materials only). ext holds the pending
// refraction ray (o, d) while the reflection child runs, then -- the ray read
// -- the reflection child's colour in its first three rows (a glass frame keeps
// 6 rows, not 9: a third fewer dirty lines written back per frame). The CORE
// fields (Lw, kr, packed) of the first P.lds_levels levels live in LDS
// instead, ext of the first P.lds_full levels too; the rest live in HBM.
enum { FRAME_FIELDS = 15, CORE = 5, EXT_ROWS = 6, FR_EXT = 3, FR_COL = 11, FR_REFL = 14 };
enum { CHUNK = 64, TILE = 8, WG = 256, WAVES_PER_WG = WG / 64 };
// Work queue: pixels per dequeue -- one 8x8 tile, or with pixel quads a 4x4
// quarter of one (16 quads = one wave's lanes) -- from QHEADS queue heads
// (chunk c belongs to head c mod QHEADS; a workgroup dequeues from head
// blockIdx mod QHEADS, see RT_QSTEAL), so the dequeue rate
// stays below what one atomic word sustains.
#ifndef RT_QHEADS
#define RT_QHEADS 8
#endif
enum { QHEADS = RT_QHEADS /* <= 32: the drained-head mask is 32 bits */, QSTRIDE = 16 /* u32 between heads: 64 B */ };
static_assert(RT_QHEADS >= 1 && RT_QHEADS <= 32, "RT_QHEADS");
// Heads a workgroup dequeues from: its home head, then RT_QSTEAL others once
// that is drained. Every head is drained by its home workgroups, so stopping
// early never drops a chunk; it bounds the end-of-launch probes (each a
// returning atomic, serialised per head address: probing all 8 heads from
// every wave cost ~45 us per launch). A workgroup shares the heads it found
// drained through an LDS mask. One steal head: C3/C4 whole frames as with
// all 7, a one-tile-row launch 85 -> 37 us, C2 0.38 -> 0.33 ms
// (profiles/r02/qsteal). Not kept: launch-wide drained flags read before
// stealing (one line written by every overflowing wave: slower).
#ifndef RT_QSTEAL
#define RT_QSTEAL 1
#endif
enum { QSET = QHEADS * QSTRIDE /* u32 per launch set of heads */,
       QSET_ALLOC = 32 * QSTRIDE /* host: room for any RT_QHEADS build */ };
#ifndef RT_QCHUNK_PIXEL
#define RT_QCHUNK_PIXEL 64  // pixels per dequeue without quads (a multiple of 16 dividing 64)
#endif
enum { SCH = 32 };  // objects per stream chunk (RT_STREAM): SCH * GEO * 8 B + SCH * 4 B per wave
enum { ST_SHADOW = 0, ST_TRACED = 1, ST_SHADED = 2, ST_SURFERR = 3, ST_STESTS = 4, ST_COUNT = ST_STESTS + RT_NUM_KINDS,
       ST_PHASE = 16, N_PHASE = 10, ST_BVHDIAG = 26, ST_EXDIAG = 34, ST_SHDIAG = 48, ST_PASSDIAG = 54,
       ST_CLOCKSTEP = 60, ST_LANEDIAG = 61 /* 61: lanes waiting in S_DONE, summed over rounds; 62: rounds */,
       ST_WATCHDOG = 63,
       STATS_PART = 16 /* u64 per workgroup record: one 128-B line */ };
// Diagnostic build (RT_PHASE_TIMING): work-sharing events, ST_SHDIAG + k:
// 0 samples posted, 1 subtrees posted, 2 claims, 3 reclaims, 4 waits, 5 rounds
// a wave spent polling idle
enum { SH_POST_S = 0, SH_POST_T = 1, SH_CLAIM = 2, SH_RECLAIM = 3, SH_WAIT = 4, SH_SPIN = 5 };
#ifdef RT_PHASE_TIMING
#define SHDIAG(k) atomicAdd(P.stats + ST_SHDIAG + (k), 1ull)
#else
#define SHDIAG(k) (void)0
#endif  // (stats buffer: 64 entries)
enum { S_IDLE = 0, S_TRACE = 1, S_SHADE = 2, S_DONE = 3 };  // S_DONE: sample colour held for the quad
#ifndef RT_LDS_MAX
#define RT_LDS_MAX (40 * 1024)
#endif
enum { LDS_MAX_BYTES = RT_LDS_MAX };
// PCG jump table entries: (row within the 20-row strip) x (sample 0..3)
enum { JUMP_ENTRIES = 20 * 4 };

// Cost estimate (Params::est_out): sample 0 of est_pts (1 or 4) pixels per
// 8x8 tile -- its centre, or the centres of its four 4x4 quarters.
__device__ __forceinline__ int est_x(int pts, unsigned int k) { return pts == 1 ? TILE / 2 : 2 + 4 * (int)(k & 1u); }
__device__ __forceinline__ int est_y(int pts, unsigned int k) { return pts == 1 ? TILE / 2 : 2 + 4 * (int)((k >> 1) & 1u); }

struct Params {
  int lds_frames_off;  // byte offset of the LDS frame cores in dynamic LDS
  int lds_levels;      // recursion levels whose frame core lives in LDS (host: LDS left at full occupancy)
  int lds_full;        // recursion levels whose other frame fields (3..11) live in LDS too
  int lds_ext_off;     // byte offset of those fields in dynamic LDS
  int stream_off;      // byte offset of the per-wave object-record stream buffers (global linear scenes)
  int qmask_off;       // byte offset of the workgroup's drained-head mask in LDS
  int jump_off;        // byte offset of the LDS copy of the sample-0 jump rows (serial samples)
  int off_geo, off_shade, off_mats, off_lights, off_kind, off_objmat, off_pref, off_csg, off_code, off_consts,
      off_entry, blob_bytes;
  int lds_vm_off;     // LDS byte offset of the per-lane VM material records (LDS flavour)
  double* vm_global;  // per-lane VM material records (global flavour)
  const uint64_t* jump;  // [20 rows][4 samples][ahi alo chi clo]: 8*r + 2*k LCG steps
  unsigned int* queue;       // this launch's QHEADS queue heads (zero at launch)
  unsigned int* queue_next;  // the next launch's heads: zeroed here by block 0
  unsigned long long* stats;  // watchdog and diagnostic counters (atomics)
  // Frame counters ST_SHADOW .. ST_STESTS + kinds, one STATS_PART record per
  // workgroup slot, added at exit without atomics (only this workgroup writes
  // its record; launches on a context are stream-ordered); the host sums the
  // records. nullptr (the tile-cost estimate): not counted.
  unsigned long long* stats_part;
  unsigned long long* wdiag;  // diagnostic build: per wave [lifetime, chunks, cycles since last chunk grab, 0]
  double* stack;
  uint32_t* out;
  int width, height, depth, nobj, nlights, y0, y1, tiles_x;
  int trow0, trow_stride;  // trow_stride > 0: output tile row j renders image tile row trow0 + j*stride
  unsigned int total_slots;
  int frames;  // stack frames per lane (depth - 1, >= 1)
  // BVH flavour (scenes with many bounded objects)
  const float* bvh_nodes;  // internal nodes [n][BN] (see BvhBuild)
  const double* bvh_geo;   // leaf objects in BVH order: geo record, 14 = index, 15 = kind
  const int* planes;       // unbounded objects, ascending index
  int nplanes, bvh_stack_off;
  double bvh_lo[3], bvh_hi[3];  // padded box around every BVH object (far_shift)
  // Global linear scenes: maximal runs of consecutive objects of one kind,
  // [nruns][4] = first index, count, kind, 0 (brute-force scalar-load loops)
  const int* runs;
  int nruns;
  const double* arec;  // [nobj][AXIS_REC] compact records of axis-aligned spheres (runs with axis = 1)
  const double* urec;  // [nobj][UNI_REC] uniform-scale spheres: m3 m7 m11 m0 (runs with axis = 2)
  int cnt_off;    // LDS byte offset of the event counters (CNT_BYTES)
  int kind_mask;  // bit k: the scene has objects of kind k
  int board_off;  // LDS byte offset of the work-sharing board (RT_SHARE == 1)
  // device-wide work sharing (RT_SHARE == 2): slots [wave slot][lane][level]
  // of GS_REC u64, the ring of posted slot ids (GS_RING), the ring's head and
  // tail tickets (control block of GS_CTL_U64 u64)
  uint64_t* gboard;
  uint64_t* gring;
  uint64_t* gctl;
  int gset;  // this launch's counter set (0 / 1); it zeroes the other
  unsigned long long gslots;  // slots gboard holds (a ticket naming another is ignored)
  // Tile order (host: scene-setup cost estimate, most expensive first): the
  // pool's virtual tile v renders tile order[v] of the launch; nullptr = in order
  const unsigned int* order;
  // Cost-estimate launch (est_out != nullptr): est_pts units per 8x8 tile of
  // the frame, each one pixel's sample 0 traced in full; est_out[tile] counts
  // the rays traced for them. Serial-sample kernel only; nothing is written to out.
  unsigned int* est_out;
  int est_pts;  // estimate pixels per tile (1 or 4)
};
// Per-lane event counters (u64, LDS, fire-and-forget ds_add), reduced once per
// workgroup at exit: per-wave 64-bit SGPR counters pushed the kernel into
// SGPR spilling (C2 +33% time, C3 +7%).
// Unit events (traced rays, shaded hits, surface errors) are counted per wave
// (lane 0 adds the ballot's popcount); per-kind shadow-test tallies per lane.
// LDS: [NUNIT][WAVES_PER_WG] then, CNT_KIND_OFF bytes in, [RT_NUM_KINDS][WG].
enum { CNT_TRACED = 0, CNT_SHADED = 1, CNT_SURFERR = 2, NUNIT = 3, CNT_KIND_OFF = 128,
       CNT_BYTES = CNT_KIND_OFF + RT_NUM_KINDS * WG * 8 };
enum { PREF = 8 };  // u32 per prefix-count entry (RT_NUM_KINDS used, 16-B aligned)
// BVH node: child 0 box (lo xyz, hi xyz), child 1 box, then as int: ref 0,
// ref 1, smallest object index under child 0, under child 1. A ref is
// (node << 3) for an internal node, (first << 3) | count for a leaf of
// `count` (1..4) consecutive bvh_geo records.
enum { BN = 16, BVH_STACK = 64 };
// (Measured and removed in round 5: a 4-wide BVH, C4 4.20 vs 4.17 ms, C5 351
// vs 317 ms serial, profiles/r04/bvh4/; and a per-lane traversal fallback
// after 256 wave node visits, C5 126.8 vs 113.2 ms, profiles/r04/bvhv/.)

struct Ray {
  d3 o, d;
};

// rayToObjectSpace (raytracer.go:51-56) with prim.Mat4.MulPoint/MulDir
// (vec.go:298-313): m points at the 3x4 affine rows.
template <typename MP>
__device__ __forceinline__ d3 to_obj_o(MP m, d3 o) {  // MulPoint (vec.go:298-304)
  return mk(m[0] * o.x + m[1] * o.y + m[2] * o.z + m[3], m[4] * o.x + m[5] * o.y + m[6] * o.z + m[7],
            m[8] * o.x + m[9] * o.y + m[10] * o.z + m[11]);
}
template <typename MP>
__device__ __forceinline__ d3 to_obj_d(MP m, d3 d) {  // MulDir (vec.go:307-313)
  return mk(m[0] * d.x + m[1] * d.y + m[2] * d.z, m[4] * d.x + m[5] * d.y + m[6] * d.z,
            m[8] * d.x + m[9] * d.y + m[10] * d.z);
}
template <typename MP>
__device__ __forceinline__ Ray to_obj(MP m, const Ray& r) {
  Ray l;
  l.o = to_obj_o(m, r.o);
  l.d = to_obj_d(m, r.d);
  return l;
}
// rayToObjectSpace for a scale + translation (host: axis_sphere; a = m0 m3
// m5 m7 m10 m11): o' = (m0*ox + m3, m5*oy + m7, m10*oz + m11), d' = (m0*dx,
// m5*dy, m10*dz). Bit-identical to MulPoint / MulDir (vec.go:298-313) when
// axis_ray_ok(o, d): the off-diagonal entries are +-0, so with finite ray
// components their products are +-0; a direction component d != 0 with
// |d| in [2^-900, 2^900) and |m0| in [2^-100, 2^100] gives a normal non-zero
// product p = m0*d, and p + (+-0) + (+-0) = p exactly, whatever the zeros'
// signs; an origin component o is either such a number (then the row is
// p + m3 in both forms) or +-0, when the full row is a sum of signed zeros
// plus m3 != 0, i.e. m3, as is +-0 + m3. Where some lane's ray fails the
// test the wave takes the full form (wave-uniform choice).
__device__ __forceinline__ bool ax_mag(double x, bool zero_ok) {
  const uint32_t e = ((uint32_t)__double2hiint(x) >> 20) & 0x7ffu;  // biased exponent
  return e - 123u < 1800u || (zero_ok && x == 0.0);                  // |x| in [2^-900, 2^900)
}
__device__ __forceinline__ bool axis_o_ok(d3 o) { return ax_mag(o.x, true) && ax_mag(o.y, true) && ax_mag(o.z, true); }
__device__ __forceinline__ bool axis_d_ok(d3 d) { return ax_mag(d.x, false) && ax_mag(d.y, false) && ax_mag(d.z, false); }
__device__ __forceinline__ d3 axis_o(const double* a, d3 o) {
  return mk(a[0] * o.x + a[1], a[2] * o.y + a[3], a[4] * o.z + a[5]);
}
__device__ __forceinline__ d3 axis_d(const double* a, d3 d) { return mk(a[0] * d.x, a[2] * d.y, a[4] * d.z); }

// Object records read through the constant address space: a wave-uniform
// index then compiles to scalar loads (s_load_dwordx16 + x8 for the 12
// WorldToObject doubles), which land in SGPRs and feed the FP64 VALU ops as
// their scalar operand -- no LDS or vector-memory bandwidth per object.
typedef const __attribute__((address_space(4))) double* cdptr;
typedef const __attribute__((address_space(4))) float* cfptr;
typedef const __attribute__((address_space(4))) int* ciptr;
// the FP32 words of a double record, in the record's address space
__device__ __forceinline__ const float* as_f(const double* p) { return reinterpret_cast<const float*>(p); }
__device__ __forceinline__ cfptr as_f(cdptr p) { return (cfptr)p; }
__device__ __forceinline__ const int* as_i(const double* p) { return reinterpret_cast<const int*>(p); }
__device__ __forceinline__ ciptr as_i(cdptr p) { return (ciptr)p; }
template <int N>
struct RecN {
  double m[N];
};
typedef RecN<12> Rec12;  // WorldToObject rows (geo records, GEO doubles apart)
typedef RecN<6> Rec6;    // axis-aligned sphere: m0 m3 m5 m7 m10 m11 (arec, AXIS_REC doubles apart)
typedef RecN<3> Rec3;    // uniform-scale sphere of a run: m3 m7 m11 (urec, UNI_REC doubles apart)
enum { AXIS_REC = 8, UNI_REC = 4 };
// Uniform-scale sphere runs (runs with axis = 2; host: m0 == m5 == m10, the
// same value for every sphere of the run -- C5's spheres are all uscale 0.04):
// axis_o / axis_d with a[0] = a[2] = a[4] = s make the object-space direction
// s*d and a = dot(s*d, s*d) the same for every sphere of the run, and the
// origin's products s*o too, so a run forms them once per ray and a sphere
// costs o' = (s*o) + t (3 adds, bit-identical to axis_o's s*o + t) plus the
// quadratic's c, halfB and discriminant: 17 FP64 operations instead of 28, and
// a 24-B record instead of 48.
template <int N, typename PT>
__device__ __forceinline__ RecN<N> ld_rec(PT p) {
  RecN<N> r;
#pragma unroll
  for (int q = 0; q < N; q++) r.m[q] = p[q];
  return r;
}
// Specialised LDS scenes: object i's geo record (GEO doubles) through scalar
// loads from the global blob instead of LDS (RT_SPEC_SGEO): the loop over
// objects is unrolled, so the record lands in SGPRs and feeds the culls and
// the FP64 transform as scalar operands (C3 spec: LDS reads 266 -> 106 in the
// ISA; same-box serial frames C3 -3.0 %, c3cone -2.1 %, C2 -1.7 %,
// profiles/r04/sgeo/). RT_SPEC_SLIGHTS does the same for the lights, the
// frame constants and the plane culls' records (all kernels): no further gain
// on C3, c4csg +1.5 % -- off.
#ifndef RT_SPEC_SGEO
#define RT_SPEC_SGEO 1
#endif
#ifndef RT_SPEC_SLIGHTS
#define RT_SPEC_SLIGHTS 0
#endif
// A BVH leaf object's record (bvh_geo: GEO doubles in leaf order; 0..11
// WorldToObject, 12..13 the FP32 bounding sphere, 14 index, 15 kind) read
// through the constant address space: the index is wave-uniform, so this is
// two scalar loads into SGPRs instead of vector loads per lane.
struct LeafRec {
  RecN<12> R;
  float cx, cy, cz, cr;
  int i, k;
#if RT_AXIS_LEAF
  bool ax;  // a scale + translation sphere (host: axis_sphere)
#endif
};
template <typename PT>
__device__ __forceinline__ LeafRec ld_leaf_p(PT p) {
  LeafRec L;
  L.R = ld_rec<12>(p);
  const uint64_t b0 = (uint64_t)__double_as_longlong(p[12]), b1 = (uint64_t)__double_as_longlong(p[13]);
  L.cx = __int_as_float((int)(uint32_t)b0);
  L.cy = __int_as_float((int)(uint32_t)(b0 >> 32));
  L.cz = __int_as_float((int)(uint32_t)b1);
  L.cr = __int_as_float((int)(uint32_t)(b1 >> 32));
  const uint64_t b2 = (uint64_t)__double_as_longlong(p[14]);
  L.i = (int)(uint32_t)b2;
#if RT_AXIS_LEAF
  L.ax = (uint32_t)(b2 >> 32) != 0;
#endif
  L.k = (int)(uint32_t)(uint64_t)__double_as_longlong(p[15]);
  return L;
}
__device__ __forceinline__ LeafRec ld_leaf(const double* base, int j) {
  return ld_leaf_p((cdptr)base + (size_t)j * 16);  // wave-uniform j: scalar loads
}
// Index of the next record to prefetch, made to depend on the current record
// (an empty asm that "reads" it): scalar loads return out of order, so the
// only wait the compiler can emit is lgkmcnt(0); this places that wait before
// the next record's loads are issued instead of right after them, so they
// stay in flight while the current record is tested.
template <int N>
__device__ __forceinline__ cdptr after_rec(cdptr next, const RecN<N>& cur) {
  asm volatile("" : "+s"(next) : "s"(cur.m[0]));
  return next;
}
// body(i, rec) for the objects i = r0 .. r0 + rn - 1 in index order, records
// (N doubles, STRIDE apart) read with scalar loads, the next record in flight
// while one is tested. Two register sets alternate (no copies between
// iterations). With CHECK > 0 (even), stop() -- wave-uniform -- is asked
// every CHECK objects.
template <int CHECK, int N = 12, int STRIDE = 16, typename Body, typename Stop>
__device__ __forceinline__ void scan_records(cdptr base, int r0, int rn, Body&& body, Stop&& stop) {
  cdptr p = base + (size_t)r0 * STRIDE;
  RecN<N> A = ld_rec<N>(p);
  int j = 0;
  for (; j + 2 <= rn; j += 2, p += 2 * STRIDE) {
    if (CHECK > 0 && j > 0 && (j % CHECK) == 0 && stop()) return;
    const RecN<N> B = ld_rec<N>(after_rec(p + STRIDE, A));
    body(r0 + j, A);
    A = ld_rec<N>(after_rec(j + 2 < rn ? p + 2 * STRIDE : p + STRIDE, B));
    body(r0 + j + 1, B);
  }
  if (j < rn) {
    if (CHECK > 0 && j > 0 && (j % CHECK) == 0 && stop()) return;
    body(r0 + j, A);
  }
}

// body(i, tx, ty, tz) for the uniform-scale spheres i = r0 .. r0 + rn - 1 in
// index order (urec records, UNI_REC doubles: the translations m3 m7 m11):
// G records per scalar load group (pairs: 64 B; quads: 128 B), two groups in
// flight as in scan_records -- 2G spheres tested per wait instead of one, so
// the record latency hides behind more FP64 work (brute-force C5 band 1.85 ->
// 1.55 s with pairs). Loads may read up to 2G - 1 records past the run (the
// host pads urec with 8); only indices < r0 + rn reach the body. stop()
// (wave-uniform) is asked every CHECK objects (a multiple of 2G).
#ifndef RT_UNI_PAIRS
// quads: C5 band 1.446-1.455 -> 1.385-1.393 s once no sphere test reloads a
// spill (before that, pairs and quads measured alike; profiles/r05/unigroup_ab/)
#define RT_UNI_PAIRS 2
#endif
// after_rec for scan_uni's 16-dword groups: the dependency goes through a
// readfirstlane of the record's first dword. Under SGPR pressure (3 lights)
// the compiler kept a group in VGPRs, and the asm's "s" operand then needed
// an illegal VGPR -> SGPR copy (hipRTC aborted the process); v_readfirstlane
// is the legal copy, and it folds away when the value is in an SGPR already.
template <int N>
__device__ __forceinline__ cdptr after_rec_u(cdptr next, const RecN<N>& cur) {
  const int dep = __builtin_amdgcn_readfirstlane(__double2loint(cur.m[0]));
  asm volatile("" : "+s"(next) : "s"(dep));
  return next;
}
template <int CHECK, typename Body, typename Stop>
__device__ __forceinline__ void scan_uni(cdptr base, int r0, int rn, Body&& body, Stop&& stop) {
  // G records per load group (RT_UNI_PAIRS = 1: pairs, 2: quads), two groups
  // in flight
  constexpr int G = RT_UNI_PAIRS >= 2 ? 4 : 2, ND = G * UNI_REC;
  static_assert(UNI_REC == 4 && CHECK % (2 * G) == 0, "scan_uni: 4-double records, stop() at group boundaries");
  cdptr p = base + (size_t)r0 * UNI_REC;
  RecN<ND> A = ld_rec<ND>(p);  // records j .. j + G - 1
  int j = 0;
  for (; j + 2 * G <= rn; j += 2 * G, p += 2 * ND) {
    if (CHECK > 0 && j > 0 && (j % CHECK) == 0 && stop()) return;
    const RecN<ND> B = ld_rec<ND>(after_rec_u(p + ND, A));  // records j + G .. j + 2G - 1
#pragma unroll
    for (int q = 0; q < G; q++) body(r0 + j + q, A.m[UNI_REC * q], A.m[UNI_REC * q + 1], A.m[UNI_REC * q + 2]);
    A = ld_rec<ND>(after_rec_u(p + 2 * ND, B));
#pragma unroll
    for (int q = 0; q < G; q++) body(r0 + j + G + q, B.m[UNI_REC * q], B.m[UNI_REC * q + 1], B.m[UNI_REC * q + 2]);
  }
  if (j < rn) {
    if (CHECK > 0 && j > 0 && (j % CHECK) == 0 && stop()) return;
    const RecN<ND> B = ld_rec<ND>(after_rec_u(p + ND, A));
#pragma unroll
    for (int q = 0; q < G; q++)
      if (j + q < rn) body(r0 + j + q, A.m[UNI_REC * q], A.m[UNI_REC * q + 1], A.m[UNI_REC * q + 2]);
#pragma unroll
    for (int q = 0; q < G - 1; q++)
      if (j + G + q < rn) body(r0 + j + G + q, B.m[UNI_REC * q], B.m[UNI_REC * q + 1], B.m[UNI_REC * q + 2]);
  }
}

// True when q = num/den (den != 0, finite) is certainly <= 0, i.e. num == 0
// or the signs differ, so the reference would reject t = q (t <= 0) and the
// division can be skipped. NaN operands return false (the division runs and
// the NaN flows through exactly as in the reference).
__device__ __forceinline__ bool t_nonpos(double num, double den) {
#if RT_DIV_SKIP
  return (num == 0.0 && !__builtin_isnan(den)) || (num < 0.0 && den > 0.0) || (num > 0.0 && den < 0.0);
#else
  return false;
#endif
}

// Sphere.Intersect (raytracer.go:58-104): unit sphere, near root only.
// c = O.O - 1 depends on the ray origin only (shared by the shadow rays of a
// hit, see shadow_sweep); sphere_hit forms it.
__device__ __forceinline__ double sphere_c(d3 o) { return dot(o, o) - 1.0; }
__device__ __forceinline__ bool sphere_hit_c(const Ray& l, double c, double& t) {
  double a = dot(l.d, l.d);
  double hb = dot(l.o, l.d);
  double disc = hb * hb - a * c;
  if (disc < 0.0) return false;
  double sq = gsqrt(disc);
  double num = -hb - sq;
  if (t_nonpos(num, a)) return false;  // t0 <= 0: no near hit
  double t0 = num / a;
  if (t0 > 0.0) {
    t = t0;
    return true;
  }
  return false;
}
__device__ __forceinline__ bool sphere_hit(const Ray& l, double& t) { return sphere_hit_c(l, sphere_c(l.o), t); }

// Plane.Intersect (raytracer.go:164-180) on an object-space ray; no = n.O
// (origin only).
__device__ __forceinline__ bool plane_hit_c(const Ray& l, d3 n, double pd, double no, double& t) {
  double denom = dot(n, l.d);
  if (__builtin_fabs(denom) < 1e-6) return false;
  double num = -pd - no;
  if (t_nonpos(num, denom)) return false;
  double tt = num / denom;
  if (tt <= 0.0) return false;
  t = tt;
  return true;
}
__device__ __forceinline__ bool plane_hit(const Ray& l, d3 n, double pd, double& t) {
  return plane_hit_c(l, n, pd, dot(n, l.o), t);
}

// Cube.Intersect (raytracer.go:214-240) over prim.PlanesForUnitCube
// (internal/prim/plane.go:29-38). Every face re-transforms the ray with the
// same matrix in the reference, so one transform gives identical values.
// With RT_CUBE_FAST the face planes' dot products are evaluated on the one
// non-zero axis: for a finite ray, n.v = (0*a + 0*b) + (+-1)*c equals +-c
// exactly whenever c != 0, and when c == 0 both forms are a zero that is
// rejected identically (|denom| < 1e-6, or t = 0 <= 0), so hits, T and
// PointObj are bit-identical to the generic dot products.
__device__ __forceinline__ bool cube_face(const Ray& l, int f, double& best, int& bf, bool& found) {
  // face f: axis, sign of the normal, -D (D = -normal.Dot(point))
  const int ax = (f < 2) ? 2 : ((f < 4) ? 0 : 1);
  const bool pos = (f == 1 || f == 3 || f == 4);
  const double negD = (f == 1 || f == 3 || f == 4) ? 1.0 : 0.0;
  double dA = ax == 0 ? l.d.x : (ax == 1 ? l.d.y : l.d.z);
  double oA = ax == 0 ? l.o.x : (ax == 1 ? l.o.y : l.o.z);
  double denom = pos ? dA : -dA;
  if (__builtin_fabs(denom) < 1e-6) return false;
  double nO = pos ? oA : -oA;
  double num = negD - nO;
  if (t_nonpos(num, denom)) return false;
  double tt = num / denom;
  if (tt <= 0.0) return false;
  d3 p = add(l.o, scale(l.d, tt));
  if (p.x < 0 || p.x > 1 || p.y < 0 || p.y > 1 || p.z < 0 || p.z > 1) return false;
  if (!found || tt < best) {
    found = true;
    best = tt;
    bf = f;
  }
  return true;
}

__device__ __forceinline__ bool cube_hit(const Ray& l, double& t, int& face) {
  bool found = false;
  double best = 0.0;
  int bf = 0;
#if RT_CUBE_FAST
#pragma unroll
  for (int f = 0; f < 6; f++) cube_face(l, f, best, bf, found);
#else
  const double N[6][3] = {{0, 0, -1}, {0, 0, 1}, {-1, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, -1, 0}};
  const double D[6] = {-0.0, -1.0, -0.0, -1.0, -1.0, -0.0};
#pragma unroll
  for (int f = 0; f < 6; f++) {
    double ft;
    if (!plane_hit(l, mk(N[f][0], N[f][1], N[f][2]), D[f], ft)) continue;
    if (ft < 0.0) continue;
    d3 p = add(l.o, scale(l.d, ft));
    if (p.x < 0 || p.x > 1 || p.y < 0 || p.y > 1 || p.z < 0 || p.z > 1) continue;
    if (!found || ft < best) {
      found = true;
      best = ft;
      bf = f;
    }
  }
#endif
  if (found) {
    t = best;
    face = bf;
  }
  return found;
}

// Cylinder.Intersect (raytracer.go:279-337).
// Cylinder.Intersect (raytracer.go:279-337) and, with cone = true, the
// contest-extension cone (oracle/rt_oracle.c cone_intersect; not in the
// reference): the same quadric-plus-caps structure, so one routine (the flag
// is wave-uniform) keeps register pressure at the cylinder's. Every quantity
// is formed in the oracle's op order: the cone's a, halfB, c0 append
// "- dy*dy", "- oy*dy", "- oy*oy" where the cylinder has nothing / "- 1.0".
// c0: the origin-only term (quadric_c0).
__device__ __forceinline__ double quadric_c0(d3 o, bool cone) {
  const double c0 = o.x * o.x + o.z * o.z;
  return cone ? c0 - o.y * o.y : c0 - 1.0;
}
__device__ __forceinline__ bool quadric_hit_c(const Ray& l, double c0, double& t, int& face, bool cone) {
  double bestT = __builtin_inf();
  int bestFace = -1;
  double a = l.d.x * l.d.x + l.d.z * l.d.z;
  double hb = l.o.x * l.d.x + l.o.z * l.d.z;
  if (cone) {
    a = a - l.d.y * l.d.y;
    hb = hb - l.o.y * l.d.y;
  }
  if (__builtin_fabs(a) > 1e-12) {  // cylinder: a >= 0, the reference's a > 1e-12
    double disc = hb * hb - a * c0;
    if (disc >= 0.0) {
      double sq = gsqrt(disc);
      // consider() ignores t <= 0 (raytracer.go:287), so a root whose sign is
      // known to be non-positive needs no division.
      double n0 = -hb - sq, n1 = -hb + sq;
      if (!t_nonpos(n0, a)) {
        double t0 = n0 / a;
        double y0 = l.o.y + l.d.y * t0;
        if (y0 >= 0.0 && y0 <= 1.0 && t0 > 0.0 && t0 < bestT) {
          bestT = t0;
          bestFace = 0;
        }
      }
      if (!t_nonpos(n1, a)) {
        double t1 = n1 / a;
        double y1 = l.o.y + l.d.y * t1;
        if (y1 >= 0.0 && y1 <= 1.0 && t1 > 0.0 && t1 < bestT) {
          bestT = t1;
          bestFace = 0;
        }
      }
    }
  } else if (cone && __builtin_fabs(hb) > 1e-12) {  // cone: ray parallel to a generator
    double n0 = -c0, den = 2.0 * hb;
    if (!t_nonpos(n0, den)) {
      double t0 = n0 / den;
      double y0 = l.o.y + l.d.y * t0;
      if (y0 >= 0.0 && y0 <= 1.0 && t0 > 0.0 && t0 < bestT) {
        bestT = t0;
        bestFace = 0;
      }
    }
  }
  if (__builtin_fabs(l.d.y) > 1e-12) {
    double nTop = 1.0 - l.o.y;
    if (!t_nonpos(nTop, l.d.y)) {
      double tTop = nTop / l.d.y;
      double px = l.o.x + l.d.x * tTop, pz = l.o.z + l.d.z * tTop;
      if (px * px + pz * pz <= 1.0 && tTop > 0.0 && tTop < bestT) {
        bestT = tTop;
        bestFace = 1;
      }
    }
    double nBot = -l.o.y;
    if (!cone && !t_nonpos(nBot, l.d.y)) {
      double tBot = nBot / l.d.y;
      double px = l.o.x + l.d.x * tBot, pz = l.o.z + l.d.z * tBot;
      if (px * px + pz * pz <= 1.0 && tBot > 0.0 && tBot < bestT) {
        bestT = tBot;
        bestFace = 2;
      }
    }
  }
  if (bestFace < 0) return false;
  t = bestT;
  face = bestFace;
  return true;
}
__device__ __forceinline__ bool quadric_hit(const Ray& l, double& t, int& face, bool cone) {
  return quadric_hit_c(l, quadric_c0(l.o, cone), t, face, cone);
}


// (branch-free forms of these tests, RT_BRANCHFREE, measured -35 M scalar and
// +45 M vector instructions on C3 and no faster: removed)

// One SceneObject.Intersect on a world-space ray; k is wave-uniform.
__device__ __forceinline__ bool object_hit(int k, const double* g, const Ray& r, double& t, int& face) {
  Ray l = to_obj(g, r);
  face = 0;
  // (kinds the specialised scene lacks fold away; the generic build keeps all)
  if (spec_kind(RT_SPHERE) && k == RT_SPHERE) return sphere_hit(l, t);
  if (spec_kind(RT_PLANE) && k == RT_PLANE) return plane_hit(l, mk(g[12], g[13], g[14]), g[15], t);
  if (spec_kind(RT_CUBE) && k == RT_CUBE) return cube_hit(l, t, face);
  if (!spec_kind(RT_CYLINDER) && !spec_kind(RT_CONE)) return false;  // unreachable for the scene's kinds
  return quadric_hit(l, t, face, spec_kind(RT_CONE) && (!spec_kind(RT_CYLINDER) || k == RT_CONE));
}

// The origin-only term of kind k's Intersect for object-space origin o
// (sphere c, cylinder / cone c0, plane n.O; cube: none).
__device__ __forceinline__ double object_oc(int k, const double* g, d3 o) {
  if (spec_kind(RT_SPHERE) && k == RT_SPHERE) return sphere_c(o);
  if (spec_kind(RT_PLANE) && k == RT_PLANE) return dot(mk(g[12], g[13], g[14]), o);
  if (spec_kind(RT_CYLINDER) && k == RT_CYLINDER) return quadric_c0(o, false);
  if (spec_kind(RT_CONE) && k == RT_CONE) return quadric_c0(o, true);
  return 0.0;
}
// object_hit on an object-space ray l whose origin term oc = object_oc(k, g,
// l.o) is given: the same operations, so the same result.
__device__ __forceinline__ bool object_hit_l(int k, const double* g, const Ray& l, double oc, double& t, int& face) {
  face = 0;
  if (spec_kind(RT_SPHERE) && k == RT_SPHERE) return sphere_hit_c(l, oc, t);
  if (spec_kind(RT_PLANE) && k == RT_PLANE) return plane_hit_c(l, mk(g[12], g[13], g[14]), g[15], oc, t);
  if (spec_kind(RT_CUBE) && k == RT_CUBE) return cube_hit(l, t, face);
  if (!spec_kind(RT_CYLINDER) && !spec_kind(RT_CONE)) return false;
  return quadric_hit_c(l, oc, t, face, spec_kind(RT_CONE) && (!spec_kind(RT_CYLINDER) || k == RT_CONE));
}

// Wave votes on a lane predicate, straight from its lane mask (HIP's
// __any / __ballot take an int: the predicate is first rematerialised as 0/1
// in a VGPR and compared again).
__device__ __forceinline__ uint64_t wave_ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }
__device__ __forceinline__ bool wave_any(bool b) { return __builtin_amdgcn_ballot_w64(b) != 0; }
__device__ __forceinline__ uint64_t popc_ballot(bool b) { return (uint64_t)__popcll(wave_ballot(b)); }

// Conservative FP32 test: can the segment o + t*d, 0 < t < tmax (d ~ unit)
// come within the padded bounding sphere (centre c, radius^2 r2)? The exact
// FP64 test can only report a hit whose point lies inside the object's
// bounding sphere (to ~1e-12 relative); the host pads the radius by 0.01%
// plus 1e-4*(1+|c|+|L|) and tmax carries 1e-4 relative slack, ~100x FP32
// rounding at scene scales, so `false` proves the exact test misses (or, for
// closestHit, cannot beat the current best).
struct F3 {
  float x, y, z;
};
__device__ __forceinline__ F3 f3(d3 v) { return F3{(float)v.x, (float)v.y, (float)v.z}; }
// `slack` (ray_slack) widens the radius by the FP32 rounding scale of the
// ray origin, so origins far from the object stay conservative.
template <typename DP>
__device__ __forceinline__ bool may_hit(F3 o, F3 d, float tmax, DP g, float slack) {
  const auto b = as_f(g + 12);
  // (fused multiply-adds: only less rounding than the bound allows for)
  float ox = b[0] - o.x, oy = b[1] - o.y, oz = b[2] - o.z;
  float tc = __builtin_fmaf(ox, d.x, __builtin_fmaf(oy, d.y, oz * d.z));
  tc = fminf(fmaxf(tc, 0.0f), tmax);
  float qx = __builtin_fmaf(-tc, d.x, ox), qy = __builtin_fmaf(-tc, d.y, oy), qz = __builtin_fmaf(-tc, d.z, oz);
  const float R = b[3] + slack;
  return __builtin_fmaf(qx, qx, __builtin_fmaf(qy, qy, qz * qz)) <= R * R;
}
// The culls with the lane's activity folded into the final compare (an
// inactive lane compares against an unreachable bound), so the result is one
// compare's lane mask: the wave's any-lane test reads it directly (a && of
// two lane masks is rematerialised through a VGPR before a ballot).
// (c: the bounding sphere's centre and padded radius, b[0..3] of may_hit)
__device__ __forceinline__ bool may_hit_s(bool act, F3 o, F3 d, float tmax, float cx, float cy, float cz, float cr,
                                          float slack) {
  float ox = cx - o.x, oy = cy - o.y, oz = cz - o.z;
  float tc = __builtin_fmaf(ox, d.x, __builtin_fmaf(oy, d.y, oz * d.z));
  tc = fminf(fmaxf(tc, 0.0f), tmax);
  float qx = __builtin_fmaf(-tc, d.x, ox), qy = __builtin_fmaf(-tc, d.y, oy), qz = __builtin_fmaf(-tc, d.z, oz);
  const float R = cr + slack;
  return __builtin_fmaf(qx, qx, __builtin_fmaf(qy, qy, qz * qz)) <= (act ? R * R : -1.0f);
}
__device__ __forceinline__ bool may_hit_a(bool act, F3 o, F3 d, float tmax, const double* g, float slack) {
  const float* b = reinterpret_cast<const float*>(g + 12);
  return may_hit_s(act, o, d, tmax, b[0], b[1], b[2], b[3], slack);
}
__device__ __forceinline__ float ray_slack(F3 o) {
  return 1e-5f * (1.0f + __builtin_fabsf(o.x) + __builtin_fabsf(o.y) + __builtin_fabsf(o.z));
}
// Conservative FP32 slab test against a BVH node box (built from the padded
// bounding spheres, rounded outwards), widened by the lane's slack. A
// component 0 * inf = NaN is ignored by fminf/fmaxf, i.e. a ray parallel to a
// slab is constrained only by the other axes (it lies on or beyond the
// widened face otherwise).
__device__ __forceinline__ bool may_hit_box(F3 o, F3 id, float slack, float tmax, const float* nb, float& tn) {
  const float x0 = (nb[0] - slack - o.x) * id.x, x1 = (nb[3] + slack - o.x) * id.x;
  const float y0 = (nb[1] - slack - o.y) * id.y, y1 = (nb[4] + slack - o.y) * id.y;
  const float z0 = (nb[2] - slack - o.z) * id.z, z1 = (nb[5] + slack - o.z) * id.z;
  tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
  const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
  return tn <= tf && tf >= 0.0f && tn <= tmax;
}
// may_hit_box as one compare, the lane's activity folded in: for tmax >= 0,
// tn <= tf && tf >= 0 && tn <= tmax  <=>  max(tn, 0) <= min(tf, tmax); an
// inactive lane's bound is -1 (a NaN tn or tmax can only admit more nodes:
// still conservative).
__device__ __forceinline__ bool may_hit_box6_a(bool act, F3 o, F3 id, float slack, float tmax, float lx, float ly,
                                               float lz, float hx, float hy, float hz, float& tn) {
  const float x0 = (lx - slack - o.x) * id.x, x1 = (hx + slack - o.x) * id.x;
  const float y0 = (ly - slack - o.y) * id.y, y1 = (hy + slack - o.y) * id.y;
  const float z0 = (lz - slack - o.z) * id.z, z1 = (hz + slack - o.z) * id.z;
  tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
  const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
  return fmaxf(tn, 0.0f) <= fminf(tf, act ? tmax : -1.0f);
}
// a float's bits as an unsigned key in the float's order (finite values)
__device__ __forceinline__ uint32_t f_order_key(int b) { return (uint32_t)(b >= 0 ? b ^ (int)0x80000000 : ~b); }
template <typename FP>
__device__ __forceinline__ bool may_hit_box_a(bool act, F3 o, F3 id, float slack, float tmax, FP nb, float& tn) {
  const float x0 = (nb[0] - slack - o.x) * id.x, x1 = (nb[3] + slack - o.x) * id.x;
  const float y0 = (nb[1] - slack - o.y) * id.y, y1 = (nb[4] + slack - o.y) * id.y;
  const float z0 = (nb[2] - slack - o.z) * id.z, z1 = (nb[5] + slack - o.z) * id.z;
  tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
  const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
  return fmaxf(tn, 0.0f) <= fminf(tf, act ? tmax : -1.0f);
}
// Per-wave traversal stack in LDS: node refs and the lanes still active there.
struct WaveStack {
  int* ref;
  uint64_t* mask;
  // r and m are wave-uniform: every active lane stores the same value, so
  // the entry is written whichever lanes are active (a lane-0-only store was
  // lost when lane 0 was inactive here: profiles/r04/generic/)
  __device__ __forceinline__ void push(int& sp, int lane, int r, uint64_t m) {
    (void)lane;
    ref[sp] = r;
    mask[sp] = m;
    sp++;
  }
};
// Binary BVH step with the first child kept in registers (RT_BVH_CONT): the
// child the stack order would pop next is visited directly and only the other
// is pushed, so a descent skips the LDS store and reload between a node and
// its first child. Nodes are visited in the same order as with two pushes.
// Same-box serial frames: C5 119.7 -> 113.5 ms, C4 4.11 -> 4.05 ms
// (profiles/r04/bvhv/; measured before the far-origin shift it was lost in
// C5's tail).
#ifndef RT_BVH_CONT
#define RT_BVH_CONT 1
#endif
__device__ __forceinline__ void bvh_next(WaveStack& st, int& sp, int lane, bool c1_first, int r0, int r1, uint64_t m0,
                                         uint64_t m1, int& nr, uint64_t& nm, bool& have) {
  const int fr = c1_first ? r1 : r0, sr = c1_first ? r0 : r1;
  const uint64_t fm = c1_first ? m1 : m0, sm = c1_first ? m0 : m1;
  if (fm) {
    if (sm) st.push(sp, lane, sr, sm);
    nr = fr;
    nm = fm;
    have = true;
  } else if (sm) {
    nr = sr;
    nm = sm;
    have = true;
  }
}
// Rays from far away (a ground-plane hit near the horizon can lie 1e7 units
// out): the FP32 culls widen every box and sphere by the origin's rounding
// scale (ray_slack), which then exceeds the scene and turns the BVH into a
// brute-force sweep over every leaf. For the BVH culls only, such a lane's
// origin moves (FP64) to just before where the ray enters the box of all BVH
// objects, o' = o + t0 d, and its bounds become tmax - t0; a lane whose ray
// misses that box takes no part. Objects lie in the box, so every cull that
// could pass for o passes for o' (both conservative); the exact tests still
// use the reference's ray, so hits and counters do not change.
#ifndef RT_FAR_SHIFT
#define RT_FAR_SHIFT 1
#endif
__device__ __forceinline__ void far_shift(bool& act, const Ray& r, const double* lo, const double* hi, F3& of,
                                          float& slack, double& t0) {
  if (!RT_FAR_SHIFT || !wave_any(act && slack > 1e-3f)) return;
  if (act && slack > 1e-3f) {
    const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    double tn = 0.0, tf = __builtin_inf();
#pragma unroll
    for (int a = 0; a < 3; a++) {
      // d = 0: +-inf (inside the slab: no bound; outside: empty); 0/0 = NaN is
      // ignored by fmin/fmax
      const double ta = (lo[a] - o[a]) / d[a], tb = (hi[a] - o[a]) / d[a];
      tn = __builtin_fmax(tn, __builtin_fmin(ta, tb));
      tf = __builtin_fmin(tf, __builtin_fmax(ta, tb));
    }
    if (!(tn <= tf)) {
      act = false;
    } else {
      t0 = tn * (1.0 - 1e-9);
      const d3 os = add(r.o, scale(r.d, t0));
      of = f3(os);
      slack = ray_slack(of);
    }
  }
}
__device__ __forceinline__ F3 f3_rcp(F3 d) {
  return F3{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z)};
}

// ---- CSG composites (contest extension; oracle/rt_oracle.c leaf_interval,
// csg_member, csg_intersect restate the same semantics op for op) ----
// One convex leaf's interval [a, b] along the ray and the faces it enters /
// leaves by: f = fa | fb << 4 | 256 when non-empty.
template <typename DP>
__device__ __forceinline__ void leaf_interval(int kind, DP g, const Ray& r, double& a, double& b, int& f) {
  const Ray l = to_obj(g, r);
  a = -__builtin_inf();
  b = __builtin_inf();
  int fa = 0, fb = 0;
  bool ok = true;
  if (spec_kind(RT_SPHERE) && kind == RT_SPHERE) {
    const double qa = dot(l.d, l.d), hb = dot(l.o, l.d), c = dot(l.o, l.o) - 1.0;
    const double disc = hb * hb - qa * c;
    if (disc < 0.0) {
      ok = false;
    } else {
      const double sq = __builtin_sqrt(disc);
      a = (-hb - sq) / qa;
      b = (-hb + sq) / qa;
    }
  } else if (spec_kind(RT_CUBE) && kind == RT_CUBE) {
    const double o3[3] = {l.o.x, l.o.y, l.o.z}, d3v[3] = {l.d.x, l.d.y, l.d.z};
    const int flo[3] = {2, 5, 0}, fhi[3] = {3, 4, 1};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (d3v[k] == 0.0) {
        if (o3[k] < 0.0 || o3[k] > 1.0) ok = false;
        continue;
      }
      const double ta = (0.0 - o3[k]) / d3v[k], tb = (1.0 - o3[k]) / d3v[k];
      double lo = ta, hi = tb;
      int fl = flo[k], fh = fhi[k];
      if (d3v[k] < 0.0) {
        lo = tb;
        hi = ta;
        fl = fhi[k];
        fh = flo[k];
      }
      if (lo > a) {
        a = lo;
        fa = fl;
      }
      if (hi < b) {
        b = hi;
        fb = fh;
      }
    }
    if (a > b) ok = false;
  } else if (spec_kind(RT_CYLINDER) && kind == RT_CYLINDER) {
    const double qa = l.d.x * l.d.x + l.d.z * l.d.z;
    if (qa > 1e-12) {
      const double hb = l.o.x * l.d.x + l.o.z * l.d.z;
      const double c0 = l.o.x * l.o.x + l.o.z * l.o.z - 1.0;
      const double disc = hb * hb - qa * c0;
      if (disc < 0.0) {
        ok = false;
      } else {
        const double sq = __builtin_sqrt(disc);
        a = (-hb - sq) / qa;
        b = (-hb + sq) / qa;
      }
    } else if (l.o.x * l.o.x + l.o.z * l.o.z > 1.0) {
      ok = false;
    }
    if (ok) {
      if (__builtin_fabs(l.d.y) > 1e-12) {
        const double tb0 = (0.0 - l.o.y) / l.d.y, tt = (1.0 - l.o.y) / l.d.y;
        double lo = tb0, hi = tt;
        int fl = 2, fh = 1;
        if (l.d.y < 0.0) {
          lo = tt;
          hi = tb0;
          fl = 1;
          fh = 2;
        }
        if (lo > a) {
          a = lo;
          fa = fl;
        }
        if (hi < b) {
          b = hi;
          fb = fh;
        }
      } else if (l.o.y < 0.0 || l.o.y > 1.0) {
        ok = false;
      }
      if (a > b) ok = false;
    }
  } else {  // RT_PLANE: the half-space n.p + D <= 0
    const d3 n = mk(g[12], g[13], g[14]);
    const double denom = dot(n, l.d);
    if (__builtin_fabs(denom) < 1e-6) {
      if (dot(n, l.o) + g[15] > 0.0) ok = false;
    } else {
      const double tt = (-g[15] - dot(n, l.o)) / denom;
      if (denom < 0.0)
        a = tt;
      else
        b = tt;
    }
  }
  f = fa | (fb << 4) | (ok ? 256 : 0);
}

// Membership of the composite given its leaves' inside mask m (bit j: leaf j
// contains the point), by the host-compiled program (rt_kernel.hip
// csg_mask_program): the postfix program with union-only / intersect-only
// groups of leaves collapsed into one mask test (bit stacks, depth <=
// RT_CSG_MAX_LEAVES).
enum { RT_CSG_ANY = -4, RT_CSG_ALL = -5 };
// composites with at least this many leaves get spatial leaf groups (host)
#ifndef RT_CSG_GROUP_MIN
#define RT_CSG_GROUP_MIN 16
#endif
enum { CSG_GROUP_MIN = RT_CSG_GROUP_MIN };
// The composite search's wave-uniform reads (postfix program, leaf groups,
// leaf kinds and records) through scalar loads from the global blob instead
// of LDS (c4csg serial, same box: 15.33 -> 14.68 ms; the composite's fields
// made wave-uniform with readfirstlane first: 16.32 -> 15.33 ms, VGPR spills
// of the CSG quads kernel 95 -> 60; profiles/r04/csg/ab_c4csg_scalar.log)
#ifndef RT_CSG_SCALAR
#define RT_CSG_SCALAR 1
#endif
#ifndef RT_CSG_FAR
#define RT_CSG_FAR 1  // far-origin shift of the composite search's culls (csg_hit)
#endif
template <typename IP>
__device__ __forceinline__ bool csg_eval(IP code, int n, uint64_t m0, uint64_t m1) {
  uint64_t st0 = 0, st1 = 0;
  int sp = 0;
  auto get = [&](int i) -> bool { return ((i < 64 ? st0 >> i : st1 >> (i - 64)) & 1) != 0; };
  auto set = [&](int i, bool v) {
    if (i < 64)
      st0 = v ? (st0 | (1ull << i)) : (st0 & ~(1ull << i));
    else
      st1 = v ? (st1 | (1ull << (i - 64))) : (st1 & ~(1ull << (i - 64)));
  };
  for (int k = 0; k < n; k++) {
    const int op = code[k];
    bool v;
    if (op >= 0) {
      v = ((op < 64 ? m0 >> op : m1 >> (op - 64)) & 1) != 0;
    } else if (op <= RT_CSG_ANY) {
      const uint64_t k0 = (uint32_t)code[k + 1] | ((uint64_t)(uint32_t)code[k + 2] << 32);
      const uint64_t k1 = (uint32_t)code[k + 3] | ((uint64_t)(uint32_t)code[k + 4] << 32);
      k += 4;
      v = op == RT_CSG_ANY ? ((m0 & k0) | (m1 & k1)) != 0 : ((m0 & k0) == k0 && (m1 & k1) == k1);
    } else {
      sp -= 2;
      const bool x = get(sp), y = get(sp + 1);
      v = op == RT_CSG_UNION ? (x || y) : (op == RT_CSG_INTERSECT ? (x && y) : (x && !y));
    }
    set(sp, v);
    sp++;
  }
  return (st0 & 1) != 0;
}

// Composite hit: the first leaf end point t > 0 (lowest leaf, entry first,
// on ties) where membership changes. face = leaf << 4 | flip << 3 | leaf face.
// Candidates only grow, so the scan stops once te * cut_m reaches cut_lim
// (strictly beyond, or at-or-beyond when !cut_strict): the caller cannot use
// such a hit (closest hit: t > best; shadow: t * |d| >= dist), so stopping
// there changes no result.
template <typename DP, typename IP, typename GP>
__device__ __forceinline__ bool csg_hit_all(DP geo, IP kinds, IP code, int nobj,
                                            GP g, const Ray& r, double& t, int& face, double cut_m,
                                            double cut_lim, bool cut_strict) {
  const auto ci = as_i(g + 14);
  const int first = nobj + ci[0], count = ci[1];
  const auto prog = code + ci[2] + 1 + 6 * code[ci[2]];  // past the leaf groups (csg_hit)
  const int plen = ci[3];
  double A[RT_CSG_MAX_LEAVES], B[RT_CSG_MAX_LEAVES];
  int F[RT_CSG_MAX_LEAVES];
  // A leaf whose padded bounding sphere the ray cannot reach for t >= 0 has
  // an empty interval or one behind the origin: it changes neither the
  // membership nor the candidates for t > 0, so it is skipped (exact).
  const F3 of = f3(r.o), df = f3(r.d);
  const float slack = ray_slack(of);
  uint64_t live0 = 0, live1 = 0;  // leaves with a non-empty interval, in registers
  for (int j = 0; j < count; j++) {
    const int k = kinds[first + j];
    const auto lg = geo + (size_t)(first + j) * GEO;
    if (k != RT_PLANE && !may_hit(of, df, 3.0e38f, lg, slack)) continue;
    leaf_interval(k, lg, r, A[j], B[j], F[j]);
    if (F[j] & 256) {
      if (j < 64)
        live0 |= 1ull << j;
      else
        live1 |= 1ull << (j - 64);
    }
  }
  double tc = 0.0;
  for (;;) {
    double te = __builtin_inf();
    int je = -1, jend = 0;
    // ascending leaf order over the live set (lowest leaf wins ties)
    for (int w = 0; w < 2; w++) {
      uint64_t m = w ? live1 : live0;
      while (m) {
        const int j = w * 64 + __builtin_ctzll(m);
        m &= m - 1;
        if (A[j] > tc && A[j] < te) {
          te = A[j];
          je = j;
          jend = 0;
        }
        if (B[j] > tc && B[j] < te) {
          te = B[j];
          je = j;
          jend = 1;
        }
      }
    }
    if (je < 0) return false;
    if (cut_strict ? te * cut_m > cut_lim : te * cut_m >= cut_lim) return false;
    // leaves containing the points just before / just after te
    uint64_t b0 = 0, b1 = 0, a0 = 0, a1 = 0;
    for (int w = 0; w < 2; w++) {
      uint64_t m = w ? live1 : live0, bm = 0, am = 0;
      while (m) {
        const int q = __builtin_ctzll(m);
        m &= m - 1;
        const int j = w * 64 + q;
        if (A[j] < te && te <= B[j]) bm |= 1ull << q;
        if (A[j] <= te && te < B[j]) am |= 1ull << q;
      }
      if (w) {
        b1 = bm;
        a1 = am;
      } else {
        b0 = bm;
        a0 = am;
      }
    }
    const bool before = csg_eval(prog, plen, b0, b1), after = csg_eval(prog, plen, a0, a1);
    if (before != after) {
      const int flip = ((jend == 0) != after) ? 1 : 0;
      t = te;
      face = (je << 4) | (flip << 3) | (jend ? (F[je] >> 4) & 15 : F[je] & 15);
      return true;
    }
    tc = te;
  }
}

#ifdef RT_CSG_DIAG
__device__ unsigned long long g_csg_diag[8];  // diagnostic build: searches, overflows, live leaves, group loop shapes
#undef RT_CSG_DIAG
#define RT_CSG_DIAG g_csg_diag
#endif
// The same search over a register-resident list of the live leaves (at most
// RT_CSG_LIVE per lane, ascending leaf order, so every tie breaks as above):
// a ray meets only a few of a composite's leaves, and the per-lane interval
// arrays of csg_hit_all live in scratch memory. A lane with more live leaves
// redoes the search with csg_hit_all (identical result).
#ifndef RT_CSG_LIVE
#define RT_CSG_LIVE 6  // 0: always the scratch-array search
#endif
template <typename DP, typename IP, typename GP>
__device__ __forceinline__ bool csg_hit_all_call(DP geo, IP kinds, IP code, int nobj,
                                              GP g, const Ray& r, double& t, int& face, double cut_m,
                                              double cut_lim, bool cut_strict) {
  return csg_hit_all(geo, kinds, code, nobj, g, r, t, face, cut_m, cut_lim, cut_strict);
}
// Callers pass a WAVE-UNIFORM composite g (every lane searches the same
// composite): its fields are read through readfirstlane below. That holds
// because composites never become BVH leaves (the host keeps them in the
// unbounded-objects list, P.planes) and every other object loop is
// wave-uniform; a per-lane object loop must not call this.
// LF packs the leaf number in 8 bits (and the host's leaf groups use 0xff as
// the end marker), hence:
static_assert(RT_CSG_MAX_LEAVES < 255, "csg_hit packs leaf numbers in 8 bits");
template <typename DP, typename IP, typename GP>
__device__ __forceinline__ bool csg_hit(DP geo, IP kinds, IP code, int nobj,
                                        GP g, const Ray& r, double& t, int& face, double cut_m = 1.0,
                                        double cut_lim = __builtin_inf(), bool cut_strict = true) {
  constexpr int K = RT_CSG_LIVE > 0 ? RT_CSG_LIVE : 1;
  if constexpr (RT_CSG_LIVE == 0) return csg_hit_all(geo, kinds, code, nobj, g, r, t, face, cut_m, cut_lim, cut_strict);
  const auto ci = as_i(g + 14);
  // (the composite's fields are wave-uniform: readfirstlane keeps the reads
  // below them scalar)
  const int first = __builtin_amdgcn_readfirstlane(nobj + ci[0]), count = __builtin_amdgcn_readfirstlane(ci[1]);
  // leaf groups (host: spatial, <= 8 leaves, FP32 bounding sphere): a group
  // no lane's ray can reach is skipped as a whole; the live list then fills
  // out of leaf order, so the search below breaks ties on the leaf index
  const auto hdr = code + __builtin_amdgcn_readfirstlane(ci[2]);
  const int ngroups = __builtin_amdgcn_readfirstlane(hdr[0]);
  const auto prog = hdr + 1 + 6 * ngroups;
  const int plen = __builtin_amdgcn_readfirstlane(ci[3]);
  F3 of = f3(r.o);
  const F3 df = f3(r.d);
  float slack = ray_slack(of);
  // A far origin (see far_shift) moves the group and leaf culls' origin to a
  // lower bound t0 of the ray's entry into the composite's padded bounding
  // sphere, and the search starts there: outside that sphere no point belongs
  // to the composite, so no membership change (hit) lies before t0, and a
  // leaf the shifted segment cannot reach holds no point beyond it.
  double tc = 0.0;
  if (RT_CSG_FAR && slack > 1e-3f) {
    const auto cb = as_f(g + 12);
    if (cb[3] < 3.0e38f) {
      const double dd = dot(r.d, r.d);
      const double tm = dot(sub(mk(cb[0], cb[1], cb[2]), r.o), r.d) / dd - (double)cb[3] / __builtin_sqrt(dd);
      const double t0 = tm - 1e-6 * __builtin_fabs(tm) - 1e-6;
      if (t0 > 0.0) {
        tc = t0;
        of = f3(add(r.o, scale(r.d, t0)));
        slack = ray_slack(of);
      }
    }
  }
  double LA[K], LB[K];
  int LF[K];  // leaf index | entry face << 8 | exit face << 12
#pragma unroll
  for (int s = 0; s < K; s++) {
    LA[s] = LB[s] = 0.0;
    LF[s] = 0;
  }
  int n = 0;
  auto add_leaf = [&](int j) {
    const int k = kinds[first + j];
    const auto lg = geo + (size_t)(first + j) * GEO;
    if (k != RT_PLANE && !may_hit(of, df, 3.0e38f, lg, slack)) return;
    double a, b;
    int f;
    leaf_interval(k, lg, r, a, b, f);
    if (f & 256) {
#pragma unroll
      for (int s = 0; s < K; s++)
        if (s == n) {
          LA[s] = a;
          LB[s] = b;
          LF[s] = j | ((f & 0xff) << 8);
        }
      n++;
    }
  };
  if (ngroups == 0) {
    for (int j = 0; j < count; j++) add_leaf(j);
  } else {
    for (int q = 0; q < ngroups; q++) {
      const auto gr = hdr + 1 + 6 * q;
      const bool gh = may_hit_s(true, of, df, 3.0e38f, __int_as_float(gr[0]), __int_as_float(gr[1]),
                                __int_as_float(gr[2]), __int_as_float(gr[3]), slack);
      if (!wave_any(gh)) continue;
#ifdef RT_CSG_DIAG
      {
        // the group's leaf loop as it runs (one iteration per leaf any lane
        // may hit) vs lane-major (each lane its own next candidate: the most
        // candidates one lane has), and the lane-leaf work both share
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane(gr[4]),
                       d1 = (uint32_t)__builtin_amdgcn_readfirstlane(gr[5]);
        int cand = 0, leaf_major = 0;
        for (int e = 0; e < 8; e++) {
          const int j = (int)(((e < 4 ? d0 : d1) >> (8 * (e & 3))) & 0xffu);
          if (j == 0xff) break;
          const int k = kinds[first + j];
          const auto lg = geo + (size_t)(first + j) * GEO;
          const bool pc = gh && (k == RT_PLANE || may_hit(of, df, 3.0e38f, lg, slack));
          cand += pc ? 1 : 0;
          leaf_major += wave_any(pc) ? 1 : 0;
        }
        int lane_major = 0;
        for (int v = 0; v < 8; v++)
          if (wave_any(cand > v)) lane_major = v + 1;
        const int lid = (int)__lane_id();
        if (__builtin_amdgcn_readfirstlane(lid) == lid) {
          atomicAdd(RT_CSG_DIAG + 3, (unsigned long long)leaf_major);
          atomicAdd(RT_CSG_DIAG + 4, (unsigned long long)lane_major);
          atomicAdd(RT_CSG_DIAG + 6, 1ull);  // (wave, group) visits
        }
        atomicAdd(RT_CSG_DIAG + 5, (unsigned long long)cand);
      }
#endif
      if (gh) {
        const uint32_t w0 = (uint32_t)__builtin_amdgcn_readfirstlane(gr[4]),
                       w1 = (uint32_t)__builtin_amdgcn_readfirstlane(gr[5]);
        for (int e = 0; e < 8; e++) {
          const int j = (int)(((e < 4 ? w0 : w1) >> (8 * (e & 3))) & 0xffu);
          if (j == 0xff) break;
          add_leaf(j);
        }
      }
    }
  }
#ifdef RT_CSG_DIAG
  atomicAdd(RT_CSG_DIAG + 0, 1ull);  // composite searches
  if (n > K) atomicAdd(RT_CSG_DIAG + 1, 1ull);  // ... that overflowed the register list
  atomicAdd(RT_CSG_DIAG + 2, (unsigned long long)n);  // live leaves
#endif
  if (n > K) return csg_hit_all_call(geo, kinds, code, nobj, g, r, t, face, cut_m, cut_lim, cut_strict);
  for (;;) {
    double te = __builtin_inf();
    int se = -1, jend = 0, je = 0x7fffffff;
#pragma unroll
    for (int s = 0; s < K; s++) {
      if (s < n) {
        // the first end point past tc; ties: the lowest leaf, then its entry
        // (what csg_hit_all's scan in leaf order gives)
        const int lj = LF[s] & 0xff;
        if (LA[s] > tc && (LA[s] < te || (LA[s] == te && lj < je))) {
          te = LA[s];
          se = s;
          jend = 0;
          je = lj;
        }
        if (LB[s] > tc && (LB[s] < te || (LB[s] == te && lj < je))) {
          te = LB[s];
          se = s;
          jend = 1;
          je = lj;
        }
      }
    }
    if (se < 0) return false;
    if (cut_strict ? te * cut_m > cut_lim : te * cut_m >= cut_lim) return false;
    uint64_t b0 = 0, b1 = 0, a0 = 0, a1 = 0;
    int fe = 0;
#pragma unroll
    for (int s = 0; s < K; s++) {
      if (s < n) {
        const int j = LF[s] & 0xff;
        const uint64_t bit = 1ull << (j & 63);
        const uint64_t bb = (LA[s] < te && te <= LB[s]) ? bit : 0ull;
        const uint64_t ab = (LA[s] <= te && te < LB[s]) ? bit : 0ull;
        if (j < 64) {
          b0 |= bb;
          a0 |= ab;
        } else {
          b1 |= bb;
          a1 |= ab;
        }
      }
      if (s == se) fe = LF[s];
    }
    const bool before = csg_eval(prog, plen, b0, b1), after = csg_eval(prog, plen, a0, a1);
    if (before != after) {
      const int flip = ((jend == 0) != after) ? 1 : 0;
      t = te;
      face = ((fe & 0xff) << 4) | (flip << 3) | (jend ? (fe >> 12) & 15 : (fe >> 8) & 15);
      return true;
    }
    tc = te;
  }
}


// Conservative FP32 test for a plane: can the segment o + t*d, 0 < t < tmax,
// cross the plane? c = world-space plane (A^T n, n.b + D for WorldToObject
// p -> A p + b) followed by its term-magnitude scale (sum_r |n_r||a_rc|,
// sum_r |n_r||b_r| + |D|). The reference decides a hit from the signs of
// f(0) = n.o_obj + D and f(tmax) (t = -f(0)/denom compared with tmax), each
// computed in FP64 with error ~1e-15 of that scale; here both are evaluated
// in FP32 and `false` needs them to agree in sign with a 1e-4 margin, so the
// exact test misses (or cannot beat the current best). tmax >= 1e30 means no
// bound: then f(0) and the slope must agree in sign (the root lies behind).
// The origin-only half (f(0) and its term scale), shared by the shadow rays
// of one hit (shadow_sweep); may_hit_plane_d finishes the test.
struct PlaneO {
  float f0, a0;
};
template <typename DP>
__device__ __forceinline__ PlaneO may_hit_plane_o(F3 o, DP sh) {
  const auto c = as_f(sh + 16);
  PlaneO r;
  r.f0 = __builtin_fmaf(c[0], o.x, __builtin_fmaf(c[1], o.y, __builtin_fmaf(c[2], o.z, c[3])));
  r.a0 = __builtin_fmaf(c[4], __builtin_fabsf(o.x),
                        __builtin_fmaf(c[5], __builtin_fabsf(o.y), __builtin_fmaf(c[6], __builtin_fabsf(o.z), c[7])));
  return r;
}
template <typename DP>
__device__ __forceinline__ bool may_hit_plane_d(PlaneO po, F3 d, float tmax, DP sh) {
  const auto c = as_f(sh + 16);
  const float f0 = po.f0, a0 = po.a0;
  const float sl = __builtin_fmaf(c[0], d.x, __builtin_fmaf(c[1], d.y, c[2] * d.z));
  const float a1 = __builtin_fmaf(c[4], __builtin_fabsf(d.x), __builtin_fmaf(c[5], __builtin_fabsf(d.y), c[6] * __builtin_fabsf(d.z)));
  float f1, m0, m1;
  if (tmax >= 1e30f) {
    f1 = sl;
    m0 = __builtin_fmaf(1e-4f, a0, 1e-30f);
    m1 = __builtin_fmaf(1e-4f, a1, 1e-30f);
  } else {
    f1 = __builtin_fmaf(tmax, sl, f0);
    m0 = __builtin_fmaf(1e-4f, __builtin_fmaf(tmax, a1, a0), 1e-30f);
    m1 = m0;
  }
  return !((f0 > m0 && f1 > m1) || (f0 < -m0 && f1 < -m1));
}
template <typename DP>
__device__ __forceinline__ bool may_hit_plane(F3 o, F3 d, float tmax, DP sh) {
  return may_hit_plane_d(may_hit_plane_o(o, sh), d, tmax, sh);
}

// Diagnostic build only (-DRT_PHASE_TIMING): wave cycles per phase, stamped
// with s_memtime into per-wave scalar sums; never enabled in the product.
#ifdef RT_PHASE_TIMING
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define PH_BEGIN() uint64_t ph_t0_ = stamp()
// (the asm comment names the phase that ends here in the ISA listing:
// scripts/isa_phases.py splits the diagnostic kernel's code at these marks)
#define PH_MARK(k)                        \
  do {                                    \
    uint64_t t_ = stamp();                \
    asm volatile("; @phase_end " #k ::: "memory"); \
    ph_acc[k] += t_ - ph_t0_;             \
    ph_t0_ = t_;                          \
  } while (0)
#else
#define PH_BEGIN() (void)0
#define PH_MARK(k) (void)0
#endif

// Diagnostic build: lanes reaching an exact FP64 Intersect after culling,
// per kind and loop (trace 0 / shadow 1), and wave batches per loop
// (global atomics: build with RT_EXACT_DIAG only when phase times don't matter).
#ifdef RT_EXACT_DIAG
#define EXDIAG(k, sh, b)                                                                    \
  do {                                                                                      \
    const uint64_t act_ = wave_ballot(1), m_ = wave_ballot(b);                                    \
    if ((int)(threadIdx.x & 63) == __ffsll((long long)act_) - 1) {                          \
      atomicAdd(P.stats + ST_EXDIAG + 2 * (k) + (sh), (unsigned long long)__popcll(m_));    \
      atomicAdd(P.stats + ST_EXDIAG + 2 * RT_NUM_KINDS + (sh), 1ull);                       \
    }                                                                                       \
  } while (0)
#else
#define EXDIAG(k, sh, b) (void)0
#endif

// Frame stack: lane-interleaved so that one field of one frame is a
// contiguous 512-B row for the wave.
__device__ __forceinline__ double* frame_ptr(double* base, int frame) { return base + (size_t)frame * FRAME_FIELDS * 64; }
__device__ __forceinline__ void st3(double* f, int field, d3 v) {
  f[(field + 0) * 64] = v.x;
  f[(field + 1) * 64] = v.y;
  f[(field + 2) * 64] = v.z;
}
__device__ __forceinline__ d3 ld3(const double* f, int field) {
  return mk(f[(field + 0) * 64], f[(field + 1) * 64], f[(field + 2) * 64]);
}

// CORE field c (0..2 Lw, 3 kr, 4 packed) -> global field index.
__device__ __forceinline__ int core_gfield(int c) { return c < 3 ? c : (c == 3 ? 9 : 10); }

// Frame flags (packed with the material index): packed = material << PK_MAT |
// board slot << PK_SLOT | flags. FL_FORKED: the pending refraction child was
// posted to the board (slot PK_SLOT: 24 bits, the device-wide board's slots
// are per (wave slot, lane, level)) for another lane to trace.
// FL_TASK: a sentinel below a claimed subtree -- its colour goes to slot
// PK_SLOT (the subtree runs at its own absolute levels, so the depth limit
// and the frame layout are those of the owner's tree).
enum { FL_TMODE = 1, FL_HASR = 2, FL_HAST = 4, FL_STAGE = 8, FL_VMMAT = 16, FL_FORKED = 32, FL_TASK = 64 };
enum { PK_SLOT = 8, PK_MAT = 32 };
#define PK_SLOT_OF(packed) ((int)(((packed) >> PK_SLOT) & 0xffffff))

// ---------------------------------------------------------------------------
// Work sharing at the tail of a launch (RT_SHARE). Once the queue is drained a
// lane that finished its last pixel is idle, while other lanes of the group
// still run the longest pixels: 4 samples one after another, each a binary
// tree of up to 2^depth - 1 rays when a material both reflects and refracts
// (raytracer.go:512-556). The lanes of a workgroup share a board in LDS:
//   * an owner lane posts work it has not started -- the next-to-last of its
//     pixel's unstarted samples, or the pending refraction child of its
//     shallowest binary frame -- into a free slot of its wave's range;
//   * an idle lane of any of the group's waves claims a slot, traces that
//     sample (PCG state jumped to the sample, raytracer.go:632-643) or subtree
//     (depth offset = the child's level) on its own stack, and delivers the
//     colour into the slot;
//   * the owner joins when it reaches that sample / child: it takes the
//     delivered colour, or reclaims a slot nobody claimed and traces it itself,
//     or waits (S_WAIT). The combine and the sample sum then run exactly as
//     without sharing ((((0 + s0) + s1) + s2) + s3, raytracer.go:651; the
//     per-level clamp, :557-561), so pixels and counters are unchanged.
// Slot state lives in two 64-bit LDS masks (posted, delivered) changed by
// atomics; a wave allocates and frees only the slots of its own range.
// ---------------------------------------------------------------------------
// Off by default: in this register-saturated kernel (168 VGPRs at 3 waves per
// SIMD) the board's code costs C3 ~10 % in every round (spills, +5 % VALU and
// +13 % SALU instructions, PMC), more than the tail gains; rt_set_work_sharing
// compiles it into a context's specialised kernel.
#ifndef RT_SHARE
#define RT_SHARE 0
#endif
#ifdef RT_COST_MAP
#undef RT_SHARE
#define RT_SHARE 0  // the cost-map diagnostic charges a pixel's work to its own lane
#endif
#ifndef RT_SHARE_SPINS
#define RT_SHARE_SPINS (1 << 16)  // idle rounds (s_sleep'd) a drained wave waits for work before leaving
#endif
#ifndef RT_SHARE_SLEEP
#define RT_SHARE_SLEEP 127  // s_sleep per idle round (x64 cycles): a polling wave keeps the issue slots of
                            // other workgroups' waves on its SIMD almost free
#endif
#ifndef RT_SHARE_SAMPLES
#define RT_SHARE_SAMPLES 1  // post unstarted samples (serial schedule), not only refraction subtrees
#endif
enum { NSLOT = 64, SLOTS_PER_WAVE = NSLOT / WAVES_PER_WG, S_WAIT = 4, S_RESUME = 5 };
// S_ADV (serial samples): the lane finished a sample (its colour added to sum);
// the next one is chosen at the top of the main loop (advance_sample), in one
// place rather than in each unwind site (instruction-cache footprint).
enum { S_ADV = 6 };
struct Board {
  unsigned long long post;           // slots holding a task nobody has claimed
  unsigned long long done;           // slots whose colour has been delivered
  unsigned int wfree[WAVES_PER_WG];  // per wave: free slots of its range (bit j: slot SLOTS_PER_WAVE * w + j)
  int nidle;                         // idle lanes of drained waves (helpers available)
  int nactive;                       // waves with busy lanes
  int pad[2];
  // subtree task: the pending refraction ray (origin, direction), read by the
  // helper when it claims the slot; then the delivered colour (res = ray[0..2])
  double ray[NSLOT][6];
  int meta[NSLOT][2];  // subtree: level of the child, 0; sample: x | k << 16 | 1 << 30, y
  // Per lane, the rarely used sample bookkeeping (kept out of the registers
  // of a kernel that uses all of them): bits 0-2 own_end (the lane traces
  // samples [0, own_end) of its pixel itself), 3-9 claimed sample task's slot
  // + 1 (0: its own pixel), 10-27 the slots of posted samples 1..3.
  uint32_t lw[WG];
};
__device__ __forceinline__ int lw_own_end(uint32_t w) { return (int)(w & 7u); }
__device__ __forceinline__ int lw_task(uint32_t w) { return (int)((w >> 3) & 127u) - 1; }
__device__ __forceinline__ int lw_fork(uint32_t w, int k) { return (int)((w >> (10 + 6 * (k - 1))) & 63u); }
enum { BOARD_BYTES = (int)sizeof(Board), META_SAMPLE = 1 << 30 };
#define RT_WG_SCOPE __HIP_MEMORY_SCOPE_WORKGROUP
__device__ __forceinline__ bool board_reclaim(Board* b, int q) {  // owner: take back a task nobody claimed
  const unsigned long long old = __hip_atomic_fetch_and(&b->post, ~(1ull << q), __ATOMIC_ACQUIRE, RT_WG_SCOPE);
  return ((old >> q) & 1ull) != 0;
}
__device__ __forceinline__ bool board_done(Board* b, int q) {
  return ((__hip_atomic_load(&b->done, __ATOMIC_ACQUIRE, RT_WG_SCOPE) >> q) & 1ull) != 0;
}
__device__ __forceinline__ void board_free(Board* b, int q) {
  __hip_atomic_fetch_or(&b->wfree[q / SLOTS_PER_WAVE], 1u << (q % SLOTS_PER_WAVE), __ATOMIC_RELAXED, RT_WG_SCOPE);
}
// owner: the delivered colour of slot q (after board_done), slot freed
__device__ __forceinline__ d3 board_take(Board* b, int q) {
  const d3 r = mk(b->ray[q][0], b->ray[q][1], b->ray[q][2]);
  __hip_atomic_fetch_and(&b->done, ~(1ull << q), __ATOMIC_RELAXED, RT_WG_SCOPE);
  board_free(b, q);
  return r;
}
__device__ __forceinline__ void board_deliver(Board* b, int q, d3 c) {  // helper
  b->ray[q][0] = c.x;
  b->ray[q][1] = c.y;
  b->ray[q][2] = c.z;
  __hip_atomic_fetch_or(&b->done, 1ull << q, __ATOMIC_RELEASE, RT_WG_SCOPE);
}
// Position of the r-th set bit of m (r < popcount(m)).
__device__ __forceinline__ int nth_bit(uint64_t m, int r) {
  for (int i = 0; i < r; i++) m &= m - 1;
  return __builtin_ctzll(m);
}
// The lowest n set bits of m.
__device__ __forceinline__ uint64_t low_bits(uint64_t m, int n) {
  uint64_t r = 0;
  for (int i = 0; i < n && m; i++) {
    const uint64_t b = m & (~m + 1);
    r |= b;
    m ^= b;
  }
  return r;
}

// ---------------------------------------------------------------------------
// Device-wide work sharing (RT_SHARE == 2). The workgroup board above lets an
// idle lane take only its own group's work, and at the tail of a launch the
// groups still running deep glass trees (raytracer.go:512-556: reflect +
// refract at every level, up to 2^depth - 1 rays per sample) are few, while
// every other group has left. Here any idle lane of any drained wave on the
// device can take a posted refraction subtree:
//   * slots in global memory, one per (wave slot, lane, level) -- a frame is
//     posted at most once, so slot ids need no allocation; record = the
//     pending refraction ray (o, d), the child's level, the state word;
//   * a ring of posted slot ids with monotone 64-bit head / tail tickets (per
//     context, never reset: a stale ticket names a slot whose state is no
//     longer POSTED, and its claim just fails);
//   * claim = CAS POSTED -> CLAIMED on the slot; the owner reclaims a slot
//     nobody claimed with CAS POSTED -> FREE and traces it itself, or takes
//     the delivered colour (DONE -> FREE), or waits (S_WAIT);
//   * the board lives in UNCACHED device memory (hipDeviceMallocUncached:
//     no XCD's L2 keeps a copy -- with ordinary memory the zeroing memset
//     left clean lines in some L2s, and sc1 polls served from them never saw
//     another XCD's update: idle waves spun to their limit, 8-rank c4csg
//     shares took 140 ms instead of 5); every access to the shared words is
//     an agent-scope relaxed atomic (sc1, past the CU's L1), and a writer
//     drains its stores (s_waitcnt vmcnt(0)) before the state or ticket that
//     publishes them. The launch's idle-lane and active-wave counters are in
//     the same block (two sets, launches alternate, each zeroing the next).
// Pixels and counters are those of the serial recursion: the owner combines
// the child's colour at its own frame exactly as it would its own (the
// reference's per-level clamp, raytracer.go:557-561).
// ---------------------------------------------------------------------------
#ifndef RT_GS_MIN_LEVELS
#define RT_GS_MIN_LEVELS 3  // post only refraction children with >= this many levels below them
#endif
// Sharded by XCD (RT_GS_SHARDS rings; a workgroup posts to ring blockIdx mod
// shards -- blocks are dealt round-robin over the 8 XCDs, so a ring's posters
// share an L2 and a memory path; placement only affects speed): each ring
// has its own head / tail words, and the idle-lane count is replicated per
// shard (an update adds to every replica, one wave instruction with a lane
// per replica), so a busy wave's poll reads words only its shard's waves read.
#ifndef RT_GS_SHARDS
#define RT_GS_SHARDS 8
#endif
enum { GS_FREE = 0, GS_POSTED = 1, GS_CLAIMED = 2, GS_DONE = 3, GS_REC = 8 /* u64 per slot */,
       GS_RING = 1 << 20 /* ring entries (u64), all shards */, GS_SH = RT_GS_SHARDS,
       GS_RSH = GS_RING / GS_SH /* entries per shard's ring */,
       // control block (u64 indices; the words 4 KB apart, so no two share a
       // memory channel): shard k's ring head / tail at GS_SHARD * k + 0 / 512,
       // then two counter sets: active waves, helper waves, idle lanes per shard
       GS_SHARD = 1024, GS_HEAD = 0, GS_TAIL = 512, GS_SET = GS_SHARD * GS_SH /* set s at GS_SET + GS_SETSZ * s */,
       GS_ACTIVE = 0, GS_HELPERS = 512, GS_NIDLE = 1024 /* + 512 * shard */, GS_SETSZ = 1024 + 512 * GS_SH,
       GS_CTL_U64 = GS_SET + 2 * GS_SETSZ };
static_assert(GS_SH >= 1 && GS_SH <= 32 && (GS_RING % GS_SH) == 0 && (GS_RSH & (GS_RSH - 1)) == 0, "RT_GS_SHARDS");
#ifndef RT_GS_POLL
// a busy wave reads the board's words every (RT_GS_POLL + 1)-th round
// (c4csg 8-rank share, profiles/r05/gpoll: 1.77-1.79 ms at 3, 1.77-1.81 at
// 1, 1.83 at 0, 1.95 at 15; sharded rings make frequent polls cheap)
#define RT_GS_POLL 3
#endif
#ifndef RT_GS_HELPERS
#define RT_GS_HELPERS 16  // drained waves that stay to help (device-wide); the others leave at once
#endif
#define RT_AG_SCOPE __HIP_MEMORY_SCOPE_AGENT
__device__ __forceinline__ uint64_t gs_ld(uint64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, RT_AG_SCOPE); }
__device__ __forceinline__ void gs_st(uint64_t* p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, RT_AG_SCOPE); }
__device__ __forceinline__ unsigned int gs_ld32(unsigned int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, RT_AG_SCOPE);
}
// Ordering. Publication is release / acquire by construction, without the
// L2 writeback / invalidate the compiler emits for agent-scope release /
// acquire on ordinary memory (buffer_wbl2 / buffer_inv: an agent-scope fence
// per sample cost round 3's sample-unit experiment 41 ms), which the board
// does not need: it is uncached (MTYPE UC), so no L2 of any XCD holds a line
// of it, and every access reaches memory.
//   * release (gs_drain before the publishing store -- POSTED, DONE, the
//     ticket): s_waitcnt vmcnt(0) waits until every earlier store of the lane
//     has been acknowledged by memory, and its "memory" clobber stops the
//     compiler moving any memory operation across it;
//   * acquire (gs_acquire after the load or CAS that observed POSTED / DONE,
//     before the payload loads): the same wait -- the observing access has
//     returned before any later load issues -- and the same compiler barrier,
//     so no payload load is hoisted above the observation.
// Every shared word is still accessed with agent-scope atomics (no tearing,
// past the CU's L1).
__device__ __forceinline__ void gs_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void gs_acquire() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ bool gs_cas(uint64_t* p, uint64_t from, uint64_t to) {
  return __hip_atomic_compare_exchange_strong(p, &from, to, __ATOMIC_RELAXED, __ATOMIC_RELAXED, RT_AG_SCOPE);
}
// the claim: CAS POSTED -> CLAIMED, then (acquire) the slot's payload may be read
__device__ __forceinline__ bool gs_claim(uint64_t* r) {
  const bool ok = gs_cas(r + 7, GS_POSTED, GS_CLAIMED);
  gs_acquire();
  return ok;
}
__device__ __forceinline__ uint64_t* gs_slot(uint64_t* board, int q) { return board + (size_t)q * GS_REC; }
// owner: take back a slot nobody claimed
__device__ __forceinline__ bool gs_reclaim(uint64_t* board, int q) { return gs_cas(gs_slot(board, q) + 7, GS_POSTED, GS_FREE); }
// owner: has the helper delivered? (acquire: gs_take's colour loads follow)
__device__ __forceinline__ bool gs_done(uint64_t* board, int q) {
  const bool d = gs_ld(gs_slot(board, q) + 7) == GS_DONE;
  gs_acquire();
  return d;
}
// owner: the delivered colour (after gs_done); the slot is free again
__device__ __forceinline__ d3 gs_take(uint64_t* board, int q) {
  uint64_t* r = gs_slot(board, q);
  const d3 c = mk(__longlong_as_double((long long)gs_ld(r)), __longlong_as_double((long long)gs_ld(r + 1)),
                  __longlong_as_double((long long)gs_ld(r + 2)));
  gs_st(r + 7, GS_FREE);
  return c;
}
// helper: the subtree's colour into the slot, then DONE
__device__ __forceinline__ void gs_deliver(uint64_t* board, int q, d3 c) {
  uint64_t* r = gs_slot(board, q);
  gs_st(r, (uint64_t)__double_as_longlong(c.x));
  gs_st(r + 1, (uint64_t)__double_as_longlong(c.y));
  gs_st(r + 2, (uint64_t)__double_as_longlong(c.z));
  gs_drain();
  gs_st(r + 7, GS_DONE);
}


// ---------------------------------------------------------------------------
// Closure-surface VM: executes a straight-line register
// program compiled on the host from a GML surface function
// (go-raytracer_amd/gml/surface_compiler.py) -- the device counterpart of
// EvalSurfaceFn (evaluator.go:672-727). Registers are 64-bit (f64 / i64 /
// bool); r0..r9 = Material, r10 = face, r11 = u, r12 = v. Go semantics:
// int64 wraparound, truncating divi/modi, floor/frac via amd64 float->int,
// Cephes sin/cos on degrees * (Pi/180). Returns true on a run-time error
// (the reference would panic).
// ---------------------------------------------------------------------------
enum VmOp {
  VM_NOP, VM_CONST, VM_MOV, VM_ADDF, VM_SUBF, VM_MULF, VM_DIVF, VM_NEGF, VM_ADDI, VM_SUBI, VM_MULI, VM_DIVI,
  VM_MODI, VM_NEGI, VM_LTF, VM_EQF, VM_LTI, VM_EQI, VM_SEL, VM_FLOOR, VM_FRAC, VM_SQRT, VM_SIN, VM_COS,
  VM_CLAMPF, VM_CLAMPI, VM_TBL, VM_AND, VM_OR, VM_NOT, VM_ERR, VM_RET
};
enum { VM_REGS = 64, VM_MAX_STEPS = 8192 };
static_assert(VM_CONST == RT_VM_CONST && VM_SEL == RT_VM_SEL && VM_TBL == RT_VM_TBL && VM_ERR == RT_VM_ERR &&
                  VM_RET == RT_VM_RET,
              "surface bytecode opcodes of include/rt_abi.h");

// Inlined: as an out-of-line call reading the LDS-staged program through
// generic pointers it rendered wrong pixels on gfx950 (measured: the global
// blob path and the inlined call are exact), and inlining needs less scratch.
__device__ __forceinline__ bool run_vm(const uint32_t* code, const uint64_t* consts, int pc, long long face, double u,
                                    double v, double* out) {
  uint64_t R[VM_REGS];
  R[10] = (uint64_t)face;
  R[11] = (uint64_t)__double_as_longlong(u);
  R[12] = (uint64_t)__double_as_longlong(v);
  bool err = false;
#define F_(r) __longlong_as_double((long long)R[r])
#define I_(r) ((long long)R[r])
#define SETF(x) R[d] = (uint64_t)__double_as_longlong(x)
  for (int steps = 0; steps < VM_MAX_STEPS; steps++, pc += 2) {
    const uint32_t w0 = code[pc], c = code[pc + 1];
    const int op = (int)(w0 & 0xff), d = (int)((w0 >> 8) & 0x3f), a = (int)((w0 >> 16) & 0x3f),
              b = (int)((w0 >> 24) & 0x3f);
    switch (op) {
      case VM_RET:
        for (int k = 0; k < 10; k++) out[k] = F_(k);
        return err;
      case VM_CONST: R[d] = consts[c]; break;
      case VM_MOV: R[d] = R[a]; break;
      case VM_ADDF: SETF(F_(a) + F_(b)); break;
      case VM_SUBF: SETF(F_(a) - F_(b)); break;
      case VM_MULF: SETF(F_(a) * F_(b)); break;
      case VM_DIVF: SETF(F_(a) / F_(b)); break;
      case VM_NEGF: SETF(-F_(a)); break;
      case VM_ADDI: R[d] = R[a] + R[b]; break;
      case VM_SUBI: R[d] = R[a] - R[b]; break;
      case VM_MULI: R[d] = R[a] * R[b]; break;
      case VM_DIVI: {  // Go: truncating; MinInt64 / -1 wraps; /0 is checked by ERR
        long long x = I_(a), y = I_(b);
        R[d] = y == 0 ? 0 : (y == -1 ? (uint64_t)0 - (uint64_t)x : (uint64_t)(x / y));
        break;
      }
      case VM_MODI: {
        long long x = I_(a), y = I_(b);
        R[d] = (y == 0 || y == -1) ? 0 : (uint64_t)(x % y);
        break;
      }
      case VM_NEGI: R[d] = (uint64_t)0 - R[a]; break;
      case VM_LTF: R[d] = F_(a) < F_(b); break;
      case VM_EQF: R[d] = F_(a) == F_(b); break;
      case VM_LTI: R[d] = I_(a) < I_(b); break;
      case VM_EQI: R[d] = R[a] == R[b]; break;
      case VM_SEL: R[d] = R[a] ? R[b] : R[c & 0x3f]; break;
      case VM_FLOOR: {
        double x = F_(a);
        R[d] = (uint64_t)go_f2i(__builtin_isfinite(x) ? __builtin_floor(x) : x);
        break;
      }
      case VM_FRAC: {
        double x = F_(a);
        SETF(x - (double)go_f2i(x));
        break;
      }
      case VM_SQRT: SETF(__builtin_sqrt(F_(a))); break;
      case VM_SIN: SETF(go_sin(0.017453292519943295 * F_(a))); break;
      case VM_COS: SETF(go_cos(0.017453292519943295 * F_(a))); break;
      case VM_CLAMPF: {
        double x = F_(a);
        SETF(x < 0 ? 0.0 : (x > 1 ? 1.0 : x));
        break;
      }
      case VM_CLAMPI: {
        long long x = I_(a);
        R[d] = (uint64_t)(x < 0 ? 0 : (x > 1 ? 1 : x));
        break;
      }
      case VM_TBL: {  // consts[c] = n, then n entries; bounds are checked by ERR
        long long n = (long long)consts[c], i = I_(a);
        i = i < 0 ? 0 : (i >= n ? n - 1 : i);
        R[d] = consts[c + 1 + i];
        break;
      }
      case VM_AND: R[d] = (R[a] != 0) && (R[b] != 0); break;
      case VM_OR: R[d] = (R[a] != 0) || (R[b] != 0); break;
      case VM_NOT: R[d] = R[a] == 0; break;
      case VM_ERR: err = err || (R[a] != 0); break;
      default: return true;
    }
  }
#undef F_
#undef I_
#undef SETF
  return true;  // malformed program (no RET)
}

// traceRay's final combine (raytracer.go:557-561).
__device__ __forceinline__ d3 combine(bool tmode, d3 lw, d3 col, double refl, double kr, d3 R, d3 Tr) {
  if (!tmode) return clamp(mul(add(lw, scale(R, refl)), col));
  return clamp(mul(add(lw, add(scale(R, kr), scale(Tr, 1.0 - kr))), col));
}

struct View {
  const int* entry;
  const uint32_t* code;
  const uint64_t* consts;
  const double* geo;
  const double* shade;
  const double* mats;
  const double* lights;
  const int* kind;
  const int* objmat;
  const uint32_t* pref;  // [nobj + 1][PREF]: objects of each kind with index < i
  const int* csg;        // CSG postfix programs (extension)
};

// QUADS (pixel quads): a pixel's 4 samples run at once in 4 adjacent lanes,
// not one after another in one lane -- 4x shorter per-pixel latency, so the
// deep, branching trees of glass at depth >= 7 no longer leave a few waves
// running long after the rest (host choice per scene, rt_kernel.hip).
template <bool LDS, bool BVH, bool CSG, bool QUADS>
#ifndef RT_MIN_WAVES
#if RT_CULL
#define RT_MIN_WAVES 3  // 168 VGPRs -> 3 waves/SIMD (C3 on par with 4; C2 -10%, C4 (BVH) -4%)
#else
#define RT_MIN_WAVES 5  // brute force (scalar-load sweep): 5 waves/SIMD, C5 band -7..-14 % vs 3 (profiles/r02/minwaves_ab)
#endif
#endif
__global__ __launch_bounds__(WG, RT_MIN_WAVES) void rt_render_kernel(const char* __restrict__ blob, Params P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef RT_COST_MAP
  constexpr bool QD = false;  // the cost-map diagnostic charges all of a pixel's work to one lane
  constexpr bool PR = false;
#else
  constexpr bool QD = QUADS;
  constexpr bool PR = !QUADS && RT_PAIRS && RT_SHARE != 1;  // pixel pairs (the workgroup board assumes one owner lane)
#endif
  // pixels per dequeue: 16 quads, 32 pairs (an 8x4 half tile) or 64 pixels
  constexpr unsigned int QCHUNK = QD ? 16u : PR ? 32u : (unsigned int)RT_QCHUNK_PIXEL;
  const char* base;
  // Stage the scene (LDS flavour) once per workgroup (the only block-wide
  // barrier).
  // PCG jump table: with quads every sample starts from entry (row, sample),
  // read from HBM (2.5 KB, cache resident: a whole LDS copy cost C4 a
  // workgroup per CU and C3 a level of LDS frame cores); serial samples start
  // at sample 0, whose 20 rows are staged in LDS
  uint64_t* jrows = reinterpret_cast<uint64_t*>(smem + P.jump_off);
  if constexpr (!QD)
    for (int i = threadIdx.x; i < 20 * 4; i += WG) jrows[i] = P.jump[(i >> 2) * 16 + (i & 3)];
  // drained-head mask of this workgroup
  unsigned int* qdrained = reinterpret_cast<unsigned int*>(smem + P.qmask_off);
  if (threadIdx.x == 0) *qdrained = 0u;
  // per-wave unit counters: zeroed before the barrier (any wave's lane 0 adds)
  if (threadIdx.x < NUNIT * WAVES_PER_WG) reinterpret_cast<unsigned long long*>(smem + P.cnt_off)[threadIdx.x] = 0ull;
  Board* Bd = reinterpret_cast<Board*>(smem + P.board_off);
  if constexpr (RT_SHARE == 1) {
    if (threadIdx.x == 0) {
      Bd->post = 0ull;
      Bd->done = 0ull;
      Bd->nidle = 0;
      Bd->nactive = WAVES_PER_WG;  // every wave starts busy (my_active)
    }
    if (threadIdx.x < WAVES_PER_WG) Bd->wfree[threadIdx.x] = (1u << SLOTS_PER_WAVE) - 1u;
  }
  if (blockIdx.x == 0 && threadIdx.x < QHEADS) atomicExch(P.queue_next + threadIdx.x * QSTRIDE, 0u);
  // device-wide sharing: this launch's idle-lane / active-wave counters
  // (device-wide sharing) this workgroup's shard: its ring, its replica of
  // the idle-lane count
  const int gshard = (int)(blockIdx.x % (unsigned)GS_SH);
  uint64_t* const g_ring = P.gring + (size_t)gshard * GS_RSH;
  uint64_t* const g_head = P.gctl + GS_SHARD * gshard + GS_HEAD;
  uint64_t* const g_tail = P.gctl + GS_SHARD * gshard + GS_TAIL;
  uint64_t* const g_set = P.gctl + GS_SET + GS_SETSZ * P.gset;
  unsigned int* g_nidle = reinterpret_cast<unsigned int*>(g_set + GS_NIDLE + 512 * gshard);
  unsigned int* g_active = reinterpret_cast<unsigned int*>(g_set + GS_ACTIVE);
  unsigned int* g_helpers = reinterpret_cast<unsigned int*>(g_set + GS_HELPERS);
  // idle-lane count updates go to every shard's replica (lane k: replica k)
  auto nidle_add = [&](int delta) {
    if ((int)(threadIdx.x & 63) < GS_SH)
      atomicAdd(reinterpret_cast<unsigned int*>(g_set + GS_NIDLE + 512 * (threadIdx.x & 63)), (unsigned int)delta);
  };
  if constexpr (RT_SHARE == 2) {
    // the next launch's counters start at zero; every wave of this launch
    // counts itself active
    if (blockIdx.x == 0 && threadIdx.x < 2 + GS_SH)
      atomicExch(reinterpret_cast<unsigned int*>(P.gctl + GS_SET + GS_SETSZ * (1 - P.gset) + 512 * threadIdx.x), 0u);
    if ((threadIdx.x & 63) == 0) atomicAdd(g_active, 1u);
  }
  // (device-wide sharing) this wave's view of the board, refreshed every 4th
  // round (every round while it is a helper): idle helper lanes, ring head /
  // tail; whether it stays as a helper after draining
  int gs_nid = 0;
  uint64_t gs_h = 0, gs_t = 0;
  bool gs_helper = false;
  if constexpr (LDS) {
    const int n16 = P.blob_bytes / 16;
    for (int i = threadIdx.x; i < n16; i += WG)
      reinterpret_cast<uint4*>(smem)[i] = reinterpret_cast<const uint4*>(blob)[i];
    base = smem;
  } else {
    base = blob;
  }
  __syncthreads();
  View S;
  S.geo = reinterpret_cast<const double*>(base + P.off_geo);
  S.shade = reinterpret_cast<const double*>(base + P.off_shade);
  S.mats = reinterpret_cast<const double*>(base + P.off_mats);
  // lights section: a 16-double record of per-frame constants, then the lights
#if RT_SPEC_SLIGHTS
  const cdptr G = (cdptr)(blob + P.off_lights);
  S.lights = reinterpret_cast<const double*>(base + P.off_lights) + GLOB;
#else
  const double* G = reinterpret_cast<const double*>(base + P.off_lights);
  S.lights = G + GLOB;
#endif
  S.kind = reinterpret_cast<const int*>(base + P.off_kind);
  S.objmat = reinterpret_cast<const int*>(base + P.off_objmat);
  S.pref = reinterpret_cast<const uint32_t*>(base + P.off_pref);
  S.csg = reinterpret_cast<const int*>(base + P.off_csg);
  S.code = reinterpret_cast<const uint32_t*>(base + P.off_code);
  S.entry = reinterpret_cast<const int*>(base + P.off_entry);
  S.consts = reinterpret_cast<const uint64_t*>(base + P.off_consts);
#if RT_SPEC_SGEO && defined(RT_SPEC_NOBJ)
  const cdptr sgeo = (cdptr)(blob + P.off_geo);  // object records through scalar loads
#endif
#if RT_CSG_SCALAR
  // composite programs, leaf groups and leaf records through scalar loads
  const cdptr cs_geo = (cdptr)(blob + P.off_geo);
  const ciptr cs_kind = (ciptr)(blob + P.off_kind);
  const ciptr cs_csg = (ciptr)(blob + P.off_csg);
#define CSG_ARGS cs_geo, cs_kind, cs_csg
#define CSG_G(i, g) (cs_geo + (size_t)(i) * GEO)
#else
#define CSG_ARGS S.geo, S.kind, S.csg
#define CSG_G(i, g) (g)
#endif
#if RT_SPEC_SLIGHTS
  // wave-uniform records through scalar loads: lights, plane culls
  const cdptr slights = G + GLOB;
  const cdptr sshade = (cdptr)(blob + P.off_shade);
#define LTP(li) (slights + (size_t)(li) * LGT)
#define SHP(i) (sshade + (size_t)(i) * SHD)
#else
#define LTP(li) (S.lights + (size_t)(li) * LGT)
#define SHP(i) (S.shade + (size_t)(i) * SHD)
#endif

  const int lane = (int)(threadIdx.x & 63);
  const int wslot = (int)(blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6));
  double* stk = P.stack + (size_t)wslot * ((size_t)P.frames * FRAME_FIELDS * 64) + lane;
  const int lds_lv = P.lds_levels;
  double* lfr = reinterpret_cast<double*>(smem + P.lds_frames_off) +
                (size_t)(threadIdx.x >> 6) * (lds_lv * CORE * 64) + lane;
  // frame core accessors: level < lds_levels in LDS, deeper in HBM
  auto core_ld = [&](int level, int c) -> double {
    if (level < lds_lv) return lfr[(level * CORE + c) * 64];
    return frame_ptr(stk, level)[core_gfield(c) * 64];
  };
  // ext rows of `level` (pending refraction ray, then the first child's
  // colour; LDS for level < lds_full).
  const int lds_full = P.lds_full;
  double* lext = reinterpret_cast<double*>(smem + P.lds_ext_off) + (size_t)(threadIdx.x >> 6) * (lds_full * EXT_ROWS * 64) + lane;
  auto ext = [&](int level) -> double* {
    return level < lds_full ? lext + (size_t)level * EXT_ROWS * 64 : frame_ptr(stk, level) + FR_EXT * 64;
  };
  auto core_st = [&](int level, int c, double v) {
    if (level < lds_lv)
      lfr[(level * CORE + c) * 64] = v;
    else
      frame_ptr(stk, level)[core_gfield(c) * 64] = v;
  };
  // Per-lane material record written by the surface VM (same layout as mats).
  double* vmrec;
  if constexpr (LDS)
    vmrec = reinterpret_cast<double*>(smem + P.lds_vm_off) + (size_t)threadIdx.x * MAT;
  else
    vmrec = P.vm_global + ((size_t)wslot * 64 + lane) * MAT;
  // Global linear scenes (scene too large for LDS, no BVH, no CSG): object
  // records and kinds stream through a per-wave LDS buffer in chunks of SCH,
  // the next chunk's 16-B loads in flight while the current chunk is tested
  // (the in-order loop the reference runs, with the record latency hidden).
  // body(i, kind, record) returns false to stop (a wave-uniform decision).
  constexpr bool STREAM = !LDS && !BVH && !CSG && RT_STREAM;
  double* sbuf = reinterpret_cast<double*>(smem + P.stream_off) + (size_t)(threadIdx.x >> 6) * (SCH * GEO);
  int* skind = reinterpret_cast<int*>(smem + P.stream_off + WAVES_PER_WG * SCH * GEO * (int)sizeof(double)) +
               (threadIdx.x >> 6) * SCH;
  auto stream_objects = [&](auto&& body) {
    constexpr int PER = SCH * GEO * (int)sizeof(double) / 16 / 64;  // 16-B pieces per lane per chunk
    const uint4* src = reinterpret_cast<const uint4*>(S.geo);
    uint4* dst = reinterpret_cast<uint4*>(sbuf);
    const int lane_ = (int)(threadIdx.x & 63);
    uint4 pre[PER];
    int pk = 0;
    auto fetch = [&](int c0) {
      const int n16 = min(SCH, P.nobj - c0) * (GEO * (int)sizeof(double) / 16);
#pragma unroll
      for (int q = 0; q < PER; q++) {
        const int idx = lane_ + q * 64;
        pre[q] = idx < n16 ? src[(size_t)c0 * (GEO * sizeof(double) / 16) + idx] : make_uint4(0, 0, 0, 0);
      }
      pk = lane_ < min(SCH, P.nobj - c0) ? S.kind[c0 + lane_] : 0;
    };
    auto store = [&]() {
#pragma unroll
      for (int q = 0; q < PER; q++) dst[lane_ + q * 64] = pre[q];
      if (lane_ < SCH) skind[lane_] = pk;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    };
    if (P.nobj <= 0) return;
    fetch(0);
    store();
    for (int c0 = 0; c0 < P.nobj; c0 += SCH) {
      const int n = min(SCH, P.nobj - c0);
      const bool more = c0 + SCH < P.nobj;
      if (more) fetch(c0 + SCH);
#if RT_STREAM_PREFETCH
      // record j + 1 read from LDS while record j is tested (registers)
      double rec[GEO], nxt[GEO];
#pragma unroll
      for (int q = 0; q < GEO; q++) rec[q] = sbuf[q];
      int kc = skind[0];
      for (int j = 0; j < n; j++) {
        const int jn = j + 1 < n ? j + 1 : j;
#pragma unroll
        for (int q = 0; q < GEO; q++) nxt[q] = sbuf[(size_t)jn * GEO + q];
        const int kn = skind[jn];
        if (!body(c0 + j, kc, rec)) return;
#pragma unroll
        for (int q = 0; q < GEO; q++) rec[q] = nxt[q];
        kc = kn;
      }
#else
      for (int j = 0; j < n; j++)
        if (!body(c0 + j, skind[j], sbuf + (size_t)j * GEO)) return;
#endif
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // every lane done reading the chunk
      if (more) store();
    }
  };
  const d3 eye = mk(0.0, 0.0, -1.0);  // raytracer.go:605-609

  // lane state
  int state = S_IDLE;
  bool need_gen = false;  // lane waits for its next sample ray
  int px = 0, py = 0, sample = 0, sp = 0;
  unsigned int pout = 0;  // output pixel index
  // Finished pixel held for the wave's next batched framebuffer store
  // (RT_PIX_BATCH): index (~0u = none) and RGBA8 value.
  uint32_t held_px = ~0u, held_val = 0u;
  // One store instruction for every lane's held pixel (wave-uniform call).
  auto flush_pixels = [&]() {
    if (held_px != ~0u) P.out[held_px] = held_val;
    held_px = ~0u;
  };
  // work sharing (RT_SHARE): per-lane sample bookkeeping in Bd->lw (Board)
// the wave index through readfirstlane (an SGPR) in the BVH and CSG kernels:
// C4 -1.0 %, c4csg -2.2 %; C3 +0.5..1.2 %, C2 +1.3..2.2 % (profiles/r05/wave_ab/)
#ifndef RT_WAVE_SGPR
#define RT_WAVE_SGPR (BVH || CSG)
#endif
  const int wave = RT_WAVE_SGPR ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : (int)(threadIdx.x >> 6);
  int my_idle = 0, spins = 0;  // wave-uniform: idle lanes this wave reports, idle rounds
  bool my_active = true;       // wave-uniform: counted in Bd->nactive
  // wave-uniform: the tail has begun for this wave (it drained the queue, or
  // another wave of the group reported idle lanes); until then the board is
  // only looked at every 4th round
  bool sh_live = false;
  int hit_i = 0, hit_f = 0;
  double hit_t = 0.0;
  Pcg rng{0, 0};
  d3 sum = mk(0, 0, 0);
  d3 sum2 = mk(0, 0, 0);  // pixel pairs: the odd lane's sample-3 colour (sample 2's is in sum)
  Ray ray;
  ray.o = mk(0, 0, 0);
  ray.d = mk(0, 0, 1);

  // wave-uniform pool and counters
  unsigned int pool_next = 0, pool_end = 0;
  int qhead = 0;  // queue heads tried so far (QHEADS)
  bool exhausted = false;
  unsigned long long* cnt = reinterpret_cast<unsigned long long*>(smem + P.cnt_off);
  unsigned long long* kcnt = reinterpret_cast<unsigned long long*>(smem + P.cnt_off + CNT_KIND_OFF);
  for (int k = 0; k < RT_NUM_KINDS; k++) kcnt[k * WG + threadIdx.x] = 0;
  // The counters' LDS addresses in the BVH and CSG kernels are formed at each
  // use from a scalar base that the empty asm hides from loop-invariant
  // hoisting: hoisted, they were held in VGPRs across the main loop and
  // spilled, and each pass paid a scratch reload and a vmcnt(0) wait per
  // counter. C4 -1.0 %, c4csg -0.9 %; the small linear scenes (C3 within
  // noise, C2 +2 %) keep the plain form (profiles/r05/remat_ab/).
#ifndef RT_CNT_REMAT
#define RT_CNT_REMAT (BVH || CSG)
#endif
  auto opaque_s = [](uint32_t b) {  // (b is wave-uniform: readfirstlane makes that explicit)
    b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
    asm volatile("" : "+s"(b));
    return b;
  };
  // shadow tests of kind k (per lane): kcnt[k * WG + threadIdx.x]
  auto cnt_kind = [&](int k, uint64_t v) {
    if constexpr (RT_CNT_REMAT) {
      uint32_t l;  // the lane number from mbcnt at the use (a hoisted one was spilled too)
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
      const uint32_t a = opaque_s((uint32_t)P.cnt_off + (uint32_t)(CNT_KIND_OFF + (k * WG + wave * 64) * 8)) + l * 8u;
      atomicAdd(reinterpret_cast<unsigned long long*>(smem + a), (unsigned long long)v);
    } else {
      atomicAdd(&kcnt[k * WG + threadIdx.x], (unsigned long long)v);
    }
  };
  // a unit event on the lanes where b holds (wave-uniform call): cnt[k * WAVES_PER_WG + wave]
  auto cnt_unit = [&](int k, bool b) {
    const unsigned int n = (unsigned int)__popcll(wave_ballot(b));
    if (lane == 0 && n) {
      if constexpr (RT_CNT_REMAT)
        atomicAdd(reinterpret_cast<unsigned long long*>(
                      smem + opaque_s((uint32_t)P.cnt_off + (uint32_t)((k * WAVES_PER_WG + wave) * 8))),
                  (unsigned long long)n);
      else
        atomicAdd(&cnt[k * WAVES_PER_WG + wave], (unsigned long long)n);
    }
  };
  WaveStack bst;
  bst.mask = reinterpret_cast<uint64_t*>(smem + P.bvh_stack_off) + (threadIdx.x >> 6) * BVH_STACK;
  bst.ref = reinterpret_cast<int*>(smem + P.bvh_stack_off + WAVES_PER_WG * BVH_STACK * 8) + (threadIdx.x >> 6) * BVH_STACK;
#ifdef RT_PHASE_TIMING
  uint64_t ph_acc[N_PHASE] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t bd_tnodes = 0, bd_snodes = 0, bd_tleaf = 0, bd_sleaf = 0, bd_trays = 0, bd_srays = 0;
  // passes and their working lanes: TRACE (tracing lanes), SHADE (hit lanes), gen (new sample rays)
  uint64_t pd_tr = 0, pd_trl = 0, pd_sh = 0, pd_shl = 0, pd_gen = 0, pd_genl = 0;
  uint64_t ld_done = 0, ld_rounds = 0;  // lanes holding a finished quad / pair sample (S_DONE) per round
#ifdef RT_COST_MAP
  uint32_t lane_cost = 0;  // node visits charged to this lane's pixel (diagnostic)
#endif
#endif

  const double W1 = (double)(P.width - 1), H1 = (double)(P.height - 1);

  // New sample ray: raytracer.go:642-649.
  auto gen_ray = [&]() {
    double dx = pcg_float64(rng) - 0.5;
    double dy = pcg_float64(rng) - 0.5;
    const double vw = G[9], vh = G[10];
    double u = ((double)px + dx) / W1 * vw - vw / 2.0;
    double v = ((double)py + dy) / H1 * vh - vh / 2.0;
    ray.o = mk(u, -v, 0.0);
    ray.d = norm(sub(ray.o, eye));
  };

  // PCG state at the start of sample k of pixel (x, y): the strip seed
  // (raytracer.go:632-634) jumped 8*(y mod 20) + 2*k draws.
  auto sample_rng = [&](int x, int y, int k) {
    const int ry = y % 20;
    const uint64_t* j = P.jump + (ry * 4 + k) * 4;
    return pcg_jump(Pcg{0xDEADULL ^ (uint64_t)x, 0xBEEFULL ^ (uint64_t)(y - ry)}, j[0], j[1], j[2], j[3]);
  };
  // The board slot a waiting owner (S_WAIT) waits on: its posted sample
  // `sample` (at sp == 0), else the posted refraction child of frame sp - 1.
  auto wait_slot = [&]() -> int {
    if (RT_SHARE == 1 && !QD && sp == 0) return lw_fork(Bd->lw[threadIdx.x], sample);
    return PK_SLOT_OF(__double_as_longlong(core_ld(sp - 1, 4)));
  };
  // Serial samples: account sample `sample` onwards after the lane finished
  // the one before -- run it (own), take a helper's colour, reclaim a posted
  // sample nobody claimed, or wait; quantise once all 4 are summed.
  auto advance_sample = [&](uint32_t w) {  // w: the lane's Bd->lw word
    for (;;) {
      if (P.est_out && sample == 1) {  // cost estimate: one sample per tile
        state = S_IDLE;
        return;
      }
      if (PR && sample == ((lane & 1) ? 4 : 2)) {  // this lane's two samples are done: the pair adds them
        state = S_DONE;
        return;
      }
      if (sample == 4) {
        d3 c = scale(sum, 1.0 / 4.0);  // raytracer.go:656 -> vec.go:104-107
        uint32_t r8 = go_f64_to_u32(c.x * 65535.0) >> 8;
        uint32_t g8 = go_f64_to_u32(c.y * 65535.0) >> 8;
        uint32_t b8 = go_f64_to_u32(c.z * 65535.0) >> 8;
#ifdef RT_COST_MAP
        P.out[pout] = lane_cost;
        lane_cost = 0;
#else
        const uint32_t v = (r8 & 0xffu) | ((g8 & 0xffu) << 8) | ((b8 & 0xffu) << 16) | 0xff000000u;
        if (RT_PIX_BATCH) {  // (the S_ADV block flushed a previously held pixel)
          held_px = pout;
          held_val = v;
        } else {
          P.out[pout] = v;
        }
#endif
        state = S_IDLE;
        return;
      }
      if (RT_SHARE != 1 || __builtin_expect(sample < lw_own_end(w), 1)) {
        need_gen = true;  // next sample ray, generated in one uniform block
        state = S_TRACE;
        return;
      }
      const int q = lw_fork(w, sample);
      if (board_reclaim(Bd, q)) {  // nobody took it: trace it here
        SHDIAG(SH_RECLAIM);
        board_free(Bd, q);
        Bd->lw[threadIdx.x] = (w & ~7u) | (uint32_t)(sample + 1);  // own_end = sample + 1
        rng = sample_rng(px, py, sample);
        need_gen = true;
        state = S_TRACE;
        return;
      }
      if (!board_done(Bd, q)) {
        SHDIAG(SH_WAIT);
        state = S_WAIT;  // (the slot is found again from Bd->lw: wait_slot)
        return;
      }
      sum = add(sum, board_take(Bd, q));  // raytracer.go:651, in sample order
      sample++;
    }
  };

  // Propagate a finished traceRay colour up the lane's frame stack
  // (post-order, raytracer.go:528/554/557-561); ends with the lane either
  // tracing its next ray (pending refraction child / next sample), waiting
  // for a helper (S_WAIT) or idle.
  auto unwind = [&](bool have_res, d3 res, bool pf_valid, long long pf_packed, d3 pf_lw, double pf_kr) {
    while (wave_any(have_res)) {
      if (have_res) {
        if (sp == 0) {
          if constexpr (QD) {
            sum = res;  // this sample's colour, summed by the quad's first lane (main loop)
            state = S_DONE;
          } else {
            // raytracer.go:651 (a claimed sample's helper starts from sum = -0:
            // -0 + c == c for every c, so sum is exactly its colour); a pair's
            // odd lane keeps samples 2 and 3 apart for the even lane's sum
            if (PR && (lane & 1))
              (sample == 2 ? sum : sum2) = res;
            else
              sum = add(sum, res);
            sample++;
            state = S_ADV;
          }
          have_res = false;
        } else {
          double* f = frame_ptr(stk, sp - 1);
          long long packed;
          if (pf_valid)
            packed = pf_packed;
          else
            packed = __double_as_longlong(core_ld(sp - 1, 4));
          int fl = (int)(packed & 0xff);
          if (RT_SHARE && __builtin_expect((fl & FL_TASK) != 0, 0)) {  // a claimed subtree is done: hand its colour to the owner
            if constexpr (RT_SHARE == 2)
              gs_deliver(P.gboard, PK_SLOT_OF(packed), res);
            else
              board_deliver(Bd, PK_SLOT_OF(packed), res);
            sp = 0;
            state = S_IDLE;
            have_res = false;
          } else if ((fl & FL_HASR) && (fl & FL_HAST) && !(fl & FL_STAGE)) {
            // reflection child done; trace the pending refraction child.
            // Its colour takes the pending ray's rows once the ray is read.
            double* e = ext(sp - 1);
            const d3 first = res;
            bool here = true;
            core_st(sp - 1, 4, __longlong_as_double(packed | FL_STAGE));
            if (RT_SHARE && __builtin_expect((fl & FL_FORKED) != 0, 0)) {
              const int q = PK_SLOT_OF(packed);
              if (RT_SHARE == 2 ? gs_reclaim(P.gboard, q) : board_reclaim(Bd, q)) {  // nobody took it: trace it here
                SHDIAG(SH_RECLAIM);
                if (RT_SHARE == 1) board_free(Bd, q);
              } else if (RT_SHARE == 2 ? gs_done(P.gboard, q) : board_done(Bd, q)) {
                here = false;
                res = RT_SHARE == 2 ? gs_take(P.gboard, q) : board_take(Bd, q);  // the next round combines (FL_STAGE set)
              } else {
                SHDIAG(SH_WAIT);
                here = false;
                state = S_WAIT;  // (the slot is found again from the frame: wait_slot)
                have_res = false;
              }
            }
            if (here) {
              ray.o = ld3(e, 0);
              ray.d = ld3(e, 3);
              state = S_TRACE;
              have_res = false;
            }
            st3(e, 0, first);
          } else {
            const double* FM = S.mats + (size_t)(packed >> PK_MAT) * MAT;
            d3 R = mk(0, 0, 0), Tr = mk(0, 0, 0);
            if ((fl & FL_HASR) && (fl & FL_HAST)) {
              R = ld3(ext(sp - 1), 0);
              Tr = res;
            } else if (fl & FL_HASR) {
              R = res;
            } else {
              Tr = res;
            }
            d3 lw;
            double kr;
            if (pf_valid) {
              lw = pf_lw;
              kr = pf_kr;
            } else {
              lw = mk(core_ld(sp - 1, 0), core_ld(sp - 1, 1), core_ld(sp - 1, 2));
              kr = core_ld(sp - 1, 3);
            }
            d3 fcol;
            double frefl;
            if (spec_feat(SF_VM) && (fl & FL_VMMAT)) {
              fcol = ld3(f, FR_COL);
              frefl = f[FR_REFL * 64];
            } else {
              fcol = mk(FM[0], FM[1], FM[2]);
              frefl = FM[3];
            }
            res = combine((fl & FL_TMODE) != 0, lw, fcol, frefl, kr, R, Tr);
            sp--;
          }
          pf_valid = false;
        }
      }
    }
  };

  PH_BEGIN();
#ifdef RT_PHASE_TIMING
  const uint64_t life_t0 = ph_t0_;
  uint64_t last_grab = life_t0, nchunk_taken = 0;
#endif
  uint32_t guard_iters = 0;
  for (;;) {
    // watchdog: a wave that has not finished after 2^26 scheduling rounds
    // (far beyond any frame) stops and reports instead of hanging the device
    if (++guard_iters > (1u << 26)) {
      if (lane == 0) atomicAdd(P.stats + ST_WATCHDOG, 1ull);
      break;
    }
    // ---- serial samples: a lane that finished a sample goes on with the next
    // one (or hands a claimed sample's colour to its owner) ----
    if constexpr (!QD) {
      if (wave_any(state == S_ADV)) {
        // a lane about to finish a pixel while it still holds one: every
        // held pixel goes out in one store first (with sharing a lane may also
        // finish by taking helpers' colours, so any advancing holder flushes)
        if (RT_PIX_BATCH && wave_any(state == S_ADV && held_px != ~0u && (RT_SHARE || (!PR && sample == 4)))) flush_pixels();
        if (state == S_ADV) {
          const uint32_t w = RT_SHARE == 1 ? Bd->lw[threadIdx.x] : 4u;
          if (RT_SHARE == 1 && __builtin_expect(lw_task(w) >= 0, 0)) {
            board_deliver(Bd, lw_task(w), sum);
            Bd->lw[threadIdx.x] = 0u;
            state = S_IDLE;
          } else {
            advance_sample(w);
          }
        }
      }
    }
    // ---- quads whose 4 samples are all done: the first lane adds the
    // colours in sample order (raytracer.go:651) and quantises
    // (raytracer.go:656, vec.go:104-107); the quad becomes idle ----
    if constexpr (QD) {
      const uint64_t dn = wave_ballot(state == S_DONE);
      const uint64_t qd = dn & (dn >> 1) & (dn >> 2) & (dn >> 3) & 0x1111111111111111ull;
      if (qd) {
        // running sum (((0 + s0) + s1) + s2) + s3, one neighbour's colour at a time
        d3 sm = add(mk(0, 0, 0), sum);
#pragma unroll
        for (int k = 1; k < 4; k++) {
          const int lk = (lane + k) & 63;
          sm = add(sm, mk(__shfl(sum.x, lk), __shfl(sum.y, lk), __shfl(sum.z, lk)));
        }
        if (RT_PIX_BATCH && wave_any(((qd >> lane) & 1) && held_px != ~0u)) flush_pixels();
        if ((qd >> lane) & 1) {
          const d3 c = scale(sm, 1.0 / 4.0);
          const uint32_t r8 = go_f64_to_u32(c.x * 65535.0) >> 8;
          const uint32_t g8 = go_f64_to_u32(c.y * 65535.0) >> 8;
          const uint32_t b8 = go_f64_to_u32(c.z * 65535.0) >> 8;
          const uint32_t v = (r8 & 0xffu) | ((g8 & 0xffu) << 8) | ((b8 & 0xffu) << 16) | 0xff000000u;
          if (RT_PIX_BATCH) {
            held_px = pout;
            held_val = v;
          } else {
            P.out[pout] = v;
          }
        }
        if ((qd >> (lane & ~3)) & 1) state = S_IDLE;
      }
    }
    // ---- pairs whose 4 samples are all done: the even lane adds
    // (((0 + s0) + s1) + s2) + s3 -- its own running sum, then its
    // neighbour's two colours (raytracer.go:651) -- and quantises
    // (raytracer.go:656, vec.go:104-107); the pair becomes idle ----
    if constexpr (PR) {
      const uint64_t dn = wave_ballot(state == S_DONE);
      const uint64_t pd = dn & (dn >> 1) & 0x5555555555555555ull;
      if (pd) {
        const int lb = (lane + 1) & 63;
        const d3 c2 = mk(__shfl(sum.x, lb), __shfl(sum.y, lb), __shfl(sum.z, lb));
        const d3 c3 = mk(__shfl(sum2.x, lb), __shfl(sum2.y, lb), __shfl(sum2.z, lb));
        const d3 sm = add(add(sum, c2), c3);
        if (RT_PIX_BATCH && wave_any(((pd >> lane) & 1) && held_px != ~0u)) flush_pixels();
        if ((pd >> lane) & 1) {
          const d3 c = scale(sm, 1.0 / 4.0);
          const uint32_t r8 = go_f64_to_u32(c.x * 65535.0) >> 8;
          const uint32_t g8 = go_f64_to_u32(c.y * 65535.0) >> 8;
          const uint32_t b8 = go_f64_to_u32(c.z * 65535.0) >> 8;
          const uint32_t v = (r8 & 0xffu) | ((g8 & 0xffu) << 8) | ((b8 & 0xffu) << 16) | 0xff000000u;
          if (RT_PIX_BATCH) {
            held_px = pout;
            held_val = v;
          } else {
            P.out[pout] = v;
          }
        }
        if ((pd >> (lane & ~1)) & 1) state = S_IDLE;
      }
    }
    // ---- refill idle lanes from the wave pool (one 8x8 tile per chunk) ----
    for (;;) {
      // with quads a pixel goes to a quad whose 4 lanes are all idle, sample k
      // to lane 4p+k; mask = the idle lanes / the idle quads' first lanes
      const uint64_t il = wave_ballot(state == S_IDLE);
      const uint64_t mask = QD   ? il & (il >> 1) & (il >> 2) & (il >> 3) & 0x1111111111111111ull
                            : PR ? il & (il >> 1) & 0x5555555555555555ull
                                 : il;
      const bool need = ((mask >> (QD ? (lane & ~3) : PR ? (lane & ~1) : lane)) & 1) != 0;
      if (mask == 0 || exhausted) break;
      if (pool_next >= pool_end) {
        const unsigned int nchunks = (P.total_slots + QCHUNK - 1) / QCHUNK;
        unsigned int c = nchunks;
        const int nheads = gridDim.x >= QHEADS ? min(QHEADS, RT_QSTEAL + 1) : QHEADS;
        while (qhead < nheads) {
          const unsigned int h = (blockIdx.x + qhead) % QHEADS;
          const unsigned int dm = __builtin_amdgcn_readfirstlane(__atomic_load_n(qdrained, __ATOMIC_RELAXED));
          if ((dm >> h) & 1u) {  // another wave of the group found it drained
            qhead++;
            continue;
          }
          unsigned int n = 0;
          if (lane == 0) n = atomicAdd(P.queue + h * QSTRIDE, 1u);
          c = __builtin_amdgcn_readfirstlane(n) * QHEADS + h;
          if (c < nchunks) break;
          if (lane == 0) atomicOr(qdrained, 1u << h);
          qhead++;  // this head is drained: try the next one
        }
        if (qhead >= nheads) {
          exhausted = true;
          break;
        }
#ifdef RT_PHASE_TIMING
        last_grab = stamp();
        nchunk_taken++;
#endif
        pool_next = c * QCHUNK;
        pool_end = min(pool_next + (unsigned int)QCHUNK, P.total_slots);
      }
      // idle lanes (quads) before mine
      const unsigned int rank = QD   ? (unsigned int)__popcll(mask & ((1ull << (lane & ~3)) - 1ull))
                                : PR ? (unsigned int)__popcll(mask & ((1ull << (lane & ~1)) - 1ull))
                                     : __builtin_amdgcn_mbcnt_hi((unsigned int)(mask >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((unsigned int)mask, 0u));
      unsigned int take = min((unsigned int)__popcll(mask), pool_end - pool_next);
      if (!QD && !PR && P.est_out) {  // cost estimate: unit u = pixel (u mod est_pts) of frame tile u / est_pts
        if (need && rank < take) {
          const unsigned int u = pool_next + rank, t = u / (unsigned)P.est_pts, k = u % (unsigned)P.est_pts;
          px = min((int)(t % (unsigned)P.tiles_x) * TILE + est_x(P.est_pts, k), P.width - 1);
          py = min((int)(t / (unsigned)P.tiles_x) * TILE + est_y(P.est_pts, k), P.y1 - 1);
          pout = t;
          const int ry = py % 20;
          rng = pcg_jump(Pcg{0xDEADULL ^ (uint64_t)px, 0xBEEFULL ^ (uint64_t)(py - ry)}, jrows[ry * 4],
                         jrows[ry * 4 + 1], jrows[ry * 4 + 2], jrows[ry * 4 + 3]);
          sample = 0;
          if (RT_SHARE == 1) Bd->lw[threadIdx.x] = 1u;  // own_end = 1
          sum = mk(0, 0, 0);
          sp = 0;
          need_gen = true;
          state = S_TRACE;
        }
        pool_next += take;
        continue;
      }
      // a pool never crosses a tile: the tile's position is wave-uniform
      unsigned int tile = pool_next / (TILE * TILE);
      if (P.order) tile = P.order[tile];
      const int trow = (int)(tile / (unsigned)P.tiles_x);
      const int x0 = (int)((tile % (unsigned)P.tiles_x) * TILE);
      const int orow0 = trow * TILE;
      const int y0t = P.trow_stride > 0 ? (P.trow0 + trow * P.trow_stride) * TILE : P.y0 + orow0;
      const int r0t = y0t % 20;  // the tile's first row within its 20-row strip
      if (need && rank < take) {
        const unsigned int within = pool_next % (TILE * TILE) + rank;
        // quads: a 16-pixel chunk is a 4x4 quarter of the tile
        const int tx = QD ? (int)(((within >> 4) & 1u) * 4u + (within & 3u)) : (int)(within % TILE);
        const int ty = QD ? (int)((within >> 5) * 4u + ((within >> 2) & 3u)) : (int)(within / TILE);
        const int x = x0 + tx;
        const int orow = orow0 + ty;
        const int y = y0t + ty;
        if (x < P.width && y < P.y1) {
          px = x;
          py = y;
          pout = (unsigned int)orow * (unsigned int)P.width + (unsigned int)x;
          // rng = PCG(0xDEAD^x, 0xBEEF^ymin) advanced 8*(y%20) + 2*sample
          // draws (raytracer.go:632-643: 2 draws per sample, 4 samples per row)
          const int ry = r0t + ty >= 20 ? r0t + ty - 20 : r0t + ty;  // y % 20 (ty < 8)
          const int ymin = y - ry;
          Pcg s0{0xDEADULL ^ (uint64_t)x, 0xBEEFULL ^ (uint64_t)ymin};
          sample = QD ? (lane & 3) : PR ? (lane & 1) * 2 : 0;
          const uint64_t* j = (QD || PR) ? P.jump + (ry * 4 + sample) * 4 : jrows + ry * 4;
          rng = pcg_jump(s0, j[0], j[1], j[2], j[3]);
          sum = mk(0, 0, 0);
          sp = 0;
          if (RT_SHARE == 1) Bd->lw[threadIdx.x] = 4u;  // own_end = 4, nothing posted
          need_gen = true;
          state = S_TRACE;
        }
      }
      pool_next += take;
    }
    if (RT_SHARE == 1 && !sh_live && !exhausted && (guard_iters & 3u) == 0u)
      sh_live = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&Bd->nidle, __ATOMIC_RELAXED, RT_WG_SCOPE)) > 0;
    if (RT_SHARE == 2 && !sh_live && !exhausted && (guard_iters & 7u) == 0u)
      sh_live = __builtin_amdgcn_readfirstlane(lane == 0 ? (int)gs_ld32(g_nidle) : 0) > 0;
    if (RT_SHARE && !sh_live && exhausted) sh_live = true;
    if (RT_SHARE && !sh_live) {
      // steady state: the refill left no lane idle (else the queue is drained)
    } else if constexpr (RT_SHARE == 2) {
      // ---- device-wide work sharing (see gs_*) ----
      auto rfl64 = [](uint64_t v) {
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
               (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
      };
      // (a) waiting owners whose helper delivered resume (the TRACE pass
      // takes the colour and combines it at the frame)
      if (__builtin_expect(wave_any(state == S_WAIT), 0)) {
        if (state == S_WAIT && gs_done(P.gboard, wait_slot())) state = S_RESUME;
      }
      // the launch's idle helper lanes and posted, unclaimed tickets: a busy
      // wave reads them every 4th round; a helper polls the tail every round
      // and the others when it moved, or every 8th round
      if (gs_helper || (guard_iters & (unsigned)RT_GS_POLL) == 0u) {
        int nid = 0;
        uint64_t gh = 0, gt = 0;
        if (lane == 0) {
          gt = gs_ld(g_tail);
          if (!gs_helper || (guard_iters & 7u) == 0u || gt != gs_t) {
            nid = (int)gs_ld32(g_nidle);
            gh = gs_ld(g_head);
          } else {
            nid = gs_nid;
            gh = gs_h;
          }
        }
        gs_nid = __builtin_amdgcn_readfirstlane(nid);
        gs_h = rfl64(gh);
        gs_t = rfl64(gt);
      }
      const int nid = gs_nid;
      const uint64_t gh = gs_h, gt = gs_t;
      const long long outstanding = (long long)(gt - gh);
      // (b) owners post the pending refraction child of their shallowest
      // binary frame (frames above a claimed subtree's sentinel only) while
      // idle lanes anywhere on the device outnumber the posted tickets
      const int want = nid - (int)min(outstanding, (long long)(1 << 30));
      if (__builtin_expect(want > 0 && outstanding < GS_RSH / 2, 0)) {
        const bool busy_lane = state == S_TRACE || state == S_SHADE || state == S_WAIT;
        int L = -1;
        // (a child at level L + 1 roots at most 2^(depth - L - 1) - 1 rays:
        // only subtrees of RT_GS_MIN_LEVELS levels or more are worth a hand-off)
        if (busy_lane)
          for (int l = min(sp - 1, P.depth - 1 - RT_GS_MIN_LEVELS); l >= 0; l--) {
            const int f = (int)(__double_as_longlong(core_ld(l, 4)) & 0xff);
            if (f & FL_TASK) break;
            if ((f & (FL_HASR | FL_HAST | FL_STAGE | FL_FORKED)) == (FL_HASR | FL_HAST)) L = l;
          }
        const uint64_t cm = wave_ballot(L >= 0);
        if (cm) {
          const int npost = min((int)__popcll(cm), want);
          const int rk = (int)__builtin_amdgcn_mbcnt_hi((unsigned int)(cm >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned int)cm, 0u));
          const bool post = L >= 0 && rk < npost;
          int q = 0;
          if (post) {
            SHDIAG(SH_POST_T);
            q = (wslot * 64 + lane) * P.frames + L;
            uint64_t* r = gs_slot(P.gboard, q);
            const double* e = ext(L);
            const d3 o = ld3(e, 0), dd = ld3(e, 3);
            gs_st(r + 0, (uint64_t)__double_as_longlong(o.x));
            gs_st(r + 1, (uint64_t)__double_as_longlong(o.y));
            gs_st(r + 2, (uint64_t)__double_as_longlong(o.z));
            gs_st(r + 3, (uint64_t)__double_as_longlong(dd.x));
            gs_st(r + 4, (uint64_t)__double_as_longlong(dd.y));
            gs_st(r + 5, (uint64_t)__double_as_longlong(dd.z));
            gs_st(r + 6, (uint64_t)(L + 1));
            gs_drain();
            gs_st(r + 7, GS_POSTED);
            const long long pk = __double_as_longlong(core_ld(L, 4));
            core_st(L, 4, __longlong_as_double(pk | FL_FORKED | ((long long)q << PK_SLOT)));
          }
          gs_drain();  // every posted slot's state has landed before its ticket
          uint64_t t0 = 0;
          if (lane == 0) t0 = __hip_atomic_fetch_add(g_tail, (uint64_t)npost, __ATOMIC_RELAXED, RT_AG_SCOPE);
          t0 = rfl64(t0);
          if (post) {
            const uint64_t t = t0 + (uint64_t)rk;
            gs_st(g_ring + (t & (GS_RSH - 1)), (t << 32) | (uint32_t)q);
          }
        }
      }
      // (c) idle lanes of a drained wave claim tickets: from its own shard's
      // ring, or -- a helper whose ring is empty, every 4th round -- from the
      // first other shard with tickets (one load per shard, a lane each)
      uint64_t il = exhausted ? wave_ballot(state == S_IDLE) : 0ull;
      int cshard = gshard;
      uint64_t ch = gh;
      bool ctry = outstanding > 0;
      if (GS_SH > 1 && il != 0 && !ctry && gs_helper && (guard_iters & 3u) == 0u && !P.est_out) {
        const int k = lane < GS_SH ? (gshard + 1 + lane) % GS_SH : gshard;
        uint64_t ot = 0, oh = 0;
        if (lane < GS_SH - 1) {
          ot = gs_ld(P.gctl + GS_SHARD * k + GS_TAIL);
          oh = gs_ld(P.gctl + GS_SHARD * k + GS_HEAD);
        }
        const uint64_t hasm = wave_ballot(lane < GS_SH - 1 && ot > oh);
        if (hasm) {
          const int fl = __builtin_ctzll(hasm);
          cshard = (gshard + 1 + fl) % GS_SH;
          ch = rfl64(__shfl(oh, fl));
          ctry = true;
        }
      }
      if (__builtin_expect(il != 0 && ctry && !P.est_out, 0)) {
        uint64_t* const c_head = P.gctl + GS_SHARD * cshard + GS_HEAD;
        uint64_t* const c_tail = P.gctl + GS_SHARD * cshard + GS_TAIL;
        uint64_t* const c_ring = P.gring + (size_t)cshard * GS_RSH;
        const int nil = (int)__popcll(il);
        uint64_t h = 0;
        int k = 0;
        if (lane == 0) {
          uint64_t hh = ch;
          for (int tries = 0; tries < 4; tries++) {
            const uint64_t tt = gs_ld(c_tail);
            const int kk = tt > hh ? (int)min((uint64_t)nil, tt - hh) : 0;
            if (kk <= 0) break;
            if (__hip_atomic_compare_exchange_strong(c_head, &hh, hh + (uint64_t)kk, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, RT_AG_SCOPE)) {
              h = hh;
              k = kk;
              break;
            }
          }
        }
        h = rfl64(h);
        k = __builtin_amdgcn_readfirstlane(k);
        if (k > 0) {
          const int rk = (int)__builtin_amdgcn_mbcnt_hi((unsigned int)(il >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned int)il, 0u));
          if (state == S_IDLE && rk < k) {
            const uint64_t t = h + (uint64_t)rk;
            uint64_t e = 0;
            // the poster writes the ticket's entry right after taking it
            for (int w_ = 0; w_ < (1 << 14); w_++) {
              e = gs_ld(c_ring + (t & (GS_RSH - 1)));
              if ((uint32_t)(e >> 32) == (uint32_t)t) break;
              __builtin_amdgcn_s_sleep(1);
            }
            if ((uint32_t)(e >> 32) == (uint32_t)t && (uint32_t)e < P.gslots) {
              const int q = (int)(uint32_t)e;
              uint64_t* r = gs_slot(P.gboard, q);
              if (gs_claim(r)) {  // (else its owner took it back)
                SHDIAG(SH_CLAIM);
                ray.o = mk(__longlong_as_double((long long)gs_ld(r + 0)), __longlong_as_double((long long)gs_ld(r + 1)),
                           __longlong_as_double((long long)gs_ld(r + 2)));
                ray.d = mk(__longlong_as_double((long long)gs_ld(r + 3)), __longlong_as_double((long long)gs_ld(r + 4)),
                           __longlong_as_double((long long)gs_ld(r + 5)));
                const int m0 = (int)gs_ld(r + 6);
                // a sentinel below the subtree (its colour goes to slot q); the
                // subtree runs at its own absolute levels
                core_st(m0 - 1, 4, __longlong_as_double((long long)FL_TASK | ((long long)q << PK_SLOT)));
                sp = m0;
                state = S_TRACE;
              }
            }
          }
          il = wave_ballot(state == S_IDLE);
        }
      }
      // (d) bookkeeping: helpers available (idle lanes of drained waves),
      // waves still busy
      const int cur_idle = (exhausted && !P.est_out) ? (int)__popcll(il) : 0;
      if (cur_idle != my_idle) {
        nidle_add(cur_idle - my_idle);
        my_idle = cur_idle;
      }
      const bool busy = wave_any(state != S_IDLE);
      if (busy != my_active) {
        if (lane == 0) atomicAdd(g_active, busy ? 1u : 0xffffffffu);
        my_active = busy;
      }
      if (__builtin_expect(!busy, 0)) {
        // drained: the first RT_GS_HELPERS such waves stay while the launch
        // may still post work, the others leave at once (thousands of pollers
        // would saturate the board's words); a helper leaves once no wave is
        // busy -- a posted or claimed subtree's owner is busy until it has
        // the colour, so then nothing is left to take (stale tickets of
        // reclaimed slots may remain) -- or after RT_SHARE_SPINS idle rounds
        if (!gs_helper) {
          unsigned int old = 0;
          if (lane == 0) old = atomicAdd(g_helpers, 1u);
          gs_helper = __builtin_amdgcn_readfirstlane((int)old) < RT_GS_HELPERS;
          if (!gs_helper) {
            if (my_idle) nidle_add(-my_idle);
            break;
          }
        }
        const int na = (spins & 7) ? 1 : __builtin_amdgcn_readfirstlane(lane == 0 ? (int)gs_ld32(g_active) : 0);
        if (na == 0 || ++spins > RT_SHARE_SPINS) {
#ifdef RT_PHASE_TIMING
          if (lane == 0) atomicAdd(P.stats + ST_SHDIAG + SH_SPIN, (unsigned long long)spins);
#endif
          if (my_idle) nidle_add(-my_idle);
          break;
        }
        __builtin_amdgcn_s_sleep(RT_SHARE_SLEEP);
        continue;
      }
      spins = 0;
      if (__builtin_expect(!wave_any(state == S_TRACE || state == S_SHADE || state == S_RESUME), 0)) {
        __builtin_amdgcn_s_sleep(RT_SHARE_SLEEP / 4);  // only waiting (or quad-holding) lanes
        continue;
      }
    } else if constexpr (RT_SHARE == 1) {
      // ---- work sharing within the workgroup (see Board) ----
      // (a) owners whose helper delivered take the colour; it is propagated
      // by the TRACE pass's unwind (a posted sample is added in sample order
      // at sp == 0, a posted refraction child combined at its frame)
      if (__builtin_expect(wave_any(state == S_WAIT), 0)) {
        if (state == S_WAIT && board_done(Bd, wait_slot())) state = S_RESUME;
      }
      // (b) owners post work they have not started, while drained waves of
      // the group have idle lanes to take it
      const int nid = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&Bd->nidle, __ATOMIC_RELAXED, RT_WG_SCOPE));
      const uint64_t pmp = nid > 0 ? __hip_atomic_load(&Bd->post, __ATOMIC_RELAXED, RT_WG_SCOPE) : 0ull;
      const int want = nid - (int)__popcll(((uint64_t)__builtin_amdgcn_readfirstlane((int)(pmp >> 32)) << 32) |
                                           (uint32_t)__builtin_amdgcn_readfirstlane((int)pmp));
      if (__builtin_expect(want > 0, 0)) {
        const bool busy_lane = state == S_TRACE || state == S_SHADE || state == S_WAIT;
        // candidates: an unstarted own sample (serial samples), else the
        // shallowest frame whose refraction child is pending and not posted
        // (frames above a claimed subtree's sentinel only)
        const uint32_t w = busy_lane ? Bd->lw[threadIdx.x] : 0u;
        const bool cs = !QD && RT_SHARE_SAMPLES && busy_lane && lw_task(w) < 0 && lw_own_end(w) - 1 > sample;
        int L = -1;
        if (busy_lane && !cs)
          for (int l = sp - 1; l >= 0; l--) {
            const int f = (int)(__double_as_longlong(core_ld(l, 4)) & 0xff);
            if (f & FL_TASK) break;
            if ((f & (FL_HASR | FL_HAST | FL_STAGE | FL_FORKED)) == (FL_HASR | FL_HAST)) L = l;
          }
        const bool cand = cs || L >= 0;
        const uint64_t cm = wave_ballot(cand);
        if (cm) {
          const uint32_t wf = (uint32_t)__builtin_amdgcn_readfirstlane(
              (int)__hip_atomic_load(&Bd->wfree[wave], __ATOMIC_RELAXED, RT_WG_SCOPE));
          const int npost = min(min((int)__popcll(cm), (int)__popc(wf)), want);
          if (npost > 0) {
            const uint32_t used = (uint32_t)low_bits(wf, npost);
            const int rk = (int)__builtin_amdgcn_mbcnt_hi((unsigned int)(cm >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((unsigned int)cm, 0u));
            if (cand && rk < npost) {
              const int q = wave * SLOTS_PER_WAVE + nth_bit(wf, rk);
              if (cs) {  // the last of the lane's unstarted samples
                SHDIAG(SH_POST_S);
                const int k = lw_own_end(w) - 1;
                Bd->meta[q][0] = px | (k << 16) | META_SAMPLE;
                Bd->meta[q][1] = py;
                const int sh = 10 + 6 * (k - 1);
                Bd->lw[threadIdx.x] = (w & ~7u & ~(63u << sh)) | (uint32_t)k | ((uint32_t)q << sh);
              } else {  // the pending refraction child of frame L, traced at level L + 1
                SHDIAG(SH_POST_T);
                const double* e = ext(L);
                const d3 o = ld3(e, 0), dd = ld3(e, 3);
                Bd->ray[q][0] = o.x;
                Bd->ray[q][1] = o.y;
                Bd->ray[q][2] = o.z;
                Bd->ray[q][3] = dd.x;
                Bd->ray[q][4] = dd.y;
                Bd->ray[q][5] = dd.z;
                Bd->meta[q][0] = L + 1;
                Bd->meta[q][1] = 0;
                const long long pk = __double_as_longlong(core_ld(L, 4));
                core_st(L, 4, __longlong_as_double(pk | FL_FORKED | ((long long)q << PK_SLOT)));
              }
            }
            if (lane == 0) {
              __hip_atomic_fetch_and(&Bd->wfree[wave], ~used, __ATOMIC_RELAXED, RT_WG_SCOPE);
              __hip_atomic_fetch_or(&Bd->post, (uint64_t)used << (wave * SLOTS_PER_WAVE), __ATOMIC_RELEASE,
                                    RT_WG_SCOPE);
            }
          }
        }
      }
      // (c) idle lanes of a drained wave claim posted tasks
      uint64_t il = exhausted ? wave_ballot(state == S_IDLE) : 0ull;
      if (__builtin_expect(il != 0, 0)) {
        const uint64_t pm0 = __hip_atomic_load(&Bd->post, __ATOMIC_RELAXED, RT_WG_SCOPE);
        const uint64_t pm = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(pm0 >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)pm0);
        if (pm) {
          const uint64_t want = low_bits(pm, (int)__popcll(il));
          uint64_t old = 0;
          if (lane == 0) old = __hip_atomic_fetch_and(&Bd->post, ~want, __ATOMIC_ACQUIRE, RT_WG_SCOPE);
          const uint64_t got = want & (((uint64_t)__builtin_amdgcn_readfirstlane((int)(old >> 32)) << 32) |
                                       (uint32_t)__builtin_amdgcn_readfirstlane((int)old));
          const int rk = (int)__builtin_amdgcn_mbcnt_hi((unsigned int)(il >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned int)il, 0u));
          if (state == S_IDLE && rk < (int)__popcll(got)) {
            const int q = nth_bit(got, rk);
            SHDIAG(SH_CLAIM);
            const int m0 = Bd->meta[q][0];
            if (m0 & META_SAMPLE) {  // sample k of pixel (x, y)
              px = m0 & 0xffff;
              py = Bd->meta[q][1];
              sample = (m0 >> 16) & 3;
              Bd->lw[threadIdx.x] = (uint32_t)(sample + 1) | ((uint32_t)(q + 1) << 3);
              sum = mk(-0.0, -0.0, -0.0);
              rng = sample_rng(px, py, sample);
              need_gen = true;
              sp = 0;
            } else {  // a refraction subtree at level m0 >= 1, under a sentinel frame
              ray.o = mk(Bd->ray[q][0], Bd->ray[q][1], Bd->ray[q][2]);
              ray.d = mk(Bd->ray[q][3], Bd->ray[q][4], Bd->ray[q][5]);
              core_st(m0 - 1, 4, __longlong_as_double((long long)FL_TASK | ((long long)q << PK_SLOT)));
              Bd->lw[threadIdx.x] = 0u;
              sp = m0;
            }
            state = S_TRACE;
          }
          il = wave_ballot(state == S_IDLE);
        }
      }
      // (d) bookkeeping for the board: helpers available, waves still busy
      const int cur_idle = P.est_out ? 0 : (int)__popcll(il);
      if (cur_idle != my_idle) {
        if (lane == 0) __hip_atomic_fetch_add(&Bd->nidle, cur_idle - my_idle, __ATOMIC_RELAXED, RT_WG_SCOPE);
        my_idle = cur_idle;
      }
      const bool busy = wave_any(state != S_IDLE);
      if (busy != my_active) {
        if (lane == 0) __hip_atomic_fetch_add(&Bd->nactive, busy ? 1 : -1, __ATOMIC_RELAXED, RT_WG_SCOPE);
        my_active = busy;
      }
      if (__builtin_expect(!busy, 0)) {
        // drained (the refill found nothing): wait while the group may still
        // post work; leave once no wave is busy and nothing is posted
        const int na = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&Bd->nactive, __ATOMIC_RELAXED, RT_WG_SCOPE));
        const uint64_t pm = __hip_atomic_load(&Bd->post, __ATOMIC_RELAXED, RT_WG_SCOPE);
        if ((na == 0 && __builtin_amdgcn_readfirstlane((int)(pm >> 32)) == 0 &&
             __builtin_amdgcn_readfirstlane((int)pm) == 0) ||
            ++spins > RT_SHARE_SPINS) {
#ifdef RT_PHASE_TIMING
          if (lane == 0) atomicAdd(P.stats + ST_SHDIAG + SH_SPIN, (unsigned long long)spins);
#endif
          if (lane == 0 && my_idle) __hip_atomic_fetch_add(&Bd->nidle, -my_idle, __ATOMIC_RELAXED, RT_WG_SCOPE);
          break;
        }
        __builtin_amdgcn_s_sleep(RT_SHARE_SLEEP);
        continue;
      }
      spins = 0;
      if (__builtin_expect(!wave_any(state == S_TRACE || state == S_SHADE || state == S_RESUME), 0)) {  // only waiting (or quad-holding) lanes
        __builtin_amdgcn_s_sleep(RT_SHARE_SLEEP / 4);
        continue;
      }
    } else {
      if (!wave_any(state != S_IDLE)) break;
    }
#ifdef RT_PHASE_TIMING
    ld_done += (uint64_t)__popcll(wave_ballot(state == S_DONE));
    ld_rounds++;
#endif
    PH_MARK(0);
    // ---- new sample rays for every lane that needs one, in one block ----
    if (wave_any(need_gen)) {
#ifdef RT_PHASE_TIMING
      pd_gen++;
      pd_genl += (uint64_t)__popcll(wave_ballot(need_gen));
#endif
      if (need_gen) {
        gen_ray();
        need_gen = false;
      }
    }
    PH_MARK(1);

    // ---- TRACE pass: closestHit over all objects (raytracer.go:469-483) ----
    if (wave_any(state == S_TRACE || (RT_SHARE && state == S_RESUME))) {
      const bool tr = state == S_TRACE;
      // Prefetch the parent frame: a ray that misses pops it right after
      // this pass, and the load latency hides under the object loop.
      bool pf = false;
      long long pf_packed = 0;
      d3 pf_lw = mk(0, 0, 0);
      double pf_kr = 0.0;
#if RT_FRAME_PREFETCH
      if (tr && sp > 0) {
        pf = true;
        pf_packed = __double_as_longlong(core_ld(sp - 1, 4));
        pf_lw = mk(core_ld(sp - 1, 0), core_ld(sp - 1, 1), core_ld(sp - 1, 2));
        pf_kr = core_ld(sp - 1, 3);
      }
#endif
      bool found = false;
      double best_t = 0.0;
      int best_i = 0, best_f = 0;
      const F3 of = f3(ray.o), df = f3(ray.d);
      const float slack = ray_slack(of);
      // One closestHit candidate (object i, wave-uniform) for the lanes in `act`.
      // The linear loop visits objects in index order (strict <, the first
      // index wins ties); the BVH visits them in any order and breaks ties on
      // the index explicitly, which selects the same object.
      auto trace_exact = [&](int i, int k, const double* g, bool test) {
        EXDIAG(k, 0, test);
        if (test) {
          double t;
          int f;
          bool h;
          if constexpr (CSG)
            h = k == RT_CSG ? csg_hit(CSG_ARGS, P.nobj, CSG_G(i, g), ray, t, f, 1.0,
                                      found ? best_t : __builtin_inf(), true)
                            : object_hit(k, g, ray, t, f);
          else
            h = object_hit(k, g, ray, t, f);
          if (h) {
            if (!found || t < best_t || (BVH && t == best_t && i < best_i)) {
              found = true;
              best_t = t;
              best_i = i;
              best_f = f;
            }
          }
        }
      };
      auto trace_obj = [&](int i, int k, const double* g, bool act) {
        bool test = act;
#if RT_CULL
        // an object entered beyond the lane's current best cannot win (strict <)
        const float tmax = found ? (float)best_t * 1.0001f + 1e-4f : 3.0e38f;
        test = k != RT_PLANE ? may_hit_a(test, of, df, tmax, g, slack)
                             : CULL_AND(test, may_hit_plane(of, df, tmax, SHP(i)));
        if (!wave_any(test)) return;
#endif
        trace_exact(i, k, g, test);
      };
      if constexpr (!BVH) {
#ifdef RT_SPEC_NOBJ
        {
#pragma unroll
          for (int i = 0; i < RT_SPEC_NOBJ; i++) {
#if RT_SPEC_SGEO
            // (scalar loads, see RT_SPEC_SGEO)
            double gl[GEO];
#pragma unroll
            for (int q = 0; q < GEO; q++) gl[q] = sgeo[i * GEO + q];
            trace_obj(i, spec_kinds[i], gl, tr);
#else
            trace_obj(i, spec_kinds[i], S.geo + (size_t)i * GEO, tr);
#endif
          }
        }
#else
        if constexpr (STREAM) {
#if RT_STREAM_SMEM && !RT_CULL
          // Brute force over a global linear scene, in kind runs. A sphere run
          // is a scalar-load loop with the next record in flight: every lane
          // forms the quadratic (Sphere.Intersect, raytracer.go:58-104) and only
          // lanes with a real root take the sqrt/division branch; index order,
          // strict < (closestHit, raytracer.go:469-483).
          const cdptr cgeo = (cdptr)S.geo;
          auto tsphere = [&](int i, const Ray& l) {
            const double a = dot(l.d, l.d);
            const double hb = dot(l.o, l.d);
            const double c = dot(l.o, l.o) - 1.0;
            const double disc = hb * hb - a * c;
            if (tr && !(disc < 0.0)) {
              const double t0 = (-hb - gsqrt(disc)) / a;
              if (t0 > 0.0 && (!found || t0 < best_t)) {
                found = true;
                best_t = t0;
                best_i = i;
                best_f = 0;
              }
            }
          };
          // scale + translation spheres take the diagonal transform (exact, see axis_o)
          const bool rax = wave_all(!tr || (axis_o_ok(ray.o) && axis_d_ok(ray.d)));
          for (int r = 0; r < P.nruns; r++) {
            // (wave-uniform run fields: readfirstlane keeps the record addresses in SGPRs)
            const int r0 = __builtin_amdgcn_readfirstlane(P.runs[4 * r]), rn = __builtin_amdgcn_readfirstlane(P.runs[4 * r + 1]),
                      rk = __builtin_amdgcn_readfirstlane(P.runs[4 * r + 2]), rax_k = __builtin_amdgcn_readfirstlane(P.runs[4 * r + 3]);
            if (spec_kind(RT_SPHERE) && rk == RT_SPHERE && rax_k == 2 && rax) {
              // uniform scale s for the whole run (see UNI_REC)
              const double sc = ((cdptr)P.urec)[(size_t)r0 * UNI_REC + 3];
              const d3 so = mk(sc * ray.o.x, sc * ray.o.y, sc * ray.o.z);
              Ray l;
              l.d = mk(sc * ray.d.x, sc * ray.d.y, sc * ray.d.z);
              const double a = dot(l.d, l.d);
              auto ubody = [&](int i, double tx, double ty, double tz) {
                l.o = mk(so.x + tx, so.y + ty, so.z + tz);
                const double hb = dot(l.o, l.d);
                const double c = dot(l.o, l.o) - 1.0;
                const double disc = hb * hb - a * c;
                if (tr && !(disc < 0.0)) {
                  const double t0 = (-hb - gsqrt(disc)) / a;
                  if (t0 > 0.0 && (!found || t0 < best_t)) {
                    found = true;
                    best_t = t0;
                    best_i = i;
                    best_f = 0;
                  }
                }
              };
              if (RT_UNI_PAIRS)
                scan_uni<0>((cdptr)P.urec, r0, rn, ubody, [] { return false; });
              else
                scan_records<0, 3, UNI_REC>((cdptr)P.urec, r0, rn, [&](int i, const Rec3& R) { ubody(i, R.m[0], R.m[1], R.m[2]); },
                                            [] { return false; });
            } else if (spec_kind(RT_SPHERE) && rk == RT_SPHERE && rax_k && rax) {
              scan_records<0, 6, AXIS_REC>((cdptr)P.arec, r0, rn, [&](int i, const Rec6& R) {
                Ray l;
                l.o = axis_o(R.m, ray.o);
                l.d = axis_d(R.m, ray.d);
                tsphere(i, l);
              }, [] { return false; });
            } else if (spec_kind(RT_SPHERE) && rk == RT_SPHERE) {
              scan_records<0>(cgeo, r0, rn, [&](int i, const Rec12& R) { tsphere(i, to_obj(R.m, ray)); },
                              [] { return false; });
            } else {
              for (int i = r0; i < r0 + rn; i++) trace_obj(i, rk, S.geo + (size_t)i * GEO, tr);
            }
          }
#else
          stream_objects([&](int i, int k, const double* g) {
            trace_obj(i, k, g, tr);
            return true;
          });
#endif
        } else {
          for (int i = 0; i < P.nobj; i++) trace_obj(i, S.kind[i], S.geo + (size_t)i * GEO, tr);
        }
#endif
      } else {
        for (int p = 0; p < P.nplanes; p++) {  // unbounded objects: planes, unbounded CSG
          const int i = P.planes[p];
          trace_obj(i, S.kind[i], S.geo + (size_t)i * GEO, tr);
        }
        const F3 idf = f3_rcp(df);
        // far origins: the BVH culls' origin, slack and bounds (see far_shift)
        F3 bof = of;
        float bslack = slack;
        double bt0 = 0.0;
        bool btr = tr;
        far_shift(btr, ray, P.bvh_lo, P.bvh_hi, bof, bslack, bt0);
#if RT_AXIS_LEAF
        // leaves' scale + translation spheres take the diagonal transform (exact, see axis_o)
        const bool rax = wave_all(!tr || (axis_o_ok(ray.o) && axis_d_ok(ray.d)));
#endif
#ifdef RT_PHASE_TIMING
        bd_trays++;
#endif
        int ssp = 0;
#if RT_BVH_CONT
        int nr = 0;  // the node visited next, kept in registers (see RT_BVH_CONT)
        uint64_t nm = wave_ballot(btr);
        bool have = true;
        for (;;) {
          int r;
          uint64_t m;
          if (have) {
            r = nr;
            m = nm;
            have = false;
          } else {
            if (ssp == 0) break;
            ssp--;
            r = __builtin_amdgcn_readfirstlane(bst.ref[ssp]);
            m = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(bst.mask[ssp] >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((int)bst.mask[ssp]);
          }
#else
        bst.push(ssp, lane, 0, wave_ballot(btr));
        while (ssp > 0) {
          ssp--;
          const int r = __builtin_amdgcn_readfirstlane(bst.ref[ssp]);
          const uint64_t m = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(bst.mask[ssp] >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((int)bst.mask[ssp]);
#endif
          const bool act = btr && ((m >> lane) & 1);
#ifdef RT_PHASE_TIMING
          bd_tnodes++;
#ifdef RT_COST_MAP
          if (tr) lane_cost++;
#endif
#endif
          if (r & 7) {  // leaf
#ifdef RT_PHASE_TIMING
            bd_tleaf++;
#endif
            const int first = r >> 3, count = r & 7;
            for (int j = first; j < first + count; j++) {
              // the leaf's record through scalar loads (wave-uniform index)
              const LeafRec L = ld_leaf(P.bvh_geo, j);
              const float tmax = found ? (float)(best_t - bt0) * 1.0001f + 1e-4f : 3.0e38f;
              const bool test = may_hit_s(act, bof, df, tmax, L.cx, L.cy, L.cz, L.cr, bslack);
              if (!wave_any(test)) continue;
#if RT_AXIS_LEAF
              if (spec_kind(RT_SPHERE) && L.k == RT_SPHERE && L.ax && rax) {
                // scale + translation sphere: diagonal transform (exact, see axis_o)
                EXDIAG(RT_SPHERE, 0, test);
                if (test) {
                  const double a[6] = {L.R.m[0], L.R.m[3], L.R.m[5], L.R.m[7], L.R.m[10], L.R.m[11]};
                  Ray l;
                  l.o = axis_o(a, ray.o);
                  l.d = axis_d(a, ray.d);
                  double t;
                  if (sphere_hit(l, t) && (!found || t < best_t || (t == best_t && L.i < best_i))) {
                    found = true;
                    best_t = t;
                    best_i = L.i;
                    best_f = 0;
                  }
                }
                continue;
              }
#endif
              trace_exact(L.i, L.k, L.R.m, test);
            }
          } else {
            const cfptr nb = (cfptr)P.bvh_nodes + (size_t)(r >> 3) * BN;  // scalar loads
            const ciptr ni = (ciptr)(nb + 12);
            const float tmax = found ? (float)(best_t - bt0) * 1.0001f + 1e-4f : 3.0e38f;
            float t0 = 0.0f, t1 = 0.0f;  // (set by may_hit_box when it returns true)
            const bool a0 = may_hit_box_a(act, bof, idf, bslack, tmax, nb, t0);
            const bool a1 = may_hit_box_a(act, bof, idf, bslack, tmax, nb + 6, t1);
            const uint64_t m0 = wave_ballot(a0), m1 = wave_ballot(a1);
            // near child popped first: the one most lanes enter first
            const bool c1_first = 2 * __popcll(wave_ballot(a0 && a1 && t1 < t0)) > __popcll(m0 & m1);
#if RT_BVH_CONT
            bvh_next(bst, ssp, lane, c1_first, ni[0], ni[1], m0, m1, nr, nm, have);
#else
            if (c1_first) {
              if (m0) bst.push(ssp, lane, ni[0], m0);
              if (m1) bst.push(ssp, lane, ni[1], m1);
            } else {
              if (m1) bst.push(ssp, lane, ni[1], m1);
              if (m0) bst.push(ssp, lane, ni[0], m0);
            }
#endif
          }
        }
      }
      cnt_unit(CNT_TRACED, tr);
#ifdef RT_PHASE_TIMING
      pd_tr++;
      pd_trl += (uint64_t)__popcll(wave_ballot(tr));
#endif
      if (!QD && P.est_out && tr) atomicAdd(P.est_out + pout, 1u);
      PH_MARK(2);
      d3 res = mk(0, 0, 0);
      if (tr) {
        if (found) {
          state = S_SHADE;
          hit_i = best_i;
          hit_f = best_f;
          hit_t = best_t;
        } else {  // background gradient, raytracer.go:493-497
          double t = 0.5 * (ray.d.y + 1.0);
          res = lerp(mk(G[3], G[4], G[5]), mk(G[6], G[7], G[8]), t);
        }
      }
      const bool resumed = RT_SHARE && state == S_RESUME;  // a waiting owner's helper delivered
      if (__builtin_expect(resumed, 0))  // (not tracing: pf is false)
        res = RT_SHARE == 2 ? gs_take(P.gboard, wait_slot()) : board_take(Bd, wait_slot());
      unwind((tr && !found) || resumed, res, pf, pf_packed, pf_lw, pf_kr);
      PH_MARK(3);
    }

    // ---- SHADE pass, once enough lanes hold a hit ----
    const uint64_t nsh = popc_ballot(state == S_SHADE);
    // (a lane that finished a sample and starts the next one at the loop top,
    // S_ADV, counts as tracing: leaving it out ran SHADE with fewer lanes,
    // lane utilisation 0.83 -> 0.74 and C3 +5 %)
    const uint64_t ntr = popc_ballot(state == S_TRACE ||
                                     (!QD && state == S_ADV && (RT_SHARE || sample < (PR && !(lane & 1) ? 2 : 4))));
    if (nsh == 0 || (ntr != 0 && nsh * RT_SHADE_DEN < (nsh + ntr) * RT_SHADE_NUM)) continue;

    const bool hit = state == S_SHADE;
    cnt_unit(CNT_SHADED, hit);
#ifdef RT_PHASE_TIMING
    pd_sh++;
    pd_shl += (uint64_t)__popcll(wave_ballot(hit));
#endif
    // ComputeSurfaceProps (raytracer.go:106-122, 182-194, 242-260, 339-370)
    d3 pw = mk(0, 0, 0), nw = mk(0, 0, 1);
    int mat = 0;
    bool surf_bad = false;
    if (hit) {
      int si = hit_i, sf = hit_f;  // the surface: the object, or a CSG composite's leaf
      bool flip = false;
      if constexpr (CSG) {
        if (S.kind[hit_i] == RT_CSG) {
          const int* ci = reinterpret_cast<const int*>(S.geo + (size_t)hit_i * GEO + 14);
          si = P.nobj + ci[0] + (hit_f >> 4);
          flip = ((hit_f >> 3) & 1) != 0;
          sf = hit_f & 7;
        }
      }
      const double* g = S.geo + (size_t)si * GEO;
      const double* s = S.shade + (size_t)si * SHD;
      const int k = S.kind[si];
      Ray l = to_obj(g, ray);
      d3 p = add(l.o, scale(l.d, hit_t));  // Hit.PointObj
      pw = mk(s[0] * p.x + s[1] * p.y + s[2] * p.z + s[3], s[4] * p.x + s[5] * p.y + s[6] * p.z + s[7],
              s[8] * p.x + s[9] * p.y + s[10] * p.z + s[11]);
      if (spec_kind(RT_SPHERE) && k == RT_SPHERE) {
        nw = p;
      } else if ((spec_kind(RT_CYLINDER) && k == RT_CYLINDER) || (spec_kind(RT_CONE) && k == RT_CONE)) {
        d3 n = sf == 0 ? (k == RT_CONE ? mk(p.x, -p.y, p.z) : mk(p.x, 0, p.z)) : (sf == 1 ? mk(0, 1, 0) : mk(0, -1, 0));
        // NormalMat = WorldToObject^T (raytracer.go:814): MulDir then Normalize.
        nw = norm(mk(g[0] * n.x + g[4] * n.y + g[8] * n.z, g[1] * n.x + g[5] * n.y + g[9] * n.z,
                     g[2] * n.x + g[6] * n.y + g[10] * n.z));
      } else {
        nw = mk(s[12 + sf * 3], s[13 + sf * 3], s[14 + sf * 3]);
      }
      if (flip) nw = neg(nw);  // the composite's outward normal
      mat = S.objmat[(size_t)si * OMAT + sf];
      if (spec_feat(SF_VM) && mat < 0) {
        // Closure surface: (face, u, v) as ComputeSurfaceProps computes them
        // (raytracer.go:124-150, 196-205, 249, 339-359), then the VM.
        double u, v;
        bool bad = false;
        long long face = (k == RT_PLANE) ? 0 : sf;
        if (k == RT_SPHERE) {
          bad = __builtin_fabs(p.y) > 1;
          v = (p.y + 1.0) / 2.0;
          u = go_acos(p.z / __builtin_sqrt(1.0 - p.y * p.y)) / 6.283185307179586;
        } else if ((k == RT_CYLINDER || k == RT_CONE) && sf == 0) {
          u = (go_atan2(p.x, p.z) + 3.141592653589793) / 6.283185307179586;
          v = p.y;
        } else {
          u = p.x;
          v = p.z;
        }
        double r[10];
        bad = run_vm(S.code, S.consts, S.entry[-mat - 1], face, u, v, r) || bad;
        if (bad)  // counted; the material reads as all-zero (oracle convention)
          for (int k = 0; k < 10; k++) r[k] = 0.0;
        vmrec[0] = r[0];
        vmrec[1] = r[1];
        vmrec[2] = r[2];
        vmrec[3] = r[3];
        const double fz = r[4];
        if (fz >= 0) {  // baked constant fuzz offset (raytracer.go:516-522)
          const double cf = go_cos(fz), sf = go_sin(fz);
          vmrec[4] = fz * cf * cf;
          vmrec[5] = fz * sf * sf;
          vmrec[6] = 1.0;
        } else {
          vmrec[4] = vmrec[5] = vmrec[6] = 0.0;
        }
        vmrec[7] = r[5];
        vmrec[8] = r[6];
        vmrec[9] = r[7];
        vmrec[10] = r[8];
        vmrec[11] = r[9];
        vmrec[12] = 1.0 / vmrec[8];  // (the host's per-material terms, see rt_set_scene)
        const double r0 = (1.0 - vmrec[8]) / (1.0 + vmrec[8]);
        vmrec[13] = r0 * r0;
        surf_bad = bad;
      }
    }
    cnt_unit(CNT_SURFERR, surf_bad);

    // computeLighting + inShadow (raytracer.go:372-429)
    PH_MARK(4);
    const double* M = (!spec_feat(SF_VM) || mat >= 0) ? S.mats + (size_t)mat * MAT : vmrec;
    d3 L = mk(0, 0, 0);
    if (hit) L = scale(mk(G[0], G[1], G[2]), M[9]);
    const double rlen = len(ray.d);
#if RT_STMAX_F32
    const float rlen_rcpf = __builtin_amdgcn_rcpf((float)rlen);
#endif
    const d3 sorig = add(pw, scale(nw, 1e-4));
// (hoisting the plane culls' origin half out of the light loop measured
// +4.6 % on C3, profiles/r05/c3_ab: not kept)
#define SH_PLANE_CULL(i, d, tmax) may_hit_plane(sof, d, tmax, SHP(i))
// (the culls' origin-to-centre vectors hoisted out of the light loop
// measured -1.5 % VALU but C3 +2..3 % from spills: not kept)
    uint32_t sc0 = 0, sc1 = 0, sc2 = 0, sc3 = 0;  // this hit's shadow tests per kind (cones: below)
    // Direction and distance to a light (raytracer.go:378-380).
    auto light_dir = [&](auto lt, d3& ldir, double& dist) {
      if (spec_feat(SF_LDIR) && (int)lt[9] == RT_LIGHT_DIRECTIONAL) {  // extension: light at infinity
        ldir = mk(lt[6], lt[7], lt[8]);
        dist = __builtin_inf();
      } else {
        d3 lth = sub(mk(lt[0], lt[1], lt[2]), pw);
        ldir = norm_len(lth, dist);  // dist = len(lth)
      }
    };
// (lighting after all shadow verdicts, RT_LIGHT_SPLIT, measured +2.4 % VALU
// instructions: removed)
#ifdef RT_SPEC_NLIGHTS
    // Specialised: every light's direction up front -- independent sqrt and
    // division chains the scheduler interleaves -- and the light loop unrolled.
    d3 ldir_a[RT_SPEC_NLIGHTS];
    double dist_a[RT_SPEC_NLIGHTS];
    // (one shared fix-up branch for all lights' normalisations measured
    // C3 +0.2..1 %: not kept)
#pragma unroll
    for (int li = 0; li < RT_SPEC_NLIGHTS; li++) light_dir(LTP(li), ldir_a[li], dist_a[li]);
    PH_MARK(5);
// (at most 4 lights: with 5-8 the joint sweep's per-light state broke the
// backend -- "illegal VGPR to SGPR copy", which aborts the process inside
// hipRTC -- in round 4's code as in this one; scripts/spec_matrix.sh)
#if RT_STREAM_SMEM && !RT_CULL && RT_SHADOW_JOINT && !defined(RT_SPEC_NOBJ) && RT_SPEC_NLIGHTS <= 4
#define RT_JOINT_SWEEP 1
#else
#define RT_JOINT_SWEEP 0
#endif
#if RT_JOINT_SWEEP
    // Brute force over a global linear scene: one sweep over the objects for
    // every light's shadow ray of this hit (inShadow per light, raytracer.go:
    // 411-429, each stopping at its own first occluder). The rays share their
    // origin, so the object-space origin and c = |o|^2 - 1 are formed once per
    // object -- the same operations as one to_obj + Sphere.Intersect per light
    // (raytracer.go:51-56, 58-104), so verdicts and counts are bit-identical.
    bool jopen[RT_SPEC_NLIGHTS];
    int jsend[RT_SPEC_NLIGHTS];
#pragma unroll
    for (int li = 0; li < RT_SPEC_NLIGHTS; li++) {
      jopen[li] = hit;
      jsend[li] = P.nobj;
    }
    if constexpr (STREAM) {
      const cdptr cgeo = (cdptr)S.geo;
      // wave-uniform: bit li = light li still has an open lane (one scalar
      // mask: an array of 8 such flags was kept in VGPRs and its branches then
      // needed an illegal VGPR -> SGPR copy)
      int lonm = 0;
      auto refresh = [&]() {
        int m = 0;
#pragma unroll
        for (int li = 0; li < RT_SPEC_NLIGHTS; li++) m |= wave_any(jopen[li]) ? (1 << li) : 0;
        lonm = __builtin_amdgcn_readfirstlane(m);
        return lonm != 0;
      };
      // one object against every light's shadow ray: lo = the shared
      // object-space origin; ldir(li) = light li's object-space direction
      auto jsphere = [&](int i, const d3 lo, auto&& ldir) {
        const double c = dot(lo, lo) - 1.0;
#pragma unroll
        for (int li = 0; li < RT_SPEC_NLIGHTS; li++) {
          if (!((lonm >> li) & 1)) continue;
          const d3 ld = ldir(li);
          const double a = dot(ld, ld);
          const double hb = dot(lo, ld);
          const double disc = hb * hb - a * c;
          if (jopen[li] && !(disc < 0.0)) {  // (i != hit_i: see ssphere)
            const double t0 = (-hb - gsqrt(disc)) / a;
            if (t0 > 0.0 && t0 * rlen < dist_a[li] && i != hit_i) {
              jopen[li] = false;
              jsend[li] = i + 1;
            }
          }
        }
      };
      // scale + translation spheres take the diagonal transform (exact, see axis_o)
      bool sax_l = !hit || axis_o_ok(sorig);
#pragma unroll
      for (int li = 0; li < RT_SPEC_NLIGHTS; li++) sax_l = sax_l && (!hit || axis_d_ok(ldir_a[li]));
      const bool sax = wave_all(sax_l);
      for (int r = 0; r < P.nruns; r++) {
        if (!refresh()) break;
        // (wave-uniform run fields: readfirstlane keeps the record addresses in SGPRs)
            const int r0 = __builtin_amdgcn_readfirstlane(P.runs[4 * r]), rn = __builtin_amdgcn_readfirstlane(P.runs[4 * r + 1]),
                      rk = __builtin_amdgcn_readfirstlane(P.runs[4 * r + 2]), rax_k = __builtin_amdgcn_readfirstlane(P.runs[4 * r + 3]);
        if (spec_kind(RT_SPHERE) && rk == RT_SPHERE && rax_k == 2 && sax) {
          // uniform scale s for the run (see UNI_REC): every light's s*d and
          // a = dot(s*d, s*d) once per run, the origin's s*o once
          const double sc = ((cdptr)P.urec)[(size_t)r0 * UNI_REC + 3];
          const d3 so = mk(sc * sorig.x, sc * sorig.y, sc * sorig.z);
          d3 uld[RT_SPEC_NLIGHTS];
          double ua[RT_SPEC_NLIGHTS];
#pragma unroll
          for (int li = 0; li < RT_SPEC_NLIGHTS; li++) {
            uld[li] = mk(sc * ldir_a[li].x, sc * ldir_a[li].y, sc * ldir_a[li].z);
            ua[li] = dot(uld[li], uld[li]);
          }
          auto ubody = [&](int i, double tx, double ty, double tz) {
            const d3 lo = mk(so.x + tx, so.y + ty, so.z + tz);
            const double c = dot(lo, lo) - 1.0;
#pragma unroll
            for (int li = 0; li < RT_SPEC_NLIGHTS; li++) {
              if (!((lonm >> li) & 1)) continue;
              const double hb = dot(lo, uld[li]);
              const double disc = hb * hb - ua[li] * c;
              if (jopen[li] && !(disc < 0.0)) {  // (i != hit_i: see ssphere)
                const double t0 = (-hb - gsqrt(disc)) / ua[li];
                if (t0 > 0.0 && t0 * rlen < dist_a[li] && i != hit_i) {
                  jopen[li] = false;
                  jsend[li] = i + 1;
                }
              }
            }
          };
          if (RT_UNI_PAIRS)
            scan_uni<RT_SHADOW_CHECK>((cdptr)P.urec, r0, rn, ubody, [&] { return !refresh(); });
          else
            scan_records<RT_SHADOW_CHECK, 3, UNI_REC>((cdptr)P.urec, r0, rn,
                                                      [&](int i, const Rec3& R) { ubody(i, R.m[0], R.m[1], R.m[2]); },
                                                      [&] { return !refresh(); });
        } else if (spec_kind(RT_SPHERE) && rk == RT_SPHERE && rax_k && sax) {
          scan_records<RT_SHADOW_CHECK, 6, AXIS_REC>((cdptr)P.arec, r0, rn, [&](int i, const Rec6& R) {
            jsphere(i, axis_o(R.m, sorig), [&](int li) { return axis_d(R.m, ldir_a[li]); });
          }, [&] { return !refresh(); });
        } else if (spec_kind(RT_SPHERE) && rk == RT_SPHERE) {
          scan_records<RT_SHADOW_CHECK>(cgeo, r0, rn, [&](int i, const Rec12& R) {
            jsphere(i, to_obj_o(R.m, sorig), [&](int li) { return to_obj_d(R.m, ldir_a[li]); });
          }, [&] { return !refresh(); });
        } else {
          for (int i = r0; i < r0 + rn; i++) {
#pragma unroll
            for (int li = 0; li < RT_SPEC_NLIGHTS; li++) {
              if (jopen[li] && i != hit_i) {
                Ray sr;
                sr.o = sorig;
                sr.d = ldir_a[li];
                double t;
                int f;
                if (object_hit(rk, S.geo + (size_t)i * GEO, sr, t, f) && t * rlen < dist_a[li]) {
                  jopen[li] = false;
                  jsend[li] = i + 1;
                }
              }
            }
          }
        }
      }
    }
#endif
// (one culled sweep over the objects for every light's shadow ray of a hit,
// RT_JOINT_CULL, measured C3 +6 % from 38 spilled VGPRs: removed)
#pragma unroll
    for (int li = 0; li < RT_SPEC_NLIGHTS; li++) {
      const auto lt = LTP(li);
      const int lkind = (int)lt[9];  // wave-uniform
      const d3 ldir = ldir_a[li];
      const double dist = dist_a[li];
#else
    for (int li = 0; li < P.nlights; li++) {
      const auto lt = LTP(li);
      const int lkind = (int)lt[9];  // wave-uniform
      d3 ldir;
      double dist;
      light_dir(lt, ldir, dist);
#endif
      bool open = hit;  // lanes still looking for an occluder
      Ray sr;
      sr.o = sorig;
      sr.d = ldir;
      const F3 sof = f3(sorig), sdf = f3(ldir);
      const float sslack = ray_slack(sof);
      // occluders must lie within t < dist / |ray.d| (raytracer.go:424)
#if RT_STMAX_F32
      // FP32 reciprocal instead of an FP64 division: relative error < 4 ulp(f32)
      // ~ 2.4e-7, far inside the 1e-4 margin (NaN / inf cases as in FP64;
      // dist = 0 culls everything, and nothing can occlude within t*|d| < 0)
      const float stmax = (float)dist * rlen_rcpf * 1.0001f + 1e-4f;
#else
      const float stmax = (float)(dist / rlen) * 1.0001f + 1e-4f;
#endif
      // inShadow's test count is #{i < end, i != hit} with end = first
      // occluder + 1 (or nobj); counted per kind from the prefix table below.
      int send = P.nobj;
      if constexpr (!BVH) {
#ifdef RT_SPEC_NOBJ
#pragma unroll
        for (int i = 0; i < RT_SPEC_NOBJ; i++) {
          if (!wave_any(open)) break;
          const int k = spec_kinds[i];
#else
        if constexpr (STREAM) {
#if defined(RT_SPEC_NLIGHTS) && RT_JOINT_SWEEP
          open = jopen[li];  // the joint sweep above
          send = jsend[li];
#elif RT_STREAM_SMEM && !RT_CULL
          // Brute force in kind runs (see the TRACE pass); inShadow stops at the
          // first occluder (raytracer.go:411-429), the wave once no lane is open
          // (tested every RT_SHADOW_CHECK objects: a closed lane never reopens).
          const cdptr cgeo = (cdptr)S.geo;
          auto ssphere = [&](int i, const Ray& l) {
            const double a = dot(l.d, l.d);
            const double hb = dot(l.o, l.d);
            const double c = dot(l.o, l.o) - 1.0;
            const double disc = hb * hb - a * c;
            // The hit's own object (i == hit_i, raytracer.go:416) is excluded
            // after the rare real-root branch, not before it: the lane's hit
            // index is then read only there (the brute-force kernel keeps it in
            // scratch, and a compare per sphere cost a scratch reload and a
            // vmcnt(0) wait per sphere and light). Its sqrt and division have
            // no side effect; verdicts and counts are unchanged.
            if (open && !(disc < 0.0)) {
              const double t0 = (-hb - gsqrt(disc)) / a;
              if (t0 > 0.0 && t0 * rlen < dist && i != hit_i) {
                open = false;
                send = i + 1;
              }
            }
          };
          const bool sax = wave_all(!hit || (axis_o_ok(sr.o) && axis_d_ok(sr.d)));
          for (int r = 0; r < P.nruns; r++) {
            if (!wave_any(open)) break;
            // (wave-uniform run fields: readfirstlane keeps the record addresses in SGPRs)
            const int r0 = __builtin_amdgcn_readfirstlane(P.runs[4 * r]), rn = __builtin_amdgcn_readfirstlane(P.runs[4 * r + 1]),
                      rk = __builtin_amdgcn_readfirstlane(P.runs[4 * r + 2]), rax_k = __builtin_amdgcn_readfirstlane(P.runs[4 * r + 3]);
            if (spec_kind(RT_SPHERE) && rk == RT_SPHERE && rax_k == 2 && sax) {
              const double sc = ((cdptr)P.urec)[(size_t)r0 * UNI_REC + 3];  // (see UNI_REC)
              const d3 so = mk(sc * sr.o.x, sc * sr.o.y, sc * sr.o.z);
              Ray l;
              l.d = mk(sc * sr.d.x, sc * sr.d.y, sc * sr.d.z);
              scan_records<RT_SHADOW_CHECK, 3, UNI_REC>((cdptr)P.urec, r0, rn, [&](int i, const Rec3& R) {
                l.o = mk(so.x + R.m[0], so.y + R.m[1], so.z + R.m[2]);
                ssphere(i, l);
              }, [&] { return !wave_any(open); });
            } else if (spec_kind(RT_SPHERE) && rk == RT_SPHERE && rax_k && sax) {
              scan_records<RT_SHADOW_CHECK, 6, AXIS_REC>((cdptr)P.arec, r0, rn, [&](int i, const Rec6& R) {
                Ray l;
                l.o = axis_o(R.m, sr.o);
                l.d = axis_d(R.m, sr.d);
                ssphere(i, l);
              }, [&] { return !wave_any(open); });
            } else if (spec_kind(RT_SPHERE) && rk == RT_SPHERE) {
              scan_records<RT_SHADOW_CHECK>(cgeo, r0, rn, [&](int i, const Rec12& R) { ssphere(i, to_obj(R.m, sr)); },
                                            [&] { return !wave_any(open); });
            } else {
              for (int i = r0; i < r0 + rn; i++) {
                if (!wave_any(open)) break;
                if (open && i != hit_i) {
                  double t;
                  int f;
                  if (object_hit(rk, S.geo + (size_t)i * GEO, sr, t, f) && t * rlen < dist) {
                    open = false;
                    send = i + 1;
                  }
                }
              }
            }
          }
#else
          stream_objects([&](int i, int k, const double* g) {
            if (!wave_any(open)) return false;
            bool test = CULL_AND(open, i != hit_i);
#if RT_CULL
            test = k != RT_PLANE ? may_hit_a(test, sof, sdf, stmax, g, sslack)
                                 : CULL_AND(test, may_hit_plane(sof, sdf, stmax, SHP(i)));
            if (!wave_any(test)) return true;
#endif
            EXDIAG(k, 1, test);
            if (test) {
              double t;
              int f;
              if (object_hit(k, g, sr, t, f) && t * rlen < dist) {
                open = false;
                send = i + 1;
              }
            }
            return true;
          });
#endif
        }
        for (int i = STREAM ? P.nobj : 0; i < P.nobj; i++) {
          if (!wave_any(open)) break;
          const int k = S.kind[i];
#endif
#if RT_SPEC_SGEO && defined(RT_SPEC_NOBJ)
          double gl[GEO];
#pragma unroll
          for (int q = 0; q < GEO; q++) gl[q] = sgeo[i * GEO + q];
          const double* g = gl;
#else
          const double* g = S.geo + (size_t)i * GEO;
#endif
          bool test = CULL_AND(open, i != hit_i);
#if RT_CULL
          test = k != RT_PLANE ? may_hit_a(test, sof, sdf, stmax, g, sslack)
                               : CULL_AND(test, SH_PLANE_CULL(i, sdf, stmax));
          if (!wave_any(test)) continue;
#endif
          EXDIAG(k, 1, test);
          if (test) {
            double t;
            int f;
            bool h;
            if constexpr (CSG)
              h = k == RT_CSG ? csg_hit(CSG_ARGS, P.nobj, CSG_G(i, g), sr, t, f, rlen, dist, false)
                              : object_hit(k, g, sr, t, f);
            else
              h = object_hit(k, g, sr, t, f);
            if (h) {
              if (t * rlen < dist) {
                open = false;
                send = i + 1;
              }
            }
          }
        }
      } else {
        // The reference stops at the first occluder in index order and its
        // test count is #{i <= that index, i != hit}; the BVH finds the
        // lowest-index occluder (pruning subtrees whose smallest index is not
        // lower than the best so far) and derives the count from prefix
        // counts per kind. The shadow verdict is the same either way.
        int occ = 0x7fffffff;
        auto shadow_exact = [&](int i, int k, const double* g, bool test) {
          EXDIAG(k, 1, test);
          if (test) {
            double t;
            int f;
            bool h;
            if constexpr (CSG)
              h = k == RT_CSG ? csg_hit(CSG_ARGS, P.nobj, CSG_G(i, g), sr, t, f, rlen, dist, false)
                              : object_hit(k, g, sr, t, f);
            else
              h = object_hit(k, g, sr, t, f);
            if (h) {
              if (t * rlen < dist) occ = i;
            }
          }
        };
        auto shadow_obj = [&](int i, int k, const double* g, bool act) {
          bool test = CULL_AND(CULL_AND(act, i != hit_i), i < occ);
          test = k != RT_PLANE ? may_hit_a(test, sof, sdf, stmax, g, sslack)
                               : CULL_AND(test, may_hit_plane(sof, sdf, stmax, SHP(i)));
          if (!wave_any(test)) return;
          shadow_exact(i, k, g, test);
        };
        for (int p = 0; p < P.nplanes; p++) {
          const int i = P.planes[p];
          shadow_obj(i, S.kind[i], S.geo + (size_t)i * GEO, hit);
        }
        const F3 sidf = f3_rcp(sdf);
        // far origins: the BVH culls' origin, slack and bound (see far_shift)
        F3 sbof = sof;
        float sbslack = sslack;
        double sbt0 = 0.0;
        bool sact = hit;
        far_shift(sact, sr, P.bvh_lo, P.bvh_hi, sbof, sbslack, sbt0);
        const float sbtmax = sbt0 == 0.0 ? stmax : (float)(dist / rlen - sbt0) * 1.0001f + 1e-4f;
#if RT_AXIS_LEAF
        const bool sax = wave_all(!hit || (axis_o_ok(sr.o) && axis_d_ok(sr.d)));
#endif
#ifdef RT_PHASE_TIMING
        bd_srays++;
#endif
        int ssp = 0;
#if RT_BVH_CONT
        int nr = 0;
        uint64_t nm = wave_ballot(sact);
        bool have = true;
        for (;;) {
          int r;
          uint64_t m;
          if (have) {
            r = nr;
            m = nm;
            have = false;
          } else {
            if (ssp == 0) break;
            ssp--;
            r = __builtin_amdgcn_readfirstlane(bst.ref[ssp]);
            m = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(bst.mask[ssp] >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((int)bst.mask[ssp]);
          }
#else
        bst.push(ssp, lane, 0, wave_ballot(sact));
        while (ssp > 0) {
          ssp--;
          const int r = __builtin_amdgcn_readfirstlane(bst.ref[ssp]);
          const uint64_t m = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(bst.mask[ssp] >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((int)bst.mask[ssp]);
#endif
          const bool act = sact && ((m >> lane) & 1);
#ifdef RT_PHASE_TIMING
          bd_snodes++;
#ifdef RT_COST_MAP
          if (hit) lane_cost++;
#endif
#endif
          if (r & 7) {  // leaf
#ifdef RT_PHASE_TIMING
            bd_sleaf++;
#endif
            const int first = r >> 3, count = r & 7;
            for (int j = first; j < first + count; j++) {
              const LeafRec L = ld_leaf(P.bvh_geo, j);  // scalar loads
              const bool test = may_hit_s(CULL_AND(CULL_AND(act, L.i != hit_i), L.i < occ), sbof, sdf, sbtmax, L.cx,
                                          L.cy, L.cz, L.cr, sbslack);
              if (!wave_any(test)) continue;
#if RT_AXIS_LEAF
              if (spec_kind(RT_SPHERE) && L.k == RT_SPHERE && L.ax && sax) {
                // scale + translation sphere: diagonal transform (exact, see axis_o)
                EXDIAG(RT_SPHERE, 1, test);
                if (test) {
                  const double a[6] = {L.R.m[0], L.R.m[3], L.R.m[5], L.R.m[7], L.R.m[10], L.R.m[11]};
                  Ray l;
                  l.o = axis_o(a, sr.o);
                  l.d = axis_d(a, sr.d);
                  double t;
                  if (sphere_hit(l, t) && t * rlen < dist) occ = L.i;
                }
                continue;
              }
#endif
              shadow_exact(L.i, L.k, L.R.m, test);
            }
          } else {
            const cfptr nb = (cfptr)P.bvh_nodes + (size_t)(r >> 3) * BN;  // scalar loads
            const ciptr ni = (ciptr)(nb + 12);
            float t0 = 0.0f, t1 = 0.0f;
            const bool a0 = may_hit_box_a(CULL_AND(act, ni[2] < occ), sbof, sidf, sbslack, sbtmax, nb, t0);
            const bool a1 = may_hit_box_a(CULL_AND(act, ni[3] < occ), sbof, sidf, sbslack, sbtmax, nb + 6, t1);
            const uint64_t m0 = wave_ballot(a0), m1 = wave_ballot(a1);
#ifndef RT_SHADOW_NEAR_FIRST
#define RT_SHADOW_NEAR_FIRST 0  // measured: near-first shadow order is slower (C5 695 -> 822 ms)
#endif
#if RT_SHADOW_NEAR_FIRST
            // nearer subtree popped first: finds an occluder soonest
            const bool c1_first = 2 * __popcll(wave_ballot(a0 && a1 && t1 < t0)) > __popcll(m0 & m1);
#else
            // lower-index subtree popped first: it can prune the other
            const bool c1_first = ni[3] < ni[2];
#endif
#if RT_BVH_CONT
            bvh_next(bst, ssp, lane, c1_first, ni[0], ni[1], m0, m1, nr, nm, have);
#else
            if (c1_first) {
              if (m0) bst.push(ssp, lane, ni[0], m0);
              if (m1) bst.push(ssp, lane, ni[1], m1);
            } else {
              if (m1) bst.push(ssp, lane, ni[1], m1);
              if (m0) bst.push(ssp, lane, ni[0], m0);
            }
#endif
          }
        }
        open = hit && occ == 0x7fffffff;
        send = open ? P.nobj : occ + 1;
      }
      if (hit) {
        const uint4 pe = *reinterpret_cast<const uint4*>(S.pref + (size_t)send * PREF);
        const uint32_t pe4 = S.pref[(size_t)send * PREF + 4];
        const int hk = hit_i < send ? S.kind[hit_i] : -1;
        sc0 += pe.x - (hk == 0 ? 1u : 0u);
        sc1 += pe.y - (hk == 1 ? 1u : 0u);
        sc2 += pe.z - (hk == 2 ? 1u : 0u);
        sc3 += pe.w - (hk == 3 ? 1u : 0u);
        if (spec_kind(4) && (P.kind_mask & 16)) cnt_kind(4, pe4 - (hk == 4 ? 1u : 0u));  // cones, CSG: rare, flushed per light
        if (spec_kind(5) && (P.kind_mask & 32)) cnt_kind(5, S.pref[(size_t)send * PREF + 5] - (hk == 5 ? 1u : 0u));
      }
      PH_MARK(6);
      if (hit && open) {
        d3 lcol = mk(lt[3], lt[4], lt[5]);
        if (spec_feat(SF_LSPOT) && lkind == RT_LIGHT_SPOT) {  // extension: cone falloff
          const double ca = dot(neg(ldir), mk(lt[6], lt[7], lt[8]));
          lcol = scale(lcol, ca >= lt[10] ? go_pow(ca, lt[11], (int)G[11]) : 0.0);
        }
        double ndl = go_max0(dot(nw, ldir));
        d3 diffuse = scale(lcol, ndl * M[9]);
        d3 H = norm(add(neg(ray.d), ldir));
        double spec = go_max0(dot(nw, H));
        d3 specular = scale(lcol, M[10] * go_pow(spec, M[11], (int)G[11]));
        L = add(add(L, diffuse), specular);
      }
      PH_MARK(7);
    }
    if (hit) {
      if (spec_kind(0) && (P.kind_mask & 1)) cnt_kind(0, sc0);
      if (spec_kind(1) && (P.kind_mask & 2)) cnt_kind(1, sc1);
      if (spec_kind(2) && (P.kind_mask & 4)) cnt_kind(2, sc2);
      if (spec_kind(3) && (P.kind_mask & 8)) cnt_kind(3, sc3);
    }

    // traceRay body after lighting (raytracer.go:505-561)
    bool have_res = false;
    d3 res = mk(0, 0, 0);
    if (hit) {
      d3 col = mk(M[0], M[1], M[2]);
      double refl = M[3], T = M[7];
      if (refl == 0 && T == 0) {
        res = clamp(mul(L, col));
        have_res = true;
      } else {
        bool hasR = refl > 0;
        Ray rr;
        rr.o = mk(0, 0, 0);
        rr.d = mk(0, 0, 1);
        if (hasR) {
          d3 rd = sub(ray.d, scale(nw, 2.0 * dot(ray.d, nw)));
          if (M[6] != 0.0) rd = add(rd, mk(M[4], M[5], 0.0));
          rr.o = sorig;  // (= add(pw, scale(nw, 1e-4)), raytracer.go:526)
          rr.d = norm(rd);
        }
        bool tmode = T > 0;
        bool hasT = false;
        Ray trr;
        trr.o = mk(0, 0, 0);
        trr.d = mk(0, 0, 1);
        double kr = 0.0;
        d3 lw = L;
        if (tmode) {
          // n1 / n2: 1 / ior from outside (M[12]), ior / 1 = ior from inside
          double ratio = M[12];
          d3 nn = nw;
          if (dot(ray.d, nn) > 0.0) {
            ratio = M[8];
            nn = scale(nn, -1.0);
          }
          // refract (raytracer.go:438-450)
          double cosI = -dot(nn, ray.d);
          double sinT2 = ratio * ratio * (1.0 - cosI * cosI);
          if (!(sinT2 > 1.0)) {
            double cosT = gsqrt(1.0 - sinT2);
            d3 td = add(scale(ray.d, ratio), scale(nn, ratio * cosI - cosT));
            if (!iszero(td)) {
              hasT = true;
              trr.o = sub(pw, scale(nn, 1e-4));
              trr.d = td;
            }
          }
          // fresnel (raytracer.go:456-467) on the unflipped normal
          double cosi = dot(ray.d, nw) / (rlen * len(nw));  // (rlen = len(ray.d), above)
          const double r0 = M[13];  // ((1 - ior) / (1 + ior))^2
          double cost = __builtin_fabs(cosi);
          kr = r0 + (1 - r0) * go_pow(1 - cost, 5);
          lw = scale(L, 1.0 - T);
        }
        const int d = P.depth - sp;  // depth of the current ray
        if (d - 1 > 0 && (hasR || hasT)) {
          core_st(sp, 0, lw.x);
          core_st(sp, 1, lw.y);
          core_st(sp, 2, lw.z);
          if (hasR && hasT) {
            st3(ext(sp), 0, trr.o);
            st3(ext(sp), 3, trr.d);
          }
          core_st(sp, 3, kr);
          if (spec_feat(SF_VM) && mat < 0) {  // the VM record is per lane: keep what the combine needs
            double* f = frame_ptr(stk, sp);
            st3(f, FR_COL, col);
            f[FR_REFL * 64] = refl;
          }
          long long packed = ((long long)(mat < 0 ? 0 : mat) << PK_MAT) | (mat < 0 ? FL_VMMAT : 0) |
                             (tmode ? FL_TMODE : 0) | (hasR ? FL_HASR : 0) | (hasT ? FL_HAST : 0);
          core_st(sp, 4, __longlong_as_double(packed));
          sp++;
          ray = hasR ? rr : trr;
          state = S_TRACE;
        } else {
          res = combine(tmode, lw, col, refl, kr, mk(0, 0, 0), mk(0, 0, 0));
          have_res = true;
        }
      }
    }
    PH_MARK(8);
    unwind(have_res, res, false, 0, mk(0, 0, 0), 0.0);
    PH_MARK(9);
  }
  if (RT_PIX_BATCH) flush_pixels();

  if (lane == 0) {
#ifdef RT_PHASE_TIMING
    for (int k = 0; k < N_PHASE; k++) atomicAdd(P.stats + ST_PHASE + k, (unsigned long long)ph_acc[k]);
    atomicAdd(P.stats + ST_BVHDIAG + 0, (unsigned long long)bd_tnodes);
    atomicAdd(P.stats + ST_BVHDIAG + 1, (unsigned long long)bd_snodes);
    atomicAdd(P.stats + ST_BVHDIAG + 2, (unsigned long long)bd_tleaf);
    atomicAdd(P.stats + ST_BVHDIAG + 3, (unsigned long long)bd_sleaf);
    atomicAdd(P.stats + ST_BVHDIAG + 4, (unsigned long long)bd_trays);
    atomicAdd(P.stats + ST_BVHDIAG + 5, (unsigned long long)bd_srays);
    atomicAdd(P.stats + ST_PASSDIAG + 0, (unsigned long long)pd_tr);
    atomicAdd(P.stats + ST_PASSDIAG + 1, (unsigned long long)pd_trl);
    atomicAdd(P.stats + ST_PASSDIAG + 2, (unsigned long long)pd_sh);
    atomicAdd(P.stats + ST_PASSDIAG + 3, (unsigned long long)pd_shl);
    atomicAdd(P.stats + ST_PASSDIAG + 4, (unsigned long long)pd_gen);
    atomicAdd(P.stats + ST_PASSDIAG + 5, (unsigned long long)pd_genl);
    atomicAdd(P.stats + ST_LANEDIAG + 0, (unsigned long long)ld_done);
    atomicAdd(P.stats + ST_LANEDIAG + 1, (unsigned long long)ld_rounds);
    // wave lifetimes (main loop): mean vs max shows the load imbalance. A
    // wave whose end stamp reads below its start (the shader clock stepped
    // back under it: round 5 saw 1.8e19-cycle "lifetimes" in the first launch
    // of a run) is counted in ST_CLOCKSTEP and left out of the mean and max.
    const uint64_t t_end = stamp();
    const bool clock_ok = t_end >= life_t0;
    const uint64_t life = clock_ok ? t_end - life_t0 : 0;
    if (clock_ok) {
      atomicAdd(P.stats + ST_BVHDIAG + 6, (unsigned long long)life);
      atomicMax(P.stats + ST_BVHDIAG + 7, (unsigned long long)life);
    } else {
      atomicAdd(P.stats + ST_CLOCKSTEP, 1ull);
    }
    if (P.wdiag) {
      P.wdiag[(size_t)wslot * 4 + 0] = life;
      P.wdiag[(size_t)wslot * 4 + 1] = nchunk_taken;
      P.wdiag[(size_t)wslot * 4 + 2] = stamp() - last_grab;
    }
#endif
  }
  // Workgroup reduction of the per-lane counters (every wave of the group
  // leaves the main loop, so all reach the barrier).
  // (768 workgroups adding ~8 counters each to one 128-B line at the end of
  // a launch serialised on one L2 channel: ~5 us per launch, C1 45.9 -> 41.2 us)
  __syncthreads();
  unsigned long long* part = P.stats_part + (size_t)blockIdx.x * STATS_PART;
  if (!P.stats_part) {
  } else if (threadIdx.x < RT_NUM_KINDS) {
    unsigned long long sum = 0;
    for (int j = 0; j < WG; j++) sum += kcnt[threadIdx.x * WG + j];
    if (sum) part[ST_STESTS + threadIdx.x] += sum;
  } else if (threadIdx.x < RT_NUM_KINDS + NUNIT) {
    const int k = (int)threadIdx.x - RT_NUM_KINDS;
    unsigned long long sum = 0;
    for (int j = 0; j < WAVES_PER_WG; j++) sum += cnt[k * WAVES_PER_WG + j];
    const int slot = k == CNT_TRACED ? ST_TRACED : (k == CNT_SHADED ? ST_SHADED : ST_SURFERR);
    if (sum) part[slot] += sum;
    // one inShadow call per (shaded hit, light)
    if (k == CNT_SHADED && sum) part[ST_SHADOW] += sum * (unsigned long long)P.nlights;
  }
}

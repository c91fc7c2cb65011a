/*
 * rt_abi.h -- C ABI of the MI355X-native renderer for the ICFP-2000 GML
 * raytracer (drop-in for the per-pixel Render() hot path of
 * timdestan/go-raytracer).
 *
 * What this replaces (reference file:line, relative to the reference repo):
 *   - raytracer.go:589-682   func Render(scene *Scene) image.Image
 *   - raytracer.go:724-830   ConvertRenderArgsToScene / convertGMLSceneObjects
 *                            (matrix inverse, normal matrices, plane D and
 *                            NormalWorld, cube face expansion) -- done inside
 *                            the library from the flattened object list below
 *   - raytracer.go:38-370    the SceneObject plug-in (Sphere/Plane/Cube/Cylinder
 *                            Intersect + ComputeSurfaceProps)
 *   - raytracer.go:372-562   computeLighting / inShadow / refract / fresnel /
 *                            closestHit / traceRay
 * The GML interpreter (internal/gml) stays on the host: it produces
 * gml.RenderArgs (evaluator.go:14-28); the host flattens RenderArgs.Scene in
 * the same BFS order as raytracer.go:776-828 and bakes each object's surface
 * into per-face constant materials (gml.Material, evaluator.go:136-150).
 *
 * Conventions: plain C, no exceptions cross this boundary; every entry point
 * returns RT_OK (0) or a negative RT_E* code, and rt_last_error() gives a
 * thread-local message. The output framebuffer has the exact layout of Go's
 * image.RGBA.Pix (row-major RGBA8, stride 4*width, alpha 255), so a cgo shim
 * can wrap it without copying.
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#ifndef __HIPCC_RTC__ /* hipRTC (scene specialisation) provides size_t itself */
#include <stddef.h>
#endif
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 6
#define RT_MAX_DEVICES 16 /* devices one rt_render_ex call may use */
#define RT_EXP_AMD64_FMA 0
#define RT_EXP_AMD64 1
#define RT_EXP_PORTABLE 2

/* Status codes. */
#define RT_OK 0
#define RT_E_INVALID (-1)   /* bad argument / malformed scene             */
#define RT_E_SINGULAR (-2)  /* transform has det == 0 (prim/vec.go:343)   */
#define RT_E_DEVICE (-3)    /* HIP runtime error                          */
#define RT_E_NOMEM (-4)     /* device allocation failed                   */

/* Primitive kinds (the concrete SceneObject types, raytracer.go:43-277). */
#define RT_SPHERE 0
#define RT_PLANE 1
#define RT_CUBE 2
#define RT_CYLINDER 3
/* Contest extension (ICFP 2000 GML `cone`; not in the reference renderer, so
 * parity-unpinned): apex at the origin, x^2 + z^2 = y^2 for 0 <= y <= 1,
 * base disk at y = 1. Faces 0 side, 1 base. */
#define RT_CONE 4
/* Contest extension (GML `intersect` / `difference`; the reference renderer
 * rejects Difference, raytracer.go:825-826): one composite solid. Its leaves
 * are rt_scene.csg_leaves[csg_first .. csg_first + csg_count) (spheres, cubes,
 * cylinders, planes as half-spaces n.p + D <= 0) combined by a postfix program
 * rt_scene.csg_code[csg_code .. csg_code + csg_code_len): v >= 0 pushes leaf v
 * (relative to csg_first), RT_CSG_UNION / _INTERSECT / _DIFFERENCE pop two.
 * The hit is the first interval end point t > 0 at which the composite's
 * membership changes (oracle/rt_oracle.c csg_intersect). */
#define RT_CSG 5
#define RT_NUM_KINDS 6
#define RT_CSG_UNION (-1)
#define RT_CSG_INTERSECT (-2)
#define RT_CSG_DIFFERENCE (-3)
#define RT_CSG_MAX_LEAVES 128

#define RT_MAX_FACES 6 /* prim.NUM_CUBE_SIDES, internal/prim/plane.go:27 */

/* gml.Material (internal/gml/evaluator.go:136-150), field for field. */
typedef struct rt_material {
    double color[3];
    double reflectivity;
    double fuzziness;
    double transparency;
    double refractive_index;
    double kd;
    double ks;
    double specular_exponent;
} rt_material;

/* gml.PointLight (internal/gml/evaluator.go:289-292). */
typedef struct rt_point_light {
    double position[3];
    double color[3];
} rt_point_light;

/* Lights of the contest extensions (GML `light`, `spotlight`; not in the
 * reference renderer, parity-unpinned). Point lights here behave exactly like
 * rt_point_light. Directional: direction = the way the light travels; the
 * shading vector is normalize(-direction) and shadow rays are unbounded.
 * Spot: at position, aimed at `direction` (a point), cutoff half-angle in
 * degrees, intensity colour * Pow(cos(angle), exponent) inside the cone and 0
 * outside (shadow rays are traced either way, one per light). No distance
 * attenuation, matching the reference's point lights. */
#define RT_LIGHT_POINT 0
#define RT_LIGHT_DIRECTIONAL 1
#define RT_LIGHT_SPOT 2
typedef struct rt_light {
    int32_t kind;
    int32_t reserved;
    double position[3];
    double direction[3]; /* directional: direction; spot: the point aimed at */
    double color[3];
    double cutoff;       /* spot: degrees */
    double exponent;     /* spot */
} rt_light;

/* One flattened scene object (a leaf of gml.RenderArgs.Scene after the BFS
 * union flattening of raytracer.go:776-828).
 *   transform      gml.<Kind>.TransformMat, row-major prim.Mat4
 *                  (object -> world); ignored when has_transform == 0 (nil
 *                  TransformMat => identity, raytracer.go:757-762).
 *   material[f]    index into rt_scene.materials for face f (the value
 *                  EvalSurfaceFn returns for that face; constant surfaces use
 *                  the same index for every face). Faces: sphere/plane 0;
 *                  cylinder 0 side, 1 top, 2 bottom (raytracer.go:263-267);
 *                  cube 0..5 = prim.CubeSide (internal/prim/plane.go:14-25).
 *   plane_point,
 *   plane_normal   RT_PLANE only: gml.Plane.Plane (evaluator.go:813-821 builds
 *                  point (0,0,0), normal (0,1,0)). */
/* Closure surfaces (GML surface functions that depend on face/u/v) run on the
 * device as straight-line register programs compiled by the host
 * (go-raytracer_amd/gml/surface_compiler.py). A face whose material index is
 * negative uses program (-material[f] - 1): it receives face (i64), u, v (f64)
 * as computed by the reference's ComputeSurfaceProps (raytracer.go:124-150,
 * 196-205, 339-359) and yields the 10 gml.Material fields, exactly what
 * EvalSurfaceFn (evaluator.go:672-727) returns for that hit. */
/* Surface-program bytecode: the contract a host compiles a GML surface
 * closure to (go-raytracer_amd/gml/surface_compiler.py is one compiler; a Go
 * or C host may emit the same words; tests/c/abi_render.c hand-assembles one).
 * Instruction = 2 x uint32: w0 = op | dst << 8 | a << 16 | b << 24, w1 = c.
 * 64 registers of 64 bits per lane (f64 bits, wrapping i64, or bool 0/1).
 * Entry: r10 = face (i64), r11 = u (f64), r12 = v (f64), as the reference's
 * ComputeSurfaceProps passes them. RET: r0..r9 = the gml.Material fields in
 * rt_material order (colour r g b, reflectivity, fuzziness, transparency,
 * refractive index, kd, ks, n), i.e. what EvalSurfaceFn returns
 * (evaluator.go:672-727; for `color kd ks n` results Reflectivity = ks and
 * fuzziness / transparency / refractive index are 0). Go semantics: one
 * rounding per f64 op, no fusion. The library validates every program at
 * rt_set_scene (opcodes, register / constant / table ranges, a reachable
 * RET within 8192 steps). */
#define RT_VM_NOP 0
#define RT_VM_CONST 1  /* r[d] = consts[c] (64-bit pattern) */
#define RT_VM_MOV 2    /* r[d] = r[a] */
#define RT_VM_ADDF 3   /* r[d] = r[a] + r[b] (f64); SUBF, MULF, DIVF likewise */
#define RT_VM_SUBF 4
#define RT_VM_MULF 5
#define RT_VM_DIVF 6
#define RT_VM_NEGF 7   /* r[d] = -r[a] */
#define RT_VM_ADDI 8   /* wrapping i64 */
#define RT_VM_SUBI 9
#define RT_VM_MULI 10
#define RT_VM_DIVI 11  /* truncating; x / 0 yields 0 (guard with ERR); MinInt64 / -1 wraps */
#define RT_VM_MODI 12  /* truncating remainder; x % 0 and x % -1 yield 0 */
#define RT_VM_NEGI 13
#define RT_VM_LTF 14   /* bool r[a] < r[b] (f64) */
#define RT_VM_EQF 15
#define RT_VM_LTI 16   /* i64 */
#define RT_VM_EQI 17
#define RT_VM_SEL 18   /* r[d] = r[a] ? r[b] : r[c & 63] */
#define RT_VM_FLOOR 19 /* i64 of floor(x) (amd64 float64 -> int64 conversion) */
#define RT_VM_FRAC 20  /* x - float64(int64(x)) */
#define RT_VM_SQRT 21
#define RT_VM_SIN 22   /* Go math.Sin(0.017453292519943295 * x), one product (evaluator.go:932 DegToRad): GML angles are degrees */
#define RT_VM_COS 23   /* Go math.Cos(0.017453292519943295 * x) */
#define RT_VM_CLAMPF 24 /* f64 clamped to [0, 1] */
#define RT_VM_CLAMPI 25 /* i64 clamped to [0, 1] */
#define RT_VM_TBL 26   /* r[d] = consts[c + 1 + clamp(r[a], 0, n - 1)], n = consts[c] (guard with ERR) */
#define RT_VM_AND 27   /* bool */
#define RT_VM_OR 28
#define RT_VM_NOT 29
#define RT_VM_ERR 30   /* the evaluation fails (counted in surface_errors) if r[a] != 0 */
#define RT_VM_RET 31
#define RT_VM_INSN(op, d, a, b) ((uint32_t)(op) | ((uint32_t)(d) << 8) | ((uint32_t)(a) << 16) | ((uint32_t)(b) << 24))

typedef struct rt_object {
    int32_t kind;
    int32_t has_transform;
    int32_t material[RT_MAX_FACES];
    double transform[16];
    double plane_point[3];
    double plane_normal[3];
    /* RT_CSG only (see RT_CSG) */
    int32_t csg_first, csg_count, csg_code, csg_code_len;
} rt_object;

/* gml.RenderArgs (internal/gml/evaluator.go:14-28) with the scene already
 * flattened. depth <= 0 => 3 and fov <= 0 => 90 are applied by the library
 * exactly as raytracer.go:592-600 does. */
typedef struct rt_scene {
    int32_t width;
    int32_t height;
    int32_t depth;
    int32_t num_lights;
    double fov;          /* degrees */
    double ambient[3];
    double bg_start[3];  /* BgColorStart (zero when plain `render`) */
    double bg_end[3];    /* BgColorEnd */
    const rt_point_light *lights;
    const rt_object *objects;
    const rt_material *materials;
    int32_t num_objects;
    int32_t num_materials;
    /* surface programs (may be empty): instruction words of all programs,
     * each 2 x uint32 (w0 = op | dst<<8 | a<<16 | b<<24, w1 = c); entry word
     * offset per program; one shared constant pool of 64-bit patterns. */
    const uint32_t *program_code;
    const uint64_t *program_consts;
    const int32_t *program_entry;
    int32_t num_programs;
    int32_t program_code_words;
    int32_t program_const_count;
    /* ABI 3: which math.Exp / math.Log a fractional math.Pow exponent
     * (raytracer.go:395 specular n, spot exponents) runs -- Go dispatches them
     * per platform: RT_EXP_AMD64_FMA (0, default) exp_amd64.s with FMA, what
     * the reference runs on an x86-64 CPU with AVX2+FMA; RT_EXP_AMD64 (1) the
     * same without FMA; RT_EXP_PORTABLE (2) exp.go / log.go (platforms with
     * no assembly Exp). Integer exponents never reach Exp. */
    int32_t exp_mode;
    /* ABI 2: when num_ext_lights > 0 these are the scene's lights, in program
     * order, and lights / num_lights are ignored. */
    const rt_light *ext_lights;
    int32_t num_ext_lights;
    int32_t reserved1;
    /* ABI 2: CSG composites (RT_CSG objects) */
    const rt_object *csg_leaves;
    const int32_t *csg_code;
    int32_t num_csg_leaves;
    int32_t csg_code_words;
} rt_scene;

/* Work counters, identical in the CPU oracle and the GPU path.
 *   primary_rays     top-level traceRay calls (4 per pixel, raytracer.go:639)
 *   secondary_rays   recursive traceRay calls entered with depth > 0
 *                    (raytracer.go:528,554; depth 0 returns at :488-491)
 *   shadow_rays      inShadow calls: one per (shaded hit, light)
 *                    (raytracer.go:383)
 *   tests[k]         Intersect calls on kind k made by closestHit
 *   shadow_tests[k]  Intersect calls on kind k made by inShadow (early exit)
 *   shaded_hits      ComputeSurfaceProps + computeLighting evaluations
 *   surface_errors   closure-surface evaluations that raised an error */
typedef struct rt_stats {
    uint64_t primary_rays;
    uint64_t secondary_rays;
    uint64_t shadow_rays;
    uint64_t tests[RT_NUM_KINDS];
    uint64_t shadow_tests[RT_NUM_KINDS];
    uint64_t shaded_hits;
    uint64_t surface_errors; /* hits whose surface evaluation failed; the
                              * reference panics on the first one
                              * (raytracer.go:499-501) */
    double kernel_ms;    /* device time of the last render (GPU path; with
                          * several devices the slowest device's span)    */
    /* ABI 6: the devices of the last frame (rt_render / rt_render_ex; 1 for
     * rt_read_stats) and, per device in rt_render_opts order, the GPU span of
     * its share of the frame; gather_ms = host wall time from the moment every
     * device's share had rendered to the frame complete in the caller's
     * buffer (the gather and copy work the renders did not hide). */
    int32_t devices;
    int32_t reserved2;
    double device_kernel_ms[RT_MAX_DEVICES];
    double gather_ms;
} rt_stats;

/* Opaque per-device context: owns the converted scene on the device, the
 * work-queue counters and the stats buffer. Re-usable across renders (the
 * reference REPL renders many times per process, cmd/gml/main.go:104-115). */
typedef struct rt_context rt_context;

/* ABI version of the loaded library (RT_ABI_VERSION). */
int rt_abi_version(void);

/* Thread-local description of the last failure on this thread. */
const char *rt_last_error(void);

/* Create a context on HIP device `device` (the caller's current device when
 * device < 0). */
int rt_create(int device, rt_context **out);
void rt_destroy(rt_context *ctx);

/* Convert the flattened scene exactly as ConvertRenderArgsToScene
 * (raytracer.go:724-830) and upload it to the context's device. The scene is
 * read only during the call. Replaces any previous scene. */
int rt_set_scene(rt_context *ctx, const rt_scene *scene);

/* Enqueue the render of image rows [y0, y1) on `stream` (a hipStream_t; NULL
 * = the null stream) into device memory `d_rgba` (row y0 first, stride
 * 4*width bytes). Asynchronous; device pointers only. The per-row pixels are
 * identical to rows y0..y1-1 of a full-frame Render(): RNG state depends only
 * on (x, 20-row strip) (raytracer.go:627-634). Launches on one context run in
 * submission order: a launch on another stream than the previous launch
 * waits for that launch to end. */
int rt_render_rows_async(rt_context *ctx, int y0, int y1, void *d_rgba,
                         void *stream);

/* Interleaved variant for load-balanced multi-GPU sharding: render `ntrows`
 * 8-row tile rows, output tile row j being image rows
 * [(trow0 + j*trow_stride)*8, +8) clipped to the image, into d_rgba packed
 * contiguously (output row j*8 + r, stride 4*width; rows past the image are
 * left untouched). Same pixels as a full-frame render. */
int rt_render_tile_rows_async(rt_context *ctx, int trow0, int trow_stride, int ntrows,
                              void *d_rgba, void *stream);

/* Read (and optionally reset) the work counters accumulated on the device
 * since the last reset. Synchronises the given stream. If the render
 * watchdog stopped a wave (a kernel bug: a frame left unfinished) it returns
 * RT_E_DEVICE and resets the counters whatever `reset` says. */
int rt_read_stats(rt_context *ctx, void *stream, int reset, rt_stats *out);

/* Device time (ms) of the most recent rt_render_rows_async on this context,
 * measured with HIP events on the stream it was launched on. Synchronises. */
int rt_last_kernel_ms(rt_context *ctx, double *ms_out);

/* Scene specialisation (MI355X-specific, no reference counterpart). With
 * enable != 0 the context compiles, through hipRTC, a variant of the render
 * kernel with the current and every later scene's object count and primitive
 * kinds as compile-time constants, when the scene is small and linear (at most
 * 8 objects, no BVH, no CSG, scene resident in LDS); other scenes keep the
 * generic kernel. Output is bit-identical either way; the one-off compile
 * (seconds, cached per process) pays off for scenes rendered many times.
 * Returns RT_E_DEVICE with the compiler log if hipRTC is unavailable or fails.
 * Takes effect immediately for the current scene and in every rt_set_scene. */
int rt_set_specialize(rt_context *ctx, int enable);

/* Acceleration of the exact search (MI355X-specific; pixels and counters are
 * identical either way): RT_ACCEL_BVH builds a BVH over the bounded objects of
 * scenes with >= 12 of them (takes effect at the next rt_set_scene);
 * RT_ACCEL_CULL lets the kernel skip Intersect calls an FP32 bound proves to
 * miss (specialised kernels only; the generic kernel always culls). Default:
 * both. 0 runs the reference's brute-force search -- every ray tests every
 * object in FP64 -- e.g. to measure the FP64 roofline of the Intersect loop. */
#define RT_ACCEL_BVH 1
#define RT_ACCEL_CULL 2
int rt_set_accel(rt_context *ctx, int flags);

/* How pixels are dealt to the device lanes (MI355X-specific; pixels and
 * counters are identical in every mode). RT_SCHED_PIXEL: a lane renders a
 * pixel's 4 samples one after another (raytracer.go:645-651), 64 pixels per
 * dequeue. RT_SCHED_QUADS: a pixel's 4 samples run at once in 4 adjacent
 * lanes whose first lane adds them in sample order, 16 pixels per dequeue --
 * 4x shorter per-pixel latency, so deep branching glass trees do not leave a
 * few waves running long after the rest. RT_SCHED_AUTO (default): quads for
 * depth >= 7, and for launches that give each lane few pixels (a
 * strong-scaling share of a frame). Takes effect at the next launch (the
 * specialised kernel of the other schedule is compiled on first use). */
#define RT_SCHED_AUTO 0
#define RT_SCHED_PIXEL 1
#define RT_SCHED_QUADS 2
/* RT_SCHED_PAIRS: a pixel's samples 0-1 in one lane and 2-3 in the next, the
 * first lane adding all four in sample order -- half the quads' per-pixel
 * parallelism at half their idle-lane cost (specialised kernels,
 * rt_set_specialize; the generic kernels run quads for it). */
#define RT_SCHED_PAIRS 3
int rt_set_schedule(rt_context *ctx, int mode);

/* Frames in flight (MI355X-specific; pixels and counters are identical): a
 * host rendering a stream of frames keeps n >= 2 contexts with the same scene
 * and alternates its launches over them, one stream each, so one frame's
 * last waves share the chip with the next frame's first.
 * Telling each context n lets RT_SCHED_AUTO trade per-pixel latency for
 * fewer idle lanes where the overlap hides the longer tail (scenes in LDS
 * without CSG): serial samples instead of quads for launches of >= 32 pixels
 * per lane at depth >= 7, and with the specialised kernel pixel pairs for
 * branching scenes at 8-16 pixels per lane (depth < 7) or >= 16 (depth >= 7). Default 1. Takes effect at once. No reference
 * counterpart (Render is one synchronous frame, raytracer.go:589). */
int rt_set_frames_in_flight(rt_context *ctx, int n);

/* Tile order (MI355X-specific; pixels and counters are identical either
 * way). With enable != 0 (default) rt_set_scene also traces sample 0 of four
 * pixels per 8x8 tile of the frame at full depth and counts its rays (none of
 * them reach rt_read_stats); every launch then deals the costliest quarter of
 * its tiles first, in cost order, and the rest in tile order, so the deep
 * glass trees start early instead of keeping a few waves running after the
 * rest, while most tiles keep their neighbours' locality. Scenes staged in
 * LDS only: a scene read from HBM (a large BVH) loses more cache locality
 * than it gains. Applies to the current scene at once; rt_tile_order_info
 * reports whether an order is active and the estimate's wall time. */
int rt_set_tile_order(rt_context *ctx, int enable);
/* Work sharing at the tail of a launch (MI355X-specific; pixels and counters
 * are identical either way; default RT_SHARE_AUTO, below). With enable =
 * RT_SHARE_GROUP the context's
 * specialised kernel (rt_set_specialize) is compiled with a per-workgroup
 * board in LDS: once the work queue is drained, a lane still tracing a pixel
 * posts the samples it has not started and the pending refraction children
 * of its binary (reflect + refract, raytracer.go:512-556) frames, idle lanes
 * of any wave of the group trace them, and the owner joins their colours in
 * the reference's order. RT_SHARE_AUTO (the default, below) never picks this
 * workgroup board: its code costs every round of the kernel more than the
 * tail gains on the BASELINE configs. Applies to the current
 * scene at once. */
#define RT_SHARE_OFF 0
#define RT_SHARE_GROUP 1
/* RT_SHARE_DEVICE (ABI 5): the board is device-wide, in uncached HBM -- an
 * idle lane of any drained wave on the device (any workgroup, any XCD) takes
 * a posted refraction subtree; a few drained waves stay to help until no wave
 * of the launch is busy. Subtrees only (no sample posting).
 * RT_SHARE_AUTO (ABI 5, the default): RT_SHARE_DEVICE for scenes with CSG
 * composites at depth >= 7 on launches of fewer than 16 pixels per lane (a
 * strong-scaling share) or without frames in flight, else off. */
#define RT_SHARE_DEVICE 2
#define RT_SHARE_AUTO 3
int rt_set_work_sharing(rt_context *ctx, int enable);
/* Whether the current scene has a tile order, and the estimate's wall time
 * (ms) at scene setup. */
int rt_tile_order_info(rt_context *ctx, int *active, double *estimate_ms);

/* How the current scene is laid out for the device (bit flags), e.g. for
 * tests that must exercise one kernel flavour: RT_INFO_LDS the scene blob is
 * staged in LDS per workgroup; RT_INFO_BVH a BVH over the bounded objects;
 * RT_INFO_CSG CSG composites; RT_INFO_STREAM a large linear scene whose
 * object records are read from global memory in index order (per-wave LDS
 * chunks, or scalar loads in the brute-force kernel); RT_INFO_WAVEFRONT the
 * scene's kernel shares work across the lanes and waves of a workgroup at
 * the tail of a launch (rt_set_work_sharing); RT_INFO_ORDERED launches deal
 * tiles most expensive first (rt_set_tile_order). */
#define RT_INFO_LDS 1
#define RT_INFO_BVH 2
#define RT_INFO_CSG 4
#define RT_INFO_STREAM 8
#define RT_INFO_WAVEFRONT 16
#define RT_INFO_ORDERED 32
#define RT_INFO_SHARE_DEVICE 64 /* the work-sharing board is device-wide (RT_SHARE_DEVICE) */
int rt_scene_info(rt_context *ctx, int *flags);

/* Whether the current scene runs a specialised kernel, and the compile time
 * (ms) that preparing it cost (0 on a cache hit). Either pointer may be NULL. */
int rt_specialized(rt_context *ctx, int *active, double *compile_ms);

/* Compile (no device needed) and cache, for this process, the specialised
 * kernel for a scene of nobj (1..8) objects of the given kinds in object
 * order and the given RT_SPEC_* feature bits, e.g. to move the compile out of
 * a latency-critical rt_set_scene. */
#define RT_SPEC_SURFACES 1    /* the scene has closure (surface program) materials */
#define RT_SPEC_DIRECTIONAL 2 /* ... directional lights */
#define RT_SPEC_SPOT 4        /* ... spot lights */
#define RT_SPEC_LIGHTS(n) ((n) << 8) /* ... exactly n (1..8) lights, as every scene with 1..8
                                        lights is specialised (0: the generic light loop) */
int rt_spec_precompile(int nobj, const int *kinds, int features, double *compile_ms);

/* Diagnostic (tests, no device): compile the specialised variant named by
 * the library's internal key "lds:bvh:csg:nobj:kinds:kmask:feat:nlights:
 * pow_bits:nocull:schedule:share:far" (schedule 0 serial, 1 quads, 2 pairs;
 * share an RT_SHARE_* mode) exactly as a launch would ask for it. Every
 * compile runs in the helper process csrc/rt_spec_cc (RT_SPEC_INPROC=1: in
 * this process), so a compiler abort is a failed compile, not a dead caller. */
int rt_debug_spec_compile(const char *key, double *compile_ms);

/* Diagnostic (tests, no device): the value of environment variable `name` as
 * the library sees it -- its copy of the process environment taken when the
 * library was loaded (every RT_* knob, the compile helper's environment and
 * the in-process compiler's come from it; changes made after loading are not
 * seen) -- or NULL. The string lives as long as the process. */
const char *rt_debug_getenv(const char *name);

/* Diagnostic (tests): run surface program `program` of the context's scene on
 * n (face, u, v) inputs on the device; out10 receives n x 10 Material fields
 * (rt_material order), err n flags (1 = the reference would raise). */
int rt_debug_run_surface(rt_context *ctx, int program, int n, const long long *face,
                         const double *u, const double *v, double *out10, int *err);

/* SSIM of two RGBA8 frames in device memory (width x height, stride 4W), the
 * reference's parity metric prim.SSIM (internal/prim/ssim.go:27-182; used by
 * raytracer_test.go:42 with threshold 0.99). Synchronous on `stream`.
 * RT_E_INVALID "images are too small" below 11x11; NaN at exactly 11 wide or
 * high (no window visited, as in the reference). */
int rt_ssim_rgba8(rt_context *ctx, const uint8_t *d_a, const uint8_t *d_b, int width, int height,
                  double *out_ssim, void *stream);

/* Synchronous whole-frame Render() into host memory (width*height*4 bytes,
 * caller-owned, e.g. Go's image.RGBA.Pix): the replacement of
 * func Render(*Scene) image.Image (raytracer.go:589-682), called from the
 * EvalState.Render hook (evaluator.go:48). Same as rt_render_ex(scene, NULL,
 * rgba_out, stats): the caller's current HIP device. */
int rt_render(const rt_scene *scene, uint8_t *rgba_out, rt_stats *stats);

/* ABI 6: Render() over one or several GPUs of this process.
 *
 * Devices (first match): device_mask != 0 -> the devices whose bit is set, in
 * ascending order; else device_count > 0 with RT_RENDER_DEVICE_LIST in flags
 * -> devices[0 .. device_count) (an ordinal may repeat: the same GPU then
 * renders several shares at once, each with its own contexts, which exercises
 * the multi-device path on one GPU); else device_count > 0 -> devices
 * 0 .. device_count-1; else the caller's current device. opts may be NULL.
 *
 * Partition: the frame's 8-row tile rows are dealt
 * round-robin, tile row t to device t mod N, so every device gets the same
 * mix of sky, floor and glass; pixels and counters are those of a one-device
 * frame (RNG state depends only on (x, 20-row strip), raytracer.go:627-634).
 * Each device renders its share into its own HBM, densely packed, as row
 * bands alternating over two contexts and streams.
 *
 * Gather (the `gather` field):
 *   RT_GATHER_HOST  each device DMAs each finished band of its share straight
 *                   to the band's final rows of a pinned frame, over its own
 *                   PCIe link, and the host copies finished bands on to
 *                   rgba_out while later bands render (N links in parallel);
 *   RT_GATHER_PEER  every share is copied to the first device over xGMI
 *                   (hipMemcpyPeerAsync, peer access enabled where the
 *                   devices allow it) and de-interleaved there into one
 *                   frame, which one DMA brings to the host -- or, with
 *                   RT_RENDER_OUT_DEVICE, which IS rgba_out;
 *   RT_GATHER_AUTO  (0) HOST for host output, PEER with RT_RENDER_OUT_DEVICE.
 * flags: RT_RENDER_OUT_DEVICE -- rgba_out is device memory of the first
 * device (H x 4W bytes); RT_RENDER_GENERIC -- the ahead-of-time kernel only
 * (no hipRTC); RT_RENDER_SPEC_SYNC -- a new scene shape waits for its
 * specialised kernel instead of rendering with the generic one meanwhile.
 * bands: row bands per device (0: one per ~2 M pixels of the share, <= 4;
 * RT_RENDER_BANDS in the environment overrides the automatic count). Bands
 * decrease in size (weights n, n-1, ..., 1; RT_RENDER_BAND_SHAPE=0: equal), so
 * the exposed copy after the last band is the smallest band's. Environment
 * knobs are read from the library's load-time copy of the environment.
 *
 * Kept per device between calls: two contexts with the last scene (an
 * unchanged scene -- byte-equal arrays -- is not converted, uploaded or
 * estimated again; a changed one is converted once and cloned to every
 * context), the share buffer, streams and events; one pinned frame. Scene
 * specialisation: a call never waits for hipRTC unless RT_RENDER_SPEC_SYNC --
 * a new shape renders with the generic kernel (same pixels and counters)
 * while its specialised kernel compiles on a background thread, and later
 * calls switch to it (rt_render_timing.specialized / .pending_compiles);
 * a failed compile is logged once and the generic kernel stays;
 * RT_RENDER_SPECIALIZE=0 in the environment keeps the generic kernel.
 * stats may be NULL: the counters summed over every device and context;
 * kernel_ms = the slowest device's GPU span; devices, device_kernel_ms[],
 * gather_ms as documented at rt_stats. Synchronous; calls are serialised. */
#define RT_GATHER_AUTO 0
#define RT_GATHER_HOST 1
#define RT_GATHER_PEER 2
#define RT_RENDER_DEVICE_LIST 1
#define RT_RENDER_OUT_DEVICE 2
#define RT_RENDER_GENERIC 4
#define RT_RENDER_SPEC_SYNC 8
typedef struct rt_render_opts {
    int32_t device_count;
    uint32_t device_mask;
    int32_t devices[RT_MAX_DEVICES];
    int32_t gather;     /* RT_GATHER_* */
    int32_t flags;      /* RT_RENDER_* */
    int32_t bands;      /* row bands per device, 0 = automatic */
    int32_t reserved[5];
} rt_render_opts;
int rt_render_ex(const rt_scene *scene, const rt_render_opts *opts, uint8_t *rgba_out, rt_stats *stats);

/* Diagnostic (tests, no device): the host side of the multi-device assembly
 * rt_render_ex runs, on host buffers. shares[d] holds device d's share as
 * rt_render_ex renders it (its tile rows d, d+N, ... of an N-device frame,
 * packed, stride 4*width, the last tile row clipped to the image); the frame
 * is assembled into out with exactly the copy plan -- bands, strided DMA
 * segments, row clipping -- the device path uses, for `bands` bands per
 * device (0 = automatic). */
int rt_debug_assemble(int width, int height, int ndev, int bands, const uint8_t *const *shares, uint8_t *out);

/* ABI 5: the parts of the calling thread's last rt_render call, on one host
 * timeline (setup + render_wait + copy_tail = total):
 *   setup_ms        scene compare (and, if it changed, conversion, upload,
 *                   specialisation, tile-cost estimate) and the launches
 *   render_wait_ms  until the frame's last band has rendered (the earlier
 *                   bands' host copies run inside it)
 *   copy_tail_ms    the last band's DMA and host copy, and the counters
 *   gpu_ms          GPU span of the frame (first band's start to last end)
 * bands: row bands the frame was rendered in (over all devices);
 * scene_reused: the scene was unchanged; specialized: every launch of the
 * call ran a specialised kernel. ABI 6: devices of the call; pending_compiles:
 * specialised kernels still compiling in the background when the call ended
 * (the call itself rendered with the generic kernel where they were missing). */
typedef struct rt_render_timing {
    double total_ms;
    double setup_ms;
    double render_wait_ms;
    double copy_tail_ms;
    double gpu_ms;
    int32_t bands;
    int32_t scene_reused;
    int32_t specialized;
    int32_t devices;
    int32_t pending_compiles;
    int32_t reserved;
} rt_render_timing;
int rt_render_last_timing(rt_render_timing *out);

#ifdef __cplusplus
}
#endif

#endif /* RT_ABI_H */

"""ctypes mirror of include/rt_abi.h (the C ABI of the renderer).

Struct layouts must match include/rt_abi.h exactly; tests/test_abi.py checks
sizes and offsets against the compiled library's expectations.
"""
import ctypes as C

RT_ABI_VERSION = 6  # include/rt_abi.h
RT_MAX_DEVICES = 16
RT_EXP_AMD64_FMA, RT_EXP_AMD64, RT_EXP_PORTABLE = 0, 1, 2  # rt_scene.exp_mode

RT_OK = 0
RT_E_INVALID = -1
RT_E_SINGULAR = -2
RT_E_DEVICE = -3
RT_E_NOMEM = -4

RT_SPHERE, RT_PLANE, RT_CUBE, RT_CYLINDER, RT_CONE, RT_CSG = 0, 1, 2, 3, 4, 5
RT_NUM_KINDS = 6
RT_MAX_FACES = 6
KIND_NAMES = ("sphere", "plane", "cube", "cylinder", "cone", "csg")
RT_CSG_UNION, RT_CSG_INTERSECT, RT_CSG_DIFFERENCE = -1, -2, -3
RT_CSG_MAX_LEAVES = 128
RT_SPEC_SURFACES, RT_SPEC_DIRECTIONAL, RT_SPEC_SPOT = 1, 2, 4  # rt_spec_precompile feature bits
RT_ACCEL_BVH, RT_ACCEL_CULL = 1, 2  # rt_set_accel flags
RT_SCHED_AUTO, RT_SCHED_PIXEL, RT_SCHED_QUADS, RT_SCHED_PAIRS = 0, 1, 2, 3  # rt_set_schedule modes
RT_INFO_LDS, RT_INFO_BVH, RT_INFO_CSG, RT_INFO_STREAM, RT_INFO_WAVEFRONT, RT_INFO_ORDERED = 1, 2, 4, 8, 16, 32  # rt_scene_info
RT_INFO_SHARE_DEVICE = 64
RT_SHARE_OFF, RT_SHARE_GROUP, RT_SHARE_DEVICE, RT_SHARE_AUTO = 0, 1, 2, 3  # rt_set_work_sharing
RT_GATHER_AUTO, RT_GATHER_HOST, RT_GATHER_PEER = 0, 1, 2  # rt_render_opts.gather
RT_RENDER_DEVICE_LIST, RT_RENDER_OUT_DEVICE, RT_RENDER_GENERIC, RT_RENDER_SPEC_SYNC = 1, 2, 4, 8  # rt_render_opts.flags


def RT_SPEC_LIGHTS(n):
    """rt_spec_precompile feature bits for exactly n (1..8) lights (include/rt_abi.h)."""
    return int(n) << 8
RT_LIGHT_POINT, RT_LIGHT_DIRECTIONAL, RT_LIGHT_SPOT = 0, 1, 2


class rt_material(C.Structure):
    _fields_ = [
        ("color", C.c_double * 3),
        ("reflectivity", C.c_double),
        ("fuzziness", C.c_double),
        ("transparency", C.c_double),
        ("refractive_index", C.c_double),
        ("kd", C.c_double),
        ("ks", C.c_double),
        ("specular_exponent", C.c_double),
    ]


class rt_point_light(C.Structure):
    _fields_ = [("position", C.c_double * 3), ("color", C.c_double * 3)]


class rt_light(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("reserved", C.c_int32),
        ("position", C.c_double * 3),
        ("direction", C.c_double * 3),
        ("color", C.c_double * 3),
        ("cutoff", C.c_double),
        ("exponent", C.c_double),
    ]


class rt_object(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("has_transform", C.c_int32),
        ("material", C.c_int32 * RT_MAX_FACES),
        ("transform", C.c_double * 16),
        ("plane_point", C.c_double * 3),
        ("plane_normal", C.c_double * 3),
        ("csg_first", C.c_int32),
        ("csg_count", C.c_int32),
        ("csg_code", C.c_int32),
        ("csg_code_len", C.c_int32),
    ]


class rt_scene(C.Structure):
    _fields_ = [
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("depth", C.c_int32),
        ("num_lights", C.c_int32),
        ("fov", C.c_double),
        ("ambient", C.c_double * 3),
        ("bg_start", C.c_double * 3),
        ("bg_end", C.c_double * 3),
        ("lights", C.POINTER(rt_point_light)),
        ("objects", C.POINTER(rt_object)),
        ("materials", C.POINTER(rt_material)),
        ("num_objects", C.c_int32),
        ("num_materials", C.c_int32),
        ("program_code", C.POINTER(C.c_uint32)),
        ("program_consts", C.POINTER(C.c_uint64)),
        ("program_entry", C.POINTER(C.c_int32)),
        ("num_programs", C.c_int32),
        ("program_code_words", C.c_int32),
        ("program_const_count", C.c_int32),
        ("exp_mode", C.c_int32),  # RT_EXP_*
        ("ext_lights", C.POINTER(rt_light)),
        ("num_ext_lights", C.c_int32),
        ("reserved1", C.c_int32),
        ("csg_leaves", C.POINTER(rt_object)),
        ("csg_code", C.POINTER(C.c_int32)),
        ("num_csg_leaves", C.c_int32),
        ("csg_code_words", C.c_int32),
    ]


class rt_stats(C.Structure):
    _fields_ = [
        ("primary_rays", C.c_uint64),
        ("secondary_rays", C.c_uint64),
        ("shadow_rays", C.c_uint64),
        ("tests", C.c_uint64 * RT_NUM_KINDS),
        ("shadow_tests", C.c_uint64 * RT_NUM_KINDS),
        ("shaded_hits", C.c_uint64),
        ("surface_errors", C.c_uint64),
        ("kernel_ms", C.c_double),
        # ABI 6: rt_render_ex's devices, per-device GPU span, exposed gather time
        ("devices", C.c_int32),
        ("reserved2", C.c_int32),
        ("device_kernel_ms", C.c_double * RT_MAX_DEVICES),
        ("gather_ms", C.c_double),
    ]

    def as_dict(self):
        return {
            "primary_rays": int(self.primary_rays),
            "secondary_rays": int(self.secondary_rays),
            "shadow_rays": int(self.shadow_rays),
            "tests": [int(v) for v in self.tests],
            "shadow_tests": [int(v) for v in self.shadow_tests],
            "shaded_hits": int(self.shaded_hits),
            "surface_errors": int(self.surface_errors),
        }

    def total_rays(self):
        return int(self.primary_rays) + int(self.secondary_rays) + int(self.shadow_rays)


class rt_render_timing(C.Structure):
    """Parts of the calling thread's last rt_render call (ABI 5), one host
    timeline: setup + render_wait + copy_tail = total."""
    _fields_ = [
        ("total_ms", C.c_double),
        ("setup_ms", C.c_double),
        ("render_wait_ms", C.c_double),
        ("copy_tail_ms", C.c_double),
        ("gpu_ms", C.c_double),
        ("bands", C.c_int32),
        ("scene_reused", C.c_int32),
        ("specialized", C.c_int32),
        ("devices", C.c_int32),
        ("pending_compiles", C.c_int32),
        ("reserved", C.c_int32),
    ]

    def as_dict(self):
        return {k: (round(getattr(self, k), 4) if isinstance(getattr(self, k), float) else int(getattr(self, k)))
                for k, _ in self._fields_ if k != "reserved"}


class rt_render_opts(C.Structure):
    """rt_render_ex options (ABI 6): devices, gather mode, flags, bands."""
    _fields_ = [
        ("device_count", C.c_int32),
        ("device_mask", C.c_uint32),
        ("devices", C.c_int32 * RT_MAX_DEVICES),
        ("gather", C.c_int32),
        ("flags", C.c_int32),
        ("bands", C.c_int32),
        ("reserved", C.c_int32 * 5),
    ]


class PackedScene:
    """Owns the ctypes arrays an rt_scene points into (keeps them alive)."""

    def __init__(self, scene, lights, objects, materials, programs=None, ext_lights=None):
        self.scene = scene
        self._lights = lights
        self._ext_lights = ext_lights
        self._objects = objects
        self._materials = materials
        # (code, consts, entry ctypes arrays, [(SurfaceFn, EvalState stack)] per program)
        self.programs = programs

    @property
    def width(self):
        return int(self.scene.width)

    @property
    def height(self):
        return int(self.scene.height)

    def ref(self):
        return C.byref(self.scene)


# Algorithmic FP64 flops per Intersect call, by kind (SURVEY.md §8(d):
# +,-,*,/,sqrt = 1 each, compares 0; miss-path counts, i.e. a lower bound).
# sphere: 33 (ray->object) + 19 (a, halfB, c, discriminant) = 52
# plane : 33 + 5 (denom) + 7 (numerator) ... = 45 on the non-parallel path
# cube  : 6 planes = 270 (the reference re-transforms the ray per face)
# cylinder: 33 + ~51 = 84
# cone (extension): 33 + a, halfB, c (15) + discriminant (3) + base cap (~10) = 61
# csg (extension): counted as one test of the composite; lower bound = its
# bounding-sphere-culled leaf work is not modelled (0)
FLOPS_PER_TEST = (52, 45, 270, 84, 61, 0)
# Per shaded hit: surface props + ambient (21); per light: lighting (68).
FLOPS_PER_SHADE = 21
FLOPS_PER_LIGHT = 68


def algorithmic_flops(stats, num_lights):
    """Sum of count x flops over the work the render did (lower bound)."""
    f = 0
    for k in range(RT_NUM_KINDS):
        f += (int(stats.tests[k]) + int(stats.shadow_tests[k])) * FLOPS_PER_TEST[k]
    f += int(stats.shaded_hits) * (FLOPS_PER_SHADE + FLOPS_PER_LIGHT * num_lights)
    return f


def sum_stats(stats):
    """One rt_stats holding the field-wise sum of several (the counters of the
    contexts that rendered frames in flight); kernel_ms is the largest."""
    out = rt_stats()
    for st in stats:
        out.primary_rays += st.primary_rays
        out.secondary_rays += st.secondary_rays
        out.shadow_rays += st.shadow_rays
        for k in range(RT_NUM_KINDS):
            out.tests[k] += st.tests[k]
            out.shadow_tests[k] += st.shadow_tests[k]
        out.shaded_hits += st.shaded_hits
        out.surface_errors += st.surface_errors
        out.kernel_ms = max(out.kernel_ms, st.kernel_ms)
    return out

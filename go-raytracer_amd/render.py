"""Render(): the reference's entry point (raytracer.go:589) over the C ABI.

The only compute path is the HIP library csrc/librtamd.so (gfx950). There is
no CPU fallback: if the library or a HIP device is missing, every call raises.
PyTorch is used only for device memory and streams.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from . import scene as _scene

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "csrc", "librtamd.so")

_lib = None


class RenderError(RuntimeError):
    pass


def load_library(path=None):
    """Load librtamd.so and declare the include/rt_abi.h signatures.
    RT_AMD_LIB overrides the in-tree path (A/B builds of the same ABI)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("RT_AMD_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RenderError("HIP renderer library not built: %s (run __graft_entry__.build())" % path)
    # torch bundles its own libamdhip64 (same soname as /opt/rocm's): load it
    # first so librtamd binds to that one runtime; loading the library first
    # would put two HIP runtimes in the process and the second finds no device.
    import torch  # noqa: F401
    l = C.CDLL(path)
    vp, i = C.c_void_p, C.c_int
    l.rt_abi_version.argtypes = []
    l.rt_abi_version.restype = i
    l.rt_last_error.argtypes = []
    l.rt_last_error.restype = C.c_char_p
    l.rt_create.argtypes = [i, C.POINTER(vp)]
    l.rt_create.restype = i
    l.rt_destroy.argtypes = [vp]
    l.rt_destroy.restype = None
    l.rt_set_scene.argtypes = [vp, vp]
    l.rt_set_scene.restype = i
    l.rt_render_rows_async.argtypes = [vp, i, i, vp, vp]
    l.rt_render_rows_async.restype = i
    l.rt_render_tile_rows_async.argtypes = [vp, i, i, i, vp, vp]
    l.rt_render_tile_rows_async.restype = i
    l.rt_read_stats.argtypes = [vp, vp, i, vp]
    l.rt_read_stats.restype = i
    l.rt_last_kernel_ms.argtypes = [vp, C.POINTER(C.c_double)]
    l.rt_last_kernel_ms.restype = i
    l.rt_debug_run_surface.argtypes = [vp, i, i, vp, vp, vp, vp, vp]
    l.rt_debug_run_surface.restype = i
    l.rt_ssim_rgba8.argtypes = [vp, vp, vp, i, i, C.POINTER(C.c_double), vp]
    l.rt_ssim_rgba8.restype = i
    l.rt_set_specialize.argtypes = [vp, i]
    l.rt_set_specialize.restype = i
    l.rt_set_accel.argtypes = [vp, i]
    l.rt_set_accel.restype = i
    l.rt_set_schedule.argtypes = [vp, i]
    l.rt_set_schedule.restype = i
    l.rt_scene_info.argtypes = [vp, C.POINTER(i)]
    l.rt_scene_info.restype = i
    l.rt_specialized.argtypes = [vp, C.POINTER(i), C.POINTER(C.c_double)]
    l.rt_specialized.restype = i
    l.rt_spec_precompile.argtypes = [i, C.POINTER(i), i, C.POINTER(C.c_double)]
    l.rt_spec_precompile.restype = i
    l.rt_set_work_sharing.argtypes = [vp, i]
    l.rt_set_work_sharing.restype = i
    l.rt_set_tile_order.argtypes = [vp, i]
    l.rt_set_tile_order.restype = i
    l.rt_set_frames_in_flight.argtypes = [vp, i]
    l.rt_set_frames_in_flight.restype = i
    l.rt_tile_order_info.argtypes = [vp, C.POINTER(i), C.POINTER(C.c_double)]
    l.rt_tile_order_info.restype = i
    l.rt_render.argtypes = [vp, vp, vp]
    l.rt_render.restype = i
    l.rt_render_last_timing.argtypes = [vp]
    l.rt_render_last_timing.restype = i
    l.rt_render_ex.argtypes = [vp, vp, vp, vp]
    l.rt_render_ex.restype = i
    l.rt_debug_assemble.argtypes = [i, i, i, i, vp, vp]
    l.rt_debug_assemble.restype = i
    l.rt_debug_spec_compile.argtypes = [C.c_char_p, C.POINTER(C.c_double)]
    l.rt_debug_spec_compile.restype = i
    l.rt_debug_getenv.argtypes = [C.c_char_p]
    l.rt_debug_getenv.restype = C.c_char_p
    if l.rt_abi_version() != abi.RT_ABI_VERSION:
        raise RenderError("librtamd ABI version mismatch")
    _lib = l
    return l


def _check(rc, what):
    if rc != abi.RT_OK:
        msg = _lib.rt_last_error() if _lib is not None else b""
        raise RenderError("%s failed (%d): %s" % (what, rc, (msg or b"").decode(errors="replace")))


def _packed(scene_or_args):
    if isinstance(scene_or_args, abi.PackedScene):
        return scene_or_args
    return _scene.convert(scene_or_args)


class RenderContext:
    """One device context: scene resident in HBM, renders rows on a torch stream."""

    def __init__(self, device=None, specialize=False):
        import torch
        if not torch.cuda.is_available():
            raise RenderError("no HIP device visible: the renderer has no CPU path")
        self.torch = torch
        self.lib = load_library()
        self.device = torch.cuda.current_device() if device is None else int(device)
        with torch.cuda.device(self.device):
            h = C.c_void_p()
            _check(self.lib.rt_create(self.device, C.byref(h)), "rt_create")
        self.handle = h
        self.packed = None
        if specialize:
            self.set_specialize(True)

    def close(self):
        if self.handle:
            self.lib.rt_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, scene_or_args):
        self.packed = _packed(scene_or_args)
        _check(self.lib.rt_set_scene(self.handle, self.packed.ref()), "rt_set_scene")
        return self.packed

    def set_specialize(self, enable=True):
        """Render with a kernel compiled for the scene's shape (hipRTC, ~1-2 s
        once per scene shape and process; bit-identical output). Raises
        RenderError if hipRTC fails."""
        _check(self.lib.rt_set_specialize(self.handle, int(bool(enable))), "rt_set_specialize")

    def set_accel(self, flags):
        """abi.RT_ACCEL_BVH | abi.RT_ACCEL_CULL (default both). 0 = the
        reference's brute-force search (every ray tests every object in FP64;
        identical pixels and counters). The BVH choice applies at the next
        set_scene; culling applies to specialised kernels."""
        _check(self.lib.rt_set_accel(self.handle, int(flags)), "rt_set_accel")

    def set_schedule(self, mode):
        """abi.RT_SCHED_AUTO (default: pixel quads for depth >= 7),
        RT_SCHED_PIXEL or RT_SCHED_QUADS -- how pixels are dealt to lanes;
        identical pixels and counters. Applies at the next set_scene."""
        _check(self.lib.rt_set_schedule(self.handle, int(mode)), "rt_set_schedule")

    def set_tile_order(self, enable=True):
        """Deal each launch's tiles most expensive first (default on; the
        estimate -- one centre sample per 8x8 tile -- runs at scene setup);
        identical pixels and counters either way. Applies at once."""
        _check(self.lib.rt_set_tile_order(self.handle, int(bool(enable))), "rt_set_tile_order")

    def set_frames_in_flight(self, n):
        """This context is one of n whose launches overlap (frames in flight,
        dist.DistributedRenderer with a list of contexts): the automatic
        schedule may then prefer serial samples at depth >= 7. Identical
        pixels and counters. Applies at once."""
        _check(self.lib.rt_set_frames_in_flight(self.handle, int(n)), "rt_set_frames_in_flight")

    def set_work_sharing(self, enable=True):
        """Work sharing at the tail of a launch (specialised kernel only;
        identical pixels and counters; applies at once). True / 1 the
        workgroup board (RT_SHARE_GROUP), 2 the device-wide one
        (RT_SHARE_DEVICE); the library default is RT_SHARE_AUTO: the device
        board for CSG scenes at depth >= 7 on strong-scaling shares or without
        frames in flight, else off."""
        # True / 1: the workgroup board; 2 (abi.RT_SHARE_DEVICE): device-wide
        mode = int(enable)
        _check(self.lib.rt_set_work_sharing(self.handle, mode), "rt_set_work_sharing")

    def tile_order_info(self):
        """(active, estimate_ms): whether the current scene's launches use a
        tile order, and the estimate's wall time at scene setup."""
        a, ms = C.c_int(), C.c_double()
        _check(self.lib.rt_tile_order_info(self.handle, C.byref(a), C.byref(ms)), "rt_tile_order_info")
        return bool(a.value), ms.value

    def scene_info(self):
        """rt_scene_info flags of the current scene (abi.RT_INFO_*): which
        kernel flavour renders it."""
        f = C.c_int()
        _check(self.lib.rt_scene_info(self.handle, C.byref(f)), "rt_scene_info")
        return f.value

    def specialized(self):
        """(active, compile_ms): whether the current scene runs a specialised
        kernel and what preparing it cost (0 on a cache hit)."""
        a, ms = C.c_int(), C.c_double()
        _check(self.lib.rt_specialized(self.handle, C.byref(a), C.byref(ms)), "rt_specialized")
        return bool(a.value), ms.value

    def render_rows_async(self, y0, y1, out, stream=None):
        """Enqueue rows [y0, y1) into the uint8 CUDA tensor `out` ([y1-y0, W, 4])."""
        torch = self.torch
        W = self.packed.width
        assert out.dtype == torch.uint8 and out.is_cuda and out.is_contiguous()
        assert out.numel() == (y1 - y0) * W * 4, "output tensor shape does not match rows"
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        _check(self.lib.rt_render_rows_async(self.handle, int(y0), int(y1), C.c_void_p(out.data_ptr()),
                                             C.c_void_p(s.cuda_stream)), "rt_render_rows_async")

    def render_tile_rows_async(self, trow0, stride, ntrows, out, stream=None):
        """Enqueue `ntrows` interleaved 8-row tile rows (image tile rows trow0 + j*stride)
        into the uint8 CUDA tensor `out` ([ntrows*8, W, 4])."""
        torch = self.torch
        W = self.packed.width
        assert out.dtype == torch.uint8 and out.is_cuda and out.is_contiguous()
        assert out.numel() == ntrows * 8 * W * 4, "output tensor shape does not match tile rows"
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        _check(self.lib.rt_render_tile_rows_async(self.handle, int(trow0), int(stride), int(ntrows),
                                                  C.c_void_p(out.data_ptr()), C.c_void_p(s.cuda_stream)),
               "rt_render_tile_rows_async")

    def read_stats(self, reset=True, stream=None):
        s = self.torch.cuda.current_stream(self.device) if stream is None else stream
        st = abi.rt_stats()
        _check(self.lib.rt_read_stats(self.handle, C.c_void_p(s.cuda_stream), int(reset), C.byref(st)),
               "rt_read_stats")
        return st

    def last_kernel_ms(self):
        ms = C.c_double()
        _check(self.lib.rt_last_kernel_ms(self.handle, C.byref(ms)), "rt_last_kernel_ms")
        return ms.value

    def debug_run_surface(self, program, face, u, v):
        """Diagnostic: run one surface program on the device for arrays of inputs."""
        face = np.ascontiguousarray(face, dtype=np.int64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        v = np.ascontiguousarray(v, dtype=np.float64)
        n = len(face)
        out = np.zeros((n, 10), dtype=np.float64)
        err = np.zeros(n, dtype=np.int32)
        _check(self.lib.rt_debug_run_surface(self.handle, int(program), n, face.ctypes.data, u.ctypes.data,
                                             v.ctypes.data, out.ctypes.data, err.ctypes.data), "rt_debug_run_surface")
        return out, err

    def ssim(self, a, b):
        """prim.SSIM (internal/prim/ssim.go:27-182) of two RGBA8 frames on the
        device. a, b: uint8 [H, W, 4] (or [H, W, 3]) torch tensors or numpy
        arrays; host arrays are uploaded."""
        torch = self.torch
        dev = "cuda:%d" % self.device

        def prep(x):
            t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.array(x, dtype=np.uint8, copy=True))
            if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] not in (3, 4):
                raise ValueError("ssim: expected uint8 [H, W, 3|4] images")
            t = t.to(dev)
            if t.shape[2] == 3:
                t = torch.cat([t, torch.full_like(t[..., :1], 255)], dim=2)
            return t.contiguous()

        ta, tb = prep(a), prep(b)
        if ta.shape != tb.shape:
            raise ValueError("images are not the same size")  # ssim.go:29-31
        out = C.c_double()
        stream = torch.cuda.current_stream(self.device)
        _check(self.lib.rt_ssim_rgba8(self.handle, C.c_void_p(ta.data_ptr()), C.c_void_p(tb.data_ptr()),
                                      int(ta.shape[1]), int(ta.shape[0]), C.byref(out),
                                      C.c_void_p(stream.cuda_stream)), "rt_ssim_rgba8")
        return out.value

    def render(self, y0=0, y1=None):
        """Synchronous render of rows [y0, y1) -> numpy uint8 [rows, W, 4]."""
        torch = self.torch
        if y1 is None:
            y1 = self.packed.height
        out = torch.empty((y1 - y0, self.packed.width, 4), dtype=torch.uint8, device="cuda:%d" % self.device)
        self.render_rows_async(y0, y1, out)
        torch.cuda.synchronize(self.device)
        return out.cpu().numpy()


def kernel_source_id():
    """Identifier of the device code and its launch configuration (sha256 of
    the kernel sources and of rt_kernel.hip -- occupancy bounds, hipRTC flags,
    schedule choice, tile order, grid sizing -- 16 hex digits): stored with
    committed PMC summaries so that a bench line only quotes counters recorded
    with the kernel and launches it times."""
    import hashlib
    h = hashlib.sha256()
    root = os.path.dirname(PKG_DIR)
    for rel in ("include/rt_abi.h", "go-raytracer_amd/csrc/rt_device.h", "go-raytracer_amd/csrc/rt_render.h",
                "go-raytracer_amd/csrc/rt_kernel.hip"):
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def spec_precompile(kinds, features=0, nlights=0):
    """Compile (no device needed) the specialised kernel for a scene whose
    objects have these primitive kinds, in order, RT_SPEC_* feature bits
    (abi.RT_SPEC_SURFACES / _DIRECTIONAL / _SPOT) and light count (1..8; the
    scene's own count, which rt_set_scene specialises on); returns the compile
    time (ms, 0 if already cached in this process)."""
    lib = load_library()
    features = int(features) | (int(nlights) << 8)
    arr = (C.c_int * len(kinds))(*[int(k) for k in kinds])
    ms = C.c_double()
    _check(lib.rt_spec_precompile(len(kinds), arr, int(features), C.byref(ms)), "rt_spec_precompile")
    return ms.value


def render_opts(devices=None, gather="auto", out_device=False, generic=False, spec_sync=False, bands=0):
    """abi.rt_render_opts for rt_render_ex. devices: None (the current
    device), an int N (devices 0..N-1) or a list of ordinals (repeats allowed:
    one GPU rendering several shares, each with its own contexts)."""
    o = abi.rt_render_opts()
    flags = 0
    if isinstance(devices, int):
        o.device_count = devices
    elif devices is not None:
        devices = [int(d) for d in devices]
        if not 1 <= len(devices) <= abi.RT_MAX_DEVICES:
            raise ValueError("1..%d devices" % abi.RT_MAX_DEVICES)
        o.device_count = len(devices)
        for k, d in enumerate(devices):
            o.devices[k] = d
        flags |= abi.RT_RENDER_DEVICE_LIST
    o.gather = {"auto": abi.RT_GATHER_AUTO, "host": abi.RT_GATHER_HOST, "peer": abi.RT_GATHER_PEER}[gather]
    flags |= (abi.RT_RENDER_OUT_DEVICE if out_device else 0) | (abi.RT_RENDER_GENERIC if generic else 0) | \
        (abi.RT_RENDER_SPEC_SYNC if spec_sync else 0)
    o.flags = flags
    o.bands = int(bands)
    return o


def render_frame(scene_or_args, devices=None, gather="auto", generic=False, spec_sync=False, bands=0, out=None):
    """One synchronous frame through rt_render_ex (include/rt_abi.h): the
    Render() seam over one or several GPUs of this process. Returns (image
    numpy uint8 [H, W, 4], abi.rt_stats, abi.rt_render_timing). `out`: a
    caller-owned host array to render into (reused across calls)."""
    lib = load_library()
    p = _packed(scene_or_args)
    if out is None:
        out = np.empty((p.height, p.width, 4), np.uint8)
    assert out.dtype == np.uint8 and out.flags.c_contiguous and out.size == p.height * p.width * 4
    o = render_opts(devices, gather, False, generic, spec_sync, bands)
    st = abi.rt_stats()
    _check(lib.rt_render_ex(p.ref(), C.byref(o), out.ctypes.data_as(C.c_void_p), C.byref(st)), "rt_render_ex")
    tm = abi.rt_render_timing()
    _check(lib.rt_render_last_timing(C.byref(tm)), "rt_render_last_timing")
    return out, st, tm


def debug_assemble(width, height, shares, bands=0):
    """The host side of rt_render_ex's multi-device assembly on host buffers
    (include/rt_abi.h rt_debug_assemble; no device): shares[d] = device d's
    packed tile rows. Returns the assembled frame."""
    lib = load_library()
    shares = [np.ascontiguousarray(s, dtype=np.uint8) for s in shares]
    ptrs = (C.c_void_p * len(shares))(*[s.ctypes.data for s in shares])
    out = np.zeros((height, width, 4), np.uint8)
    _check(lib.rt_debug_assemble(int(width), int(height), len(shares), int(bands), ptrs,
                                 out.ctypes.data_as(C.c_void_p)), "rt_debug_assemble")
    return out


def Render(scene_or_args, return_stats=False):
    """Render(scene) -> RGBA8 image as numpy [H, W, 4] (Go image.RGBA.Pix layout),
    raytracer.go:589-682. Runs on the current HIP device."""
    ctx = RenderContext()
    try:
        ctx.set_scene(scene_or_args)
        ctx.read_stats(reset=True)
        img = ctx.render()
        st = ctx.read_stats(reset=True)
    finally:
        ctx.close()
    return (img, st) if return_stats else img

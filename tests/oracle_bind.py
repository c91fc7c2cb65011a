"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None
SURFACE_CB = C.CFUNCTYPE(C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.POINTER(C.c_double))
_cb_keep = None


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build_oracle()
        l = C.CDLL(ORACLE_SO)
        l.oracle_render_rows.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        l.oracle_render_rows.restype = C.c_int
        l.oracle_intersect.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                       C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int)]
        l.oracle_intersect.restype = C.c_int
        l.oracle_surface_normal.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double),
                                            C.POINTER(C.c_double), C.POINTER(C.c_double)]
        l.oracle_surface_normal.restype = C.c_int
        for fn in ("oracle_go_pow",):
            getattr(l, fn).argtypes = [C.c_double, C.c_double]
            getattr(l, fn).restype = C.c_double
        l.oracle_go_pow_mode.argtypes = [C.c_double, C.c_double, C.c_int]
        l.oracle_go_pow_mode.restype = C.c_double
        l.oracle_go_exp_amd64.argtypes = [C.c_double, C.c_int]
        l.oracle_go_exp_amd64.restype = C.c_double
        l.oracle_go_log_amd64.argtypes = [C.c_double]
        l.oracle_go_log_amd64.restype = C.c_double
        for fn in ("oracle_go_tan", "oracle_go_sin", "oracle_go_cos", "oracle_go_exp", "oracle_go_log"):
            getattr(l, fn).argtypes = [C.c_double]
            getattr(l, fn).restype = C.c_double
        l.oracle_pcg_float64.argtypes = [C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
        l.oracle_pcg_float64.restype = None
        for fn in ("oracle_go_acos",):
            getattr(l, fn).argtypes = [C.c_double]
            getattr(l, fn).restype = C.c_double
        l.oracle_go_atan2.argtypes = [C.c_double, C.c_double]
        l.oracle_go_atan2.restype = C.c_double
        l.oracle_set_surface_callback.argtypes = [SURFACE_CB]
        l.oracle_set_surface_callback.restype = None
        _lib = l
    return _lib


def render_rows(packed, y0=0, y1=None, threads=8):
    """Oracle render of rows [y0, y1): returns (uint8[rows, W, 4], rt_stats)."""
    from importlib import import_module
    abi = import_module("go_raytracer_amd.abi")
    if y1 is None:
        y1 = packed.height
    out = np.zeros((y1 - y0, packed.width, 4), dtype=np.uint8)
    st = abi.rt_stats()
    _install_surfaces(packed)
    rc = lib().oracle_render_rows(C.addressof(packed.scene), y0, y1, threads,
                                  out.ctypes.data_as(C.c_void_p), C.addressof(st))
    if rc != 0:
        raise RuntimeError("oracle_render_rows failed: %d" % rc)
    return out, st


def _install_surfaces(packed):
    """Closure surfaces: the oracle calls back into the GML interpreter
    (gml.eval_surface_fn, the restatement of EvalSurfaceFn) per hit."""
    global _cb_keep
    if not packed.programs:
        return
    from go_raytracer_amd import gml
    sfs = packed.programs[3]
    state = packed.programs[4].clone() if packed.programs[4] is not None else gml.EvalState()

    def cb(prog, face, u, v, out):
        try:
            m = gml.eval_surface_fn(face, u, v, state, sfs[prog])
        except gml.GMLError:
            return 1
        vals = list(m.color) + [m.reflectivity, m.fuzziness, m.transparency, m.refractive_index,
                                m.kd, m.ks, m.specular_exponent]
        for k in range(10):
            out[k] = float(vals[k])
        return 0

    _cb_keep = SURFACE_CB(cb)
    lib().oracle_set_surface_callback(_cb_keep)

"""Where a fresh process's first Render() goes (GPU box): HIP runtime
initialisation (hipGetDeviceCount + hipFree(0) through libamdhip64 directly),
then the first rt_render_ex call's parts (rt_render_last_timing), then a
second call. usage: python3 scripts/first_call_parts.py [config]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402

t0 = time.perf_counter()
rt = load_package()
lib = rt.render.load_library()
t_load = time.perf_counter()
hip = ctypes.CDLL("libamdhip64.so")
n = ctypes.c_int(0)
hip.hipGetDeviceCount(ctypes.byref(n))
t_count = time.perf_counter()
hip.hipFree(ctypes.c_void_p(0))
t_init = time.perf_counter()
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
p = rt.scene.convert(rt.configs.CONFIGS[cfg]())
t_conv = time.perf_counter()
out = None
res = {"config": cfg, "load_ms": (t_load - t0) * 1e3, "hip_device_count_ms": (t_count - t_load) * 1e3,
       "hip_context_ms": (t_init - t_count) * 1e3, "host_convert_ms": (t_conv - t_init) * 1e3}
for k in range(2):
    t = time.perf_counter()
    img, st, tm = rt.render_frame(p, out=out)
    out = img
    res["call%d_ms" % k] = (time.perf_counter() - t) * 1e3
    res["call%d_parts" % k] = tm.as_dict()
print(json.dumps(res))

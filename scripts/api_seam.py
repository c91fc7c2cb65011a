#!/usr/bin/env python3
"""rt_render (the Render() seam) on C3 4K under several band counts and host
copy thread counts: median of the last calls, with the library's own parts
(rt_render_last_timing). Usage: python3 scripts/api_seam.py [config]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402


def main():
    pkg = load_package()
    import numpy as np
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    packed = pkg.scene.convert(pkg.configs.CONFIGS[cfg]())
    lib = pkg.render.load_library()
    out = np.empty((packed.height, packed.width, 4), np.uint8)
    st = pkg.abi.rt_stats()
    res = []
    for bands in (1, 2, 4, 8):
        for threads in (1, 4, 8):
            os.environ["RT_RENDER_BANDS"] = str(bands)
            os.environ["RT_RENDER_COPY_THREADS"] = str(threads)
            calls = []
            for _ in range(15):
                t0 = time.perf_counter()
                rc = lib.rt_render(packed.ref(), out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st))
                wall = (time.perf_counter() - t0) * 1e3
                assert rc == 0, lib.rt_last_error()
                tm = pkg.abi.rt_render_timing()
                lib.rt_render_last_timing(ctypes.byref(tm))
                calls.append((wall, tm.as_dict()))
            last = sorted(calls[-9:], key=lambda c: c[0])
            wall, parts = last[len(last) // 2]
            r = {"bands": bands, "threads": threads, "wall_ms": round(wall, 3), "parts": parts}
            print(json.dumps(r), flush=True)
            res.append(r)
    best = min(res, key=lambda r: r["wall_ms"])
    print("best", json.dumps(best), flush=True)


if __name__ == "__main__":
    main()

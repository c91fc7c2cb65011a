"""A/B several builds of librtamd.so in ONE process (interleaved rounds).

usage: python scripts/ab.py --config c3 --rounds 5 lib1.so lib2.so ...
Each variant renders the same frame; outputs must be byte-identical to the
first variant's. Prints per-variant median / min kernel ms and Mrays/s.
"""
import argparse
import ctypes as C
import json
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--specialize", type=int, default=1, help="rt_set_specialize on each context (default 1)")
    ap.add_argument("--frames", type=int, default=3, help="serial frames per variant per round")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    pkg = load_package()
    import torch
    torch.cuda.set_device(0)
    kw = {}
    if a.width:
        kw["width"] = a.width
    if a.height:
        kw["height"] = a.height
    args = pkg.configs.CONFIGS[a.config](**kw)
    packed = pkg.scene.convert(args)
    H, W = packed.height, packed.width
    ctxs = []
    tmp = tempfile.mkdtemp()
    for i, path in enumerate(a.libs):
        cp = os.path.join(tmp, "v%d_%s" % (i, os.path.basename(path)))
        shutil.copy(path, cp)
        lib = pkg.render.load_library.__wrapped__(cp) if hasattr(pkg.render.load_library, "__wrapped__") else None
        l = C.CDLL(cp)
        l.rt_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        l.rt_set_scene.argtypes = [C.c_void_p, C.c_void_p]
        l.rt_render_rows_async.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        l.rt_last_kernel_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        l.rt_read_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        l.rt_last_error.restype = C.c_char_p
        h = C.c_void_p()
        assert l.rt_create(0, C.byref(h)) == 0, l.rt_last_error()
        l.rt_set_specialize.argtypes = [C.c_void_p, C.c_int]
        assert l.rt_set_specialize(h, a.specialize) == 0, l.rt_last_error()
        assert l.rt_set_scene(h, packed.ref()) == 0, l.rt_last_error()
        ctxs.append((path, l, h))
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    ref = None
    times = {p: [] for p, _, _ in ctxs}
    rays = {}
    for r in range(a.rounds + 1):
        for path, l, h in ctxs:
            st = pkg.abi.rt_stats()
            l.rt_read_stats(h, C.c_void_p(stream.cuda_stream), 1, C.byref(st))
            for _f in range(a.frames):
                out.zero_()
                assert l.rt_render_rows_async(h, 0, H, C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream)) == 0
                ms = C.c_double()
                l.rt_last_kernel_ms(h, C.byref(ms))
                if r > 0:
                    times[path].append(ms.value)
            l.rt_read_stats(h, C.c_void_p(stream.cuda_stream), 1, C.byref(st))
            img = out.cpu()
            if ref is None:
                ref = img.clone()
            elif not torch.equal(img, ref):
                print("MISMATCH", path, int((img != ref).any(-1).sum()), "pixels", flush=True)
            rays[path] = st.total_rays() // a.frames
    res = []
    for path, _, _ in ctxs:
        t = sorted(times[path])
        med = t[len(t) // 2]
        res.append({"lib": os.path.basename(path), "median_ms": round(med, 4), "min_ms": round(t[0], 4),
                    "Mrays_s": round(rays[path] / (med * 1e-3) / 1e6, 1), "rays": rays[path]})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()

"""Closure-surface debugging: GPU vs oracle on small GML scenes (diff maps, counters).

usage: RT_AMD_LIB=path/to/librtamd.so python scripts/dbg_closure.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from __graft_entry__ import load_package  # noqa: E402

ERR_SRC = """
[ 0.0 1.0 ] /tab
{ /v /u /face tab u floor get /c c c c point 1.0 0.0 1.0 } plane 0.0 -1.0 0.0 translate /p
0.2 0.2 0.2 point [ ] p 1 90.0 64 48 "x.ppm" render
"""


def diffmap(a, b, cols=64):
    d = (a != b).any(axis=-1)
    H, W = d.shape
    sy, sx = max(1, H // (cols * H // W // 2 or 1)), max(1, W // cols)
    for y in range(0, H, sy):
        print("".join("#" if d[y:y + sy, x:x + sx].any() else "." for x in range(0, W, sx)))


def main():
    rt = load_package()
    import oracle_bind
    from go_raytracer_amd import gml
    ctx = rt.RenderContext(0)
    scenes = [("err", gml.run_text(ERR_SRC)[0][0][0])]
    for name in ("cube", "cylinder", "sphere"):
        args = gml.run_file(os.path.join(ROOT, "tests", "golden", "gml", name + ".gml"))[0][0][0]
        args.width, args.height = 128, 96
        scenes.append((name, args))
    for name, args in scenes:
        packed = rt.scene.convert(args)
        ctx.set_scene(packed)
        ctx.read_stats(reset=True)
        img = ctx.render()
        st = ctx.read_stats(reset=True).as_dict()
        ref, ost = oracle_bind.render_rows(packed)
        ost = ost.as_dict()
        nd = int((img != ref).any(axis=-1).sum())
        print("== %s %dx%d: %d pixels differ" % (name, packed.width, packed.height, nd))
        for k in st:
            if st[k] != ost[k]:
                print("   counter %s gpu=%s oracle=%s" % (k, st[k], ost[k]))
        if nd:
            diffmap(img, ref)
            bad = np.argwhere((img != ref).any(axis=-1))[:8]
            for y, x in bad:
                print("   (x=%d,y=%d) gpu=%s oracle=%s" % (x, y, img[y, x], ref[y, x]))
    ctx.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Generates the reduced-size golden images of the BASELINE configs
(tests/golden/synthetic/): each rendered by the CPU oracle (oracle/, pinned
byte-for-byte against the reference's own goldens, tests/test_oracle.py) and
stored as RGB8 PNG plus the oracle's work counters. Test infrastructure:
re-run after changing a config; the tests check both the oracle and the HIP
path against these bytes.

    python tests/golden/make_synthetic.py          # reduced-size goldens
    python tests/golden/make_synthetic.py --full   # full-size strips (minutes)
"""
import json
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

# name -> (config, width, height, row band or None)
CASES = {
    "c1_256x256": ("c1", 256, 256, None),
    "c2_320x180": ("c2", 320, 180, None),
    "c3_320x180": ("c3", 320, 180, None),
    "c3cone_320x180": ("c3cone", 320, 180, None),
    "c4_192x108": ("c4", 192, 108, None),
    "c4csg_128x72": ("c4csg", 128, 72, None),
    "c5_96x60_rows20-40": ("c5", 96, 60, (20, 40)),
}
# Full-size strips of configs too costly for the CPU suite to re-render (the
# oracle's brute-force 100k-sphere search: minutes on 8 threads); the GPU
# tests compare the HIP path with these committed bytes and counters.
# C5 as BASELINE.json states it: one 20-row strip (raytracer.go:632-634 strip
# seeds) of the full 7680-wide, 4320-row frame, 100 000 spheres, depth 8.
FULL = {
    "c5_7680x4320_rows2140-2160": ("c5", 7680, 4320, (2140, 2160)),
    # the horizon rows: rays that meet the ground plane up to ~1e7 units out,
    # whose shadow and reflection rays take the BVH culls' far-origin shift
    # (rt_render.h far_shift)
    "c5_7680x4320_rows2156-2164": ("c5", 7680, 4320, (2156, 2164)),
    # the top of the frame (sky above the sphere field), the lower middle
    # (ground reflections of the sphere field at depth 8, raytracer.go:512-528)
    # and the bottom rows (the nearest ground, the steepest reflections)
    "c5_7680x4320_rows0-8": ("c5", 7680, 4320, (0, 8)),
    # the upper sphere field (the nearest layer's top edge is near row 171,
    # the farthest layer's near row 1508: rays from the sky through the field)
    "c5_7680x4320_rows600-608": ("c5", 7680, 4320, (600, 608)),
    "c5_7680x4320_rows3200-3208": ("c5", 7680, 4320, (3200, 3208)),
    "c5_7680x4320_rows4312-4320": ("c5", 7680, 4320, (4312, 4320)),
}


def render(name, cases=CASES, threads=8):
    from __graft_entry__ import load_package
    import oracle_bind
    pkg = load_package()
    cfg, w, h, band = cases[name]
    packed = pkg.scene.convert(pkg.configs.CONFIGS[cfg](width=w, height=h))
    y0, y1 = band if band else (0, h)
    img, st = oracle_bind.render_rows(packed, y0, y1, threads=threads)
    return packed, (y0, y1), img, st


def write(cases, meta_name, threads=8):
    out = os.path.join(HERE, "synthetic")
    os.makedirs(out, exist_ok=True)
    meta = {}
    for name in cases:
        _, (y0, y1), img, st = render(name, cases, threads)
        assert (img[..., 3] == 255).all()
        Image.fromarray(np.ascontiguousarray(img[..., :3])).save(os.path.join(out, name + ".png"), optimize=True)
        meta[name] = {"config": cases[name][0], "width": cases[name][1], "height": cases[name][2],
                      "rows": [y0, y1], "stats": st.as_dict()}
        print(name, st.total_rays(), "rays", flush=True)
    with open(os.path.join(out, meta_name), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


def main():
    if "--full" in sys.argv:  # minutes: the 100k-sphere brute-force strip
        write(FULL, "counters_full.json", threads=os.cpu_count() or 8)
    elif "--full-only" in sys.argv:  # --full-only NAME: add one full-size strip
        name = sys.argv[sys.argv.index("--full-only") + 1]
        path = os.path.join(HERE, "synthetic", "counters_full.json")
        meta = json.load(open(path)) if os.path.exists(path) else {}
        write({name: FULL[name]}, "counters_full.json.new", threads=os.cpu_count() or 8)
        new = os.path.join(HERE, "synthetic", "counters_full.json.new")
        meta.update(json.load(open(new)))
        os.remove(new)
        with open(path, "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
    else:
        write(CASES, "counters.json")


if __name__ == "__main__":
    main()

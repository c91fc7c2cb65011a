"""Render GML programs through the HIP path and write the images.

The reference's `render` builtin calls EvalState.Render, which renders and
writes a PNG named by the program (raytracer.go:700-708, cmd/gml/main.go:
383-390). Here each render call of the program is converted and rendered on
the device as it happens (the hook runs mid-program, so later frames see the
state as it was then), then written by imageio.

usage: python -m go_raytracer_amd.cli [--out-dir DIR] [--device N] [--stats] file.gml ...
(from the repo root the package directory is go-raytracer_amd/; see
__graft_entry__.load_package)
"""
import argparse
import json
import os
import sys


def render_program(path, out_dir=None, device=0, stats=False, log=sys.stdout, extensions=False):
    from . import gml, imageio, scene
    from .render import RenderContext
    ctx = RenderContext(device)
    written = []

    def hook(e, args):
        args.state = e.clone()
        packed = scene.convert(args)
        ctx.set_scene(packed)
        ctx.read_stats(reset=True)
        img = ctx.render()
        st = ctx.read_stats(reset=True)
        name = os.path.basename(args.file) if out_dir else args.file
        dst = os.path.join(out_dir, name) if out_dir else name
        imageio.write_image(dst, img)
        written.append(dst)
        if stats:
            d = st.as_dict()
            d.update(file=dst, kernel_ms=round(st.kernel_ms, 3), width=packed.width, height=packed.height)
            print(json.dumps(d), file=log)

    try:
        st = gml.EvalState(render=hook, extensions=extensions)
        st.parse_and_eval_file(path)
    finally:
        ctx.close()
    return written


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("files", nargs="+")
    ap.add_argument("--out-dir", default=None)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--extensions", action="store_true",
                    help="enable cone, light, spotlight, real (ICFP operators the reference lacks)")
    a = ap.parse_args(argv)
    if a.out_dir:
        os.makedirs(a.out_dir, exist_ok=True)
    for f in a.files:
        for w in render_program(f, a.out_dir, a.device, a.stats, extensions=a.extensions):
            print("wrote", w)
    return 0


if __name__ == "__main__":
    sys.exit(main())

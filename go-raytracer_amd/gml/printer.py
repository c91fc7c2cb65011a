"""RenderArgs text dump (internal/gml/evaluator_test_helpers.go:15-145), used
to pin the host front end against internal/gml/testdata/*.out."""
from .. import scene as S
from .evaluator import SurfaceFn, env_string, debug_str
from .gofmt import fmt_fixed
from . import syntax as X


def render_args_lines(args, idmap):
    lines = []
    ind = [0]

    def add(s):
        lines.append("    " * ind[0] + s)

    def f3(v):
        return "%s %s %s" % (fmt_fixed(v[0]), fmt_fixed(v[1]), fmt_fixed(v[2]))

    add("render %d %d %s" % (args.width, args.height, args.file))
    ind[0] += 1
    add("fov: %s" % fmt_fixed(args.fov))
    add("depth: %d" % args.depth)
    if any(c != 0 for c in args.bg_start) or any(c != 0 for c in args.bg_end):
        add("background-gradient:")
        ind[0] += 1
        add("p1: " + f3(args.bg_start))
        add("p2: " + f3(args.bg_end))
        ind[0] -= 1
    add("ambient: " + f3(args.ambient))
    for l in args.lights:
        if not isinstance(l, S.PointLight):
            raise TypeError("unknown light type %s" % type(l).__name__)
        add("light:")
        ind[0] += 1
        add("position: " + f3(l.position))
        add("color: " + f3(l.color))
        ind[0] -= 1

    def surface(fn):
        add("surface:")
        ind[0] += 1
        if isinstance(fn, SurfaceFn) and fn.closure is not None:
            add("code: " + X.token_list_string(fn.closure.code))
            env = fn.closure.env
            if env:
                add("env:")
                ind[0] += 1
                for i in sorted(env):
                    add("%s: %s" % (idmap.id_name.get(i, "%d (?)" % i), debug_str(env[i], idmap)))
                ind[0] -= 1
        else:
            m = fn.material if isinstance(fn, SurfaceFn) else fn
            add("color: " + f3(m.color))
            add("reflectivity: " + fmt_fixed(m.reflectivity))
            add("fuzz: " + fmt_fixed(m.fuzziness))
            add("transparency: " + fmt_fixed(m.transparency))
            add("refractiveIndex: " + fmt_fixed(m.refractive_index))
            add("kd: " + fmt_fixed(m.kd))
            add("ks: " + fmt_fixed(m.ks))
            add("n: " + fmt_fixed(m.specular_exponent))
        ind[0] -= 1

    def xform(m):
        add("xform:")
        ind[0] += 1
        for row in m:
            add("".join(fmt_fixed(x) for x in row))
        ind[0] -= 1

    def obj(o):
        name = {S.Sphere: "sphere", S.Cube: "cube", S.Plane: "plane"}.get(type(o))
        if name is not None:
            add(name + ":")
            ind[0] += 1
            xform(o.transform_mat)
            surface(o.surface)
            ind[0] -= 1
        elif isinstance(o, S.Union):
            add("union:")
            ind[0] += 1
            for c in o.objects:
                obj(c)
            ind[0] -= 1
        else:
            raise TypeError("unknown scene object type")

    obj(args.scene)
    return lines

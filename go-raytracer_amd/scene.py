"""Host-side scene values and the flattening into the C ABI (rt_scene).

Mirrors the reference's GML scene-object values (internal/gml/evaluator.go:
157-292) and the union flattening / surface baking that sits in front of the
render hot path (raytracer.go:724-830), so a caller holding a gml.RenderArgs
equivalent gets exactly the object order and matrices the reference renders.

Everything here is host plumbing executed once per frame; the per-pixel work
happens in the HIP kernel behind include/rt_abi.h.
"""
import ctypes as C
from dataclasses import dataclass, field, replace
from typing import List, Optional

from . import abi
from . import gomath


@dataclass(frozen=True)
class Material:
    """gml.Material (evaluator.go:136-150)."""
    color: tuple = (0.0, 0.0, 0.0)
    reflectivity: float = 0.0
    fuzziness: float = 0.0
    transparency: float = 0.0
    refractive_index: float = 0.0
    kd: float = 0.0
    ks: float = 0.0
    specular_exponent: float = 0.0


def material(color, refl, fuzz, transparency, refr, kd, ks, n):
    """The `material` builtin's argument order: color refl fuzz transparency refr kd ks n
    (evaluator.go:869-893)."""
    return Material(tuple(float(c) for c in color), float(refl), float(fuzz), float(transparency),
                    float(refr), float(kd), float(ks), float(n))


def surface(color, kd, ks, n):
    """A surface function returning the contest's `color kd ks n`: EvalSurfaceFn maps
    it to a Material with Reflectivity = ks (evaluator.go:700-726)."""
    return Material(color=tuple(float(c) for c in color), kd=float(kd), ks=float(ks),
                    specular_exponent=float(n), reflectivity=float(ks))


@dataclass(frozen=True)
class PointLight:
    """gml.PointLight (evaluator.go:289-292)."""
    position: tuple
    color: tuple


@dataclass(frozen=True)
class DirectionalLight:
    """Contest extension (GML `light`, not in the reference): light at infinity
    travelling along `direction` (include/rt_abi.h rt_light)."""
    direction: tuple
    color: tuple


@dataclass(frozen=True)
class SpotLight:
    """Contest extension (GML `spotlight`, not in the reference): at `position`,
    aimed at point `at`, cutoff half-angle in degrees, falloff exponent."""
    position: tuple
    at: tuple
    color: tuple
    cutoff: float
    exponent: float


class SceneObject:
    """gml.SceneObject (evaluator.go:152-156): Transform composes existing.MulMat(new)."""

    transform_mat = None

    def transform(self, mat):
        new = mat if self.transform_mat is None else gomath.mul_mat(self.transform_mat, mat)
        return replace(self, transform_mat=new)

    # GML builtins on scene objects (evaluator.go:1015-1062)
    def translate(self, x, y, z):
        return self.transform(gomath.translate(float(x), float(y), float(z)))

    def scale(self, x, y, z):
        return self.transform(gomath.scale(float(x), float(y), float(z)))

    def uscale(self, s):
        s = float(s)
        return self.transform(gomath.scale(s, s, s))

    def rotatex(self, deg):
        return self.transform(gomath.rotate_x(gomath.deg_to_rad(float(deg))))

    def rotatey(self, deg):
        return self.transform(gomath.rotate_y(gomath.deg_to_rad(float(deg))))

    def rotatez(self, deg):
        return self.transform(gomath.rotate_z(gomath.deg_to_rad(float(deg))))


@dataclass(frozen=True)
class Sphere(SceneObject):
    """Unit sphere at the origin (evaluator.go:157-175, builtin :755-770).
    `surface` is a Material or a per-face tuple of Materials (face 0 only)."""
    surface: object = Material()
    transform_mat: Optional[list] = None


@dataclass(frozen=True)
class Cube(SceneObject):
    """Unit cube [0,1]^3 (evaluator.go:185-204). Per-face surface: 6-tuple
    indexed by prim.CubeSide (internal/prim/plane.go:14-25)."""
    surface: object = Material()
    transform_mat: Optional[list] = None


@dataclass(frozen=True)
class Cylinder(SceneObject):
    """Unit cylinder x^2+z^2<=1, 0<=y<=1 (evaluator.go:206-223). Per-face surface:
    (side, top, bottom) (raytracer.go:263-267)."""
    surface: object = Material()
    transform_mat: Optional[list] = None


@dataclass(frozen=True)
class Cone(SceneObject):
    """Contest extension (GML `cone`, not in the reference renderer): apex at the
    origin, x^2 + z^2 = y^2 for 0 <= y <= 1, base at y = 1. Faces (side, base)."""
    surface: object = Material()
    transform_mat: Optional[list] = None


@dataclass(frozen=True)
class Plane(SceneObject):
    """Plane through point with normal (builtin: (0,0,0), (0,1,0), evaluator.go:813-821)."""
    surface: object = Material()
    transform_mat: Optional[list] = None
    point: tuple = (0.0, 0.0, 0.0)
    normal: tuple = (0.0, 1.0, 0.0)


@dataclass(frozen=True)
class Union(SceneObject):
    """gml.Union (evaluator.go:244-262). Transform distributes over members."""
    objects: tuple = ()

    def transform(self, mat):
        return Union(tuple(o.transform(mat) for o in self.objects))


def union(first, second):
    """The `union` builtin: `first second union` pops second then first and builds
    Union{Objects: [second, first]} (evaluator.go:1064-1075)."""
    return Union((second, first))


@dataclass(frozen=True)
class Difference(SceneObject):
    """gml.Difference (evaluator.go:264-287): solid a minus solid b. The
    reference renderer rejects it (raytracer.go:825-826); here it renders as a
    CSG composite (contest extension, parity-unpinned; include/rt_abi.h RT_CSG)."""
    a: object = None
    b: object = None

    def transform(self, mat):
        return Difference(self.a.transform(mat), self.b.transform(mat))


@dataclass(frozen=True)
class Intersect(SceneObject):
    """GML `intersect` (contest extension, not in the reference): a and b."""
    a: object = None
    b: object = None

    def transform(self, mat):
        return Intersect(self.a.transform(mat), self.b.transform(mat))


@dataclass
class RenderArgs:
    """gml.RenderArgs (evaluator.go:14-28)."""
    ambient: tuple
    lights: List[PointLight]
    scene: SceneObject
    depth: int
    fov: float
    width: int
    height: int
    file: str = "out.ppm"
    bg_start: tuple = (0.0, 0.0, 0.0)
    bg_end: tuple = (0.0, 0.0, 0.0)
    # GML EvalState at the render call (per-frame clone, raytracer.go:738-751):
    # closure surfaces evaluate on its stack. None for scenes built in Python.
    state: object = None
    # Which math.Exp / math.Log a fractional Pow exponent runs (rt_scene.exp_mode,
    # abi.RT_EXP_*): Go's amd64 assembly with FMA by default (the reference's
    # deployment on an x86-64 CPU with AVX2+FMA).
    exp_mode: int = 0


_NFACES = {abi.RT_SPHERE: 1, abi.RT_PLANE: 1, abi.RT_CUBE: 6, abi.RT_CYLINDER: 3, abi.RT_CONE: 2}
_KIND = {Sphere: abi.RT_SPHERE, Plane: abi.RT_PLANE, Cube: abi.RT_CUBE, Cylinder: abi.RT_CYLINDER,
         Cone: abi.RT_CONE}


def flatten(root):
    """BFS union flattening, raytracer.go:776-828 (order decides closestHit ties).
    A Difference / Intersect is kept whole: one CSG composite (extension)."""
    out = []
    queue = [root]
    while queue:
        obj = queue.pop(0)
        if isinstance(obj, Union):
            queue.extend(obj.objects)
        elif type(obj) in _KIND or isinstance(obj, (Difference, Intersect)):
            out.append(obj)
        else:
            raise TypeError("unknown scene object type %s" % type(obj).__name__)
    return out


_CSG_LEAF = (Sphere, Cube, Cylinder, Plane)


def csg_program(obj):
    """Leaves (in order) and the postfix program of a CSG composite: unions
    inside a composite are set unions (include/rt_abi.h RT_CSG)."""
    leaves, code = [], []

    def walk(o):
        if isinstance(o, Union):
            if not o.objects:
                raise ValueError("empty union inside a CSG composite")
            walk(o.objects[0])
            for c in o.objects[1:]:
                walk(c)
                code.append(abi.RT_CSG_UNION)
        elif isinstance(o, (Difference, Intersect)):
            walk(o.a)
            walk(o.b)
            code.append(abi.RT_CSG_DIFFERENCE if isinstance(o, Difference) else abi.RT_CSG_INTERSECT)
        elif isinstance(o, _CSG_LEAF):
            code.append(len(leaves))
            leaves.append(o)
        else:
            raise ValueError("%s cannot be a CSG leaf" % type(o).__name__)

    walk(obj)
    if len(leaves) > abi.RT_CSG_MAX_LEAVES:
        raise ValueError("CSG composite with %d leaves (max %d)" % (len(leaves), abi.RT_CSG_MAX_LEAVES))
    return leaves, code


def _face_materials(obj, kind):
    s = obj.surface
    n = _NFACES[kind]
    if hasattr(s, "closure") and hasattr(s, "material"):  # gml.SurfaceFn
        if s.material is not None:
            s = s.material
        else:
            return [s] * n
    if isinstance(s, Material):
        return [s] * n
    s = tuple(s)
    if len(s) != n:
        raise ValueError("%s needs %d per-face surfaces, got %d" % (type(obj).__name__, n, len(s)))
    return list(s)


def convert(args: RenderArgs) -> abi.PackedScene:
    """Flatten RenderArgs into the rt_scene the C ABI takes."""
    objs = flatten(args.scene)
    mats: List[Material] = []
    mat_index = {}

    def midx(m):
        if m not in mat_index:
            mat_index[m] = len(mats)
            mats.append(m)
        return mat_index[m]

    programs = []     # (SurfaceFn, Program)
    prog_index = {}

    def pidx(sf):
        key = id(sf.closure)
        if key not in prog_index:
            from .gml.surface_compiler import compile_surface
            stack = args.state.stack if args.state is not None else ()
            prog_index[key] = len(programs)
            programs.append((sf, compile_surface(sf, stack)))
        return -(prog_index[key] + 1)

    def fill(co, o):
        kind = _KIND[type(o)]
        co.kind = kind
        fm = _face_materials(o, kind)
        idx = [midx(m) if isinstance(m, Material) else pidx(m) for m in fm]
        for f in range(abi.RT_MAX_FACES):
            co.material[f] = idx[f] if f < len(idx) else idx[0]
        if o.transform_mat is not None:
            co.has_transform = 1
            for r in range(4):
                for c in range(4):
                    co.transform[r * 4 + c] = float(o.transform_mat[r][c])
        else:
            co.has_transform = 0
        if kind == abi.RT_PLANE:
            for k in range(3):
                co.plane_point[k] = float(o.point[k])
                co.plane_normal[k] = float(o.normal[k])

    c_objs = (abi.rt_object * max(1, len(objs)))()
    csg_leaves, csg_code = [], []
    for i, o in enumerate(objs):
        co = c_objs[i]
        if isinstance(o, (Difference, Intersect)):
            leaves, code = csg_program(o)
            co.kind = abi.RT_CSG
            co.csg_first, co.csg_count = len(csg_leaves), len(leaves)
            co.csg_code, co.csg_code_len = len(csg_code), len(code)
            csg_leaves.extend(leaves)
            csg_code.extend(code)
        else:
            fill(co, o)
    c_leaves = None
    if csg_leaves:
        c_leaves = (abi.rt_object * len(csg_leaves))()
        for j, o in enumerate(csg_leaves):
            fill(c_leaves[j], o)
    if not mats:
        mats.append(Material())
    c_mats = (abi.rt_material * len(mats))()
    for i, m in enumerate(mats):
        cm = c_mats[i]
        for k in range(3):
            cm.color[k] = float(m.color[k])
        cm.reflectivity = m.reflectivity
        cm.fuzziness = m.fuzziness
        cm.transparency = m.transparency
        cm.refractive_index = m.refractive_index
        cm.kd = m.kd
        cm.ks = m.ks
        cm.specular_exponent = m.specular_exponent
    ext = any(not isinstance(l, PointLight) for l in args.lights)
    c_lights = (abi.rt_point_light * max(1, len(args.lights)))()
    c_ext = None
    if not ext:
        for i, l in enumerate(args.lights):
            for k in range(3):
                c_lights[i].position[k] = float(l.position[k])
                c_lights[i].color[k] = float(l.color[k])
    else:  # contest-extension lights: the whole list, in program order
        c_ext = (abi.rt_light * len(args.lights))()
        for i, l in enumerate(args.lights):
            e = c_ext[i]
            for k in range(3):
                e.color[k] = float(l.color[k])
            if isinstance(l, PointLight):
                e.kind = abi.RT_LIGHT_POINT
                for k in range(3):
                    e.position[k] = float(l.position[k])
            elif isinstance(l, DirectionalLight):
                e.kind = abi.RT_LIGHT_DIRECTIONAL
                for k in range(3):
                    e.direction[k] = float(l.direction[k])
            elif isinstance(l, SpotLight):
                e.kind = abi.RT_LIGHT_SPOT
                for k in range(3):
                    e.position[k] = float(l.position[k])
                    e.direction[k] = float(l.at[k])
                e.cutoff = float(l.cutoff)
                e.exponent = float(l.exponent)
            else:
                raise TypeError("unknown light type %s" % type(l).__name__)
    sc = abi.rt_scene()
    sc.width = int(args.width)
    sc.height = int(args.height)
    sc.depth = int(args.depth)
    sc.num_lights = 0 if ext else len(args.lights)
    if ext:
        sc.ext_lights = C.cast(c_ext, C.POINTER(abi.rt_light))
        sc.num_ext_lights = len(args.lights)
    sc.fov = float(args.fov)
    for k in range(3):
        sc.ambient[k] = float(args.ambient[k])
        sc.bg_start[k] = float(args.bg_start[k])
        sc.bg_end[k] = float(args.bg_end[k])
    sc.lights = C.cast(c_lights, C.POINTER(abi.rt_point_light))
    sc.objects = C.cast(c_objs, C.POINTER(abi.rt_object))
    sc.materials = C.cast(c_mats, C.POINTER(abi.rt_material))
    sc.num_objects = len(objs)
    sc.num_materials = len(mats)
    c_csg_code = None
    if csg_leaves:
        c_csg_code = (C.c_int32 * len(csg_code))(*csg_code)
        sc.csg_leaves = C.cast(c_leaves, C.POINTER(abi.rt_object))
        sc.csg_code = C.cast(c_csg_code, C.POINTER(C.c_int32))
        sc.num_csg_leaves = len(csg_leaves)
        sc.csg_code_words = len(csg_code)
    packed_progs = None
    if programs:
        from .gml.surface_compiler import OP
        words, consts, entry = [], [], []
        for sf, prog in programs:
            base = len(consts)
            entry.append(len(words))
            for op, d, a, b, c in prog.code:
                if op in (OP["CONST"], OP["TBL"]):
                    c += base
                words.append(op | (d << 8) | (a << 16) | (b << 24))
                words.append(c & 0xFFFFFFFF)
            consts.extend(prog.consts)
        c_code = (C.c_uint32 * len(words))(*words)
        c_consts = (C.c_uint64 * max(1, len(consts)))(*consts)
        c_entry = (C.c_int32 * len(entry))(*entry)
        sc.program_code = C.cast(c_code, C.POINTER(C.c_uint32))
        sc.program_consts = C.cast(c_consts, C.POINTER(C.c_uint64))
        sc.program_entry = C.cast(c_entry, C.POINTER(C.c_int32))
        sc.num_programs = len(programs)
        sc.program_code_words = len(words)
        sc.program_const_count = len(consts)
        packed_progs = (c_code, c_consts, c_entry, [sf for sf, _ in programs], args.state)
    sc.exp_mode = int(args.exp_mode)
    packed = abi.PackedScene(sc, c_lights, c_objs, c_mats, packed_progs, c_ext)
    packed._csg = (c_leaves, c_csg_code)  # (kept alive with the scene)
    return packed


SCENE_FILE_MAGIC = b"RTSCENE1"


def write_scene_file(packed: abi.PackedScene, path):
    """Serialise an rt_scene for a non-Python host of the C ABI
    (tests/c/abi_render.c `file` mode): magic, the scalars, then every array
    the rt_scene points at as raw include/rt_abi.h structs / words, in field
    order. Little-endian, native struct layout."""
    import struct
    s = packed.scene

    def raw(ptr, ctype, n):
        if n <= 0:
            return b""
        return C.string_at(C.cast(ptr, C.c_void_p), C.sizeof(ctype) * n)

    with open(path, "wb") as f:
        f.write(SCENE_FILE_MAGIC)
        f.write(struct.pack("<4i", s.width, s.height, s.depth, s.num_lights))
        f.write(struct.pack("<10d", s.fov, *s.ambient, *s.bg_start, *s.bg_end))
        f.write(struct.pack("<9i", s.num_objects, s.num_materials, s.num_programs, s.program_code_words,
                            s.program_const_count, s.exp_mode, s.num_ext_lights, s.num_csg_leaves, s.csg_code_words))
        f.write(raw(s.lights, abi.rt_point_light, s.num_lights))
        f.write(raw(s.objects, abi.rt_object, s.num_objects))
        f.write(raw(s.materials, abi.rt_material, s.num_materials))
        f.write(raw(s.program_code, C.c_uint32, s.program_code_words if s.num_programs else 0))
        f.write(raw(s.program_consts, C.c_uint64, s.program_const_count if s.num_programs else 0))
        f.write(raw(s.program_entry, C.c_int32, s.num_programs))
        f.write(raw(s.ext_lights, abi.rt_light, s.num_ext_lights))
        f.write(raw(s.csg_leaves, abi.rt_object, s.num_csg_leaves))
        f.write(raw(s.csg_code, C.c_int32, s.csg_code_words))

"""The C-ABI library loads and exports every symbol include/rt_abi.h declares;
the ctypes mirror matches the C struct layout. No device calls (CPU-only)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import go_raytracer_amd as rt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rt_abi.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(rt_\w+)\s*\(", src, re.M)))


def test_header_declares_the_entry_points():
    names = declared_functions()
    for n in ["rt_abi_version", "rt_last_error", "rt_create", "rt_destroy", "rt_set_scene",
              "rt_render_rows_async", "rt_read_stats", "rt_last_kernel_ms", "rt_render", "rt_render_ex",
              "rt_debug_assemble"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = rt.load_library()
    for n in declared_functions():
        assert hasattr(lib, n), n
    assert lib.rt_abi_version() == rt.abi.RT_ABI_VERSION == 6


def test_struct_layout_matches_header(tmp_path):
    prog = tmp_path / "layout.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s"\n' % HEADER + r'''
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(rt_material), sizeof(rt_point_light), sizeof(rt_object),
         sizeof(rt_scene), sizeof(rt_stats), sizeof(rt_render_timing), sizeof(rt_render_opts));
  printf("%zu %zu %zu %zu\n", offsetof(rt_object, transform), offsetof(rt_object, plane_normal),
         offsetof(rt_scene, lights), offsetof(rt_scene, num_materials));
  printf("%zu %zu %zu %zu %zu %zu\n", offsetof(rt_stats, kernel_ms), offsetof(rt_stats, device_kernel_ms),
         offsetof(rt_stats, gather_ms), offsetof(rt_render_timing, pending_compiles),
         offsetof(rt_render_opts, gather), offsetof(rt_render_opts, bands));
  return 0;
}
''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(prog)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    got = [int(v) for v in out]
    a = rt.abi
    want = [C.sizeof(a.rt_material), C.sizeof(a.rt_point_light), C.sizeof(a.rt_object), C.sizeof(a.rt_scene),
            C.sizeof(a.rt_stats), C.sizeof(a.rt_render_timing), C.sizeof(a.rt_render_opts),
            a.rt_object.transform.offset, a.rt_object.plane_normal.offset,
            a.rt_scene.lights.offset, a.rt_scene.num_materials.offset,
            a.rt_stats.kernel_ms.offset, a.rt_stats.device_kernel_ms.offset, a.rt_stats.gather_ms.offset,
            a.rt_render_timing.pending_compiles.offset, a.rt_render_opts.gather.offset, a.rt_render_opts.bands.offset]
    assert got == want


def test_render_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    with pytest.raises(rt.render.RenderError):
        rt.Render(rt.configs.c1(width=8, height=8))


def test_python_constants_mirror_the_header():
    """Every integer #define of include/rt_abi.h that the ctypes mirror also
    names (kinds, status codes, schedules, work-sharing modes, info bits...)
    has the header's value."""
    src = open(HEADER).read()
    defs = {m.group(1): int(m.group(2)) for m in re.finditer(r"^#define\s+(RT_\w+)\s+\(?(-?\d+)\)?\s*(?:/\*.*)?$", src, re.M)}
    a = rt.abi
    checked = [n for n in defs if hasattr(a, n)]
    for n in checked:
        assert getattr(a, n) == defs[n], n
    for n in ["RT_SHARE_OFF", "RT_SHARE_GROUP", "RT_SHARE_DEVICE", "RT_SHARE_AUTO", "RT_INFO_SHARE_DEVICE",
              "RT_ABI_VERSION", "RT_SCHED_PAIRS", "RT_CSG", "RT_MAX_DEVICES", "RT_GATHER_HOST", "RT_GATHER_PEER",
              "RT_RENDER_DEVICE_LIST", "RT_RENDER_OUT_DEVICE", "RT_RENDER_GENERIC", "RT_RENDER_SPEC_SYNC"]:
        assert n in checked, n

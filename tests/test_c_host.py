"""A non-Python host of the C ABI: tests/c/abi_render.c (built by
tests/hip/Makefile, linked against librtamd.so) builds the flattened scenes
the reference's cgo shim would pass -- including a closure
surface hand-assembled from the bytecode contract of include/rt_abi.h -- and
calls rt_render. Its bytes must equal the reference goldens."""
import json
import os
import re
import subprocess

import numpy as np
import pytest
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "abi_render")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _build():
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "hip")], check=True)


def test_c_host_builds_and_links_the_library():
    _build()
    out = subprocess.run(["ldd", EXE], capture_output=True, text=True).stdout
    assert "librtamd.so" in out and "not found" not in out.split("librtamd.so")[1].splitlines()[0]


def test_bytecode_opcodes_match_the_compiler():
    """The opcode numbers rt_abi.h documents are the ones the host compiler emits."""
    from go_raytracer_amd.gml import surface_compiler as sc
    hdr = open(os.path.join(ROOT, "include", "rt_abi.h")).read()
    ops = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"#define RT_VM_([A-Z]+) (\d+)", hdr))
    assert len(ops) == len(sc.OPS) == 32
    for name, code in ops.items():
        assert sc.OP[name] == code, name


@pytest.mark.gpu
@pytest.mark.parametrize("scene,golden", [("canned", "example_canned.png"), ("sphere", "example_sphere.png")])
def test_c_host_rt_render_matches_reference_golden(tmp_path, scene, golden):
    _build()
    out = tmp_path / (scene + ".rgba")
    r = subprocess.run([EXE, scene, str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    st = json.loads(r.stdout.strip().splitlines()[-1])
    gold = np.asarray(Image.open(os.path.join(GOLDEN, golden)).convert("RGB"))
    img = np.fromfile(out, dtype=np.uint8).reshape(st["height"], st["width"], 4)
    assert (img[..., 3] == 255).all()
    assert np.array_equal(img[..., :3], gold)
    assert st["primary_rays"] == 4 * st["width"] * st["height"] and st["surface_errors"] == 0

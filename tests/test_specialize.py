"""Scene specialisation compile path (hipRTC, no device needed): the embedded
device sources compile for gfx950 with compile-time object kinds, and bad
requests fail loudly. Device parity of the specialised kernel is in
test_gpu_parity.py (test_specialised_*)."""
import os
import pytest

import go_raytracer_amd as rt

A = rt.abi


@pytest.mark.parametrize("kinds,feat", [
    ([A.RT_SPHERE, A.RT_CUBE, A.RT_CYLINDER, A.RT_PLANE], 0),  # C2/C3 shape
    ([A.RT_CONE, A.RT_SPHERE], A.RT_SPEC_DIRECTIONAL | A.RT_SPEC_SPOT),
    ([A.RT_CUBE], A.RT_SPEC_SURFACES),
    ([A.RT_PLANE] * 8, 7),
    ([A.RT_SPHERE, A.RT_CUBE, A.RT_CYLINDER, A.RT_PLANE], A.RT_SPEC_LIGHTS(4)),  # C3 as rt_set_scene keys it
    ([A.RT_CONE, A.RT_SPHERE], A.RT_SPEC_DIRECTIONAL | A.RT_SPEC_SPOT | A.RT_SPEC_LIGHTS(3))])
def test_precompile_builds_a_code_object(kinds, feat):
    ms = rt.spec_precompile(kinds, feat)
    assert ms >= 0
    assert rt.spec_precompile(kinds, feat) == 0.0  # cached per process


@pytest.mark.parametrize("kinds", [[], [A.RT_SPHERE] * 9, [A.RT_CSG], [7], [-1]])
def test_precompile_rejects_bad_requests(kinds):
    with pytest.raises(rt.render.RenderError):
        rt.spec_precompile(kinds)


def test_precompile_rejects_unknown_feature_bits():
    with pytest.raises(rt.render.RenderError):
        rt.spec_precompile([A.RT_SPHERE], 8)
    with pytest.raises(rt.render.RenderError):
        rt.spec_precompile([A.RT_SPHERE], A.RT_SPEC_LIGHTS(9))  # 1..8 lights


def test_brute_force_kernels_with_many_lights_compile():
    """The brute-force specialised kernel (RT_CULL=0) with 5 and 8 lights: a
    backend error there ("illegal VGPR to SGPR copy") aborts the process
    inside hipRTC instead of failing rt_set_scene, so the variants are
    compiled offline here exactly as hipRTC builds them (scripts/spec_regs.sh;
    the full matrix: scripts/spec_matrix.sh)."""
    import subprocess
    import concurrent.futures as cf
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = os.path.join(root, "scripts", "spec_regs.sh")
    cases = [("-DRT_SPEC_KMASK=15 -DRT_SPEC_FEAT=0 -DRT_SPEC_NLIGHTS=%d -DRT_SPEC_POWBITS=6 -DRT_CULL=0" % nl, q)
             for nl in (5, 8) for q in ("false",)]

    def build(c):
        r = subprocess.run(["bash", script, c[0], "false", "false", "false", c[1]], capture_output=True, text=True,
                           timeout=600)
        return c, r.returncode, r.stdout + r.stderr

    with cf.ThreadPoolExecutor(len(cases)) as ex:
        for c, rc, out in ex.map(build, cases):
            assert rc == 0 and "error" not in out, (c, out[-2000:])
            assert ".vgpr_count" in out


def test_compiler_abort_stays_in_the_helper_process():
    """A hipRTC backend error aborts the process it runs in (round 5: "illegal
    VGPR to SGPR copy" with 5-8 lights). Compiles run in the helper process
    (csrc/rt_spec_cc), so an abort there is an ordinary compile failure here:
    RT_E_DEVICE with the reason, this process alive -- forced with the
    helper's test hook, in a fresh process."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import sys
sys.path.insert(0, %r)
from __graft_entry__ import load_package
rt = load_package()
A = rt.abi
try:
    rt.spec_precompile([A.RT_CYLINDER, A.RT_SPHERE, A.RT_PLANE], 0, 7)
    print("compiled?!")
except rt.render.RenderError as e:
    print("failed as expected:", str(e)[:200])
print("process alive")
''' % root
    env = dict(os.environ, RT_SPEC_CC_ABORT="1")
    env.pop("RT_SPEC_INPROC", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "failed as expected" in r.stdout and "signal 6" in r.stdout and "process alive" in r.stdout, r.stdout


def _spec_matrix():
    """Specialisation keys a launch can ask for (rt_kernel.hip spec_key /
    pick_schedule / pick_share / spec_for), sampled over every dimension:
    flavour (small unrolled LDS scene, larger LDS scene, global linear culled
    and brute force, BVH in LDS and global with and without the far-origin
    shift, CSG in LDS and global), schedule (serial, quads, pairs), work
    sharing (off, workgroup, device), 1..8 lights, features."""
    def key(lds, bvh, csg, nobj, kinds, kmask, feat, nl, pb, nocull, sch, share, far):
        return ":".join(str(v) for v in (lds, bvh, csg, nobj, kinds, kmask, feat, nl, pb, nocull, sch, share, far))
    cases = []
    for sch in (0, 1, 2):  # C2 / C3 shape, every schedule x sharing, lights spread over 1..8
        for share in (0, 1, 2):
            if share == 1 and sch == 2:
                continue  # (spec_for turns pairs into quads under the workgroup board)
            cases.append(key(1, 0, 0, 4, "1,3,2,0", 15, 0, 1 + (3 * sch + share) % 8, 6, 0, sch, share, 1))
    cases.append(key(1, 0, 0, 8, "0,0,0,0,1,2,3,4", 31, 7, 8, 7, 0, 0, 0, 1))  # every kind, every feature
    cases.append(key(1, 0, 0, 2, "4,0", 17, 6, 3, 7, 0, 1, 0, 1))               # cone, directional + spot
    for sch in (0, 1, 2):
        cases.append(key(1, 0, 0, 0, "", 15, 1, 2, 7, 0, sch, 0, 1))            # > 8 objects in LDS, closures
    for nl in range(1, 9):                                                      # brute force, 1..8 lights
        for sch in (0, 1):
            cases.append(key(0, 0, 0, 0, "", 3 if nl % 2 else 31, 0, nl, 6, 1, sch, 0, 1))
    cases.append(key(0, 0, 0, 0, "", 15, 0, 0, 6, 1, 1, 0, 1))                  # brute force, > 8 lights
    for sch in (0, 1):
        cases.append(key(0, 0, 0, 0, "", 15, 0, 2, 6, 0, sch, 0, 1))            # culled global stream
    for lds, far in ((1, 0), (0, 1), (0, 0)):                                   # BVH (C4 / C5 shapes)
        for sch in (0, 1, 2):
            for share in (0, 2):
                cases.append(key(lds, 1, 0, 0, "", 3, 0, 2, 6, 0, sch, share, far))
    for lds in (1, 0):                                                          # CSG (c4csg shape)
        for sch in (0, 1, 2):
            for share in (0, 1, 2):
                if share == 1 and sch == 2:
                    continue
                cases.append(key(lds, 0, 1, 0, "", 39, 0, 2 if lds else 5, 6, 0, sch, share, 1))
    return cases


def test_every_kind_of_specialisation_key_compiles():
    """The key space spec_for can request, compiled through the library's own
    path (rt_debug_spec_compile: the helper process, the options a launch
    passes), 8 at a time. No variant should first fail inside a user's
    process -- and if one ever does, it fails in the helper and the render
    falls back to the generic kernel."""
    import concurrent.futures as cf
    import ctypes
    lib = rt.load_library()
    cases = _spec_matrix()
    assert len(cases) >= 60

    def build(k):
        ms = ctypes.c_double()
        rc = lib.rt_debug_spec_compile(k.encode(), ctypes.byref(ms))
        return k, rc, (lib.rt_last_error() or b"").decode(errors="replace") if rc else ""

    bad = []
    with cf.ThreadPoolExecutor(8) as ex:
        for k, rc, msg in ex.map(build, cases):
            if rc != 0:
                bad.append((k, msg[-500:]))
    assert not bad, bad


@pytest.mark.parametrize("key", ["1:0:0", "1:0:0:4:1,3,2,0:15:0:4:6:0:3:0:1", "x:0:0:0::15:0:4:6:0:0:0:1",
                                 "1:0:0:9:1:15:0:4:6:0:0:0:1"])
def test_debug_spec_compile_rejects_malformed_keys(key):
    import ctypes
    lib = rt.load_library()
    assert lib.rt_debug_spec_compile(key.encode(), ctypes.byref(ctypes.c_double())) == A.RT_E_INVALID

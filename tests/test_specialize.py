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

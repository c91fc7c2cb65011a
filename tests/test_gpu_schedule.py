"""Work distribution on the device (needs an MI355X): the tile order dealt
from the scene-setup cost estimate, work sharing at the tail of a launch
(posted samples / refraction subtrees traced by idle lanes of the workgroup)
and launches on several streams. None of them may change a byte or a
counter: every case is checked against the CPU oracle (raytracer.go:589-682
restated, tests/oracle_bind.py).
"""
import os

import numpy as np
import pytest

import go_raytracer_amd as rt
import oracle_bind

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    """generic kernel; specialised kernel; specialised kernel with work
    sharing at the tail (rt_set_work_sharing), the workgroup board; the same
    with the device-wide board (RT_SHARE_DEVICE)"""
    import torch
    assert torch.cuda.is_available()
    g = rt.RenderContext(0)
    s = rt.RenderContext(0, specialize=True)
    s.set_work_sharing(rt.abi.RT_SHARE_OFF)  # (the default, RT_SHARE_AUTO, shares CSG scenes)
    w = rt.RenderContext(0, specialize=True)
    w.set_work_sharing(rt.abi.RT_SHARE_GROUP)
    d = rt.RenderContext(0, specialize=True)
    d.set_work_sharing(rt.abi.RT_SHARE_DEVICE)
    yield g, s, w, d
    for c in (g, s, w, d):
        c.close()


def render(ctx, packed):
    ctx.set_scene(packed)
    ctx.read_stats(reset=True)
    img = ctx.render()
    st = ctx.read_stats(reset=True)
    return img, st


def assert_same(img, ref, what):
    if not np.array_equal(img, ref):
        bad = np.argwhere((img != ref).any(axis=-1))
        y, x = bad[0]
        raise AssertionError("%s: %d pixels differ; first at (x=%d,y=%d) gpu=%s oracle=%s"
                             % (what, len(bad), x, y, img[y, x], ref[y, x]))


CASES = {
    # deep binary glass trees (raytracer.go:512-556) in few pixels per lane:
    # most lanes are idle from the start, so nearly every sample and pending
    # refraction child is posted to the board
    "c4_small": lambda: rt.configs.c4(width=72, height=40),
    "c3_small": lambda: rt.configs.c3(width=96, height=56),
    "canned_small": lambda: rt.configs.canned(width=64, height=40),
    "c4csg_small": lambda: rt.configs.c4csg(width=64, height=48),
    "c3_ragged": lambda: rt.configs.c3(width=53, height=29),  # partial tiles and half tiles
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_tile_order_and_sharing_match_oracle(ctxs, case):
    packed = rt.scene.convert(CASES[case]())
    ref, ost = oracle_bind.render_rows(packed)
    ctxs[2].set_scene(packed)
    assert ctxs[2].scene_info() & rt.abi.RT_INFO_WAVEFRONT
    assert not ctxs[2].scene_info() & rt.abi.RT_INFO_SHARE_DEVICE
    ctxs[3].set_scene(packed)
    assert ctxs[3].scene_info() & rt.abi.RT_INFO_SHARE_DEVICE
    ctxs[1].set_scene(packed)
    assert not ctxs[1].scene_info() & rt.abi.RT_INFO_WAVEFRONT
    for c in ctxs:
        try:
            for order in (True, False):
                c.set_tile_order(order)
                # pairs: samples 0-1 / 2-3 in two lanes (specialised kernel;
                # the generic and the work-sharing kernels run quads for it)
                for mode in (rt.abi.RT_SCHED_PIXEL, rt.abi.RT_SCHED_QUADS, rt.abi.RT_SCHED_PAIRS):
                    c.set_schedule(mode)
                    img, st = render(c, packed)
                    what = "%s order=%s schedule=%d" % (case, order, mode)
                    assert_same(img, ref, what)
                    assert st.as_dict() == ost.as_dict(), what
        finally:
            c.set_tile_order(True)
            c.set_schedule(rt.abi.RT_SCHED_AUTO)


def test_cost_estimate_leaves_counters_alone(ctxs):
    """The scene-setup estimate launch traces rays too; they must not reach
    the frame's counters."""
    g = ctxs[0]
    packed = rt.scene.convert(rt.configs.c3(width=128, height=72))
    g.read_stats(reset=True)
    g.set_scene(packed)
    active, ms = g.tile_order_info()
    assert active and ms > 0
    st = g.read_stats(reset=True)
    assert st.total_rays() == 0 and st.shaded_hits == 0
    ref, ost = oracle_bind.render_rows(packed)
    img = g.render()
    st = g.read_stats(reset=True)
    assert_same(img, ref, "c3 after estimate")
    assert st.as_dict() == ost.as_dict()


@pytest.mark.parametrize("which", ["share", "device", "pairs"])
def test_interleaved_shares_with_order_match_full_frame(ctxs, which):
    """Strong-scaling shares (tile rows r, r + N, ...) each get their own
    tile order; gathered, they are the oracle's frame (with work sharing, and
    in the pixel-pairs schedule)."""
    import torch
    s = {"share": ctxs[2], "device": ctxs[3], "pairs": ctxs[1]}[which]
    s.set_schedule(rt.abi.RT_SCHED_PAIRS if which == "pairs" else rt.abi.RT_SCHED_AUTO)
    args = rt.configs.c4(width=160, height=96)
    packed = rt.scene.convert(args)
    ref, ost = oracle_bind.render_rows(packed)
    s.set_scene(packed)
    s.read_stats(reset=True)
    world = 3
    nt, K = rt.dist.tile_rows(packed.height, world)
    slabs = torch.zeros((world, K * 8, packed.width, 4), dtype=torch.uint8, device="cuda:0")
    for r in range(world):
        n = max(0, min(K, (nt - r + world - 1) // world))
        s.render_tile_rows_async(r, world, n, slabs[r, : n * 8])
    torch.cuda.synchronize()
    img = rt.dist.deinterleave(slabs, packed.height).cpu().numpy()
    st = s.read_stats(reset=True)
    s.set_schedule(rt.abi.RT_SCHED_AUTO)
    assert_same(img, ref, "interleaved shares (%s)" % which)
    assert st.as_dict() == ost.as_dict()


def test_launches_on_alternating_streams(ctxs):
    """Launches alternate between two sets of queue heads; a launch on
    another stream waits for the previous one, so back-to-back launches on
    different streams render every row."""
    import torch
    g = ctxs[0]
    packed = rt.scene.convert(rt.configs.c2(width=200, height=120))
    ref, ost = oracle_bind.render_rows(packed)
    g.set_scene(packed)
    g.read_stats(reset=True)
    streams = [torch.cuda.Stream(device=0) for _ in range(3)]
    outs = [torch.zeros((120, 200, 4), dtype=torch.uint8, device="cuda:0") for _ in range(6)]
    for k, o in enumerate(outs):
        g.render_rows_async(0, 120, o, stream=streams[k % 3])
    torch.cuda.synchronize()
    for k, o in enumerate(outs):
        assert_same(o.cpu().numpy(), ref, "launch %d" % k)
    st = g.read_stats(reset=True)
    for key, v in ost.as_dict().items():
        want = [6 * x for x in v] if isinstance(v, (list, tuple)) else 6 * v
        assert st.as_dict()[key] == want, key


@pytest.mark.parametrize("specialize", [False, True])
def test_frames_in_flight_hint_keeps_bytes_and_counters(specialize):
    """rt_set_frames_in_flight(ctx, 2) lets the automatic schedule deal a whole
    4K C4 frame (depth 8, LDS scene, no CSG) serially instead of in pixel
    quads; the frame and every counter equal the default schedule's (which
    the full-size oracle tests pin)."""
    packed = rt.scene.convert(rt.configs.c4())
    a = rt.RenderContext(0, specialize=specialize)
    b = rt.RenderContext(0, specialize=specialize)
    try:
        b.set_frames_in_flight(2)
        ref, st_ref = render(a, packed)
        img, st = render(b, packed)
        assert_same(img, ref, "C4 serial (frames in flight) vs quads")
        assert st.as_dict() == st_ref.as_dict()
        with pytest.raises(rt.render.RenderError):
            b.set_frames_in_flight(0)
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("cfg,world", [("c3", 4), ("c4", 2)])
def test_frames_in_flight_shares_keep_bytes_and_counters(cfg, world):
    """Strong-scaling shares where the in-flight automatic schedule picks pixel
    pairs (C3 over 4 ranks: 10 pixels per lane; C4 over 2: 21) equal the
    default schedule's shares (quads) byte for byte and counter for counter."""
    import torch
    packed = rt.scene.convert(getattr(rt.configs, cfg)())
    a = rt.RenderContext(0, specialize=True)
    b = rt.RenderContext(0, specialize=True)
    try:
        b.set_frames_in_flight(2)
        nt, K = rt.dist.tile_rows(packed.height, world)
        n = max(0, min(K, (nt + world - 1) // world))  # rank 0's tile rows
        outs = []
        for c in (a, b):
            c.set_scene(packed)
            c.read_stats(reset=True)
            buf = torch.zeros((n * 8, packed.width, 4), dtype=torch.uint8, device="cuda:0")
            c.render_tile_rows_async(0, world, n, buf)
            torch.cuda.synchronize()
            outs.append((buf.cpu().numpy(), c.read_stats(reset=True).as_dict()))
        assert_same(outs[1][0], outs[0][0], "%s rank 0 of %d: pairs vs quads" % (cfg, world))
        assert outs[1][1] == outs[0][1]
    finally:
        a.close()
        b.close()


def test_device_sharing_full_c4csg_frame_and_shares():
    """Config 4 as stated (c4csg: cube minus 64 spheres, 4K, depth 8) with the
    device-wide board: the whole frame and each of the 8 interleaved
    strong-scaling shares (where most lanes are idle early and nearly every
    pending refraction subtree is posted) equal the unshared specialised
    kernel's -- byte for byte, counter for counter; that kernel's full frame
    is pinned against the oracle in test_gpu_parity.py."""
    import torch
    packed = rt.scene.convert(rt.configs.c4csg())
    a = rt.RenderContext(0, specialize=True)
    b = rt.RenderContext(0, specialize=True)
    try:
        a.set_work_sharing(rt.abi.RT_SHARE_OFF)
        b.set_work_sharing(rt.abi.RT_SHARE_DEVICE)
        for c in (a, b):
            c.set_scene(packed)
        assert b.scene_info() & rt.abi.RT_INFO_SHARE_DEVICE
        ref, st_ref = render(a, packed)
        img, st = render(b, packed)
        assert_same(img, ref, "c4csg device sharing, whole frame")
        assert st.as_dict() == st_ref.as_dict()
        world = 8
        nt, K = rt.dist.tile_rows(packed.height, world)
        for r in range(world):
            n = max(0, min(K, (nt - r + world - 1) // world))
            outs = []
            for c in (a, b):
                c.read_stats(reset=True)
                buf = torch.zeros((n * 8, packed.width, 4), dtype=torch.uint8, device="cuda:0")
                c.render_tile_rows_async(r, world, n, buf)
                torch.cuda.synchronize()
                outs.append((buf.cpu().numpy(), c.read_stats(reset=True).as_dict()))
            assert_same(outs[1][0], outs[0][0], "c4csg share %d of %d, device sharing" % (r, world))
            assert outs[1][1] == outs[0][1]
    finally:
        a.close()
        b.close()


BOARD_STRESS = r'''
import sys
import numpy as np
import torch
sys.path.insert(0, %r); sys.path.insert(0, %r)
from __graft_entry__ import load_package
import oracle_bind
rt = load_package()
packed = rt.scene.convert(rt.configs.c4csg())
ref, ost = oracle_bind.render_rows(packed, threads=16)
c = rt.RenderContext(0, specialize=True)
c.set_work_sharing(rt.abi.RT_SHARE_DEVICE)
c.set_scene(packed)
assert c.scene_info() & rt.abi.RT_INFO_SHARE_DEVICE
c.read_stats(reset=True)
img = c.render()
st = c.read_stats(reset=True)
bad = int((img != ref).any(axis=-1).sum())
print("whole frame: %%d pixels differ, counters %%s" %% (bad, "equal" if st.as_dict() == ost.as_dict() else "DIFFER"))
ok = bad == 0 and st.as_dict() == ost.as_dict()
world = 8
nt, K = rt.dist.tile_rows(packed.height, world)
tot = rt.abi.rt_stats()
for r in range(world):
    n = max(0, min(K, (nt - r + world - 1) // world))
    buf = torch.zeros((n * 8, packed.width, 4), dtype=torch.uint8, device="cuda:0")
    c.render_tile_rows_async(r, world, n, buf)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    for j in range(n):
        t = r + j * world
        y0, y1 = t * 8, min(packed.height, t * 8 + 8)
        if not np.array_equal(got[j * 8:j * 8 + (y1 - y0)], ref[y0:y1]):
            ok = False
            print("share %%d tile row %%d differs" %% (r, t))
st = c.read_stats(reset=True)
ok = ok and st.as_dict() == ost.as_dict()
print("shares: counters %%s" %% ("equal" if st.as_dict() == ost.as_dict() else "DIFFER"))
print("board stress ok" if ok else "board stress MISMATCH")
''' % (ROOT, os.path.join(ROOT, "tests"))


def test_device_board_stress_against_oracle():
    """The device-wide board at its most contended: every drained wave of the
    device stays as a helper (RT_GS_HELPERS far above the wave count) and busy
    waves poll the board every round (RT_GS_POLL 0) -- the full 4K c4csg
    frame and its 8 interleaved shares against the CPU oracle, bytes and
    counters (in a fresh process, so that the stress flags compile)."""
    import subprocess
    import sys
    env = dict(os.environ, RT_SPEC_EXTRA_FLAGS="-DRT_GS_HELPERS=1000000 -DRT_GS_POLL=0")
    r = subprocess.run([sys.executable, "-c", BOARD_STRESS], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "board stress ok" in r.stdout, r.stdout + r.stderr

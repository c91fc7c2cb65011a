"""rt_render_ex (include/rt_abi.h, ABI 6): the Render() seam
(raytracer.go:589-682, hooked at evaluator.go:48) over one or several GPUs of
one process, against the CPU oracle -- bytes and every counter.

One GPU box has one GPU, so the multi-device path runs on repeated device
ordinals: [0, 0, 0] gives three slots, each with its own two contexts, share
buffer, streams and copies, dealt the frame's tile rows round-robin exactly as
three GPUs would be; the gather (per-device DMA to the pinned frame, or the
xGMI peer copies and the first device's de-interleave) runs unchanged."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import go_raytracer_amd as rt
import oracle_bind

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "abi_render")
THREADS = min(16, os.cpu_count() or 8)

_oracle_cache = {}


def oracle(name, **kw):
    key = (name, tuple(sorted(kw.items())))
    if key not in _oracle_cache:
        p = rt.scene.convert(rt.configs.CONFIGS[name](**kw))
        img, st = oracle_bind.render_rows(p, threads=THREADS)
        _oracle_cache[key] = (p, img, st.as_dict())
    return _oracle_cache[key]


def c_host(p, tmp_path, gather="host", devices=()):
    """The plain-C host (tests/c/abi_render.c, file mode) rendering the scene
    through rt_render_ex."""
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "hip")], check=True)
    sp, op = tmp_path / "scene.bin", tmp_path / "out.rgba"
    rt.scene.write_scene_file(p, sp)
    r = subprocess.run([EXE, "file", str(sp), str(op), gather] + [str(d) for d in devices],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    st = json.loads(r.stdout.strip().splitlines()[-1])
    img = np.fromfile(op, dtype=np.uint8).reshape(st["height"], st["width"], 4)
    return img, st


def counters(st):
    keys = ("primary_rays", "secondary_rays", "shadow_rays", "tests", "shadow_tests", "shaded_hits", "surface_errors")
    return {k: st[k] for k in keys}


@pytest.mark.parametrize("name", ["c3", "c4csg"])
def test_c_host_render_ex_one_device_full_size(name, tmp_path):
    """device_count = 1 through the C ABI from a plain-C host: the full-size
    bench frame (C3, 3840 x 2160, depth 6) and the CSG stress frame (c4csg,
    4K depth 8) byte- and counter-equal to the oracle."""
    p, ref, ost = oracle(name)
    img, st = c_host(p, tmp_path, "host", [0])
    assert st["devices"] == 1 and st["device_kernel_ms"][0] > 0
    assert np.array_equal(img, ref)
    assert counters(st) == ost


@pytest.mark.parametrize("gather,devices", [("host", [0, 0, 0]), ("peer", [0, 0])])
def test_c_host_render_ex_shares_full_size_c3(gather, devices, tmp_path):
    """The full 4K C3 frame dealt over 3 (host gather) or 2 (xGMI peer gather)
    device slots from the C host equals the oracle."""
    p, ref, ost = oracle("c3")
    img, st = c_host(p, tmp_path, gather, devices)
    assert st["devices"] == len(devices) and all(v > 0 for v in st["device_kernel_ms"])
    assert np.array_equal(img, ref)
    assert counters(st) == ost


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0], [0] * 8])
@pytest.mark.parametrize("gather", ["host", "peer"])
@pytest.mark.parametrize("name,size", [("c2", (160, 90)), ("c4", (77, 53)), ("canned", (120, 77))])
def test_render_ex_shares_equal_oracle(name, size, gather, devices):
    """Reduced frames (ragged heights) over 1/2/3/8 device slots, both gathers:
    bytes and summed counters equal the oracle; telemetry per device."""
    p, ref, ost = oracle(name, width=size[0], height=size[1])
    img, st, tm = rt.render_frame(p, devices=devices, gather=gather)
    assert np.array_equal(img, ref)
    assert st.as_dict() == ost
    assert st.devices == tm.devices == len(devices)
    trows = (size[1] + 7) // 8
    for d in range(len(devices)):
        assert (st.device_kernel_ms[d] > 0) == (d < trows)
    assert st.kernel_ms == pytest.approx(max(st.device_kernel_ms[:len(devices)]))
    assert st.gather_ms >= 0


def test_render_ex_8_slots_c4csg_full_size():
    """The CSG stress frame at its stated size over 8 device slots (its
    BASELINE row is 'row-tiled across 8 GPUs + gather'), host gather."""
    p, ref, ost = oracle("c4csg")
    img, st, tm = rt.render_frame(p, devices=[0] * 8)
    assert np.array_equal(img, ref)
    assert st.as_dict() == ost
    assert st.devices == 8


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_render_ex_device_output(devices):
    """RT_RENDER_OUT_DEVICE: the frame gathered into the caller's device
    buffer on the first device (one device: rendered straight into it)."""
    import torch
    p, ref, ost = oracle("c2", width=96, height=61)
    lib = rt.load_library()
    out = torch.full((p.height, p.width, 4), 7, dtype=torch.uint8, device="cuda:0")
    o = rt.render.render_opts(devices, gather="peer", out_device=True)
    st = rt.abi.rt_stats()
    rc = lib.rt_render_ex(p.ref(), ctypes.byref(o), ctypes.c_void_p(out.data_ptr()), ctypes.byref(st))
    assert rc == 0, lib.rt_last_error()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert st.as_dict() == ost


def test_render_ex_scene_change_reaches_every_slot():
    """A changed scene is converted once and cloned to every context of every
    slot; an in-place material change is seen on all of them."""
    p, ref, ost = oracle("c3", width=96, height=54)
    img, st, tm = rt.render_frame(p, devices=[0, 0, 0])
    assert np.array_equal(img, ref) and st.as_dict() == ost
    img, st, tm = rt.render_frame(p, devices=[0, 0, 0])
    assert tm.scene_reused == 1 and np.array_equal(img, ref)
    m = p._materials
    old = m[0].color[0]
    m[0].color[0] = 0.25 if old != 0.25 else 0.5
    try:
        ref2, ost2 = oracle_bind.render_rows(p, threads=THREADS)
        img2, st2, tm2 = rt.render_frame(p, devices=[0, 0, 0])
        assert tm2.scene_reused == 0
        assert np.array_equal(img2, ref2) and st2.as_dict() == ost2.as_dict()
    finally:
        m[0].color[0] = old


def test_render_ex_rejects_bad_options():
    lib = rt.load_library()
    p = rt.scene.convert(rt.configs.c1(width=16, height=16))
    out = np.empty((16, 16, 4), np.uint8)
    o = rt.render.render_opts([99])
    assert lib.rt_render_ex(p.ref(), ctypes.byref(o), out.ctypes.data_as(ctypes.c_void_p), None) == rt.abi.RT_E_INVALID
    o = rt.render.render_opts()
    o.flags = 1 << 20
    assert lib.rt_render_ex(p.ref(), ctypes.byref(o), out.ctypes.data_as(ctypes.c_void_p), None) == rt.abi.RT_E_INVALID
    o = rt.render.render_opts(gather="host", out_device=True)
    assert lib.rt_render_ex(p.ref(), ctypes.byref(o), out.ctypes.data_as(ctypes.c_void_p), None) == rt.abi.RT_E_INVALID


FIRST_CALL = r'''
import ctypes, json, sys, time
import numpy as np
sys.path.insert(0, %r); sys.path.insert(0, %r)
from __graft_entry__ import load_package
import oracle_bind
rt = load_package()
name, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
p = rt.scene.convert(rt.configs.CONFIGS[name](width=w, height=h))
ref, ost = oracle_bind.render_rows(p, threads=16)
out = np.empty((h, w, 4), np.uint8)
calls = []
t_end = time.time() + 120
while True:
    t0 = time.perf_counter()
    img, st, tm = rt.render_frame(p, out=out)
    calls.append({"ms": (time.perf_counter() - t0) * 1e3, "specialized": tm.specialized,
                  "pending": tm.pending_compiles, "equal": bool(np.array_equal(img, ref)),
                  "counters": st.as_dict() == ost.as_dict()})
    if tm.specialized or time.time() > t_end:
        break
    time.sleep(0.05)
print(json.dumps(calls))
''' % (ROOT, os.path.join(ROOT, "tests"))


@pytest.mark.parametrize("name,size", [("c3", (3840, 2160)), ("c4csg", (960, 540))])
def test_first_call_renders_generic_then_switches(name, size):
    """A fresh process's first Render() of a new scene shape does not wait for
    hipRTC: it renders with the generic kernel (same bytes and counters) while
    the specialised kernel compiles in the background, and a later call
    switches to it -- bytes and counters equal the oracle before and after."""
    r = subprocess.run([sys.executable, "-c", FIRST_CALL, name, str(size[0]), str(size[1])],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    calls = json.loads(r.stdout.strip().splitlines()[-1])
    assert calls[0]["specialized"] == 0 and calls[0]["pending"] >= 1, calls[0]
    assert calls[-1]["specialized"] == 1, calls[-1]
    assert all(c["equal"] and c["counters"] for c in calls), calls
    print("first call %.1f ms, %d calls to switch, steady %.1f ms" % (calls[0]["ms"], len(calls), calls[-1]["ms"]))


ENV_RACE = r'''
import ctypes, os, sys, threading, time
import numpy as np
sys.path.insert(0, %r); sys.path.insert(0, %r)
from __graft_entry__ import load_package
import oracle_bind
rt = load_package()
# Load the library and initialise the HIP runtime before the churn starts:
# the library copies the environment when it loads, and HIP's own first-call
# initialisation reads dozens of variables with glibc's lock-free getenv --
# code this library cannot guard (it segfaulted there once, mid-churn). Every
# compile and render below runs while the environment is being rewritten.
rt.render_frame(rt.scene.convert(rt.configs.c1(width=16, height=16)), generic=True)
stop = False
def churn():
    k = 0
    while not stop:
        for i in range(300):
            os.environ["RT_ENV_CHURN_%%d" %% i] = "x" * (k %% 97)
        for i in range(300):
            del os.environ["RT_ENV_CHURN_%%d" %% i]
        k += 1
t = threading.Thread(target=churn); t.start()
ok = True
try:
    for cfg in (rt.configs.c2(width=72, height=40), rt.configs.canned(width=56, height=36)):
        p = rt.scene.convert(cfg)
        ref, ost = oracle_bind.render_rows(p, threads=8)
        img, st, tm = rt.render_frame(p, spec_sync=True)
        ok = ok and tm.specialized == 1 and np.array_equal(img, ref) and st.as_dict() == ost.as_dict()
finally:
    stop = True
    t.join()
print("env race ok" if ok else "env race MISMATCH")
''' % (ROOT, os.path.join(ROOT, "tests"))


def test_hiprtc_compiles_while_another_thread_rewrites_the_environment():
    """Regression test of round 5's rt_set_scene segfault: two new-shape
    specialisations compile (synchronously, in a fresh process) and render
    while a second thread grows and shrinks os.environ by 300 keys at a time;
    the library reads only its load-time copy of the environment (knobs, the
    compile helper's and the in-process compiler's environment), and the bytes
    equal the oracle. The library is loaded and HIP initialised before the
    churn starts (HIP's initialisation reads the live environment itself)."""
    r = subprocess.run([sys.executable, "-c", ENV_RACE], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "env race ok" in r.stdout, r.stdout + r.stderr

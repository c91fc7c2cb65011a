"""The library's view of the process environment (CPU, no device): it reads a
copy taken when it loads (csrc/rt_kernel.hip env_snap), never the live
environment, so a host thread rewriting os.environ while a render or compile
runs cannot pull strings out from under it (the round-6 segfault of
tests/test_gpu_render_ex.py's environment-race test was a per-call getenv in
the band plan). Each case runs in a fresh process: the copy is per process."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LOAD = r'''
import os, sys, threading
sys.path.insert(0, %r)
from __graft_entry__ import load_package
rt = load_package()
lib = rt.render.load_library()
''' % ROOT


def _run(code, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", LOAD + code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_knobs_come_from_the_load_time_copy():
    out = _run(r'''
os.environ["RT_ENV_PROBE"] = "after"
os.environ["RT_ENV_NEW"] = "x"
del os.environ["RT_ENV_GONE"]
print(lib.rt_debug_getenv(b"RT_ENV_PROBE"), lib.rt_debug_getenv(b"RT_ENV_NEW"), lib.rt_debug_getenv(b"RT_ENV_GONE"),
      lib.rt_debug_getenv(b"RT_ENV"), lib.rt_debug_getenv(None))
''', {"RT_ENV_PROBE": "before", "RT_ENV_GONE": "still"})
    # set before the load: seen; set or removed after it: not; prefixes do not match
    assert out.split() == ["b'before'", "None", "b'still'", "None", "None"], out


def test_library_reads_survive_a_thread_rewriting_the_environment():
    out = _run(r'''
stop = False
def churn():
    k = 0
    while not stop:
        for i in range(300):
            os.environ["RT_ENV_CHURN_%d" % i] = "x" * (k % 97)
        for i in range(300):
            del os.environ["RT_ENV_CHURN_%d" % i]
        k += 1
t = threading.Thread(target=churn)
t.start()
ok = True
try:
    for _ in range(100000):
        ok = ok and lib.rt_debug_getenv(b"RT_ENV_PROBE") == b"kept" and lib.rt_debug_getenv(b"RT_ENV_CHURN_7") is None
finally:
    stop = True
    t.join()
print("ok" if ok else "changed")
''', {"RT_ENV_PROBE": "kept"})
    assert out.strip() == "ok", out

"""Generic (non-specialised) kernel of one or more library builds against the
oracle on a reduced config, in every schedule, tile order on and off, through
the bare C ABI (builds from earlier trees lack later entry points).
usage: python3 scripts/generic_parity.py CFG W H lib1.so [lib2.so ...]"""
import ctypes as C
import os
import shutil
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from __graft_entry__ import load_package  # noqa: E402


def main():
    cfg, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    pkg = load_package()
    import oracle_bind
    import torch
    torch.cuda.set_device(0)
    packed = pkg.scene.convert(pkg.configs.CONFIGS[cfg](width=w, height=h))
    ref, ost = oracle_bind.render_rows(packed)
    out = torch.empty((h, w, 4), dtype=torch.uint8, device="cuda")
    tmp = tempfile.mkdtemp()
    bad_any = False
    for k, path in enumerate(sys.argv[4:]):
        cp = os.path.join(tmp, "v%d_%s" % (k, os.path.basename(path)))
        shutil.copy(path, cp)
        l = C.CDLL(cp)
        l.rt_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        l.rt_set_scene.argtypes = [C.c_void_p, C.c_void_p]
        l.rt_set_schedule.argtypes = [C.c_void_p, C.c_int]
        l.rt_set_tile_order.argtypes = [C.c_void_p, C.c_int]
        l.rt_render_rows_async.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        l.rt_read_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        l.rt_last_error.restype = C.c_char_p
        hd = C.c_void_p()
        assert l.rt_create(0, C.byref(hd)) == 0, l.rt_last_error()
        for order in (1, 0):
            for mode in (pkg.abi.RT_SCHED_PIXEL, pkg.abi.RT_SCHED_QUADS):
                assert l.rt_set_tile_order(hd, order) == 0
                assert l.rt_set_schedule(hd, mode) == 0
                assert l.rt_set_scene(hd, packed.ref()) == 0, l.rt_last_error()
                st = pkg.abi.rt_stats()
                l.rt_read_stats(hd, None, 1, C.byref(st))
                out.zero_()
                assert l.rt_render_rows_async(hd, 0, h, C.c_void_p(out.data_ptr()), None) == 0, l.rt_last_error()
                rc = l.rt_read_stats(hd, None, 1, C.byref(st))
                img = out.cpu().numpy()
                bad = (img != ref).any(axis=-1)
                eq = st.as_dict() == ost.as_dict()
                bad_any = bad_any or bad.any() or not eq or rc != 0
                tiles = sorted({(int(y) // 8, int(x) // 8) for y, x in np.argwhere(bad)})
                print("%s order=%d mode=%d rc=%d differ=%d tiles=%d stats_equal=%s" %
                      (os.path.basename(path), order, mode, rc, int(bad.sum()), len(tiles), eq), flush=True)
    sys.exit(1 if bad_any and os.environ.get("STRICT") else 0)


if __name__ == "__main__":
    main()

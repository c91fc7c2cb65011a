"""Diagnostic: one reduced config through the generic and specialised kernels
in both schedules, tile order on and off, each compared with the oracle.
usage: python3 scripts/diag_parity.py c4 96 64"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from __graft_entry__ import load_package
rt = load_package()
import oracle_bind

cfg, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
packed = rt.scene.convert(getattr(rt.configs, cfg)(width=w, height=h))
ref, ost = oracle_bind.render_rows(packed)
for spec in (False, True):
    c = rt.RenderContext(0, specialize=spec)
    for order in (True, False):
        c.set_tile_order(order)
        for mode in (rt.abi.RT_SCHED_PIXEL, rt.abi.RT_SCHED_QUADS):
            c.set_schedule(mode)
            c.set_scene(packed)
            c.read_stats(reset=True)
            img = c.render()
            st = c.read_stats(reset=True)
            bad = (img != ref).any(axis=-1)
            print("spec=%d order=%d mode=%d differ=%d stats_equal=%s" % (spec, order, mode, bad.sum(), st.as_dict() == ost.as_dict()), flush=True)
    c.close()

if os.environ.get("DIAG_DETAIL"):
    c = rt.RenderContext(0)
    c.set_tile_order(False)
    c.set_schedule(rt.abi.RT_SCHED_PIXEL)
    c.set_scene(packed)
    c.read_stats(reset=True)
    img = c.render()
    st = c.read_stats(reset=True).as_dict()
    for k, v in ost.as_dict().items():
        if st[k] != v:
            print("counter", k, "gpu", st[k], "oracle", v)
    bad = (img != ref).any(axis=-1)
    ys, xs = np.nonzero(bad)
    tiles = sorted(set((int(y) // 8, int(x) // 8) for y, x in zip(ys, xs)))
    print("tiles (ty,tx) with differing pixels:", len(tiles), tiles[:40])
    for ty, tx in tiles[:3]:
        print("tile", ty, tx, "differing pixels:", int(bad[ty*8:ty*8+8, tx*8:tx*8+8].sum()))
    print(bad[:, :].astype(int).sum(axis=0).tolist())
    print(bad[:, :].astype(int).sum(axis=1).tolist())
    for y, x in list(zip(ys, xs))[:8]:
        print((int(x), int(y)), img[y, x].tolist(), ref[y, x].tolist())
    c.close()

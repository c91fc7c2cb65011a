"""Per-pixel BVH node-visit map (diagnostic build -DRT_COST_MAP).

usage: RT_AMD_LIB=build_variants/librtamd_cost.so python scripts/cost_map.py c5 480 270 out.npy
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402


def main():
    cfg, w, h, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    rt = load_package()
    ctx = rt.RenderContext(0)
    packed = rt.scene.convert(rt.configs.CONFIGS[cfg](width=w, height=h))
    ctx.set_scene(packed)
    img = ctx.render()
    cost = np.ascontiguousarray(img).view(np.uint32).reshape(h, w)
    np.save(out, cost)
    flat = np.sort(cost.ravel())
    print("mean %.1f p50 %d p90 %d p99 %d p99.9 %d max %d" % (
        flat.mean(), flat[len(flat) // 2], flat[int(len(flat) * 0.9)], flat[int(len(flat) * 0.99)],
        flat[int(len(flat) * 0.999)], flat[-1]))
    y, x = np.unravel_index(np.argmax(cost), cost.shape)
    print("max at x=%d y=%d" % (x, y))
    # 8x8 tile sums (one wave chunk each)
    t = cost[:h // 8 * 8, :w // 8 * 8].reshape(h // 8, 8, w // 8, 8).sum(axis=(1, 3))
    top = np.argsort(cost.ravel())[::-1][:int(os.environ.get("COST_TOP", "20"))]
    for k in top:
        yy, xx = divmod(int(k), w)
        print("  pixel x=%d y=%d cost %d" % (xx, yy, cost[yy, xx]))
    ts = np.sort(t.ravel())
    print("tile sums: mean %.0f max %d top5 %s" % (ts.mean(), ts[-1], ts[-5:].tolist()))
    ty, tx = np.unravel_index(np.argmax(t), t.shape)
    print("worst tile x=%d..%d y=%d..%d" % (tx * 8, tx * 8 + 7, ty * 8, ty * 8 + 7))
    ctx.close()


if __name__ == "__main__":
    main()

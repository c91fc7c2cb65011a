"""Strong-scaling rehearsal on ONE GPU: the kernel time of rank 0's share of a
frame (interleaved 8-row tile rows, stride = world) for world = 1, 2, 4, 8, as
bench.py --scaling strong would launch it on each rank (no collective here).
efficiency(world) = t(1) / (world * t(world)); with STRONG_ALL_RANKS=1 (default)
every rank's share is timed too and w<N>_eff_max uses the slowest one.
usage: python scripts/strong_emul.py [config] [steps]   (STRONG_WORLDS=1,2,4,8 by default;
STRONG_SHARING=1: the context compiled with work sharing)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    pkg = load_package()
    import torch
    torch.cuda.set_device(0)
    packed = pkg.scene.convert(pkg.configs.CONFIGS[cfg]())
    ctx = pkg.RenderContext(0, specialize=True)
    if os.environ.get("STRONG_SHARING") == "1":  # work sharing at the tail (rt_set_work_sharing)
        ctx.set_work_sharing(True)
    ctx.set_scene(packed)
    out = {"config": cfg}
    t1 = None
    worlds = [int(w) for w in os.environ.get("STRONG_WORLDS", "1,2,4,8").split(",")]
    all_ranks = os.environ.get("STRONG_ALL_RANKS", "1") == "1"

    def share_ms(rank, world):
        dr = pkg.dist.DistributedRenderer(ctx, packed, rank, world, torch.device("cuda", 0), mode="interleaved")
        for _ in range(3):
            dr.step(gather=False)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        t0 = time.perf_counter()
        for k in range(steps):
            dr.step(gather=False, events=ev[k])
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / steps * 1e3
        return sorted(a.elapsed_time(b) for a, b in ev)[steps // 2], wall

    for world in worlds:
        ms, wall = share_ms(0, world)
        out["w%d_wall_ms" % world] = round(wall, 4)
        t1 = t1 or ms
        out["w%d_ms" % world] = round(ms, 4)
        out["w%d_eff" % world] = round(t1 / (world * ms), 3)
        if all_ranks and world > 1:
            # the driver's step time is the slowest rank's share, not rank 0's
            mx = max([ms] + [share_ms(r, world)[0] for r in range(1, world)])
            out["w%d_max_ms" % world] = round(mx, 4)
            out["w%d_eff_max" % world] = round(t1 / (world * mx), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

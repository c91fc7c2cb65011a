"""Frames in flight on ONE GPU: wall time per frame (or per rank share of a
frame, interleaved 8-row tile rows, stride = world) when F contexts, each with
its own stream, queue sets, frame stack and output buffer, render consecutive
frames round-robin, so frame k+1's workgroups fill the CUs that frame k's tail
leaves idle. F = 1 is the serial baseline (one context, one stream).
w<N>_f<F>_eff_max = t(1 rank, F) / (N * slowest rank's share time at F): the
efficiency the driver's 1/2/4/8-GPU bench lines give (every line runs F).
usage: python scripts/inflight_emul.py [config] [steps]
       (INFLIGHT_WORLDS=1,8  INFLIGHT_F=1,2,3  INFLIGHT_RANKS=all|0  INFLIGHT_SHARE=0|1|2  INFLIGHT_SCHED=pixel|quads|pairs  INFLIGHT_HINT=1|0:
        rt_set_frames_in_flight(F) on the contexts, as bench.py does)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    pkg = load_package()
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    packed = pkg.scene.convert(pkg.configs.CONFIGS[cfg]())
    fs = [int(v) for v in os.environ.get("INFLIGHT_F", "1,2,3").split(",")]
    worlds = [int(w) for w in os.environ.get("INFLIGHT_WORLDS", "1,2,4,8").split(",")]
    all_ranks = os.environ.get("INFLIGHT_RANKS", "all") == "all"
    ctxs = []
    for _ in range(max(fs)):
        c = pkg.RenderContext(0, specialize=True)
        if os.environ.get("INFLIGHT_SHARE", "auto") != "auto":  # 0 off, 1 group, 2 device, 3 auto (default)
            c.set_work_sharing(int(os.environ["INFLIGHT_SHARE"]))
        sched = os.environ.get("INFLIGHT_SCHED")  # pixel / quads / pairs (default: auto)
        if sched:
            c.set_schedule({"pixel": pkg.abi.RT_SCHED_PIXEL, "quads": pkg.abi.RT_SCHED_QUADS,
                            "pairs": pkg.abi.RT_SCHED_PAIRS}[sched])
        c.set_scene(packed)
        ctxs.append(c)
    streams = [torch.cuda.Stream(dev) for _ in ctxs]
    out = {"config": cfg, "steps": steps, "work_sharing": os.environ.get("INFLIGHT_SHARE", "auto")}

    def wall_ms(F, rank, world):
        drs = [pkg.dist.DistributedRenderer(ctxs[i], packed, rank, world, dev, mode="interleaved")
               for i in range(F)]
        nt = drs[0].ntrows
        if os.environ.get("INFLIGHT_HINT", "1") == "1":  # rt_set_frames_in_flight, as bench.py does
            for c in ctxs[:F]:
                c.set_frames_in_flight(F)

        def launch(k):
            i = k % F
            if nt > 0:
                ctxs[i].render_tile_rows_async(rank, world, nt, drs[i].buf[: nt * 8], stream=streams[i])
        for k in range(2 * F):
            launch(k)
        torch.cuda.synchronize()
        for c in ctxs[:F]:
            c.read_stats(reset=True)
        t0 = time.perf_counter()
        for k in range(steps):
            launch(k)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps * 1e3
        rays = sum(c.read_stats(reset=True).total_rays() for c in ctxs[:F])
        return dt, rays / steps

    t1 = {}
    for world in worlds:
        for F in fs:
            ranks = range(world) if (all_ranks and world > 1) else [0]
            res = [wall_ms(F, r, world) for r in ranks]
            mx = max(ms for ms, _ in res)
            key = "w%d_f%d" % (world, F)
            out[key + "_ms"] = round(res[0][0], 4)
            out[key + "_max_ms"] = round(mx, 4)
            out[key + "_rays"] = int(sum(r for _, r in res))
            if world == 1:
                t1[F] = mx
            # the driver's efficiency: its own N=1 line runs the same F
            if t1.get(F):
                out[key + "_eff_max"] = round(t1[F] / (world * mx), 3)
            if t1.get(1):
                out[key + "_eff_vs_serial_frame"] = round(t1[1] / (world * mx), 3)
            print(key, round(res[0][0], 4), round(mx, 4), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

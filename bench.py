#!/usr/bin/env python3
"""Benchmark of the render hot path (BASELINE.json metric: Mrays/s at 4K depth 6).

One step = one frame of the workload with its 8-row tile rows dealt
round-robin across the N ranks and gathered to rank 0 over RCCL (default
--scaling strong --shard interleaved: BASELINE.json north_star's "image rows
shard across the GPUs with a final RCCL gather"; at N=1 the single rank
renders the whole frame and nothing is exchanged), or, with --scaling weak, a
batch of N frames, one per GPU, with no data-path collective. One process per
GPU. Workload = config C3 (3840x2160, depth 6, cylinder + cube +
sphere-for-cone, 4 lights).

Frames in flight (--inflight F; default 2, 3 for C3 shares at >= 4 ranks,
inflight_default): each rank holds F render contexts
with the scene and launches consecutive steps on them round-robin, one stream
each, so the next frame's workgroups take the CUs the current frame's last
waves leave idle. Each step still renders its whole frame (or share) into its
own buffer; kernel_ms (the roofline's time) is then the GPU span per frame, not
one launch's start-to-end duration, which overlaps its neighbours
(roofline.launch_ms_overlapped).

Rays = primary + secondary + shadow, counted on the device with the same rule
as the CPU oracle (include/rt_abi.h rt_stats). value = rays of all ranks per
step / max-over-ranks step time.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from __graft_entry__ import load_package  # noqa: E402

# MI355X peaks (MI355X_MICROARCH.md; FP64 vector = 256 CU x 128 flop/clk x 2.4 GHz)
PEAK_FP64_TFLOPS = 78.6
PEAK_FP64_NOFMA_TFLOPS = 39.3  # parity build: no contraction -> one mul or add per lane-op
PEAK_HBM_GBS = 8000.0
METRIC = "Mrays/s (primary+shadow+reflect) at 4K depth=6; 1/2/4/8-GPU scaling"  # BASELINE.json "metric"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="c3")
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    p.add_argument("--cpu-threads", type=int, default=8)
    p.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                   help="strong (default): one frame's rows sharded over the ranks + RCCL gather to "
                        "rank 0; weak: every rank renders its own full frame (no collective)")
    p.add_argument("--shard", choices=["interleaved", "bands"], default="interleaved",
                   help="row partition for --scaling strong")
    p.add_argument("--accel", choices=["bvh", "none"], default="bvh",
                   help="none: the reference's brute-force search (no BVH, no culling; identical pixels "
                        "and counters) -- BASELINE config 5's regime, the FP64 roofline of the Intersect loop")
    p.add_argument("--rows", default=None, metavar="Y0:Y1",
                   help="render only rows [Y0, Y1) of the full-size frame (one GPU): a full-width row "
                        "band of a config too costly to render whole (brute-force C5 at 7680x4320)")
    p.add_argument("--companion", choices=["auto", "off"], default="auto",
                   help="c3: also time c3cone (C3 with the cone) for the line's c3cone field; "
                        "off in profiling runs, whose counters must come from C3 frames only")
    p.add_argument("--inflight", type=int, default=None,
                   help="frames in flight per rank: F render contexts with the same scene on F streams "
                        "render consecutive frames round-robin, so one frame's tail overlaps the next "
                        "frame's head (every frame still rendered whole; 1 = serial launches). Default "
                        "(inflight_default): 2, or 3 for the C3 scenes' strong-scaling shares at >= 4 ranks")
    p.add_argument("--schedule", choices=["auto", "pixel", "quads", "pairs"], default="auto",
                   help="rt_set_schedule: how pixels are dealt to lanes (identical pixels and counters); "
                        "auto picks from depth, pixels per lane and frames in flight. The PMC passes run "
                        "--inflight 1 with the schedule the in-flight bench picks")
    p.add_argument("--work-sharing", choices=["auto", "on", "group", "device", "off"], default="auto",
                   help="rt_set_work_sharing: tail work sharing compiled into the specialised kernel "
                        "(on = group: a per-workgroup LDS board; device: a device-wide board in HBM; "
                        "auto, the library default: device for CSG scenes at depth >= 7 on strong-scaling "
                        "shares or without frames in flight)")
    p.add_argument("--specialize", choices=["on", "off"], default="on",
                   help="scene-specialised kernel for small linear scenes (hipRTC, compiled once "
                        "before the warmup; bit-identical output)")
    p.add_argument("--api", action="store_true",
                   help="time the reference's seam instead: ONE process renders each step through rt_render_ex "
                        "(include/rt_abi.h ABI 6, the Render() replacement) over --gpus N devices (tile rows dealt "
                        "round-robin, the frame gathered into pageable host memory); no torch.distributed")
    p.add_argument("--api-devices", default=None, metavar="D0,D1,...",
                   help="--api: explicit device ordinals (repeats allowed: one GPU rendering several shares, "
                        "a one-GPU rehearsal of the N-device path)")
    p.add_argument("--gather", choices=["auto", "host", "peer"], default="auto",
                   help="--api: host = each device DMAs its share to the pinned frame over its own PCIe link; "
                        "peer = shares copied to the first device over xGMI, one DMA to the host")
    p.add_argument("--launch-selftest", action="store_true",
                   help="CPU test of the N-rank launch and telemetry path: gloo ranks, synthetic "
                        "per-rank times, no device (tests/test_bench_launch.py)")
    return p.parse_args()


def inflight_default(args, world):
    """Frames in flight when --inflight is not given: 2, and 3 for C3 / c3cone
    shares of a strong-scaling frame over >= 4 ranks. A share there is 5-10
    pixels per lane, so its last deep-glass pixels leave the device idle for
    longer relative to the share, and a third frame fills that tail: the
    1-GPU rehearsal of every rank's C3 share (scripts/inflight_emul.py,
    profiles/r05/share_f3/) gives 8 ranks 0.446-0.451 -> 0.425-0.427 ms and
    4 ranks 0.824-0.838 -> 0.810-0.815 ms, while whole frames (3.04 vs 2.99 ms)
    and C4's shares are slower with three."""
    small_linear = args.config in ("c3", "c3cone") and args.rows is None and args.accel != "none"
    return 3 if (args.scaling == "strong" and world >= 4 and small_linear) else 2


def spawn_ranks(n):
    """`python3 bench.py --gpus N` without a launcher: start the N rank
    processes here, before anything touches a GPU (one process per GPU,
    LOCAL_RANK = RANK, rendezvous on 127.0.0.1), wait for them, and return the
    worst exit status. A rank that fails stops the others. Rank 0 prints the
    JSON line."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for q in live:  # one rank failed: the collectives of the others would hang
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def telemetry(rank_rows):
    """The N>1 line's per-rank fields from rank_table rows [render span per
    step (GPU ms), gather cost per frame (ms, -1 = none), wall time (s)]."""
    per = [{"rank": r, "render_span_ms": round(v[0], 4),
            "gather_ms": None if v[1] < 0 else round(v[1], 4),
            "wall_ms_per_step": round(v[2], 4)} for r, v in enumerate(rank_rows)]
    slow = max(range(len(per)), key=lambda r: per[r]["render_span_ms"])
    g = [p["gather_ms"] for p in per if p["gather_ms"] is not None]
    return {"per_rank_ms": per, "slowest_rank": slow,
            "gather_ms": {"mean": round(sum(g) / len(g), 4), "max": round(max(g), 4)} if g else None}


def launch_selftest(args):
    """Each rank of a gloo world reports synthetic times through the same
    rank_table / telemetry path the GPU bench uses; rank 0 prints one line."""
    import torch.distributed as dist
    pkg = load_package()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    rows = pkg.dist.rank_table([1.0 + rank, 0.25 * (rank + 1) if world > 1 else -1.0, 2.0 + rank])
    mx, sm = pkg.dist.reduce_max_sum([2.0 + rank, 10.0])
    if rank == 0:
        line = {"metric": METRIC, "n_gpus": world, "selftest": True, "max_wall": mx[0], "sum_rays": sm[1]}
        line.update(telemetry(rows))
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(config):
    """HBM bytes per launch of the render kernel from the committed rocprofv3
    --pmc passes (profiles/traffic_<config>.json, scripts/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", "traffic_%s.json" % config)
    if not os.path.exists(path):
        return None, None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("traffic_bytes"), os.path.relpath(path, ROOT), d.get("kernel_src")


def pmc_executed(key):
    """Executed-work counters of the render kernel for this workload from the
    committed rocprofv3 --pmc summary (profiles/pmc_<key>.json, written by
    scripts/pmc_roofline.py from passes over the same kernel build)."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % key)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        return json.load(f), os.path.relpath(path, ROOT)


def host_cpu():
    """(model name, logical CPUs of the machine, CPUs this process may use).
    On the GPU box nproc / os.cpu_count() count the whole machine; the job's
    share is its affinity mask, further capped by OMP_NUM_THREADS when set
    (16 per GPU there)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    ncpu = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = ncpu
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        avail = min(avail, int(omp))
    return model, ncpu, avail


def cpu_sample(packed, threads, budget_s):
    """The CPU oracle (C restatement of the Go path) on this host, `threads`
    workers over (column, 20-row) strips like raytracer.go:611-677, on a
    bounded sample: SURVEY.md 8(d)'s subset -- the first rows of the frame,
    up to 40 (two 20-row strips per column), extrapolated by ray count --
    doubled from one row until it takes about budget_s / 2; a frame the
    budget covers whole (C3: ~1.6 s) is timed whole. C5 brute force (100 k
    spheres, every ray testing all of them) reaches only a few of the 40
    rows within the budget: the line says how many."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind
    H = packed.height
    rows = 1
    while True:
        y0, y1 = 0, min(H, rows)
        t0 = time.perf_counter()
        _, st = oracle_bind.render_rows(packed, y0, y1, threads=threads)
        dt = time.perf_counter() - t0
        if dt >= budget_s / 2 or y1 == H or (y1 >= 40 and dt * (H / y1) > budget_s):
            break
        rows = min(H, rows * 2 if dt > 0.05 else rows * 8)
        if y1 >= 40 and rows > 40 and dt * (rows / y1) > budget_s and dt * (H / y1) > budget_s:
            break
    rays = st.total_rays()
    what = "full %dx%d frame" % (packed.width, H) if y1 == H else \
        "rows 0..%d (the first rows: SURVEY 8(d)'s 40-row subset%s) of the %dx%d frame" % (
            y1, "" if y1 >= 40 else ", cut to the time budget", packed.width, H)
    return rays / dt / 1e6, "%s of the same scene (%d rays, %.2f s wall)" % (what, rays, dt)


def cpu_baseline(packed, threads, budget_s=10.0):
    """cpu_baseline: `value` with the reference's fixed 8 render workers
    (raytracer.go:725 numRenderThreads) and an extra run on every CPU this job
    may use; oracle built -O3 -ffp-contract=off (oracle/Makefile)."""
    model, ncpu, avail = host_cpu()
    v, sample = cpu_sample(packed, threads, budget_s)
    out = {"value": v, "unit": "Mrays/s", "cores": threads, "kind": "port", "sample": sample,
           "cpu_model": model, "nproc": ncpu, "cpus_available": avail}
    if avail != threads:
        va, sa = cpu_sample(packed, avail, budget_s)
        out["all_cores"] = {"value": va, "cores": avail, "sample": sa}
    return out


def gpu_span_ms(evs):
    """GPU time per frame over a timed run: first launch's start event to the
    latest end event, divided by the frame count (HIP events on the launch
    streams). With frames in flight, launches overlap, so this -- not the
    average start-to-end duration of one launch -- is the kernel time a
    frame costs."""
    span = max(evs[0][0].elapsed_time(e1) for _, e1 in evs)
    return span / len(evs)


def make_contexts(pkg, dev, packed, n, specialize, accel=None, schedule="auto", sharing=None):
    ctxs = []
    for _ in range(n):
        c = pkg.RenderContext(dev.index, specialize=specialize)
        if sharing is not None:  # (None: the library's default, RT_SHARE_AUTO)
            c.set_work_sharing(int(sharing))
        if accel is not None:
            c.set_accel(accel)
        c.set_schedule({"auto": pkg.abi.RT_SCHED_AUTO, "pixel": pkg.abi.RT_SCHED_PIXEL,
                        "quads": pkg.abi.RT_SCHED_QUADS, "pairs": pkg.abi.RT_SCHED_PAIRS}[schedule])
        c.set_frames_in_flight(n)  # the automatic schedule knows the launches overlap
        c.set_scene(packed)
        ctxs.append(c)
    return ctxs


def side_config(pkg, name, dev, specialize, inflight, streams=None, steps=10, warmup=2):
    """One GPU, whole frames of another config (the C3 line's companion: C3 as
    BASELINE.json states it, with the cone the reference lacks), with the same
    frames in flight as the main line, on the main line's streams (HIP maps
    streams onto GPU_MAX_HW_QUEUES = 4 hardware queues round-robin: two more
    streams can land on one queue, which serialises their launches): value,
    ms/frame and the reference-work roofline fraction."""
    import torch
    rargs = pkg.configs.CONFIGS[name]()
    packed = pkg.scene.convert(rargs)
    ctxs = make_contexts(pkg, dev, packed, inflight, specialize)
    dr = pkg.dist.DistributedRenderer(ctxs, packed, 0, 1, dev, mode="frame",
                                      streams=streams if inflight > 1 else None)
    for _ in range(max(warmup, inflight)):
        dr.step()
    dr.flush()
    torch.cuda.synchronize()
    dr.read_stats(reset=True)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        dr.step(events=evs[k])
    dr.flush()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = dr.read_stats(reset=True)
    kavg = gpu_span_ms(evs)
    flops = pkg.abi.algorithmic_flops(st, len(rargs.lights)) / steps
    for c in ctxs:
        c.close()
    ex, exsrc = pmc_executed(name)
    executed = None
    if ex is not None and ex.get("kernel_src") == pkg.render.kernel_source_id() and kavg > 0:
        executed = {"executed_frac": round(ex["executed_fp64_flops"] / (kavg * 1e-3) / 1e12 / PEAK_FP64_TFLOPS, 4),
                    "issue_util": round(ex["issue_util"], 4), "pmc_source": exsrc}
    elif ex is not None:
        executed = {"pmc_stale": exsrc}
    return {"executed": executed, "workload": "%s: %s" % (name, pkg.configs.WORKLOADS[name]), "value": round(st.total_rays() / dt / 1e6, 2),
            "unit": "Mrays/s", "ms_per_step": round(dt / steps * 1e3, 4), "kernel_ms": round(kavg, 4),
            "rays_per_step": int(st.total_rays() / steps),
            "frac": round(flops / (kavg * 1e-3) / 1e12 / PEAK_FP64_TFLOPS, 4), "parity": "unpinned (cone: contest extension)"}


def render_api_leg(pkg, packed, reps=30, budget_s=20.0):
    """The reference's own seam, timed: rt_render (include/rt_abi.h), the
    synchronous replacement of func Render(*Scene) image.Image
    (raytracer.go:589-682, hooked at evaluator.go:48): every call compares the
    scene with the last one (converting and uploading it when it changed),
    renders one frame and copies the RGBA8 image into pageable host memory
    (numpy), like Go's image.RGBA. Reported: the first call in the process
    (context creation, scene conversion, upload, tile-cost estimate; the
    generic kernel renders while the specialised ones compile in the
    background), the calls until the specialised kernels render (at most
    `budget_s`), then the median of the last five of `reps` calls, and that
    median call's parts as the library measured them on the same call
    (rt_render_last_timing: one host timeline, so setup + render_wait +
    copy_tail = total)."""
    import ctypes
    import numpy as np
    lib = pkg.render.load_library()
    out = np.empty((packed.height, packed.width, 4), np.uint8)
    st = pkg.abi.rt_stats()

    def call():
        t0 = time.perf_counter()
        rc = lib.rt_render(packed.ref(), out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st))
        wall = (time.perf_counter() - t0) * 1e3
        if rc != 0:
            raise RuntimeError("rt_render failed: %s" % lib.rt_last_error().decode())
        tm = pkg.abi.rt_render_timing()
        lib.rt_render_last_timing(ctypes.byref(tm))
        return wall, tm.as_dict()

    first = call()
    # the calls render with the generic kernel until the bands' specialised
    # kernels (one per band schedule) have compiled in the background: the
    # steady calls are timed after that (bounded wait)
    to_spec = 1
    t_lim = time.perf_counter() + budget_s
    while not first[1]["specialized"] and time.perf_counter() < t_lim:
        w, parts = call()
        to_spec += 1
        if parts["specialized"]:
            break
        time.sleep(0.01)
    calls = [call() for _ in range(reps)]
    last = sorted(calls[-5:], key=lambda c: c[0])
    wall, parts = last[len(last) // 2]
    return {"what": "rt_render(scene, host RGBA8, stats): scene compare (+ conversion and upload when it "
                    "changed) + one frame + copy into pageable host memory, synchronous (the Render() seam, "
                    "raytracer.go:589); not part of `value`",
            "calls": len(calls), "first_call_ms": round(first[0], 3), "first_call_parts": first[1],
            "calls_until_specialised": to_spec,
            "steady_ms": round(wall, 3),
            "parts_ms": parts,
            "parts_def": "library timeline of the median steady call: setup_ms + render_wait_ms + copy_tail_ms "
                         "= total_ms (wall from Python: steady_ms); gpu_ms = GPU span of its bands",
            "rays_per_call": int(st.primary_rays + st.secondary_rays + st.shadow_rays)}


def api_main(args):
    """--api: one step = one synchronous rt_render_ex call (the Render() seam,
    raytracer.go:589-682, over N GPUs of this process, ABI 6): scene compare,
    N shares rendered, the gather into a pageable host buffer, the counters.
    The first call of the process (new scene: conversion, upload, estimate,
    the generic kernel while the specialised one compiles in the background)
    is reported apart; then calls until the specialised kernel renders, W
    warm-up calls and K timed calls. value = rays per call / wall per call."""
    import numpy as np
    pkg = load_package()
    import torch  # noqa: F401  (the HIP runtime the library binds to)
    devices = [int(x) for x in args.api_devices.split(",")] if args.api_devices else list(range(args.gpus))
    cfg = pkg.configs.CONFIGS[args.config]
    kw = {}
    if args.width:
        kw["width"] = args.width
    if args.height:
        kw["height"] = args.height
    rargs = cfg(**kw)
    packed = pkg.scene.convert(rargs)
    out = np.empty((packed.height, packed.width, 4), np.uint8)

    def call():
        return pkg.render_frame(packed, devices=devices, gather=args.gather, out=out, generic=args.specialize == "off")

    t0 = time.perf_counter()
    _, st, tm = call()
    first = {"ms": round((time.perf_counter() - t0) * 1e3, 3), "parts": tm.as_dict()}
    calls_to_switch = 1
    t_lim = time.perf_counter() + 120
    while not tm.specialized and args.specialize == "on" and time.perf_counter() < t_lim:
        _, st, tm = call()
        calls_to_switch += 1
    for _ in range(args.warmup):
        call()
    rays = 0
    dev_ms = [0.0] * len(devices)
    span = gather = 0.0
    spec_all = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, st, tm = call()
        rays += st.total_rays()
        span += st.kernel_ms
        gather += st.gather_ms
        spec_all = spec_all and bool(tm.specialized)
        for d in range(len(devices)):
            dev_ms[d] += st.device_kernel_ms[d]
    elapsed = time.perf_counter() - t0
    K = args.steps
    kavg = span / K
    flops = pkg.abi.algorithmic_flops(st, len(rargs.lights))
    achieved = flops / (kavg * 1e-3) / 1e12 if kavg > 0 else 0.0
    line = {
        "metric": METRIC, "value": round(rays / elapsed / 1e6, 2), "unit": "Mrays/s",
        "n_gpus": len(set(devices)), "steps": K, "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "%s: %s" % (args.config, pkg.configs.WORKLOADS[args.config]),
                   "width": packed.width, "height": packed.height, "depth": rargs.depth,
                   "rays_per_step": int(rays / K), "devices": devices,
                   "parallelism": "rt_render_ex: rows%d-interleaved, %s gather, one process" % (len(devices), args.gather),
                   "kernel": "specialised" if spec_all else "generic (specialisation pending or off)"},
        "seam": {"what": "rt_render_ex(scene, opts, host RGBA8, stats) per step: scene compare + the N shares + "
                         "gather into pageable host memory + counters (the Render() seam, raytracer.go:589)",
                 "first_call_ms": first["ms"], "first_call_parts": first["parts"],
                 "calls_until_specialised": calls_to_switch,
                 "device_kernel_ms": [round(v / K, 4) for v in dev_ms],
                 "gather_ms": round(gather / K, 4), "last_call_parts": tm.as_dict()},
        "roofline": {"bound": "valu-fp64", "achieved": round(achieved, 3), "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                     "frac": None, "reference_work_frac": round(achieved / PEAK_FP64_TFLOPS / max(1, len(set(devices))), 4),
                     "kernel_ms": round(kavg, 4),
                     "kernel_ms_def": "slowest device's GPU span per call (rt_stats.kernel_ms)",
                     "traffic": None},
        "cpu_baseline": None,
    }
    if args.cpu_baseline == "auto":
        line["cpu_baseline"] = cpu_baseline(packed, args.cpu_threads)
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    if args.api:
        return api_main(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher (torchrun) set the ranks up: start them here, before any
        # GPU call in this process
        sys.exit(spawn_ranks(args.gpus))
    if args.launch_selftest:
        return launch_selftest(args)
    pkg = load_package()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = pkg.configs.CONFIGS[args.config]
    kw = {}
    if args.width:
        kw["width"] = args.width
    if args.height:
        kw["height"] = args.height
    rargs = cfg(**kw)
    packed = pkg.scene.convert(rargs)
    if args.inflight is None:
        args.inflight = inflight_default(args, world)
    if args.inflight < 1:
        raise SystemExit("--inflight must be >= 1")
    ctxs = make_contexts(pkg, dev, packed, args.inflight, args.specialize == "on",
                         accel=0 if args.accel == "none" else None, schedule=args.schedule,
                         sharing={"auto": None, "off": 0, "on": 1, "group": 1, "device": 2}[args.work_sharing])
    ctx = ctxs[0]
    spec_active, spec_ms = ctx.specialized()
    order_active, order_ms = ctx.tile_order_info()
    bvh = bool(ctx.scene_info() & pkg.abi.RT_INFO_BVH)
    # CSG composites are an extension: the reference has no flop model for them
    no_ref_model = bool(ctx.scene_info() & pkg.abi.RT_INFO_CSG)
    mode = "frame" if args.scaling == "weak" else args.shard
    band = None
    if args.rows:
        if world != 1:
            raise SystemExit("--rows is a one-GPU measurement")
        band = tuple(int(v) for v in args.rows.split(":"))
        mode = "band"
    # strong scaling over several ranks: frame k's gather overlaps frame k+1's render
    dr = pkg.dist.DistributedRenderer(ctxs, packed, rank, world, dev, mode=mode, band=band,
                                      pipeline=args.scaling == "strong", gather_timing=True)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(max(args.warmup, args.inflight)):  # every context warmed up
        dr.step()
    dr.flush()
    torch.cuda.synchronize()
    dr.read_stats(reset=True)
    dr.gather_ms()  # (the warm-up gathers are not the timed ones)

    # Kernel time: torch events on the launch streams around each render launch
    # inside the timed region, read after it (no host sync per step).
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        dr.step(events=evs[k])
    dr.flush()  # every frame gathered to rank 0 inside the timed region
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    launch_ms = [e0.elapsed_time(e1) for e0, e1 in evs] if dr.has_work() else []
    span_ms = gpu_span_ms(evs) if dr.has_work() else 0.0
    st = dr.read_stats(reset=True)

    rays_local = st.total_rays()
    flops_local = pkg.abi.algorithmic_flops(st, len(rargs.lights))
    # the roofline's kernel time: GPU span per frame (= the average launch
    # duration when launches do not overlap, i.e. --inflight 1)
    kavg = span_ms
    lavg = sum(launch_ms) / len(launch_ms) if launch_ms else 0.0
    gms = dr.gather_ms()
    rank_rows = pkg.dist.rank_table([span_ms, -1.0 if gms is None else gms, elapsed / args.steps * 1e3],
                                    device=dev)
    mx, sm = pkg.dist.reduce_max_sum([elapsed, rays_local], device=dev)
    elapsed, rays_total = mx[0], sm[1]

    if rank == 0:
        per_step_rays = rays_total / args.steps
        ms_per_step = elapsed / args.steps * 1e3
        value = rays_total / elapsed / 1e6
        # roofline for the dominant (only) kernel: algorithmic FP64 flops per
        # launch / GPU time per launch (HIP events on the launch streams)
        flops_per_launch = flops_local / max(1, len(launch_ms))
        achieved_tf = flops_per_launch / (kavg * 1e-3) / 1e12 if kavg > 0 else 0.0
        out_bytes = dr.buf.numel()
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "%s: %s" % (args.config, pkg.configs.WORKLOADS[args.config]),
                       "width": packed.width, "height": packed.height, "depth": rargs.depth,
                       "lights": len(rargs.lights), "objects": int(packed.scene.num_objects),
                       "rays_per_step": int(per_step_rays),
                       "parallelism": ("rows %d:%d (band)" % band) if band else
                                      ("frame-per-gpu%d" % world) if args.scaling == "weak"
                                      else "rows%d-%s%s" % (world, args.shard, "-pipelined" if dr.pipeline else ""),
                       "frames_in_flight": args.inflight,
                       "schedule": args.schedule,
                       "work_sharing": args.work_sharing,
                       "kernel": "specialised" if spec_active else "generic",
                       "accel": "bvh+cull" if args.accel == "bvh" else "none (brute force)",
                       "spec_compile_ms": round(spec_ms, 1),
                       "tile_order_ms": round(order_ms, 2) if order_active else None},
            "roofline": {"bound": "valu-fp64", "achieved": round(achieved_tf, 3), "peak": PEAK_FP64_TFLOPS,
                         "unit": "TFLOP/s",
                         # with a BVH the kernel skips most of the reference's
                         # Intersect calls, so reference work per second is no
                         # utilisation (it can exceed 1): null, and the executed
                         # fraction (PMC) carries the roofline instead
                         "frac": None if (bvh or no_ref_model) else round(achieved_tf / PEAK_FP64_TFLOPS, 4),
                         "reference_work_frac": round(achieved_tf / PEAK_FP64_TFLOPS, 4),
                         "frac_nofma_ceiling": None if (bvh or no_ref_model) else round(achieved_tf / PEAK_FP64_NOFMA_TFLOPS, 4),
                         "kernel_ms": round(kavg, 4), "flops_per_launch": int(flops_per_launch),
                         "kernel_ms_def": "GPU span per frame: first launch's start to the last launch's end "
                                          "(HIP events on the launch streams) / frames (one launch per frame)",
                         "launch_ms_overlapped": round(lavg, 4),
                         "hbm_out_gbs": round(out_bytes / (kavg * 1e-3) / 1e9, 2) if kavg > 0 else None,
                         "traffic": None, "traffic_source": None},
            "cpu_baseline": None,
        }
        if world > 1:
            # per rank: GPU render span per step, the pipelined gather's cost
            # per frame (render end -> collective complete, the wait for the
            # slowest rank included), wall per step
            line.update(telemetry(rank_rows))
        # What the kernel executes (PMC) next to the reference-algorithmic frac
        key = args.config + ("_bf" if args.accel == "none" else "") + \
            ("_rows%d-%d" % band if band else "")
        ex, exsrc = pmc_executed(key) if (world == 1 and not args.width and not args.height) else (None, None)
        if ex is not None and ex.get("kernel_src") != pkg.render.kernel_source_id():
            # counters of another kernel build: not quoted as this run's
            line["roofline"]["pmc_stale"] = exsrc
            ex = None
        if ex is not None and kavg > 0:
            ex_tf = ex["executed_fp64_flops"] / (kavg * 1e-3) / 1e12
            line["roofline"].update({
                "executed_tflops": round(ex_tf, 3),
                "executed_frac": round(ex_tf / PEAK_FP64_TFLOPS, 4),
                "fp64_pipe_busy": round(ex["fp64_pipe_busy"], 4),
                "valu_busy": round(ex["valu_busy"], 4),
                "issue_util": round(ex["issue_util"], 4),
                "lane_util": round(ex["lane_util"], 4),
                "pmc_source": exsrc})
        # (the traffic summary of the accelerated search: not quoted for --accel none)
        tb, src, tsrc = pmc_traffic(args.config) if args.accel != "none" else (None, None, None)
        if tb is not None and tsrc != pkg.render.kernel_source_id():
            line["roofline"]["traffic_stale"] = src  # another kernel build's counters
            tb = None
        if tb is not None and world == 1 and not args.width and not args.height and not band:
            line["roofline"]["traffic"] = int(tb)
            line["roofline"]["traffic_source"] = src
        if world == 1 and args.config == "c3" and args.companion == "auto" and not (args.width or args.height or band):
            line["c3cone"] = side_config(pkg, "c3cone", dev, args.specialize == "on", args.inflight, streams=dr.streams)
        if world == 1 and args.config == "c3" and args.companion == "auto" and not (args.width or args.height or band):
            line["render_api"] = render_api_leg(pkg, packed)
        if world == 1 and args.cpu_baseline == "auto":
            line["cpu_baseline"] = cpu_baseline(packed, args.cpu_threads)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

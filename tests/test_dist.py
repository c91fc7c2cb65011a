"""Row-band sharding + gather to rank 0 (go_raytracer_amd/dist.py) on CPU with
gloo, world sizes 2 and 3 (uneven bands). Each rank renders its band with the
CPU oracle; the assembled frame must equal the single-process full frame --
the property the GPU path relies on (RNG depends only on (x, 20-row strip),
raytracer.go:627-634)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, w, h, q, mode="bands"):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from __graft_entry__ import load_package
    pkg = load_package()
    import oracle_bind
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    packed = pkg.scene.convert(pkg.configs.c2(width=w, height=h))
    if mode == "bands":
        y0, y1, per = pkg.dist.band_rows(h, rank, world)
        band = torch.zeros((per, w, 4), dtype=torch.uint8)
        if y1 > y0:
            img, _ = oracle_bind.render_rows(packed, y0, y1, threads=2)
            band[: y1 - y0] = torch.from_numpy(img)
    else:  # interleaved 8-row tile rows r, r+world, ...
        nt, K = pkg.dist.tile_rows(h, world)
        band = torch.zeros((K * 8, w, 4), dtype=torch.uint8)
        for j in range(K):
            t = rank + j * world
            if t < nt:
                y0, y1 = t * 8, min(h, t * 8 + 8)
                img, _ = oracle_bind.render_rows(packed, y0, y1, threads=2)
                band[j * 8: j * 8 + (y1 - y0)] = torch.from_numpy(img)
    frame = pkg.dist.gather_frame(band, h, mode)
    if rank == 0:
        q.put(frame.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h,mode", [(2, 64, 40, "bands"), (3, 48, 31, "bands"),
                                            (2, 64, 40, "interleaved"), (3, 40, 45, "interleaved")])
def test_gather_of_row_bands_equals_full_frame(world, w, h, mode):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind
    import go_raytracer_amd as rt
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full, _ = oracle_bind.render_rows(rt.scene.convert(rt.configs.c2(width=w, height=h)))
    assert frame.shape == full.shape
    assert np.array_equal(frame, full)


def test_band_rows_cover_the_frame_once():
    import go_raytracer_amd as rt
    for h in (1, 7, 20, 2160, 4321):
        for world in (1, 2, 3, 4, 8):
            rows = []
            for r in range(world):
                y0, y1, per = rt.dist.band_rows(h, r, world)
                assert 0 <= y0 <= y1 <= h and y1 - y0 <= per
                rows.extend(range(y0, y1))
            assert rows == list(range(h))


class _OracleCtx:
    """Stand-in for RenderContext in CPU tests: renders rows with the oracle."""

    def __init__(self, packed, oracle_bind):
        self.packed, self.ob = packed, oracle_bind
        self.calls = 0

    def render_rows_async(self, y0, y1, out, stream=None):
        self.calls += 1
        img, _ = self.ob.render_rows(self.packed, y0, y1, threads=2)
        out[: y1 - y0] = torch.from_numpy(img)

    def render_tile_rows_async(self, trow0, stride, ntrows, out, stream=None):
        self.calls += 1
        h = self.packed.height
        for j in range(ntrows):
            y0 = (trow0 + j * stride) * 8
            y1 = min(h, y0 + 8)
            if y1 > y0:
                img, _ = self.ob.render_rows(self.packed, y0, y1, threads=2)
                out[j * 8: j * 8 + (y1 - y0)] = torch.from_numpy(img)


def _weak_worker(rank, world, port, w, h, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from __graft_entry__ import load_package
    pkg = load_package()
    import oracle_bind
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    packed = pkg.scene.convert(pkg.configs.c2(width=w, height=h))
    dr = pkg.dist.DistributedRenderer(_OracleCtx(packed, oracle_bind), packed, rank, world, "cpu", mode="frame")
    assert dr.has_work()
    frame = dr.step()  # no collective in this mode
    mx, sm = pkg.dist.reduce_max_sum([rank + 1.0, 10.0 * (rank + 1)])
    q.put((rank, frame.numpy().copy(), mx, sm))
    dist.barrier()
    dist.destroy_process_group()


def test_weak_scaling_frame_per_rank():
    """bench.py --scaling weak (the default is strong): every rank renders the
    whole frame locally; timing is max over ranks, rays summed."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind
    import go_raytracer_amd as rt
    world, w, h = 2, 40, 24
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_weak_worker, args=(r, world, port, w, h, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full, _ = oracle_bind.render_rows(rt.scene.convert(rt.configs.c2(width=w, height=h)))
    for rank, frame, mx, sm in got:
        assert np.array_equal(frame, full), rank
        assert mx == [2.0, 20.0] and sm == [3.0, 30.0]


def test_reduce_max_sum_without_process_group():
    import go_raytracer_amd as rt
    assert rt.dist.reduce_max_sum([1.5, 2.0]) == ([1.5, 2.0], [1.5, 2.0])


def _pipeline_worker(rank, world, port, w, h, q, mode, inflight=1):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from __graft_entry__ import load_package
    pkg = load_package()
    import oracle_bind
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    packed = pkg.scene.convert(pkg.configs.c2(width=w, height=h))
    ctxs = [_OracleCtx(packed, oracle_bind) for _ in range(inflight)]
    dr = pkg.dist.DistributedRenderer(ctxs if inflight > 1 else ctxs[0], packed, rank, world, "cpu", mode=mode,
                                      pipeline=True, streams=[None] * inflight)
    assert dr.pipeline and len(dr.bufs) == max(2, inflight) and dr.inflight == inflight
    frames = []
    for _ in range(3):  # step 3 reuses step 1's buffer: its gather completes first
        dr.step()
        if dr.frame is not None:
            frames.append(dr.frame.numpy().copy())
    last = dr.flush()
    assert all(c.calls == len(range(i, 3, inflight)) for i, c in enumerate(ctxs))  # step k on context k mod F
    if rank == 0:
        frames.append(last.numpy().copy())
        q.put(frames)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,inflight", [(2, "interleaved", 1), (3, "bands", 1),
                                                (2, "interleaved", 2), (3, "interleaved", 3)])
def test_pipelined_gather_frames_equal_full_frame(world, mode, inflight):
    """bench.py --scaling strong over several ranks: rank buffers alternate
    and each gather is asynchronous (frame k's gather overlaps frame k+1's
    render); with frames in flight (bench --inflight, the default 2) step k
    renders on context k mod F into buffer k mod F. Every gathered frame
    equals the full-frame render."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind
    import go_raytracer_amd as rt
    w, h = 48, 36
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, w, h, q, mode, inflight))
             for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full, _ = oracle_bind.render_rows(rt.scene.convert(rt.configs.c2(width=w, height=h)))
    # with 2 buffers step 3 completed step 1's gather and flush the last one;
    # with 3 buffers in flight only flush completes one
    assert len(frames) == (2 if inflight < 3 else 1)
    for f in frames:
        assert np.array_equal(f, full)

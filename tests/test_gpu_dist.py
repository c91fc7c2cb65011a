"""The bench's multi-GPU path on a real device: a `nccl` (RCCL) process group
at world size 1, DistributedRenderer in the strong-scaling modes, the frame
assembled through the RCCL gather (forced at world size 1) equal to a
single-context full-frame render. World sizes > 1 need one GPU per rank
(RCCL rejects two ranks on one device); they are covered with gloo on the CPU
(tests/test_dist.py) and run by the driver's 8-GPU bench."""
import os
import socket

import numpy as np
import pytest

import go_raytracer_amd as rt

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_group():
    import torch
    import torch.distributed as dist
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield dist
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["interleaved", "bands", "frame"])
def test_rccl_gathered_frame_equals_full_render(nccl_group, mode):
    import torch
    packed = rt.scene.convert(rt.configs.c3(width=320, height=180))
    ctx = rt.RenderContext(0)
    try:
        ctx.set_scene(packed)
        full = ctx.render()
        dr = rt.dist.DistributedRenderer(ctx, packed, 0, 1, torch.device("cuda", 0), mode=mode)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        frame = dr.step(events=ev, collective=True)
        torch.cuda.synchronize()
        assert ev[0].elapsed_time(ev[1]) > 0
        got = frame.cpu().numpy()
        assert got.shape == full.shape
        assert np.array_equal(got, full)
    finally:
        ctx.close()


@pytest.mark.parametrize("mode", ["interleaved", "bands"])
def test_rccl_pipelined_gathers_equal_full_render(nccl_group, mode):
    """bench.py's strong-scaling loop: two rank buffers alternate, each RCCL
    gather is asynchronous and completes at the buffer's next use or flush()."""
    import torch
    packed = rt.scene.convert(rt.configs.c3(width=320, height=180))
    ctx = rt.RenderContext(0)
    try:
        ctx.set_scene(packed)
        full = ctx.render()
        dr = rt.dist.DistributedRenderer(ctx, packed, 0, 1, torch.device("cuda", 0), mode=mode, pipeline="always")
        assert dr.pipeline
        got = []
        for _ in range(3):
            dr.step()
            if dr.frame is not None:
                got.append(dr.frame.cpu().numpy())
        got.append(dr.flush().cpu().numpy())
        torch.cuda.synchronize()
        assert len(got) == 2
        for g in got:
            assert np.array_equal(g, full)
    finally:
        ctx.close()


def test_rccl_max_sum_reduction(nccl_group):
    import torch
    mx, sm = rt.dist.reduce_max_sum([1.5, 7.0], device=torch.device("cuda", 0))
    assert mx == [1.5, 7.0] and sm == [1.5, 7.0]


@pytest.mark.parametrize("inflight", [2, 3])
def test_frames_in_flight_equal_serial_frames(inflight):
    """bench.py --inflight F (default 2): F contexts with the same scene render
    consecutive frames on F streams, so launches overlap on the device. Every
    frame's pixels equal the serial render, and the summed counters equal the
    serial counters times the frame count."""
    import torch
    packed = rt.scene.convert(rt.configs.c3(width=640, height=360))
    dev = torch.device("cuda", 0)
    ref = rt.RenderContext(0, specialize=True)
    ctxs = [rt.RenderContext(0, specialize=True) for _ in range(inflight)]
    try:
        ref.set_scene(packed)
        ref.read_stats(reset=True)
        full = ref.render()
        st1 = ref.read_stats(reset=True).as_dict()
        for c in ctxs:
            c.set_scene(packed)
            c.read_stats(reset=True)
        dr = rt.dist.DistributedRenderer(ctxs, packed, 0, 1, dev, mode="frame")
        assert dr.inflight == inflight and len(dr.bufs) == inflight and len(set(dr.streams)) == inflight
        steps = 2 * inflight + 1
        for _ in range(steps):
            dr.step()
        dr.flush()
        torch.cuda.synchronize()
        for b in dr.bufs:
            assert np.array_equal(b.cpu().numpy(), full)
        st = dr.read_stats(reset=True).as_dict()
        for k, v in st1.items():
            want = [x * steps for x in v] if isinstance(v, list) else v * steps
            assert st[k] == want, k
    finally:
        ref.close()
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("inflight", [2, 3])
def test_rccl_pipelined_gathers_with_frames_in_flight(nccl_group, inflight):
    """The strong-scaling loop with two or three contexts in flight (bench.py
    uses three for C3 shares at >= 4 ranks): each RCCL gather is issued on its
    render's stream; every gathered frame equals the full render."""
    import torch
    packed = rt.scene.convert(rt.configs.c3(width=320, height=180))
    ctxs = [rt.RenderContext(0) for _ in range(inflight)]
    try:
        for c in ctxs:
            c.set_scene(packed)
        full = ctxs[0].render()
        dr = rt.dist.DistributedRenderer(ctxs, packed, 0, 1, torch.device("cuda", 0), mode="interleaved",
                                         pipeline="always")
        got = []
        for _ in range(5):
            dr.step()
            if dr.frame is not None:
                got.append(dr.frame.cpu().numpy())
        got.append(dr.flush().cpu().numpy())
        torch.cuda.synchronize()
        # a buffer's gather completes when the buffer comes round again (steps
        # F .. 4), plus the flush
        assert len(got) == 5 - inflight + 1
        for g in got:
            assert np.array_equal(g, full)
    finally:
        for c in ctxs:
            c.close()

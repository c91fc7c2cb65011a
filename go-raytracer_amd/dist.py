"""Multi-GPU rendering, one process per GPU.

Weak scaling (mode "frame", bench --scaling weak): a batch of frames, one per rank
(e.g. the frames of an animation or of independent requests); each rank renders
its whole frame into its own HBM buffer. The units (frames, and within them
pixels) are independent, so there is no data-path collective at all.

Strong scaling (the bench default, north_star's design: one frame sharded
across GPUs + gather to rank 0, RCCL over xGMI): pixels are independent and the jitter RNG depends only on (column,
20-row strip) (raytracer.go:627-634), so any row partition renders
bit-identical rows. Two partitions:

- "interleaved" (default): the image's 8-row tile rows are dealt round-robin,
  rank r owning tile rows r, r+N, r+2N, ... -- sky and ground rows are spread
  evenly, so ranks finish together. Rank 0 gathers the [K*8, W, 4] slabs and
  de-interleaves them on the device.
- "bands": contiguous bands of ceil(H/N) rows (simple; imbalanced when the
  cost varies with height).

The gather is one collective over the process group (backend "nccl" = RCCL on
ROCm; "gloo" in the CPU tests). No reduction is needed.
"""
import math

TILE = 8


def band_rows(height, rank, world):
    """Contiguous band [y0, y1) owned by `rank` (last band may be shorter/empty)."""
    per = int(math.ceil(height / float(world)))
    y0 = min(height, rank * per)
    y1 = min(height, y0 + per)
    return y0, y1, per


def tile_rows(height, world):
    """(tile rows in the image, tile rows per rank K): rank r owns tile rows
    r + j*world for j < K (those past the image are padding)."""
    nt = (height + TILE - 1) // TILE
    return nt, (nt + world - 1) // world


def deinterleave(slabs, height):
    """slabs: [world, K*8, W, 4] (rank-major) -> [height, W, 4] frame."""
    world, rows, W, ch = slabs.shape
    K = rows // TILE
    full = slabs.reshape(world, K, TILE, W, ch).permute(1, 0, 2, 3, 4).reshape(K * world * TILE, W, ch)
    return full[:height]


_recv = {}


def gather_frame(buf, height, mode="bands", group=None, collective=None, slot=None):
    """Gather every rank's buffer to rank 0 and assemble the [H, W, 4] frame
    there (None elsewhere). Rank 0 receives straight into the slices of one
    reused [world, ...] tensor per `slot` (no stacking copy; frames in flight
    on different streams use different slots, so one frame's receive tensor is
    never overwritten while another stream still reads it). With a single rank
    the buffer already is the frame and no collective runs, unless
    `collective` is True (tests: the RCCL gather at world size 1)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if collective is None:
        collective = world > 1
    if not collective or not dist.is_initialized():
        return deinterleave(buf.unsqueeze(0), height) if mode == "interleaved" else buf[:height]
    rank = dist.get_rank(group)
    if rank == 0:
        key = (tuple(buf.shape), buf.dtype, buf.device, world, "sync", slot)
        stacked = _recv.get(key)
        if stacked is None:
            stacked = _recv[key] = torch.empty((world,) + tuple(buf.shape), dtype=buf.dtype, device=buf.device)
        dist.gather(buf, gather_list=list(stacked.unbind(0)), dst=0, group=group)
        if mode == "interleaved":
            return deinterleave(stacked, height)
        return stacked.reshape(-1, *buf.shape[1:])[:height].clone()  # the receive tensor is reused
    dist.gather(buf, dst=0, group=group)
    return None


class PendingGather:
    """An in-flight gather of one rank buffer (async_op): wait() completes it
    and returns the assembled frame on rank 0 (None elsewhere). With `timing`
    (a list), wait() appends (issue, done) CUDA events: issue recorded on the
    launch stream when the gather was enqueued (= this rank's render end),
    done on the caller's stream once the collective has completed -- their
    difference is the gather's cost to this rank, waiting for the slowest
    rank included."""

    def __init__(self, work, stacked, height, mode, shape, issue=None, timing=None):
        self.work, self.stacked, self.height, self.mode, self.shape = work, stacked, height, mode, shape
        self.issue, self.timing = issue, timing

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
            if self.issue is not None and self.timing is not None:
                import torch
                done = torch.cuda.Event(enable_timing=True)
                done.record()
                self.timing.append((self.issue, done))
        if self.stacked is None:
            return None
        if self.mode == "interleaved":
            return deinterleave(self.stacked, self.height)
        return self.stacked.reshape(-1, *self.shape[1:])[:self.height].clone()


def gather_frame_async(buf, height, mode, slot, group=None, timing=None):
    """gather_frame as an async collective into receive slot `slot` (one
    receive tensor per slot on rank 0, so two frames can be in flight).
    `timing`: see PendingGather (CUDA tensors only)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    issue = None
    if timing is not None and buf.is_cuda:
        issue = torch.cuda.Event(enable_timing=True)
        issue.record()
    if dist.get_rank(group) == 0:
        key = (tuple(buf.shape), buf.dtype, buf.device, world, "slot", slot)
        stacked = _recv.get(key)
        if stacked is None:
            stacked = _recv[key] = torch.empty((world,) + tuple(buf.shape), dtype=buf.dtype, device=buf.device)
        work = dist.gather(buf, gather_list=list(stacked.unbind(0)), dst=0, group=group, async_op=True)
        return PendingGather(work, stacked, height, mode, tuple(buf.shape), issue, timing)
    return PendingGather(dist.gather(buf, dst=0, group=group, async_op=True), None, height, mode, tuple(buf.shape),
                         issue, timing)


def rank_table(values, device=None):
    """Every rank's list of floats, on every rank: [[rank 0's], [rank 1's], ...]
    (one all_reduce of a zero-padded [world, n] tensor; identity without an
    initialised process group). The N>1 bench line's per-rank telemetry."""
    import torch
    import torch.distributed as dist
    vals = [float(v) for v in values]
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [vals]
    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.zeros((world, len(vals)), dtype=torch.float64, device=device)
    t[rank] = torch.tensor(vals, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def reduce_max_sum(values, device=None):
    """(max over ranks, sum over ranks) of a list of floats (one all_reduce
    each; identity without an initialised process group). Used for the step
    time (max) and the ray totals (sum)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return t.tolist(), t.tolist()
    mx, sm = t.clone(), t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return mx.tolist(), sm.tolist()


class DistributedRenderer:
    """Per step: this rank's whole frame (mode "frame", weak scaling), or its
    share of one frame's rows ("interleaved" / "bands", strong scaling) followed
    by the gather to rank 0.

    Frames in flight: `ctx` may be a list of F render contexts holding the same
    scene (each with its own queue heads, frame stack and counters; rt_abi.h
    contexts are independent). Step k renders on context k mod F, on that
    context's stream, into buffer k mod F, so frame k+1's workgroups take the
    CUs that frame k's last waves leave idle -- the tail of a launch (a
    persistent grid draining its tile queue) overlaps the head of the next.
    Every frame is still rendered whole; pixels and counters do not change.
    F = 1 is the serial schedule on the caller's current stream."""

    def __init__(self, ctx, packed, rank, world, device, mode="interleaved", band=None, pipeline=False,
                 streams=None, gather_timing=False):
        import torch
        self.ctxs = list(ctx) if isinstance(ctx, (list, tuple)) else [ctx]
        if not self.ctxs:
            raise ValueError("no render context")
        self.ctx = self.ctxs[0]
        self.inflight = len(self.ctxs)
        if streams is None:
            streams = [None] if self.inflight == 1 else [torch.cuda.Stream(device) for _ in self.ctxs]
        if len(streams) != self.inflight:
            raise ValueError("one stream per context")
        self.streams = list(streams)
        self.packed = packed
        self.rank = rank
        self.world = world
        self.mode = mode
        self.H = packed.height
        self.W = packed.width
        if mode == "frame":
            rows = self.H
        elif mode == "band":
            # one fixed row band [y0, y1) of the full-size frame, one rank
            # (measurement of configs too costly to render whole, e.g. brute-force C5)
            if world != 1 or band is None:
                raise ValueError("mode 'band' takes band=(y0, y1) and one rank")
            self.y0, self.y1 = int(band[0]), int(band[1])
            if not 0 <= self.y0 < self.y1 <= self.H:
                raise ValueError("band %r outside the %d-row frame" % (band, self.H))
            rows = self.y1 - self.y0
        elif mode == "interleaved":
            self.nt, self.K = tile_rows(self.H, world)
            # this rank's valid tile rows (the rest of its slab is padding)
            self.ntrows = max(0, min(self.K, (self.nt - rank + world - 1) // world))
            rows = self.K * TILE
        else:
            self.y0, self.y1, rows = band_rows(self.H, rank, world)
        self.buf = torch.zeros((rows, self.W, 4), dtype=torch.uint8, device=device)
        self.frame = None
        # pipeline (strong scaling over >1 rank): rank buffers alternate and
        # each gather runs asynchronously, so frame k's gather overlaps frame
        # k+1's render; a buffer is reused only after its gather has completed
        # (pipeline="always": also at one rank -- the GPU test of the RCCL path)
        self.pipeline = (pipeline == "always" or (bool(pipeline) and world > 1)) and mode in ("interleaved", "bands")
        nbufs = max(self.inflight, 2 if self.pipeline else 1)
        if nbufs % self.inflight:
            raise ValueError("buffers must divide evenly over the contexts")
        self.bufs = [self.buf] + [torch.zeros_like(self.buf) for _ in range(nbufs - 1)]
        self.pending = [None] * nbufs
        self.k = 0
        # (issue, done) event pairs of completed pipelined gathers (telemetry,
        # opt-in: gather_timing=True, bench.py; gather_ms() empties the list)
        self.gather_events = [] if gather_timing else None

    def has_work(self):
        if self.mode in ("frame", "band"):
            return True
        return self.ntrows > 0 if self.mode == "interleaved" else self.y1 > self.y0

    def read_stats(self, reset=True):
        """Counters of every context, summed (abi.sum_stats)."""
        from . import abi
        return abi.sum_stats([c.read_stats(reset=reset) for c in self.ctxs])

    def step(self, gather=True, events=None, collective=None):
        """Render this rank's rows and gather the frame. `events` (start, end):
        torch.cuda.Events recorded on the launch stream around the render
        kernel, for kernel timing without a host sync per step."""
        import torch
        slot = self.k % len(self.bufs)
        i = self.k % self.inflight
        self.k += 1
        ctx, stream, buf = self.ctxs[i], self.streams[i], self.bufs[slot]
        if self.pending[slot] is not None:  # this buffer's previous gather must be done
            # completed (and the frame assembled) on the caller's stream, which
            # the launch stream then follows before it overwrites the buffer
            self.frame = self.pending[slot].wait()
            self.pending[slot] = None
            if stream is not None:
                stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            if events is not None:
                events[0].record()
            if self.mode in ("frame", "band"):
                if self.mode == "frame":
                    ctx.render_rows_async(0, self.H, buf, stream=stream)
                else:
                    ctx.render_rows_async(self.y0, self.y1, buf, stream=stream)
                if events is not None:
                    events[1].record()
                self.frame = buf  # rank-local rows; nothing to exchange (complete after flush())
                return self.frame
            if self.mode == "interleaved":
                if self.ntrows > 0:
                    ctx.render_tile_rows_async(self.rank, self.world, self.ntrows,
                                               buf[: self.ntrows * TILE], stream=stream)
            elif self.y1 > self.y0:
                ctx.render_rows_async(self.y0, self.y1, buf[: self.y1 - self.y0], stream=stream)
            if events is not None:
                events[1].record()
            if gather:
                if self.pipeline:
                    # issued on the launch stream: the collective waits for this render only
                    self.pending[slot] = gather_frame_async(buf, self.H, self.mode, slot, timing=self.gather_events)
                    return None  # the frame comes from flush() / a later step
                self.frame = gather_frame(buf, self.H, self.mode, collective=collective,
                                          slot=slot if self.inflight > 1 else None)
        if gather and stream is not None:
            # the frame was gathered and assembled on the launch stream: the
            # caller's stream (which reads it) is ordered after it
            torch.cuda.current_stream().wait_stream(stream)
        return self.frame

    def gather_ms(self):
        """Mean per-frame cost of the completed pipelined gathers to this rank
        (ms from its render end to the collective's completion; None if no
        timed gather ran); resets the record. Call after flush() and a sync."""
        if self.gather_events is None:
            return None
        ev, self.gather_events = self.gather_events, []
        if not ev:
            return None
        return sum(a.elapsed_time(b) for a, b in ev) / len(ev)

    def flush(self):
        """Complete every in-flight gather (pipeline mode); returns the frame of
        the last step on rank 0. Frames in flight: the caller's stream is
        ordered after every context's stream."""
        import torch
        order = [(self.k + i) % len(self.bufs) for i in range(len(self.bufs))]  # oldest first
        for slot in order:
            if self.pending[slot] is not None:
                self.frame = self.pending[slot].wait()
                self.pending[slot] = None
        if self.inflight > 1 and torch.cuda.is_available():
            cur = torch.cuda.current_stream()
            for s in self.streams:
                if s is not None:
                    cur.wait_stream(s)
        return self.frame

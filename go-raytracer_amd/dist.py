"""Row-band sharding of one frame across GPUs + gather to rank 0 (RCCL/xGMI).

Pixels are independent and the jitter RNG depends only on (column, 20-row
strip) (raytracer.go:627-634), so any row partition renders bit-identical
rows. One process per GPU; rank r renders rows [r*B, min(H, (r+1)*B)) with
B = ceil(H / world). The frame is assembled on rank 0 with one gather over
the process group (backend "nccl" = RCCL on ROCm; "gloo" on CPU tests). No
reduction is needed.
"""
import math


def band_rows(height, rank, world):
    """Rows [y0, y1) owned by `rank` (the last band may be shorter or empty)."""
    per = int(math.ceil(height / float(world)))
    y0 = min(height, rank * per)
    y1 = min(height, y0 + per)
    return y0, y1, per


def assemble(bands, height):
    """Concatenate per-rank band buffers ([per, W, 4] each, padded) into [H, W, 4]."""
    import torch
    world = len(bands)
    per = bands[0].shape[0]
    full = torch.cat(list(bands), dim=0)
    assert full.shape[0] == per * world
    return full[:height]


def gather_frame(band_buf, height, group=None):
    """Gather every rank's padded band to rank 0. Returns the [H, W, 4] frame on
    rank 0 and None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        return band_buf[:height]
    if rank == 0:
        bufs = [torch.empty_like(band_buf) for _ in range(world)]
        dist.gather(band_buf, gather_list=bufs, dst=0, group=group)
        return assemble(bufs, height)
    dist.gather(band_buf, dst=0, group=group)
    return None


class DistributedRenderer:
    """Renders one frame per step with rows sharded over the process group."""

    def __init__(self, ctx, packed, rank, world, device):
        import torch
        self.ctx = ctx
        self.packed = packed
        self.rank = rank
        self.world = world
        self.H = packed.height
        self.W = packed.width
        self.y0, self.y1, self.per = band_rows(self.H, rank, world)
        self.band = torch.zeros((self.per, self.W, 4), dtype=torch.uint8, device=device)
        self.frame = None

    def step(self, gather=True):
        n = self.y1 - self.y0
        if n > 0:
            self.ctx.render_rows_async(self.y0, self.y1, self.band[:n])
        if gather and self.world > 1:
            self.frame = gather_frame(self.band, self.H)
        elif self.world == 1:
            self.frame = self.band
        return self.frame

"""CPU tests of rt_render_ex's multi-device partition and assembly
(include/rt_abi.h rt_render_ex, rt_debug_assemble; no device): the frame's
8-row tile rows dealt round-robin over N devices, each
device's share packed, and the frame assembled with exactly the copy plan the
device path runs -- bands, strided DMA runs, the clipped last tile row, the
host copies -- equals the frame the shares were cut from."""
import numpy as np
import pytest

import go_raytracer_amd as rt

TILE = 8


def shares_of(frame, n):
    """Device d's share as rt_render_tile_rows_async writes it: tile rows
    d, d+n, ... packed, the last one clipped to the image (rows past the image
    are left untouched: poisoned here)."""
    H, W = frame.shape[:2]
    trows = (H + TILE - 1) // TILE
    out = []
    for d in range(n):
        rows = list(range(d, trows, n))
        s = np.full((max(1, len(rows)) * TILE, W, 4), 0xAB, np.uint8)
        for j, t in enumerate(rows):
            r0, r1 = t * TILE, min(H, t * TILE + TILE)
            s[j * TILE:j * TILE + (r1 - r0)] = frame[r0:r1]
        out.append(s)
    return out


@pytest.mark.parametrize("n", [1, 2, 3, 8])
@pytest.mark.parametrize("size", [(64, 48), (77, 53), (19, 9), (40, 130)])
@pytest.mark.parametrize("bands", [0, 1, 2, 3, 5])
def test_assembly_of_interleaved_shares_is_the_frame(n, size, bands):
    W, H = size
    rng = np.random.default_rng(W * 1000 + H + n)
    frame = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    got = rt.render.debug_assemble(W, H, shares_of(frame, n), bands=bands)
    assert np.array_equal(got, frame)


def test_more_devices_than_tile_rows():
    """16 devices for a 3-tile-row image: the devices past the last tile row
    render nothing and the frame is still complete."""
    W, H = 33, 20
    frame = np.random.default_rng(1).integers(0, 256, (H, W, 4), dtype=np.uint8)
    got = rt.render.debug_assemble(W, H, shares_of(frame, 16))
    assert np.array_equal(got, frame)


def test_4k_frame_over_8_devices_with_automatic_bands():
    """The bench frame (3840 x 2160) over 8 devices, automatic bands."""
    W, H = 3840, 2160
    frame = np.random.default_rng(2).integers(0, 256, (H, W, 4), dtype=np.uint8)
    for n in (2, 8):
        assert np.array_equal(rt.render.debug_assemble(W, H, shares_of(frame, n)), frame)


def test_bad_arguments_are_rejected():
    lib = rt.load_library()
    assert lib.rt_debug_assemble(0, 8, 1, 0, None, None) == rt.abi.RT_E_INVALID
    assert lib.rt_debug_assemble(8, 8, rt.abi.RT_MAX_DEVICES + 1, 0, None, None) == rt.abi.RT_E_INVALID


def test_render_opts_device_selection():
    o = rt.render.render_opts([0, 0, 1], gather="peer", generic=True)
    assert o.device_count == 3 and list(o.devices)[:3] == [0, 0, 1]
    assert o.flags == rt.abi.RT_RENDER_DEVICE_LIST | rt.abi.RT_RENDER_GENERIC
    assert o.gather == rt.abi.RT_GATHER_PEER
    o = rt.render.render_opts(4)
    assert o.device_count == 4 and o.flags == 0

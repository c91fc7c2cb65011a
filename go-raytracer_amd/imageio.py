"""Image output for rendered frames.

The reference writes PNG with Go's image/png (cmd/gml/main.go:383-390,
cmd/example/main.go:21-28); for an opaque *image.RGBA that encoder emits
8-bit truecolour (colour type 2). write_png does the same from the RGBA8
frame (alpha is 255 everywhere on the render path), with zlib instead of Go's
compress/flate, so files decode to identical pixels but are not byte-identical
to Go's. write_ppm writes binary P6, the contest's own output format.
"""
import struct
import zlib

import numpy as np


def _rgb(img):
    a = np.asarray(img)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] not in (3, 4):
        raise ValueError("expected a uint8 [H, W, 3|4] image")
    if a.shape[2] == 4:
        if not (a[..., 3] == 255).all():
            raise ValueError("frame is not opaque: the render path writes alpha 255")
        a = a[..., :3]
    return np.ascontiguousarray(a)


def encode_png(img, level=6):
    """PNG bytes (RGB8, filter 0 per row) of an opaque RGBA8/RGB8 frame."""
    rgb = _rgb(img)
    h, w, _ = rgb.shape

    def chunk(tag, data):
        c = struct.pack(">I", len(data)) + tag + data
        return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    raw = np.empty((h, 1 + 3 * w), dtype=np.uint8)
    raw[:, 0] = 0
    raw[:, 1:] = rgb.reshape(h, 3 * w)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(raw.tobytes(), level))
            + chunk(b"IEND", b""))


def write_png(path, img):
    with open(path, "wb") as f:
        f.write(encode_png(img))


def encode_ppm(img):
    rgb = _rgb(img)
    h, w, _ = rgb.shape
    return b"P6\n%d %d\n255\n" % (w, h) + rgb.tobytes()


def write_ppm(path, img):
    with open(path, "wb") as f:
        f.write(encode_ppm(img))


def write_image(path, img):
    """By extension: .ppm -> P6, anything else -> PNG (the reference always
    writes PNG, whatever the .gml file names)."""
    (write_ppm if str(path).lower().endswith(".ppm") else write_png)(path, img)


def read_ppm(path):
    data = open(path, "rb").read()
    parts = data.split(maxsplit=4)
    if parts[0] != b"P6" or int(parts[3]) != 255:
        raise ValueError("not a binary 8-bit PPM")
    w, h = int(parts[1]), int(parts[2])
    pix = np.frombuffer(parts[4][:w * h * 3] if len(parts) > 4 else b"", dtype=np.uint8)
    return pix.reshape(h, w, 3)


def read_image(path):
    """uint8 [H, W, 3] from a PNG (via PIL) or binary PPM file."""
    if str(path).lower().endswith(".ppm"):
        return read_ppm(path)
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"))


def ssim(a, b, device=0):
    """prim.SSIM of two frames, computed on the HIP device (rt_ssim_rgba8)."""
    from .render import RenderContext
    ctx = RenderContext(device)
    try:
        return ctx.ssim(a, b)
    finally:
        ctx.close()

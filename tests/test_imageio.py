"""Image output and the SSIM parity metric on the CPU:
PNG/PPM round trips, and the numpy restatement of prim.SSIM checked against
the properties the reference's own tests assert (ssim_test.go:37-67) and its
error cases (ssim.go:29-34)."""
import io
import math
import os
import sys

import numpy as np
import pytest
from PIL import Image

import go_raytracer_amd as rt

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import ssim_ref  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _rand_rgba(rng, h, w):
    img = rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    img[..., 3] = 255
    return img


def test_png_round_trip(tmp_path):
    rng = np.random.default_rng(1)
    img = _rand_rgba(rng, 37, 53)
    p = tmp_path / "x.png"
    rt.imageio.write_png(str(p), img)
    back = np.asarray(Image.open(str(p)))
    assert Image.open(str(p)).mode == "RGB"  # Go's encoder: truecolour for opaque RGBA
    assert np.array_equal(back, img[..., :3])
    assert np.array_equal(rt.imageio.read_image(str(p)), img[..., :3])


def test_ppm_round_trip(tmp_path):
    rng = np.random.default_rng(2)
    img = _rand_rgba(rng, 20, 31)
    p = tmp_path / "x.ppm"
    rt.imageio.write_image(str(p), img)
    assert open(str(p), "rb").read(2) == b"P6"
    assert np.array_equal(rt.imageio.read_image(str(p)), img[..., :3])
    assert np.array_equal(np.asarray(Image.open(str(p)).convert("RGB")), img[..., :3])


def test_non_opaque_frames_are_rejected():
    img = np.zeros((4, 4, 4), dtype=np.uint8)
    with pytest.raises(ValueError):
        rt.imageio.encode_png(img)


def test_golden_png_decodes_to_itself():
    gold = np.asarray(Image.open(os.path.join(GOLDEN, "example_canned.png")).convert("RGB"))
    data = rt.imageio.encode_png(gold)
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(data)).convert("RGB")), gold)


def test_ssim_same_image_is_one():
    # TestSSIMSameImage: >= 0.999
    img = _rand_rgba(np.random.default_rng(3), 100, 100)
    assert ssim_ref.ssim(img, img) >= 0.999


def test_ssim_different_images_below_one():
    # TestSSIMDifferentImages: <= 0.999
    rng = np.random.default_rng(4)
    assert ssim_ref.ssim(_rand_rgba(rng, 100, 100), _rand_rgba(rng, 100, 100)) < 0.999


def test_ssim_errors_and_degenerate_sizes():
    a = np.zeros((20, 20, 3), dtype=np.uint8)
    with pytest.raises(ValueError, match="same size"):
        ssim_ref.ssim(a, np.zeros((20, 21, 3), dtype=np.uint8))
    with pytest.raises(ValueError, match="too small"):
        ssim_ref.ssim(np.zeros((10, 30, 3), np.uint8), np.zeros((10, 30, 3), np.uint8))
    # exactly 11 wide: the reference visits no window (x < W - 11) -> 0/0
    assert math.isnan(ssim_ref.ssim(np.zeros((11, 30, 3), np.uint8), np.zeros((11, 30, 3), np.uint8)))


def test_ssim_windows_skip_last_row_and_column():
    # only the last column differs: no visited window covers it (ssim.go:53-58)
    rng = np.random.default_rng(5)
    a = _rand_rgba(rng, 30, 30)
    b = a.copy()
    b[:, -1, :3] = 255 - b[:, -1, :3]
    assert ssim_ref.ssim(a, b) == ssim_ref.ssim(a, a)


def test_ssim_gaussian_kernel_normalised():
    k = ssim_ref.gaussian_kernel()
    assert abs(sum(k) - 1.0) < 1e-15 and k[60] == max(k)

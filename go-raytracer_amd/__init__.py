"""MI355X-native renderer for the ICFP-2000 GML raytracer hot path.

Layout:
  csrc/rt_kernel.hip   HIP megakernel (gfx950) + the C ABI of include/rt_abi.h
  csrc/rt_ssim.hip     device SSIM (the reference's parity metric)
  abi.py               ctypes mirror of include/rt_abi.h
  scene.py             host scene values, BFS flattening, surface baking
  gomath.py            Go float64 host math (transform matrices)
  configs.py           canned.gml and the BASELINE configs C1..C5
  csrc/rt_render_api.hip  rt_render / rt_render_ex: the Render() seam over 1..16 GPUs
  render.py            Render(): the reference's entry point over the C ABI
  dist.py              tile-row / row-band sharding across GPUs + RCCL gather
  imageio.py           PNG / PPM output, SSIM
  gml/                 host GML front end + closure-surface compiler
"""
from . import abi, configs, dist, gomath, imageio, scene  # noqa: F401
from .render import Render, RenderContext, load_library, render_frame, spec_precompile  # noqa: F401

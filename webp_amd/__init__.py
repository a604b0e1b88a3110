"""webp_amd -- MI355X (gfx950) implementation of the deepteams/webp
internal/dsp hot path behind a C ABI (include/webpgpu.h).

Submodules:
  dsp     -- batched mirror of internal/dsp's function variables
  frames  -- frame-level seams (decode reconstruct+filter, import, analysis,
             fancy upsampling, plane SSIM)
"""
from . import _lib  # noqa: F401  (raises if libwebpgpu.so is missing)
from ._lib import LIB_PATH, WebpGpuError  # noqa: F401


def device_check():
    """Raise unless the current HIP device is a gfx950."""
    _lib.call("wg_device_check")

"""VP8L predictor transform on the GPU, mirroring the reference's
internal/lossless entry points:

  ResidualImage(argb, bits, quality)      encode_predictor.go:378-455
  predictor_inverse(modes, bits, resid)   decode_transform.go:202-360 (predictorInverseTransform)
  SubtractGreen(argb) / AddGreen(argb)    encode_predictor.go:461, dsp/lossless_dsp.go:12

and the cross-colour / colour-index transforms:

  ColorSpaceTransform(argb, bits)         encode_predictor.go:727-770 (in place)
  color_space_inverse(data, bits, src)    decode_transform.go:454-520
  color_index_inverse(palette, xbits, w, src)  decode_transform.go:560-612

ARGB images are (n, h, w) int32 CUDA tensors holding 0xAARRGGBB words (the
reference's []uint32; torch has no uint32 arithmetic, the bits are the same).
"""
import numpy as np
import torch

from ._lib import call, lib


def _stream():
    return torch.cuda.current_stream().cuda_stream


def subsample(size, bits):
    """VP8LSubSampleSize (internal/lossless/constants.go:212)."""
    return (size + (1 << bits) - 1) >> bits


def _batched(argb):
    assert argb.is_cuda and argb.dtype == torch.int32 and argb.is_contiguous()
    return argb if argb.dim() == 3 else argb.unsqueeze(0)


def ResidualImage(argb, bits, quality, out=None):
    """-> (modes (n, tiles_y, tiles_x) int32 = mode<<8|0xff000000, residuals like argb)."""
    a = _batched(argb)
    n, h, w = a.shape
    if out is None:
        modes = torch.empty((n, subsample(h, bits), subsample(w, bits)), dtype=torch.int32, device=a.device)
        res = torch.empty_like(a)
    else:
        modes, res = out
    call("wg_vp8l_residual_image", a.data_ptr(), w, h, h * w, bits, quality, n, modes.data_ptr(), res.data_ptr(),
         _stream())
    return modes, res


def ResidualImage_devices(argb, bits, quality, devices):
    """ResidualImage of one (h, w) HOST image (uint32 / int32 numpy) by tile-row
    bands over `devices` (wg_vp8l_residual_image_devices) -> host (modes
    (tiles_y, tiles_x), residuals (h, w)) as uint32."""
    a = np.ascontiguousarray(argb).view(np.uint32)
    h, w = a.shape
    devs = np.ascontiguousarray(devices, dtype=np.int32)
    modes = np.empty((subsample(h, bits), subsample(w, bits)), np.uint32)
    res = np.empty((h, w), np.uint32)
    call("wg_vp8l_residual_image_devices", devs.ctypes.data, len(devs), a.ctypes.data, w, h, bits, quality,
         modes.ctypes.data, res.ctypes.data)
    return modes, res


def predictor_inverse(modes, bits, residuals, out=None, check=False):
    r = _batched(residuals)
    n, h, w = r.shape
    if out is None:
        out = torch.empty_like(r)
    work = torch.empty(lib.wg_vp8l_inverse_work_bytes(w, h, n), dtype=torch.uint8, device=r.device)
    call("wg_vp8l_inverse_predictor", modes.data_ptr(), bits, w, h, h * w, n, r.data_ptr(), out.data_ptr(),
         work.data_ptr(), _stream())
    if check:
        call("wg_vp8l_inverse_status", work.data_ptr(), _stream())
    return out


def SubtractGreen(argb):
    """In place, like the reference."""
    call("wg_vp8l_green", argb.data_ptr(), argb.numel(), 0, _stream())
    return argb


def AddGreen(argb):
    call("wg_vp8l_green", argb.data_ptr(), argb.numel(), 1, _stream())
    return argb


def ColorSpaceTransform(argb, bits, data=None):
    """Forward cross-colour transform in place; -> multiplier words (n, tiles_y, tiles_x)
    (g2r | g2b << 8 | r2b << 16, packMultipliers)."""
    a = _batched(argb)
    n, h, w = a.shape
    if data is None:
        data = torch.empty((n, subsample(h, bits), subsample(w, bits)), dtype=torch.int32, device=a.device)
    call("wg_vp8l_color_space_transform", a.data_ptr(), w, h, h * w, bits, n, data.data_ptr(), _stream())
    return data


def color_space_inverse(data, bits, src, out=None):
    s = _batched(src)
    n, h, w = s.shape
    if out is None:
        out = torch.empty_like(s)
    call("wg_vp8l_color_space_inverse", data.data_ptr(), bits, w, h, h * w, n, s.data_ptr(), out.data_ptr(), _stream())
    return out


def color_index_inverse(palette, xbits, width, src, out=None):
    """src (n, h, subsample(width, xbits)) packed index words; palette (<=256,) int32
    shared by the n images.  Out-of-palette indices leave `out` untouched."""
    s = _batched(src)
    n, h, pw = s.shape
    assert pw == subsample(width, xbits)
    if out is None:
        out = torch.zeros((n, h, width), dtype=torch.int32, device=s.device)
    call("wg_vp8l_color_index_inverse", palette.data_ptr(), palette.numel(), xbits, width, h, n, s.data_ptr(), h * pw,
         out.data_ptr(), h * width, _stream())
    return out


def slog2_lut(n=65536):
    out = np.zeros(n, np.float64)
    call("wg_vp8l_slog2_lut_host", out.ctypes.data, n)
    return out


def to_argb_tensor(u32, device="cuda"):
    """numpy uint32 (.., h, w) -> int32 CUDA tensor with the same bits."""
    return torch.from_numpy(np.ascontiguousarray(u32, np.uint32).view(np.int32)).to(device)


def from_argb_tensor(t):
    return t.cpu().numpy().view(np.uint32)

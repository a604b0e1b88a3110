"""Alpha-plane filters and alpha processing on the GPU,
mirroring the reference's entry points:

  alpha_filter(filter, planes)          alphaFilter{Horizontal,Vertical,Gradient}
                                        internal/lossy/alpha.go:387-454
  alpha_unfilter(filter, planes)        alphaUnfilter* alpha.go:128-203 (in place)
  estimate_best_filter(planes)          estimateBestFilter alpha.go:321-385
                                        + getNumColors :302-317
  ApplyAlphaMultiply / MultARGBRow / ApplyAlphaMultiply4444 / DispatchAlpha /
  ExtractAlpha / HasAlpha8b / HasAlpha32b / AlphaReplace /
  DispatchAlphaToGreen / ExtractGreen / PackRGB
                                        internal/dsp/alpha_proc.go:28-238

Alpha planes are (n, h, w) or (h, w) uint8 CUDA tensors; ARGB words are int32
tensors holding the 0xAARRGGBB bits.  Results the Go functions return (bool /
int) come back as Python values after a stream synchronisation; the *_async
forms leave them on the device.
"""
import torch

from ._lib import call, lib

NONE, HORIZONTAL, VERTICAL, GRADIENT = 0, 1, 2, 3  # AlphaFilter* (alpha.go)


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _planes(t, dtype=torch.uint8):
    assert t.is_cuda and t.dtype == dtype and t.is_contiguous()
    return t if t.dim() == 3 else t.unsqueeze(0)


def alpha_filter(filter_, planes, out=None):
    p = _planes(planes)
    n, h, w = p.shape
    if out is None:
        out = torch.empty_like(planes)
    assert out.data_ptr() != p.data_ptr(), "alpha_filter: in and out must not alias"
    call("wg_alpha_filter", filter_, p.data_ptr(), out.data_ptr(), w, h, h * w, n, _stream())
    return out


def alpha_unfilter(filter_, planes, check=False):
    """In place; check=True synchronises and raises if a gradient band wait timed out."""
    p = _planes(planes)
    n, h, w = p.shape
    work = torch.empty(max(lib.wg_alpha_unfilter_work_bytes(w, h, n), 16), dtype=torch.uint8, device=p.device)
    call("wg_alpha_unfilter", filter_, p.data_ptr(), w, h, h * w, n, work.data_ptr(), _stream())
    if check and filter_ == GRADIENT and h > 1:
        call("wg_alpha_unfilter_status", work.data_ptr(), _stream())
    return planes


def estimate_best_filter_async(planes):
    """-> (best_filter int32[n], num_colors int32[n]) device tensors."""
    p = _planes(planes)
    n, h, w = p.shape
    best = torch.empty(n, dtype=torch.int32, device=p.device)
    colors = torch.empty(n, dtype=torch.int32, device=p.device)
    work = torch.empty(lib.wg_alpha_estimate_work_bytes(n), dtype=torch.uint8, device=p.device)
    call("wg_alpha_estimate_filter", p.data_ptr(), w, h, h * w, n, best.data_ptr(), colors.data_ptr(),
         work.data_ptr(), _stream())
    return best, colors


def estimate_best_filter(planes):
    best, _ = estimate_best_filter_async(planes)
    return best.tolist() if planes.dim() == 3 else int(best[0])


def get_num_colors(planes):
    _, colors = estimate_best_filter_async(planes)
    return colors.tolist() if planes.dim() == 3 else int(colors[0])


def ApplyAlphaMultiply(rgba, alpha_first, width, height, stride, inverse):
    """rgba: uint8 tensor, (n, pitch) for n images or flat for one; in place."""
    assert rgba.is_cuda and rgba.dtype == torch.uint8 and rgba.is_contiguous()
    n = rgba.shape[0] if rgba.dim() == 2 else 1
    pitch = rgba.shape[-1] if rgba.dim() == 2 else rgba.numel()
    call("wg_apply_alpha_multiply", rgba.data_ptr(), int(alpha_first), width, height, stride, pitch, n,
         int(inverse), _stream())
    return rgba


def MultARGBRow(argb, inverse):
    assert argb.is_cuda and argb.dtype == torch.int32 and argb.is_contiguous()
    call("wg_mult_argb", argb.data_ptr(), argb.numel(), int(inverse), _stream())
    return argb


def ApplyAlphaMultiply4444(data, width, height, stride):
    assert data.is_cuda and data.dtype == torch.uint8 and data.is_contiguous()
    n = data.shape[0] if data.dim() == 2 else 1
    pitch = data.shape[-1] if data.dim() == 2 else data.numel()
    call("wg_apply_alpha_multiply_4444", data.data_ptr(), width, height, stride, pitch, n, _stream())
    return data


def _flag(device):
    return torch.empty(1, dtype=torch.int32, device=device)


def DispatchAlpha(alpha, alpha_stride, width, height, dst, dst_stride, alpha_off):
    """-> True if any alpha != 0xff (alpha_proc.go:140)."""
    f = _flag(alpha.device)
    call("wg_dispatch_alpha", alpha.data_ptr(), alpha_stride, width, height, dst.data_ptr(), dst_stride, alpha_off,
         f.data_ptr(), _stream())
    return bool(f.item())


def ExtractAlpha(src, src_stride, width, height, alpha, alpha_stride, alpha_off):
    """-> 1 if every alpha is 0xff, else 0 (alpha_proc.go:158)."""
    f = _flag(src.device)
    call("wg_extract_alpha", src.data_ptr(), src_stride, width, height, alpha.data_ptr(), alpha_stride, alpha_off,
         f.data_ptr(), _stream())
    return int(f.item())


def HasAlpha8b(src, length):
    f = _flag(src.device)
    call("wg_has_alpha", src.data_ptr(), length, 1, f.data_ptr(), _stream())
    return bool(f.item())


def HasAlpha32b(src, length):
    f = _flag(src.device)
    call("wg_has_alpha", src.data_ptr(), length, 4, f.data_ptr(), _stream())
    return bool(f.item())


def AlphaReplace(argb, length, color):
    call("wg_alpha_replace", argb.data_ptr(), length, color & 0xffffffff, _stream())
    return argb


def DispatchAlphaToGreen(alpha, alpha_stride, width, height, dst, dst_stride):
    call("wg_dispatch_alpha_to_green", alpha.data_ptr(), alpha_stride, width, height, dst.data_ptr(), dst_stride,
         _stream())
    return dst


def ExtractGreen(argb, alpha, size):
    call("wg_extract_green", argb.data_ptr(), alpha.data_ptr(), size, _stream())
    return alpha


def PackRGB(r, g, b, length, step, out):
    call("wg_pack_rgb", r.data_ptr(), g.data_ptr(), b.data_ptr(), length, step, out.data_ptr(), _stream())
    return out

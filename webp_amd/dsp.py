"""Host mirror of deepteams/webp ``internal/dsp`` (dsp.go:10-37, ssim.go:251-254)
over the batched GPU entry points of libwebpgpu.so.

Every function keeps the reference's name and argument meaning, with one
batch dimension in front: ``bufs`` is a (n, L) uint8 CUDA tensor of n
independent caller-owned buffers (the reference's ``[]byte``), ``off`` is
the block origin inside each buffer, and results are written in place
exactly where the Go function writes them.  Computation always runs on the
GPU; there is no CPU path.
"""
import torch

from ._lib import WebpGpuError, call

WG_EINVAL = -1  # include/webpgpu.h


class InvalidArgument(WebpGpuError, ValueError):
    """A block call whose footprint leaves its buffer: the reference panics
    with a Go bounds-check error; the host mirror refuses it (status WG_EINVAL)
    before any device work, since the device entry points take bare pointers."""
    status = WG_EINVAL

BPS = 32  # internal/dsp/dsp.go:5
YUV_SIZE = BPS * 17 + BPS * 9  # internal/lossy/constants.go:70-75
YOFF = BPS + 8
UOFF = YOFF + BPS * 16 + BPS
VOFF = UOFF + 16

# transform kinds (webpgpu.h wg_transform)
_T_ONE, _T_TWO, _T_AC3, _T_DC, _T_UV, _T_DCUV = range(6)
# metric kinds
_M_SSE4, _M_SSE16, _M_TD4, _M_TD16 = range(4)
# filter kinds (webpgpu.h wg_filter)
FILTER_KINDS = {
    "SimpleVFilter16": 0, "SimpleHFilter16": 1, "SimpleVFilter16i": 2, "SimpleHFilter16i": 3,
    "VFilter16": 4, "HFilter16": 5, "VFilter16i": 6, "HFilter16i": 7,
    "VFilter8": 8, "HFilter8": 9, "VFilter8i": 10, "HFilter8i": 11,
}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _dev(t, dtype=None):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise TypeError("webp_amd.dsp expects CUDA (HIP) tensors")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return t


def _modes(modes, n, device):
    if isinstance(modes, int):
        modes = torch.full((n,), modes, dtype=torch.uint8, device=device)
    return _dev(modes.to(torch.uint8) if modes.dtype != torch.uint8 else modes)


def _offs(off, n, device):
    if isinstance(off, int):
        return None, off
    return _dev(off.to(torch.int32).to(device).contiguous()), 0


def _span(lo, hi, length, what):
    """Every byte offset a call touches lies in [lo, hi); the buffer has `length`."""
    if lo < 0 or hi > length:
        raise InvalidArgument(f"{what}: touches bytes [{lo}, {hi}) of a {length}-byte buffer (status {WG_EINVAL})")


def _check_offs(off, lo_rel, hi_rel, length, what):
    """Block origin(s) `off` (int, or a tensor of per-instance origins) with the
    footprint [off + lo_rel, off + hi_rel) inside every buffer."""
    if isinstance(off, int):
        _span(off + lo_rel, off + hi_rel, length, what)
    elif off.numel():
        o = off.to(torch.int64)
        _span(int(o.min()) + lo_rel, int(o.max()) + hi_rel, length, what)


def _block(off, rows, cols, stride=BPS):
    """[lo, hi) of a rows x cols block at `off` (row stride `stride`)."""
    return off, off + (rows - 1) * stride + cols


def _need_cols(t, cols, what):
    if t.dim() != 2 or t.shape[1] < cols:
        raise InvalidArgument(f"{what}: rows of {tuple(t.shape)[1:]} elements, the call uses {cols} (status {WG_EINVAL})")


# ---- intra predictors (predict_lossy.go, dsp.go:33-37) ----

_PRED_SIZE = {"wg_pred_luma4": (4, 8), "wg_pred_luma16": (16, 16), "wg_pred_chroma8": (8, 8)}


def _pred(name, modes, bufs, off):
    _dev(bufs, torch.uint8)
    n = bufs.shape[0]
    m = _modes(modes, n, bufs.device)
    # the block, its left column, the top row from the top-left corner (luma4:
    # and the 4 top-right pixels) -- predict_lossy.go's reads around off
    size, top = _PRED_SIZE[name]
    _check_offs(off, -BPS - 1, (size - 1) * BPS + size if size > 4 else max(3 * BPS + 4, -BPS + top),
                bufs.shape[1], name)
    offs, o = _offs(off, n, bufs.device)
    call(name, m.data_ptr(), bufs.data_ptr(), bufs.stride(0), offs.data_ptr() if offs is not None else None, o, n,
         _stream())


def PredLuma4(modes, bufs, off):
    """PredLuma4[mode](buf, off) for each buffer (predict_lossy.go:185-451)."""
    _pred("wg_pred_luma4", modes, bufs, off)


def PredLuma16(modes, bufs, off):
    """PredLuma16[mode](buf, off) (predict_lossy.go:27-102)."""
    _pred("wg_pred_luma16", modes, bufs, off)


def PredChroma8(modes, bufs, off):
    """PredChroma8[mode](buf, off) (predict_lossy.go:106-181)."""
    _pred("wg_pred_chroma8", modes, bufs, off)


# ---- transforms (transforms.go, dsp.go:10-24) ----

# kind -> (coefficients read, rows x cols of dst written)
_T_SHAPE = {_T_ONE: (16, 4, 4), _T_TWO: (32, 4, 8), _T_AC3: (16, 4, 4), _T_DC: (16, 4, 4), _T_UV: (64, 8, 8),
            _T_DCUV: (64, 8, 8)}


def _transform(kind, coeffs, dst, off):
    _dev(coeffs, torch.int16)
    _dev(dst, torch.uint8)
    n = dst.shape[0]
    nco, rows, cols = _T_SHAPE[kind]
    _need_cols(coeffs, nco, "wg_transform coeffs")
    if coeffs.shape[0] != n:
        raise InvalidArgument(f"wg_transform: {coeffs.shape[0]} coefficient rows for {n} buffers")
    _check_offs(off, 0, (rows - 1) * BPS + cols, dst.shape[1], "wg_transform dst")
    call("wg_transform", kind, coeffs.data_ptr(), coeffs.stride(0), dst.data_ptr() + off, dst.stride(0), n,
         _stream())


def Transform(coeffs, dst, do_two, off=0):
    """Transform(coeffs, dst[off:], doTwo) -- transformTwo (transforms.go:139)."""
    _transform(_T_TWO if do_two else _T_ONE, coeffs, dst, off)


def TransformAC3(coeffs, dst, off=0):
    _transform(_T_AC3, coeffs, dst, off)


def TransformDC(coeffs, dst, off=0):
    _transform(_T_DC, coeffs, dst, off)


def TransformUV(coeffs, dst, off=0):
    _transform(_T_UV, coeffs, dst, off)


def TransformDCUV(coeffs, dst, off=0):
    _transform(_T_DCUV, coeffs, dst, off)


def TransformWHT(inp, out):
    """TransformWHT(in[16], out[256]) (transforms.go:223): DCs land at out[16*k]."""
    _dev(inp, torch.int16)
    _dev(out, torch.int16)
    _need_cols(inp, 16, "TransformWHT in")
    _need_cols(out, 241, "TransformWHT out")
    call("wg_transform_wht", inp.data_ptr(), out.data_ptr(), inp.shape[0], _stream())


def FTransformWHT(inp, out):
    """FTransformWHT on a flat 4x4 DC array (transforms.go:500)."""
    _dev(inp, torch.int16)
    _dev(out, torch.int16)
    _need_cols(inp, 16, "FTransformWHT in")
    _need_cols(out, 16, "FTransformWHT out")
    call("wg_ftransform_wht", inp.data_ptr(), out.data_ptr(), inp.shape[0], _stream())


def ITransform(ref, inp, dst, do_two, ref_off=0, dst_off=0):
    """ITransform(ref, in, dst, doTwo) (transforms.go:256).  ref and dst are the
    same (n, L) buffer tensor at offsets ref_off / dst_off."""
    _dev(ref, torch.uint8)
    _dev(inp, torch.int16)
    _dev(dst, torch.uint8)
    assert ref.stride(0) == dst.stride(0) and inp.shape[1] == 32
    cols = 8 if do_two else 4
    _check_offs(ref_off, 0, 3 * BPS + cols, ref.shape[1], "ITransform ref")
    _check_offs(dst_off, 0, 3 * BPS + cols, dst.shape[1], "ITransform dst")
    call("wg_itransform", ref.data_ptr() + ref_off, inp.data_ptr(), dst.data_ptr() + dst_off, ref.stride(0),
         int(do_two), ref.shape[0], _stream())


def FTransform(src, ref, out, src_off=0, ref_off=0, two=False):
    """FTransform(src, ref, out) (transforms.go:371); two=True is FTransform2."""
    _dev(src, torch.uint8)
    _dev(ref, torch.uint8)
    _dev(out, torch.int16)
    assert src.stride(0) == ref.stride(0)
    cols = 8 if two else 4
    _check_offs(src_off, 0, 3 * BPS + cols, src.shape[1], "FTransform src")
    _check_offs(ref_off, 0, 3 * BPS + cols, ref.shape[1], "FTransform ref")
    _need_cols(out, 32 if two else 16, "FTransform out")
    call("wg_ftransform", src.data_ptr() + src_off, ref.data_ptr() + ref_off, src.stride(0), out.data_ptr(),
         int(two), src.shape[0], _stream())


def FTransform2(src, ref, out, src_off=0, ref_off=0):
    FTransform(src, ref, out, src_off, ref_off, two=True)


# ---- distortion (ssim.go) ----

def _metric(kind, pix, ref, pix_off, ref_off):
    _dev(pix, torch.uint8)
    _dev(ref, torch.uint8)
    assert pix.stride(0) == ref.stride(0)
    size = 4 if kind in (_M_SSE4, _M_TD4) else 16
    _check_offs(pix_off, 0, (size - 1) * BPS + size, pix.shape[1], "wg_metric pix")
    _check_offs(ref_off, 0, (size - 1) * BPS + size, ref.shape[1], "wg_metric ref")
    out = torch.empty(pix.shape[0], dtype=torch.int32, device=pix.device)
    call("wg_metric", kind, pix.data_ptr() + pix_off, ref.data_ptr() + ref_off, pix.stride(0), out.data_ptr(),
         pix.shape[0], _stream())
    return out


def SSE4x4(pix, ref, pix_off=0, ref_off=0):
    return _metric(_M_SSE4, pix, ref, pix_off, ref_off)


def SSE16x16(pix, ref, pix_off=0, ref_off=0):
    return _metric(_M_SSE16, pix, ref, pix_off, ref_off)


def TDisto4x4(a, b, a_off=0, b_off=0):
    return _metric(_M_TD4, a, b, a_off, b_off)


def TDisto16x16(a, b, a_off=0, b_off=0):
    return _metric(_M_TD16, a, b, a_off, b_off)


def SSIMGet(src1, src2, stride):
    """SSIMGet(src1, stride, src2, stride) (ssim.go:116) per buffer pair."""
    _dev(src1, torch.uint8)
    _dev(src2, torch.uint8)
    _span(0, 6 * stride + 7, min(src1.shape[1], src2.shape[1]), "SSIMGet 7x7 window")
    out = torch.empty(src1.shape[0], dtype=torch.float64, device=src1.device)
    call("wg_ssim_get", src1.data_ptr(), src2.data_ptr(), src1.stride(0), stride, None, out.data_ptr(),
         src1.shape[0], _stream())
    return out


def SSIMGetClipped(src1, src2, stride, xywh):
    """SSIMGetClipped(src1, stride, src2, stride, xo, yo, W, H) (ssim.go:132); xywh (n, 4) int32."""
    _dev(src1, torch.uint8)
    _dev(src2, torch.uint8)
    xywh = _dev(xywh.to(torch.int32).contiguous())
    out = torch.empty(src1.shape[0], dtype=torch.float64, device=src1.device)
    call("wg_ssim_get", src1.data_ptr(), src2.data_ptr(), src1.stride(0), stride, xywh.data_ptr(), out.data_ptr(),
         src1.shape[0], _stream())
    return out


# ---- loop filters (filter.go:93-242) ----

def filter_span(name, base, stride, uv_delta=0):
    """[lo, hi) of the bytes dsp.<name> reads or writes (filter.go:93-242): an
    edge filter at o with normal step h, edge step v over s positions touches
    o + a*h .. o + b*h + (s - 1)*v, (a, b) = (-2, 1) simple / (-4, 3) normal;
    the inner variants at o = base + 4k (k = 1..3, chroma k = 1) steps."""
    simple = name.startswith("Simple")
    a, b = (-2, 1) if simple else (-4, 3)
    vert = "VFilter" in name
    s = 8 if name.endswith(("8", "8i")) else 16
    h, v = (stride, 1) if vert else (1, stride)
    ks = ((1, 2, 3) if s == 16 else (1,)) if name.endswith("i") else (0,)
    origins = [base + 4 * k * h for k in ks]
    if s == 8:
        origins += [o + uv_delta for o in origins]
    return min(o + a * h for o in origins), max(o + b * h + (s - 1) * v for o in origins) + 1


def filter_edge(name, p, base, stride, thresh, ithresh=None, hev=None, uv_delta=0):
    """Apply dsp.<name>(p, base, stride, thresh[, ithresh, hevT]) to every buffer.
    For the 8-pixel chroma filters the V plane is p + uv_delta."""
    _dev(p, torch.uint8)
    n = p.shape[0]

    def vec(x):
        if x is None:
            return None
        if isinstance(x, int):
            x = torch.full((n,), x, dtype=torch.int32, device=p.device)
        return _dev(x.to(torch.int32).contiguous())
    t, it, h = vec(thresh), vec(ithresh), vec(hev)
    lo, hi = filter_span(name, base, stride, uv_delta)
    _span(lo, hi, p.shape[1], name)
    call("wg_filter", FILTER_KINDS[name], p.data_ptr(), p.stride(0), base, stride, uv_delta, t.data_ptr(),
         it.data_ptr() if it is not None else None, h.data_ptr() if h is not None else None, n, _stream())


# ---- line-pair upsampler (upsample.go:45-236, upsample_direct_amd64.go:10) ----

def _rows(t, n=None, need=0, dtype=torch.uint8):
    """A (n, L) batch of rows; each row must hold the `need` elements the call reads."""
    _dev(t, dtype)
    if t.dim() != 2 or (n is not None and t.shape[0] != n):
        raise ValueError(f"expected (n, L) rows{'' if n is None else f' with n = {n}'}, got {tuple(t.shape)}")
    if t.shape[1] < need:
        raise ValueError(f"rows of {t.shape[1]} elements, the call reads {need}")
    return t


def _plane_need(width, height, stride):
    """elements a (width x height, stride) block spans: (height - 1) * stride + width"""
    if stride < width:
        raise ValueError("stride < width")
    return 0 if width <= 0 or height <= 0 else (height - 1) * stride + width


def _line_pairs(fmt, top_y, bot_y, top_u, top_v, bot_u, bot_v, width, alpha_top=None, alpha_bot=None):
    cw = (width + 1) // 2
    n = _rows(top_y, None, width).shape[0]
    for t in (top_u, top_v, bot_u, bot_v):
        _rows(t, n, cw)
        assert t.stride(0) == top_u.stride(0)
    if bot_y is not None:
        assert _rows(bot_y, n, width).stride(0) == top_y.stride(0)
    for t in (alpha_top, alpha_bot):
        if t is not None:
            _rows(t, n, width)
    bpp = 4 if fmt else 3
    top_dst = torch.empty((n, bpp * width), dtype=torch.uint8, device=top_y.device)
    bot_dst = torch.empty_like(top_dst) if bot_y is not None else None
    if alpha_top is not None and alpha_bot is not None:
        assert alpha_top.stride(0) == alpha_bot.stride(0)
    a_step = alpha_top.stride(0) if alpha_top is not None else (alpha_bot.stride(0) if alpha_bot is not None else 0)
    call("wg_upsample_line_pairs", fmt, top_y.data_ptr(), bot_y.data_ptr() if bot_y is not None else None,
         top_y.stride(0), top_u.data_ptr(), top_v.data_ptr(), bot_u.data_ptr(), bot_v.data_ptr(), top_u.stride(0),
         top_dst.data_ptr(), bot_dst.data_ptr() if bot_dst is not None else None, top_dst.stride(0),
         alpha_top.data_ptr() if alpha_top is not None else None,
         alpha_bot.data_ptr() if alpha_bot is not None else None, a_step, width, n, _stream())
    return top_dst, bot_dst


def UpsampleLinePair(top_y, bot_y, top_u, top_v, bot_u, bot_v, width):
    """UpsampleLinePair (upsample.go:45) for n line pairs: rows are (n, L)
    uint8 CUDA tensors (bot_y None = an odd height's last row); returns
    (topDst, botDst) as (n, 3*width) RGB rows."""
    return _line_pairs(0, top_y, bot_y, top_u, top_v, bot_u, bot_v, width)


def UpsampleLinePairNRGBA(top_y, bot_y, top_u, top_v, bot_u, bot_v, width, alpha_top=None, alpha_bot=None):
    """UpsampleLinePairNRGBA (upsample_direct_amd64.go:10): (n, 4*width) NRGBA
    rows; alpha rows None -> 255."""
    return _line_pairs(1, top_y, bot_y, top_u, top_v, bot_u, bot_v, width, alpha_top, alpha_bot)


def PointSampleRow(y, u, v, width):
    """PointSampleRow(y, u, v, dst, width) (upsample.go:240) for n rows: y
    (n, >= width), u / v (n, >= (width + 1) // 2) uint8; returns dst (n, 3*width) RGB."""
    n = _rows(y, None, width).shape[0]
    _rows(u, n, (width + 1) // 2)
    assert _rows(v, n, (width + 1) // 2).stride(0) == u.stride(0)
    dst = torch.empty((n, 3 * width), dtype=torch.uint8, device=y.device)
    call("wg_point_sample_rows", y.data_ptr(), u.data_ptr(), v.data_ptr(), y.stride(0), u.stride(0), dst.data_ptr(),
         dst.stride(0), width, n, _stream())
    return dst


# ---- packed ARGB -> YUV rows (yuv.go:255-330) ----

def _argb_rows(argb, width):
    if argb.dtype == torch.int32:  # torch has no uint32 arithmetic; the bits are what count
        argb = argb.view(torch.uint32)
    return _rows(argb, None, width, torch.uint32)


def ConvertARGBToY(argb, width):
    """ConvertARGBToY(argb, y, width) (yuv.go:270): argb (n, >= width) packed
    0xAARRGGBB uint32 (or int32 bits); returns y (n, width) uint8."""
    argb = _argb_rows(argb, width)
    n = argb.shape[0]
    y = torch.empty((n, width), dtype=torch.uint8, device=argb.device)
    call("wg_convert_argb_to_y", argb.data_ptr(), argb.stride(0), y.data_ptr(), y.stride(0), width, n, _stream())
    return y


def ConvertARGBToUV(argb, src_width, do_store, u=None, v=None):
    """ConvertARGBToUV(argb, u, v, srcWidth, doStore) (yuv.go:291) for n rows:
    returns (u, v) (n, (src_width + 1) // 2); with do_store False the samples
    are averaged into u / v (given, updated in place), as the Go call does."""
    argb = _argb_rows(argb, src_width)
    n, cw = argb.shape[0], (src_width + 1) // 2
    if u is None or v is None:
        if not do_store:
            raise ValueError("doStore false averages into existing u, v rows")
        u = torch.empty((n, cw), dtype=torch.uint8, device=argb.device)
        v = torch.empty_like(u)
    _rows(u, n, cw)
    assert _rows(v, n, cw).stride(0) == u.stride(0)
    call("wg_convert_argb_to_uv", argb.data_ptr(), argb.stride(0), u.data_ptr(), v.data_ptr(), u.stride(0), src_width,
         int(bool(do_store)), n, _stream())
    return u, v


# ---- RGBA -> YUV420 chroma helpers (yuv.go:486-576, random.go) ----

def AccumulateRGBA(r, g, b, a, stride, width):
    """AccumulateRGBA(r, g, b, a, stride, dst, width) (yuv.go:486) for n row
    pairs: r/g/b/a are (n, L) uint8 planar rows (second row at +stride);
    returns dst as (n, 4 * ceil(width / 2)) uint16."""
    need = stride + width if width > 0 else 0  # the second row at +stride
    if stride < width:
        raise ValueError("stride < width")
    n = _rows(r, None, need).shape[0]
    for t in (g, b, a):
        assert _rows(t, n, need).stride(0) == r.stride(0)
    dst = torch.empty((n, 4 * ((width + 1) // 2)), dtype=torch.uint16, device=r.device)
    call("wg_accumulate_rgba", r.data_ptr(), g.data_ptr(), b.data_ptr(), a.data_ptr(), stride, r.stride(0),
         dst.data_ptr(), dst.stride(0), width, n, _stream())
    return dst


def ConvertRGBA32ToUV(rgb, width):
    """ConvertRGBA32ToUV(rgb, u, v, width) (yuv.go:553): rgb (n, >= 4*width) uint16; returns (u, v) (n, width)."""
    _rows(rgb, None, 4 * width, torch.uint16)
    n = rgb.shape[0]
    u = torch.empty((n, width), dtype=torch.uint8, device=rgb.device)
    v = torch.empty_like(u)
    call("wg_convert_rgba32_to_uv", rgb.data_ptr(), rgb.stride(0), u.data_ptr(), v.data_ptr(), u.stride(0), width, n,
         _stream())
    return u, v


RANDOM_BYTES = 232  # wg_random (VP8Random)


def InitRandom(dithering, n=1, device="cuda"):
    """InitRandom(rg, dithering) (random.go:39) -> (n, 232) uint8 CUDA tensor of wg_random states."""
    import ctypes

    import numpy as np
    from ._lib import lib
    host = np.zeros(RANDOM_BYTES, np.uint8)
    lib.wg_random_init_host(host.ctypes.data_as(ctypes.c_void_p), float(dithering))
    return torch.from_numpy(np.tile(host, (n, 1))).to(device)


def ConvertRGBA32ToUVDithered(rgb, width, states):
    """ConvertRGBA32ToUVDithered(rgb, u, v, width, rg) (yuv.go:568): row i
    draws from states[i] (InitRandom), which advance in place."""
    _rows(rgb, None, 4 * width, torch.uint16)
    _dev(states, torch.uint8)
    n = rgb.shape[0]
    assert states.shape == (n, RANDOM_BYTES)
    u = torch.empty((n, width), dtype=torch.uint8, device=rgb.device)
    v = torch.empty_like(u)
    call("wg_convert_rgba32_to_uv_dithered", rgb.data_ptr(), rgb.stride(0), u.data_ptr(), v.data_ptr(), u.stride(0),
         width, states.data_ptr(), n, _stream())
    return u, v


# ---- SSE / PSNR / DistoStats (ssim.go:12-181) ----

def SSE(pix, ref, width, height, pix_stride, ref_stride):
    """SSE(pix, ref, width, height, pixStride, refStride) (ssim.go:172) per
    buffer pair: pix / ref (n, L) uint8; returns (n,) int64 (uint64 bits)."""
    n = _rows(pix, None, _plane_need(width, height, pix_stride)).shape[0]
    _rows(ref, n, _plane_need(width, height, ref_stride))
    out = torch.empty(n, dtype=torch.int64, device=pix.device)
    call("wg_sse_planes", pix.data_ptr(), ref.data_ptr(), width, height, pix_stride, ref_stride, pix.stride(0),
         ref.stride(0), out.data_ptr(), n, _stream())
    return out


def PSNRFromSSE(sse, count):
    """PSNRFromSSE(sse, count) (ssim.go:163): sse / count (n,) int64 -> (n,) float64."""
    _dev(sse, torch.int64)
    _dev(count, torch.int64)
    out = torch.empty(sse.shape[0], dtype=torch.float64, device=sse.device)
    call("wg_psnr_from_sse", sse.data_ptr(), count.data_ptr(), out.data_ptr(), sse.shape[0], _stream())
    return out


def DistoStatsOfBlocks(pix, ref, width, height, pix_stride, ref_stride):
    """The DistoStats that SSIMFromBlocks (ssim.go:103) accumulates, per block
    pair: (n, 6) int32 holding the uint32 fields (W, Xm, Ym, Xxm, Xym, Yym)."""
    n = _rows(pix, None, _plane_need(width, height, pix_stride)).shape[0]
    _rows(ref, n, _plane_need(width, height, ref_stride))
    out = torch.empty((n, 6), dtype=torch.int32, device=pix.device)
    call("wg_disto_stats_blocks", pix.data_ptr(), ref.data_ptr(), width, height, pix_stride, ref_stride,
         pix.stride(0), ref.stride(0), out.data_ptr(), n, _stream())
    return out


def SSIMFromStats(stats, clipped=False):
    """SSIMFromStats (ssim.go:88) / SSIMFromStatsClipped (:97): (n, 6) stats -> (n,) float64."""
    _dev(stats, torch.int32)
    out = torch.empty(stats.shape[0], dtype=torch.float64, device=stats.device)
    call("wg_ssim_from_stats", stats.data_ptr(), int(bool(clipped)), out.data_ptr(), stats.shape[0], _stream())
    return out


def SSIMFromBlocks(pix, ref, width, height, pix_stride, ref_stride):
    """SSIMFromBlocks (ssim.go:103): SSIMFromStatsClipped of the blocks' DistoStats."""
    return SSIMFromStats(DistoStatsOfBlocks(pix, ref, width, height, pix_stride, ref_stride), clipped=True)

"""TEST INFRASTRUCTURE ONLY -- ctypes view of the C restatement in oracle/.

The oracle restates deepteams/webp's Go internal/dsp hot path (and the lossy
decoder/encoder loops that drive it) in plain C.  Only tests/, the graft
smoke() check and bench.py's ``cpu_baseline`` leg may import this module, as
the checker / CPU baseline.  The product (webp_amd) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")

MB_INFO_DTYPE = np.dtype([
    ("non_zero_y", "<u4"), ("non_zero_uv", "<u4"), ("imodes", "u1", (16,)),
    ("is_i4x4", "u1"), ("uv_mode", "u1"), ("skip", "u1"), ("segment", "u1"),
    ("f_limit", "u1"), ("f_ilevel", "u1"), ("f_inner", "u1"), ("hev_thresh", "u1"),
])
assert MB_INFO_DTYPE.itemsize == 32

BPS = 32
YUV_SIZE = BPS * 17 + BPS * 9
YOFF = BPS + 8
UOFF = YOFF + BPS * 16 + BPS
VOFF = UOFF + 16


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    if not os.path.exists(_SO):
        build()
    return ctypes.CDLL(_SO)


lib = _load()

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i16p = ctypes.POINTER(ctypes.c_int16)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i = ctypes.c_int

_SIGS = {
    "or_transform": (None, [_i16p, _u8p, _i]),
    "or_transform_dc": (None, [_i16p, _u8p]),
    "or_transform_ac3": (None, [_i16p, _u8p]),
    "or_transform_uv": (None, [_i16p, _u8p]),
    "or_transform_dcuv": (None, [_i16p, _u8p]),
    "or_transform_wht": (None, [_i16p, _i16p]),
    "or_itransform": (None, [_u8p, _i16p, _u8p, _i]),
    "or_ftransform": (None, [_u8p, _u8p, _i16p]),
    "or_ftransform2": (None, [_u8p, _u8p, _i16p]),
    "or_ftransform_wht": (None, [_i16p, _i16p]),
    "or_pred_luma16": (None, [_i, _u8p, _i]),
    "or_pred_chroma8": (None, [_i, _u8p, _i]),
    "or_pred_luma4": (None, [_i, _u8p, _i]),
    "or_simple_vfilter16": (None, [_u8p, _i, _i, _i]),
    "or_simple_hfilter16": (None, [_u8p, _i, _i, _i]),
    "or_simple_vfilter16i": (None, [_u8p, _i, _i, _i]),
    "or_simple_hfilter16i": (None, [_u8p, _i, _i, _i]),
    "or_vfilter16": (None, [_u8p, _i, _i, _i, _i, _i]),
    "or_hfilter16": (None, [_u8p, _i, _i, _i, _i, _i]),
    "or_vfilter16i": (None, [_u8p, _i, _i, _i, _i, _i]),
    "or_hfilter16i": (None, [_u8p, _i, _i, _i, _i, _i]),
    "or_vfilter8": (None, [_u8p, _u8p, _i, _i, _i, _i, _i, _i]),
    "or_hfilter8": (None, [_u8p, _u8p, _i, _i, _i, _i, _i, _i]),
    "or_vfilter8i": (None, [_u8p, _u8p, _i, _i, _i, _i, _i, _i]),
    "or_hfilter8i": (None, [_u8p, _u8p, _i, _i, _i, _i, _i, _i]),
    "or_yuv_to_rgb": (None, [_i, _i, _i, _u8p]),
    "or_rgb_to_y": (_i, [_i, _i, _i]),
    "or_rgb_to_u": (_i, [_i, _i, _i, _i]),
    "or_rgb_to_v": (_i, [_i, _i, _i, _i]),
    "or_gamma_to_linear": (ctypes.c_uint32, [_i]),
    "or_linear_to_gamma": (_i, [ctypes.c_uint32, _i]),
    "or_accumulate_rgba": (None, [_u8p, _u8p, _u8p, _u8p, _i, _u16p, _i]),
    "or_convert_rgba32_to_uv": (None, [_u16p, _u8p, _u8p, _i]),
    "or_convert_argb_to_y": (None, [ctypes.c_void_p, _u8p, _i]),
    "or_convert_argb_to_uv": (None, [ctypes.c_void_p, _u8p, _u8p, _i, _i]),
    "or_point_sample_row": (None, [_u8p, _u8p, _u8p, _u8p, _i]),
    "or_upsample_line_pair_nrgba": (None, [_u8p] * 10 + [_i]),
    "or_upsample_line_pair_rgb": (None, [_u8p] * 8 + [_i]),
    "or_build_nrgba": (None, [_i, _i, _u8p, _i, _u8p, _u8p, _i, _u8p, _u8p]),
    "or_sse4x4": (_i, [_u8p, _u8p]),
    "or_sse16x16": (_i, [_u8p, _u8p]),
    "or_tdisto4x4": (_i, [_u8p, _u8p]),
    "or_tdisto16x16": (_i, [_u8p, _u8p]),
    "or_ssim_get": (ctypes.c_double, [_u8p, _i, _u8p, _i]),
    "or_ssim_get_clipped": (ctypes.c_double, [_u8p, _i, _u8p, _i, _i, _i, _i, _i]),
    "or_plane_ssim": (ctypes.c_double, [_u8p, _i, _u8p, _i, _i, _i]),
    "or_sse_plane": (ctypes.c_uint64, [_u8p, _i, _u8p, _i, _i, _i]),
    "or_disto_stats": (None, [_u8p, _i, _u8p, _i, _i, _i, ctypes.c_void_p]),
    "or_ssim_from_stats": (ctypes.c_double, [ctypes.c_void_p, _i]),
    "or_psnr_from_sse": (ctypes.c_double, [ctypes.c_uint64, ctypes.c_int64]),
    "or_random_init": (None, [ctypes.c_void_p, ctypes.c_float]),
    "or_convert_rgba32_to_uv_dithered": (None, [_u16p, _u8p, _u8p, _i, ctypes.c_void_p]),
    "or_import_rgba": (None, [_u8p, _i, _i, _i, _i, _u8p, _u8p, _u8p]),
    "or_dithering_strength": (ctypes.c_float, [ctypes.c_float]),
    "or_import_rgba_dithered": (None, [_u8p, _i, _i, _i, _i, ctypes.c_float, _u8p, _u8p, _u8p]),
    "or_compute_alphas": (_i, [_u8p, _u8p, _u8p, _i, _i, _i32p, _i32p, _i32p]),
    "or_decode_reconstruct": (None, [ctypes.c_void_p, _i16p, _i, _i, _u8p, _u8p, _u8p]),
    "or_decode_filter": (None, [ctypes.c_void_p, _i, _i, _i, _u8p, _u8p, _u8p]),
    "or_decode_frame": (None, [ctypes.c_void_p, _i16p, _i, _i, _i, _u8p, _u8p, _u8p]),
    "or_go_log2": (ctypes.c_double, [ctypes.c_double]),
    "or_vp8l_slog2_lut": (None, [ctypes.c_void_p, _i]),
    "or_vp8l_predict": (ctypes.c_uint32, [_i, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "or_vp8l_estimate_entropy": (ctypes.c_double, [ctypes.c_void_p, _i, _i, _i, _i, _i, _i]),
    "or_vp8l_residual_image": (None, [ctypes.c_void_p, _i, _i, _i, _i, ctypes.c_void_p, ctypes.c_void_p]),
    "or_vp8l_inverse_predictor": (None, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, ctypes.c_void_p]),
    "or_vp8l_subtract_green": (None, [ctypes.c_void_p, ctypes.c_size_t]),
    "or_vp8l_add_green": (None, [ctypes.c_void_p, ctypes.c_size_t]),
    "or_vp8l_decode": (_i, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "or_vp8l_color_space_transform": (None, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p]),
    "or_vp8l_color_space_inverse": (None, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, ctypes.c_void_p]),
    "or_vp8l_color_index_inverse": (None, [ctypes.c_void_p, _i, _i, _i, _i, ctypes.c_void_p, ctypes.c_void_p]),
    "or_alpha_filter": (None, [_i, ctypes.c_void_p, _i, _i, ctypes.c_void_p]),
    "or_alpha_unfilter": (None, [_i, ctypes.c_void_p, _i, _i]),
    "or_alpha_estimate_best_filter": (_i, [ctypes.c_void_p, _i, _i]),
    "or_alpha_num_colors": (_i, [ctypes.c_void_p, _i, _i]),
    "or_apply_alpha_multiply": (None, [ctypes.c_void_p, _i, _i, _i, _i, _i]),
    "or_mult_argb": (None, [ctypes.c_void_p, ctypes.c_size_t, _i]),
    "or_apply_alpha_multiply_4444": (None, [ctypes.c_void_p, _i, _i, _i]),
    "or_dispatch_alpha": (_i, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, _i, _i]),
    "or_extract_alpha": (_i, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, _i, _i]),
    "or_has_alpha": (_i, [ctypes.c_void_p, ctypes.c_size_t, _i]),
    "or_alpha_replace": (None, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]),
    "or_dispatch_alpha_to_green": (None, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, _i]),
    "or_extract_green": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "or_pack_rgb": (None, [ctypes.c_void_p] * 3 + [ctypes.c_size_t, _i, ctypes.c_void_p]),
    "or_rescale_plane": (_i, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, _i, _i, _i]),
    "or_sharpyuv_tables": (None, [ctypes.c_void_p, ctypes.c_void_p]),
    "or_sharpyuv_convert_tf": (_i, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, _i, ctypes.c_void_p, ctypes.c_void_p,
                                    _i, ctypes.c_void_p, _i]),
    "or_sharpyuv_convert_standard": (None, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, _i, ctypes.c_void_p,
                                            ctypes.c_void_p, _i, ctypes.c_void_p]),
    "or_sharpyuv_gamma_to_linear": (ctypes.c_uint32, [ctypes.c_uint16, _i, _i]),
    "or_sharpyuv_linear_to_gamma": (ctypes.c_uint16, [ctypes.c_uint32, _i, _i]),
    "or_sharpyuv_tf_long_double": (None, [_i]),
    "or_setup_segment": (None, [_i] * 8 + [ctypes.c_void_p]),
    "or_fixed_costs_i4": (None, [ctypes.c_void_p]),
    "or_quantize_coeffs": (_i, [ctypes.c_void_p] * 3 + [_i]),
    "or_dequant_coeffs": (None, [ctypes.c_void_p] * 3),
    "or_rd_score": (ctypes.c_uint64, [_i, _i, _i]),
    "or_token_cost": (_i, [ctypes.c_void_p, _i, _i, ctypes.c_void_p, _i, _i]),
    "or_trellis_quantize": (_i, [ctypes.c_void_p] * 3 + [_i, _i, _i, ctypes.c_void_p, _i]),
    "or_quality_to_compression": (ctypes.c_double, [_i]),
    "or_quality_to_qindex": (_i, [_i]),
    "or_segment_quant": (_i, [_i, _i, _i]),
    "or_segment_analysis": (None, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "or_encode_frame_rd": (None, [ctypes.c_void_p] * 3 + [_i] * 4 + [ctypes.c_void_p] * 3 + [_i, _i, ctypes.c_void_p]),
    "or_sharpyuv_convert": (_i, [ctypes.c_void_p, _i, _i, _i, ctypes.c_void_p, _i, ctypes.c_void_p, ctypes.c_void_p, _i,
                                 ctypes.c_void_p]),
}
for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


def ptr(a, ctype=ctypes.c_uint8, offset=0):
    """Pointer to a[...] + offset elements (a must be C-contiguous)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.cast(a.ctypes.data + offset * a.itemsize, ctypes.POINTER(ctype))


def u8(a, offset=0):
    return ptr(a, ctypes.c_uint8, offset)


def i16(a, offset=0):
    return ptr(a, ctypes.c_int16, offset)


# ---- frame-level helpers (numpy in / numpy out) ----

def plane_dims(w, h):
    mbw, mbh = (w + 15) >> 4, (h + 15) >> 4
    return mbw, mbh


def import_rgba(rgba, has_alpha=True):
    """importImage: rgba (h, w, 4) uint8 -> padded Y, U, V planes."""
    h, w, _ = rgba.shape
    rgba = np.ascontiguousarray(rgba)
    mbw, mbh = plane_dims(w, h)
    Y = np.zeros((mbh * 16, mbw * 16), np.uint8)
    U = np.zeros((mbh * 8, mbw * 8), np.uint8)
    V = np.zeros((mbh * 8, mbw * 8), np.uint8)
    lib.or_import_rgba(u8(rgba), w, h, w * 4, int(has_alpha), u8(Y), u8(U), u8(V))
    return Y, U, V


def import_rgba_dithered(rgba, has_alpha=True, dithering=None, quality=75.0):
    """importImage with dithering (Preprocessing bit 1): dithering defaults to
    webp.Encode's strength for `quality`."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    h, w, _ = rgba.shape
    if dithering is None:
        dithering = lib.or_dithering_strength(float(quality))
    mbw, mbh = plane_dims(w, h)
    Y = np.zeros((mbh * 16, mbw * 16), np.uint8)
    U = np.zeros((mbh * 8, mbw * 8), np.uint8)
    V = np.zeros((mbh * 8, mbw * 8), np.uint8)
    lib.or_import_rgba_dithered(u8(rgba), w, h, w * 4, int(has_alpha), float(dithering), u8(Y), u8(U), u8(V))
    return Y, U, V


def compute_alphas(Y, U, V, w, h):
    mbw, mbh = plane_dims(w, h)
    alphas = np.zeros(mbw * mbh, np.int32)
    lum = np.zeros_like(alphas)
    uva = np.zeros_like(alphas)
    uvavg = lib.or_compute_alphas(u8(Y), u8(U), u8(V), w, h, ptr(alphas, ctypes.c_int32),
                                  ptr(lum, ctypes.c_int32), ptr(uva, ctypes.c_int32))
    return alphas, lum, uva, uvavg


def decode_frame(mb, coeffs, filter_type, mbw, mbh, recon=True, filt=True):
    """Reconstruct (+ loop filter) a frame of parsed macroblocks."""
    mb = np.ascontiguousarray(mb, dtype=MB_INFO_DTYPE)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.int16)
    Y = np.zeros((mbh * 16, mbw * 16), np.uint8)
    U = np.zeros((mbh * 8, mbw * 8), np.uint8)
    V = np.zeros((mbh * 8, mbw * 8), np.uint8)
    if recon and filt:
        lib.or_decode_frame(mb.ctypes.data, i16(coeffs), filter_type, mbw, mbh, u8(Y), u8(U), u8(V))
    elif recon:
        lib.or_decode_reconstruct(mb.ctypes.data, i16(coeffs), mbw, mbh, u8(Y), u8(U), u8(V))
    return Y, U, V


def filter_frame(mb, filter_type, mbw, mbh, Y, U, V):
    mb = np.ascontiguousarray(mb, dtype=MB_INFO_DTYPE)
    Y, U, V = Y.copy(), U.copy(), V.copy()
    lib.or_decode_filter(mb.ctypes.data, filter_type, mbw, mbh, u8(Y), u8(U), u8(V))
    return Y, U, V


def build_nrgba(Y, U, V, w, h, alpha=None):
    out = np.zeros((h, w, 4), np.uint8)
    Y = np.ascontiguousarray(Y)
    U = np.ascontiguousarray(U)
    V = np.ascontiguousarray(V)
    a = None if alpha is None else np.ascontiguousarray(alpha)
    lib.or_build_nrgba(w, h, u8(Y), Y.shape[1], u8(U), u8(V), U.shape[1], u8(a) if a is not None else None,
                       u8(out))
    return out


def plane_ssim(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    h, w = a.shape
    return lib.or_plane_ssim(u8(a), a.shape[1], u8(b), b.shape[1], w, h)


# ---------------- VP8L predictor transform ----------------

def vp8l_subsample(size, bits):
    return (size + (1 << bits) - 1) >> bits


def vp8l_residual_image(argb, bits, quality):
    """ResidualImage: argb (h, w) uint32 -> (modes (th, tw) uint32, residuals (h, w) uint32)."""
    argb = np.ascontiguousarray(argb, np.uint32)
    h, w = argb.shape
    modes = np.zeros((vp8l_subsample(h, bits), vp8l_subsample(w, bits)), np.uint32)
    res = np.zeros_like(argb)
    lib.or_vp8l_residual_image(argb.ctypes.data, w, h, bits, quality, modes.ctypes.data, res.ctypes.data)
    return modes, res


def vp8l_inverse_predictor(modes, bits, residuals):
    residuals = np.ascontiguousarray(residuals, np.uint32)
    modes = np.ascontiguousarray(modes, np.uint32)
    h, w = residuals.shape
    out = np.zeros_like(residuals)
    lib.or_vp8l_inverse_predictor(modes.ctypes.data, bits, w, h, residuals.ctypes.data, out.ctypes.data)
    return out


def vp8l_estimate_entropy(argb, bits, tx, ty, mode):
    argb = np.ascontiguousarray(argb, np.uint32)
    h, w = argb.shape
    return lib.or_vp8l_estimate_entropy(argb.ctypes.data, w, h, tx, ty, bits, mode)


def vp8l_slog2_lut(n=65536):
    out = np.zeros(n, np.float64)
    lib.or_vp8l_slog2_lut(out.ctypes.data, n)
    return out


def vp8l_subtract_green(argb):
    a = np.ascontiguousarray(argb, np.uint32).copy()
    lib.or_vp8l_subtract_green(a.ctypes.data, a.size)
    return a


def vp8l_color_space_transform(argb, bits):
    """ColorSpaceTransform: (h, w) uint32 -> (multiplier words (tiles_y, tiles_x), transformed argb)."""
    a = np.ascontiguousarray(argb, np.uint32).copy()
    h, w = a.shape
    data = np.zeros((vp8l_subsample(h, bits), vp8l_subsample(w, bits)), np.uint32)
    lib.or_vp8l_color_space_transform(a.ctypes.data, w, h, bits, data.ctypes.data)
    return data, a


def vp8l_color_space_inverse(data, bits, src):
    src = np.ascontiguousarray(src, np.uint32)
    h, w = src.shape
    data = np.ascontiguousarray(data, np.uint32)
    out = np.empty_like(src)
    lib.or_vp8l_color_space_inverse(data.ctypes.data, bits, w, h, src.ctypes.data, out.ctypes.data)
    return out


def vp8l_color_index_inverse(palette, xbits, width, src, fill=0):
    """colorIndexInverseTransform: src (h, subsample(width, xbits)) packed index words -> (h, width)."""
    src = np.ascontiguousarray(src, np.uint32)
    pal = np.ascontiguousarray(palette, np.uint32)
    h = src.shape[0]
    out = np.full((h, width), fill, np.uint32)
    lib.or_vp8l_color_index_inverse(pal.ctypes.data, len(pal), xbits, width, h, src.ctypes.data, out.ctypes.data)
    return out


class _VP8LInfo(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("has_alpha", ctypes.c_int), ("tw", ctypes.c_int),
                ("n_transforms", ctypes.c_int), ("type", ctypes.c_int * 4), ("bits", ctypes.c_int * 4),
                ("xsize", ctypes.c_int * 4), ("dsize", ctypes.c_int * 4)]


VP8L_PREDICTOR, VP8L_CROSS_COLOR, VP8L_SUBTRACT_GREEN, VP8L_COLOR_INDEXING = range(4)


def riff_chunk(data, fourcc):
    """The payload of the first `fourcc` chunk of a RIFF/WEBP file."""
    assert data[:4] == b"RIFF" and data[8:12] == b"WEBP"
    off = 12
    while off + 8 <= len(data):
        size = int.from_bytes(data[off + 4:off + 8], "little")
        if data[off:off + 4] == fourcc:
            return data[off + 8:off + 8 + size]
        off += 8 + size + (size & 1)
    raise ValueError("no %r chunk" % fourcc)


def vp8l_decode_entropy(data):
    """Entropy-decode a VP8L stream (a .webp file or the bare payload) up to
    the inverse transforms -> dict(width, height, tw, pixels (h, tw) uint32,
    transforms=[dict(type, bits, xsize, data)] in bitstream order; predictor /
    cross-colour data is the (tiles_y, tiles_x) sub-image, colour indexing
    data the expanded palette)."""
    payload = riff_chunk(data, b"VP8L") if data[:4] == b"RIFF" else data
    buf = np.frombuffer(payload, np.uint8).copy()
    info = _VP8LInfo()
    assert lib.or_vp8l_decode(buf.ctypes.data, len(buf), ctypes.byref(info), None, None) == 0
    h = info.height
    pixels = np.zeros((h, info.tw), np.uint32)
    tds = []
    for k in range(info.n_transforms):
        t, bits, xs = info.type[k], info.bits[k], info.xsize[k]
        if t in (VP8L_PREDICTOR, VP8L_CROSS_COLOR):
            tds.append(np.zeros((vp8l_subsample(h, bits), vp8l_subsample(xs, bits)), np.uint32))
        else:
            tds.append(np.zeros(max(info.dsize[k], 1), np.uint32))
    ptrs = (ctypes.c_void_p * 4)(*[d.ctypes.data for d in tds], *([None] * (4 - len(tds))))
    assert lib.or_vp8l_decode(buf.ctypes.data, len(buf), ctypes.byref(info), pixels.ctypes.data, ptrs) == 0
    transforms = [dict(type=info.type[k], bits=info.bits[k], xsize=info.xsize[k], data=tds[k])
                  for k in range(info.n_transforms)]
    return dict(width=info.width, height=h, has_alpha=info.has_alpha, tw=info.tw, pixels=pixels,
                transforms=transforms)


def vp8l_apply_inverse(dec):
    """applyInverseTransforms (decode_transform.go:134-156) with the
    restatement's inverses, last-read transform first -> (h, w) ARGB."""
    cur = dec["pixels"]
    for t in reversed(dec["transforms"]):
        if t["type"] == VP8L_PREDICTOR:
            cur = vp8l_inverse_predictor(t["data"], t["bits"], cur)
        elif t["type"] == VP8L_CROSS_COLOR:
            cur = vp8l_color_space_inverse(t["data"], t["bits"], cur)
        elif t["type"] == VP8L_SUBTRACT_GREEN:
            cur = cur.copy()
            lib.or_vp8l_add_green(cur.ctypes.data, cur.size)
        else:
            cur = vp8l_color_index_inverse(t["data"], t["bits"], t["xsize"], cur)
    return cur


# ---------------- alpha plane ----------------

def alpha_filter(filter_, plane):
    """alphaFilter{Horizontal,Vertical,Gradient} (filter 1/2/3; 0 copies): (h, w) uint8 -> filtered."""
    a = np.ascontiguousarray(plane, np.uint8)
    h, w = a.shape
    out = np.empty_like(a)
    lib.or_alpha_filter(filter_, a.ctypes.data, w, h, out.ctypes.data)
    return out


def alpha_unfilter(filter_, plane):
    a = np.ascontiguousarray(plane, np.uint8).copy()
    h, w = a.shape
    lib.or_alpha_unfilter(filter_, a.ctypes.data, w, h)
    return a


def alpha_estimate_best_filter(plane):
    a = np.ascontiguousarray(plane, np.uint8)
    return lib.or_alpha_estimate_best_filter(a.ctypes.data, a.shape[1], a.shape[0])


def alpha_num_colors(plane):
    a = np.ascontiguousarray(plane, np.uint8)
    return lib.or_alpha_num_colors(a.ctypes.data, a.shape[1], a.shape[0])


def apply_alpha_multiply(rgba, alpha_first, inverse, width=None):
    """ApplyAlphaMultiply on (h, stride) uint8 rows of 4-byte pixels (width defaults to stride // 4)."""
    a = np.ascontiguousarray(rgba, np.uint8).copy()
    h, stride = a.shape
    lib.or_apply_alpha_multiply(a.ctypes.data, int(alpha_first), width or stride // 4, h, stride, int(inverse))
    return a


def mult_argb(argb, inverse):
    a = np.ascontiguousarray(argb, np.uint32).copy()
    lib.or_mult_argb(a.ctypes.data, a.size, int(inverse))
    return a


def apply_alpha_multiply_4444(data, width=None):
    a = np.ascontiguousarray(data, np.uint8).copy()
    h, stride = a.shape
    lib.or_apply_alpha_multiply_4444(a.ctypes.data, width or stride // 2, h, stride)
    return a


def dispatch_alpha(alpha, dst, alpha_off, width=None):
    """DispatchAlpha: alpha (h, alpha_stride) into dst (h, dst_stride) bytes -> (dst', any transparent)."""
    al = np.ascontiguousarray(alpha, np.uint8)
    d = np.ascontiguousarray(dst, np.uint8).copy()
    h, astride = al.shape
    r = lib.or_dispatch_alpha(al.ctypes.data, astride, width or astride, h, d.ctypes.data, d.shape[1], alpha_off)
    return d, bool(r)


def extract_alpha(src, alpha, alpha_off, width=None):
    """ExtractAlpha: src (h, src_stride) bytes -> (alpha (h, alpha_stride) plane, 1 if all opaque else 0)."""
    s_ = np.ascontiguousarray(src, np.uint8)
    al = np.ascontiguousarray(alpha, np.uint8).copy()
    h, sstride = s_.shape
    r = lib.or_extract_alpha(s_.ctypes.data, sstride, width or sstride // 4, h, al.ctypes.data, al.shape[1], alpha_off)
    return al, r


def has_alpha(src, step):
    """HasAlpha8b (step 1) / HasAlpha32b (step 4) over len(src) // step entries."""
    s_ = np.ascontiguousarray(src, np.uint8)
    return bool(lib.or_has_alpha(s_.ctypes.data, s_.size // step if step == 4 else s_.size, step))


def alpha_replace(argb, color):
    a = np.ascontiguousarray(argb, np.uint32).copy()
    lib.or_alpha_replace(a.ctypes.data, a.size, color)
    return a


def dispatch_alpha_to_green(alpha, dst_stride):
    al = np.ascontiguousarray(alpha, np.uint8)
    h, w = al.shape
    out = np.zeros((h, dst_stride), np.uint32)
    lib.or_dispatch_alpha_to_green(al.ctypes.data, w, w, h, out.ctypes.data, dst_stride)
    return out


def extract_green(argb):
    a = np.ascontiguousarray(argb, np.uint32)
    out = np.empty(a.shape, np.uint8)
    lib.or_extract_green(a.ctypes.data, out.ctypes.data, a.size)
    return out


def pack_rgb(r, g, b, length, step):
    r, g, b = (np.ascontiguousarray(c, np.uint8) for c in (r, g, b))
    out = np.empty(length, np.uint32)
    lib.or_pack_rgb(r.ctypes.data, g.ctypes.data, b.ctypes.data, length, step, out.ctypes.data)
    return out


def rescale_plane(src, dst_width, dst_height):
    """Drive dsp.Rescaler (rescale.go:63-257) over a (h, w) uint8 plane.
    -> (dst (dst_height, dst_width) uint8, rows written); unwritten rows are 0."""
    s = np.ascontiguousarray(src, np.uint8)
    sh, sw = s.shape
    out = np.zeros((dst_height, dst_width), np.uint8)
    rows = lib.or_rescale_plane(s.ctypes.data, sw, sh, sw, out.ctypes.data, dst_width, dst_height, dst_width)
    return out, rows


# ---------------- SharpYUV ----------------

WEBP_MATRIX = np.array([16839, 33059, 6420, 16 << 16, -9719, -19081, 28800, 128 << 16,
                        28800, -24116, -4684, 128 << 16], np.int32)  # sharpyuv/csp.go:66-70


TRANSFER_FUNCS = (1, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18)  # sharpyuv/gamma.go:11-28


def sharpyuv_convert(rgb, matrix=WEBP_MATRIX, transfer=13, sharp=True):
    """sharpyuv.Convert: rgb (h, w, 3) uint8 -> (Y (h, w), U, V ((h+1)//2, (w+1)//2),
    iterations).  sharp=False is convertStandard (iterations 0); transfer is
    the H.273 code (13 = sRGB, the default)."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w, _ = rgb.shape
    cw, ch = (w + 1) // 2, (h + 1) // 2
    Y = np.zeros((h, w), np.uint8)
    U = np.zeros((ch, cw), np.uint8)
    V = np.zeros((ch, cw), np.uint8)
    m = np.ascontiguousarray(matrix, np.int32)
    if not sharp:
        lib.or_sharpyuv_convert_standard(rgb.ctypes.data, w, h, 3 * w, Y.ctypes.data, w, U.ctypes.data, V.ctypes.data,
                                         cw, m.ctypes.data)
        return Y, U, V, 0
    it = lib.or_sharpyuv_convert_tf(rgb.ctypes.data, w, h, 3 * w, Y.ctypes.data, w, U.ctypes.data, V.ctypes.data, cw,
                                    m.ctypes.data, int(transfer))
    return Y, U, V, it


def sharpyuv_transfer_tables(transfer, bit_depth=10):
    """GammaToLinear over [0, 2^bd) and LinearToGamma over [0, max + 1] (gamma.go:360-446)."""
    g2l = np.array([lib.or_sharpyuv_gamma_to_linear(v, bit_depth, transfer) for v in range(1 << bit_depth)], np.uint32)
    n = int(g2l.max()) + 1
    l2g = np.array([lib.or_sharpyuv_linear_to_gamma(v, bit_depth, transfer) for v in range(n)], np.uint16)
    return g2l, l2g


def sharpyuv_tables():
    g = np.zeros(1026, np.uint32)
    l = np.zeros(514, np.uint32)  # noqa: E741
    lib.or_sharpyuv_tables(g.ctypes.data, l.ctypes.data)
    return g, l


# ---------------- encoder MB RD loop (Phase A) ----------------

SQUANT_DTYPE = np.dtype([("quant", "<i4"), ("iquant", "<i4"), ("bias", "<i4"), ("zthresh", "<i4"),
                         ("dc_quant", "<i4"), ("dc_iquant", "<i4"), ("dc_bias", "<i4"), ("dc_zthresh", "<i4"),
                         ("sharpen", "<i2", (16,))])
SEGMENT_DTYPE = np.dtype([("y1", SQUANT_DTYPE), ("y2", SQUANT_DTYPE), ("uv", SQUANT_DTYPE),
                          ("lambda_i4", "<i4"), ("lambda_i16", "<i4"), ("lambda_uv", "<i4"), ("lambda_mode", "<i4"),
                          ("tlambda_i4", "<i4"), ("tlambda_i16", "<i4"), ("tlambda_uv", "<i4"), ("tlambda_sd", "<i4")])
MB_ENC_DTYPE = np.dtype([("coeffs", "<i2", (400,)), ("modes", "u1", (16,)), ("nz_y", "u1", (16,)),
                         ("nz_uv", "u1", (8,)), ("non_zero_y", "<u4"), ("non_zero_uv", "<u4"),
                         ("mb_type", "u1"), ("i16_mode", "u1"), ("uv_mode", "u1"), ("nz_dc", "u1"),
                         ("skip", "u1"), ("segment", "u1"), ("pad", "u1", (2,)), ("score", "<u8")])
assert SQUANT_DTYPE.itemsize == 64 and SEGMENT_DTYPE.itemsize == 224 and MB_ENC_DTYPE.itemsize == 864


def setup_segment(q, dq=(0, 0, 0, 0, 0), method=4, sns_strength=50):
    seg = np.zeros(1, SEGMENT_DTYPE)
    lib.or_setup_segment(q, *dq, method, sns_strength, seg.ctypes.data)
    return seg[0]


def default_proba():
    """CoeffsProba0 (internal/lossy/proba.go:45), the tables Phase A uses after ResetProba."""
    import re
    txt = open(os.path.join(_HERE, "vp8_tables.h")).read()
    body = txt[txt.index("vp8_coeffs_proba0["):]
    body = body[body.index("{") + 1:body.index("};")]
    return np.array([int(x) for x in re.findall(r"\d+", body)], np.uint8)


def encode_frame_rd(Y, U, V, width, height, segments, segs, proba, method=4, quality=75):
    """Phase A over one frame: returns (mb_enc array (mbh*mbw,), reconstructed Y, U, V)."""
    Y, U, V = (np.ascontiguousarray(p, np.uint8).copy() for p in (Y, U, V))
    mbw, mbh = Y.shape[1] // 16, Y.shape[0] // 16
    out = np.zeros(mbw * mbh, MB_ENC_DTYPE)
    seg_ids = np.ascontiguousarray(segments, np.uint8)
    segs = np.ascontiguousarray(segs, SEGMENT_DTYPE)
    proba = np.ascontiguousarray(proba, np.uint8)
    lib.or_encode_frame_rd(Y.ctypes.data, U.ctypes.data, V.ctypes.data, width, height, mbw, mbh, seg_ids.ctypes.data,
                           segs.ctypes.data, proba.ctypes.data, method, quality, out.ctypes.data)
    return out, Y, U, V


# ---------------- segment analysis (analysis() after computeAlphas) ----------------

FRAME_SEGS_DTYPE = np.dtype([("num_segments", "<i4"), ("base_quant", "<i4"), ("global_uv_alpha", "<i4"),
                             ("dq_uv_ac", "<i4"), ("dq_uv_dc", "<i4"), ("filter_level", "<i4"), ("update_map", "<i4"),
                             ("pad", "<i4"), ("quant", "<i4", (4,)), ("fstrength", "<i4", (4,)), ("alpha", "<i4", (4,)),
                             ("beta", "<i4", (4,)), ("seg_proba", "u1", (4,)), ("pad2", "<i4", (3,))])
assert FRAME_SEGS_DTYPE.itemsize == 112


def encoder_config(quality=75, method=4, sns_strength=50, filter_strength=60, filter_sharpness=0, filter_type=1,
                   segments=4, preprocessing=0):
    """The EncodeConfig fields the analysis reads; defaults = DefaultConfig(75)
    (internal/lossy/encode.go:66-86), which webp.Encode's DefaultOptions resolve to."""
    return np.array([quality, method, sns_strength, filter_strength, filter_sharpness, filter_type, segments,
                     preprocessing], np.int32)


def segment_analysis(alphas, mbw, mbh, uv_sum, cfg):
    """assignSegments + setSegmentParams + setSegmentProbas for one frame:
    returns (seg_ids uint8 (mbh*mbw,), FRAME_SEGS record, 4 SEGMENT_DTYPE quantiser records)."""
    a = np.ascontiguousarray(alphas, np.int32).reshape(-1)
    assert a.size == mbw * mbh
    cfg = np.ascontiguousarray(cfg, np.int32)
    seg_ids = np.zeros(mbw * mbh, np.uint8)
    info = np.zeros(1, FRAME_SEGS_DTYPE)
    lib.or_segment_analysis(a.ctypes.data, mbw, mbh, int(uv_sum), cfg.ctypes.data, seg_ids.ctypes.data,
                            info.ctypes.data)
    info = info[0]
    dq = (0, 0, 0, int(info["dq_uv_dc"]), int(info["dq_uv_ac"]))
    segs = np.stack([setup_segment(int(q), dq, method=int(cfg[1]), sns_strength=int(cfg[2])) for q in info["quant"]])
    return seg_ids, info, segs


def encode_frame(Y, U, V, width, height, cfg=None, proba=None):
    """The lossy encoder's DSP path after import for one frame, as
    EncodeFrame runs it: computeAlphas -> analysis() segments -> Phase A.
    Returns (mb_enc, (RY, RU, RV), seg_ids, info)."""
    cfg = encoder_config() if cfg is None else cfg
    mbw, mbh = Y.shape[1] // 16, Y.shape[0] // 16
    alphas, _, uva, _ = compute_alphas(Y, U, V, width, height)
    seg_ids, info, segs = segment_analysis(alphas, mbw, mbh, int(uva.sum()), cfg)
    proba = default_proba() if proba is None else proba
    enc, ry, ru, rv = encode_frame_rd(Y, U, V, width, height, seg_ids, segs, proba, method=int(cfg[1]),
                                      quality=int(cfg[0]))
    return enc, (ry, ru, rv), seg_ids, info


# ---------------- block-level yuv / metric helpers (tests/test_gpu_blockops_yuv.py) ----------------

RANDOM_DTYPE = np.dtype([("index1", "<i4"), ("index2", "<i4"), ("tab", "<u4", (55,)), ("amp", "<i4")])  # or_random


def random_init(dithering):
    """InitRandom (internal/dsp/random.go:39): one VP8Random state record."""
    st = np.zeros(1, RANDOM_DTYPE)
    lib.or_random_init(st.ctypes.data, float(dithering))
    return st


def accumulate_rgba(r, g, b, a, stride, width):
    """AccumulateRGBA (yuv.go:486) of one row pair: 1-D planes, row 2 at +stride."""
    out = np.zeros(4 * ((width + 1) // 2), np.uint16)
    lib.or_accumulate_rgba(u8(r), u8(g), u8(b), u8(a), stride, out.ctypes.data_as(_u16p), width)
    return out


def convert_rgba32_to_uv(rgb, width, state=None):
    """ConvertRGBA32ToUV[Dithered] (yuv.go:553, :568); `state` (RANDOM_DTYPE) is advanced in place."""
    rgb = np.ascontiguousarray(rgb, np.uint16)
    u = np.zeros(width, np.uint8)
    v = np.zeros(width, np.uint8)
    if state is None:
        lib.or_convert_rgba32_to_uv(rgb.ctypes.data_as(_u16p), u8(u), u8(v), width)
    else:
        lib.or_convert_rgba32_to_uv_dithered(rgb.ctypes.data_as(_u16p), u8(u), u8(v), width, state.ctypes.data)
    return u, v


def convert_argb_to_y(argb, width):
    """ConvertARGBToY (yuv.go:270): packed uint32 0xAARRGGBB row -> Y bytes."""
    argb = np.ascontiguousarray(argb, np.uint32)
    assert argb.size >= width
    y = np.zeros(width, np.uint8)
    lib.or_convert_argb_to_y(argb.ctypes.data, u8(y), width)
    return y


def convert_argb_to_uv(argb, src_width, do_store, u=None, v=None):
    """ConvertARGBToUV (yuv.go:291): returns (u, v) of (src_width + 1) // 2
    samples; with do_store False the samples are averaged into copies of u, v."""
    argb = np.ascontiguousarray(argb, np.uint32)
    assert argb.size >= src_width
    n = (src_width + 1) // 2
    u = np.zeros(n, np.uint8) if u is None else np.array(u[:n], np.uint8)
    v = np.zeros(n, np.uint8) if v is None else np.array(v[:n], np.uint8)
    lib.or_convert_argb_to_uv(argb.ctypes.data, u8(u), u8(v), src_width, int(bool(do_store)))
    return u, v


def point_sample_row(y, u, v, width):
    """PointSampleRow (upsample.go:240): RGB row, 3 bytes per pixel."""
    dst = np.zeros(3 * width, np.uint8)
    lib.or_point_sample_row(u8(y), u8(u), u8(v), u8(dst), width)
    return dst


def upsample_line_pair(ty, by, tu, tv, bu, bv, width, nrgba, at=None, ab=None):
    """UpsampleLinePair (upsample.go:45, RGB) / UpsampleLinePairNRGBA (:130); by may be None."""
    bpp = 4 if nrgba else 3
    td = np.zeros(bpp * width, np.uint8)
    bd = np.zeros(bpp * width, np.uint8)
    byp = u8(by) if by is not None else None
    if nrgba:
        lib.or_upsample_line_pair_nrgba(u8(ty), byp, u8(tu), u8(tv), u8(bu), u8(bv), u8(td), u8(bd),
                                        u8(at) if at is not None else None, u8(ab) if ab is not None else None, width)
    else:
        lib.or_upsample_line_pair_rgb(u8(ty), byp, u8(tu), u8(tv), u8(bu), u8(bv), u8(td), u8(bd), width)
    return td, (bd if by is not None else None)


def disto_stats(pix, ref):
    """DistoStats of SSIMFromBlocks (ssim.go:103): [w, xm, ym, xxm, xym, yym] uint32."""
    pix = np.ascontiguousarray(pix, np.uint8)
    ref = np.ascontiguousarray(ref, np.uint8)
    out = np.zeros(6, np.uint32)
    h, w = pix.shape
    lib.or_disto_stats(u8(pix), w, u8(ref), w, w, h, out.ctypes.data)
    return out


def ssim_from_stats(stats, clipped):
    st = np.ascontiguousarray(stats, np.uint32)
    return float(lib.or_ssim_from_stats(st.ctypes.data, int(clipped)))


def psnr_from_sse(sse, count):
    return float(lib.or_psnr_from_sse(int(sse), int(count)))

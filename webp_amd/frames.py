"""Frame-level entry points: the reference's row/frame seams.

  decode_frames     internal/lossy/decode.go:532-560 (reconstructRow + filterRowAt)
  import_rgba       internal/lossy/encode.go:671-943 (importImage)
  analysis_alphas   internal/lossy/encode_analysis.go:245-307 (computeAlphas)
  build_nrgba       webp.go:379-450 (buildNRGBA -> UpsampleLinePairNRGBA)
  plane_ssim        AccumulateSSIM over ssim.go:116-160

All take / return CUDA tensors; a leading batch dimension means "n images of
the same size".  Everything runs in libwebpgpu.so on the GPU.
"""
import numpy as np
import torch

from ._lib import call, lib

MB_INFO_DTYPE = np.dtype([
    ("non_zero_y", "<u4"), ("non_zero_uv", "<u4"), ("imodes", "u1", (16,)),
    ("is_i4x4", "u1"), ("uv_mode", "u1"), ("skip", "u1"), ("segment", "u1"),
    ("f_limit", "u1"), ("f_ilevel", "u1"), ("f_inner", "u1"), ("hev_thresh", "u1"),
])  # wg_mb_info, include/webpgpu.h
assert MB_INFO_DTYPE.itemsize == 32


def _stream():
    return torch.cuda.current_stream().cuda_stream


def mb_dims(w, h):
    return (w + 15) >> 4, (h + 15) >> 4


def mb_info_tensor(mb, device="cuda"):
    """numpy structured array (.., MB_INFO_DTYPE) -> (n, 32) uint8 device tensor."""
    arr = np.ascontiguousarray(mb, dtype=MB_INFO_DTYPE).reshape(-1)
    return torch.from_numpy(arr.view(np.uint8).reshape(-1, 32).copy()).to(device)


def decode_frames(mb_info, coeffs, filter_type, mbw, mbh, n_images=1, out=None, work=None, check=False):
    """Reconstruct + loop-filter n frames of parsed macroblocks.

    mb_info: (n*mbh*mbw, 32) uint8, coeffs: (n*mbh*mbw, 384) int16 (CUDA).
    Returns (Y, U, V) of shapes (n, 16*mbh, 16*mbw) and (n, 8*mbh, 8*mbw)."""
    dev = coeffs.device
    assert mb_info.is_cuda and coeffs.is_cuda and coeffs.dtype == torch.int16
    assert mb_info.numel() == 32 * n_images * mbw * mbh and coeffs.numel() == 384 * n_images * mbw * mbh
    if out is None:
        Y = torch.empty((n_images, 16 * mbh, 16 * mbw), dtype=torch.uint8, device=dev)
        U = torch.empty((n_images, 8 * mbh, 8 * mbw), dtype=torch.uint8, device=dev)
        V = torch.empty_like(U)
    else:
        Y, U, V = out
    if work is None:
        work = torch.empty(lib.wg_decode_work_bytes(mbw, mbh, n_images), dtype=torch.uint8, device=dev)
    call("wg_decode_frames", mb_info.data_ptr(), coeffs.data_ptr(), filter_type, mbw, mbh, n_images, Y.data_ptr(),
         U.data_ptr(), V.data_ptr(), work.data_ptr(), _stream())
    if check:  # synchronises: raises if an in-kernel dependency wait timed out
        call("wg_decode_status", work.data_ptr(), mbw, n_images, _stream())
    return Y, U, V


def import_rgba(rgba, has_alpha=True, out=None):
    """importImage: (n, h, w, 4) uint8 RGBA -> padded (Y, U, V) planes."""
    assert rgba.is_cuda and rgba.dtype == torch.uint8 and rgba.dim() == 4 and rgba.is_contiguous()
    n, h, w, _ = rgba.shape
    mbw, mbh = mb_dims(w, h)
    if out is None:
        Y = torch.empty((n, 16 * mbh, 16 * mbw), dtype=torch.uint8, device=rgba.device)
        U = torch.empty((n, 8 * mbh, 8 * mbw), dtype=torch.uint8, device=rgba.device)
        V = torch.empty_like(U)
    else:
        Y, U, V = out
    call("wg_import_rgba", rgba.data_ptr(), w, h, 4 * w, 4 * w * h, int(bool(has_alpha)), Y.data_ptr(), U.data_ptr(),
         V.data_ptr(), Y[0].numel(), U[0].numel(), n, _stream())
    return Y, U, V


_DITHER_PLANS = {}


def dither_plan(w, h, device="cuda"):
    """The per-size VP8Random draws of importImage's dithered path, built once
    per (padded size, device) and kept resident."""
    key = (mb_dims(w, h), str(device))
    if key not in _DITHER_PLANS:
        plan = torch.empty(lib.wg_dither_plan_bytes(w, h), dtype=torch.uint8, device=device)
        call("wg_dither_plan", w, h, plan.data_ptr(), _stream())
        _DITHER_PLANS[key] = plan
    return _DITHER_PLANS[key]


def dither_amp(quality=75.0, preprocessing=2):
    """InitRandom's amplitude for webp.Encode's dithering at this quality (0 without preprocessing bit 1)."""
    return int(lib.wg_dither_amp(float(quality), int(preprocessing)))


def import_rgba_dithered(rgba, amp, has_alpha=True, out=None):
    """importImage with dithering: (n, h, w, 4) uint8 RGBA -> padded (Y, U, V)."""
    assert rgba.is_cuda and rgba.dtype == torch.uint8 and rgba.dim() == 4 and rgba.is_contiguous()
    n, h, w, _ = rgba.shape
    mbw, mbh = mb_dims(w, h)
    if out is None:
        Y = torch.empty((n, 16 * mbh, 16 * mbw), dtype=torch.uint8, device=rgba.device)
        U = torch.empty((n, 8 * mbh, 8 * mbw), dtype=torch.uint8, device=rgba.device)
        V = torch.empty_like(U)
    else:
        Y, U, V = out
    plan = dither_plan(w, h, rgba.device)
    call("wg_import_rgba_dithered", rgba.data_ptr(), w, h, 4 * w, 4 * w * h, int(bool(has_alpha)), int(amp),
         plan.data_ptr(), Y.data_ptr(), U.data_ptr(), V.data_ptr(), Y[0].numel(), U[0].numel(), n, _stream())
    return Y, U, V


def analysis_alphas(Y, U, V, w, h, parts=False, out=None):
    """computeAlphas: per-MB mixed alpha (n, mbh*mbw) int32 and the UV alpha average per image."""
    n = Y.shape[0]
    mbw, mbh = mb_dims(w, h)
    dev = Y.device
    if out is None:
        alphas = torch.empty((n, mbw * mbh), dtype=torch.int32, device=dev)
        uv_sum = torch.empty((n,), dtype=torch.int32, device=dev)
        lum = torch.empty_like(alphas) if parts else None
        uva = torch.empty_like(alphas) if parts else None
    else:
        alphas, uv_sum, lum, uva = out
    call("wg_analysis_alphas", Y.data_ptr(), U.data_ptr(), V.data_ptr(), w, h, Y[0].numel(), U[0].numel(), n,
         alphas.data_ptr(), lum.data_ptr() if lum is not None else None,
         uva.data_ptr() if uva is not None else None, uv_sum.data_ptr(), _stream())
    if parts:
        return alphas, uv_sum, lum, uva
    return alphas, uv_sum


def build_nrgba(Y, U, V, w, h, alpha=None, out=None):
    """buildNRGBA (webp.go:379): (n, H, Ws) planes -> (n, h, w, 4) NRGBA."""
    n = Y.shape[0]
    if out is None:
        out = torch.empty((n, h, w, 4), dtype=torch.uint8, device=Y.device)
    a_ptr, a_pitch = (None, 0) if alpha is None else (alpha.data_ptr(), alpha[0].numel())
    call("wg_upsample_nrgba", Y.data_ptr(), Y.shape[-1], Y[0].numel(), U.data_ptr(), V.data_ptr(), U.shape[-1],
         U[0].numel(), a_ptr, a_pitch, w, h, out.data_ptr(), out[0].numel(), n, _stream())
    return out


def plane_ssim(a, b, work=None):
    """Sum of per-pixel clipped-window SSIM for each image pair; (n,) float64."""
    n, h, w = a.shape
    if work is None:
        work = torch.empty(lib.wg_plane_ssim_work_bytes(w, h, n), dtype=torch.uint8, device=a.device)
    out = torch.empty((n,), dtype=torch.float64, device=a.device)
    call("wg_plane_ssim", a.data_ptr(), a.shape[-1], a[0].numel(), b.data_ptr(), b.shape[-1], b[0].numel(), w, h, n,
         out.data_ptr(), work.data_ptr(), _stream())
    return out


def plane_ssim_devices(a, b, devices):
    """Plane SSIM of one (h, w) HOST uint8 pair by 16-row bands over `devices`
    (wg_plane_ssim_devices); equals plane_ssim's sum bit for bit."""
    a = np.ascontiguousarray(a, dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    h, w = a.shape
    devs = np.ascontiguousarray(devices, dtype=np.int32)
    out = np.zeros(1, np.float64)
    call("wg_plane_ssim_devices", devs.ctypes.data, len(devs), a.ctypes.data, w, b.ctypes.data, w, w, h, out.ctypes.data)
    return float(out[0])


def vp8_parse(data):
    """Parse a lossy WebP (RIFF "VP8 " chunk or raw VP8 frame) on the host:
    returns (dims dict, mb_info structured array, coeffs int16 (n_mb, 384))."""
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    dims = np.zeros(5, dtype=np.int32)
    call("wg_vp8_parse", buf.ctypes.data, buf.size, dims.ctypes.data, None, None, 0)
    n = int(dims[3]) * int(dims[4])
    mb = np.zeros(n, dtype=MB_INFO_DTYPE)
    co = np.zeros((n, 384), dtype=np.int16)
    call("wg_vp8_parse", buf.ctypes.data, buf.size, dims.ctypes.data, mb.ctypes.data, co.ctypes.data, n)
    keys = ("width", "height", "filter_type", "mbw", "mbh")
    return {k: int(v) for k, v in zip(keys, dims)}, mb, co


WEBP_MATRIX = np.array([16839, 33059, 6420, 16 << 16, -9719, -19081, 28800, 128 << 16,
                        28800, -24116, -4684, 128 << 16], np.int32)  # sharpyuv/csp.go:66-70


def sharpyuv_convert(rgb, matrix=WEBP_MATRIX, out=None, work=None, iterations=False, transfer=13, sharp=True):
    """sharpyuv.Convert: (n, h, w, 3) uint8 RGB -> Y (n, h, w), U, V (n, (h+1)//2,
    (w+1)//2).  transfer: H.273 code (13 = sRGB, the default); sharp=False is
    convertStandard.  iterations=True also returns the refinement iterations
    each image ran (numpy int32; synchronises the stream)."""
    assert rgb.is_cuda and rgb.dtype == torch.uint8 and rgb.dim() == 4 and rgb.is_contiguous()
    n, h, w, _ = rgb.shape
    cw, ch = (w + 1) // 2, (h + 1) // 2
    if out is None:
        Y = torch.empty((n, h, w), dtype=torch.uint8, device=rgb.device)
        U = torch.empty((n, ch, cw), dtype=torch.uint8, device=rgb.device)
        V = torch.empty_like(U)
    else:
        Y, U, V = out
    if work is None:
        work = torch.empty(lib.wg_sharpyuv_work_bytes(w, h, n), dtype=torch.uint8, device=rgb.device)
    m = np.ascontiguousarray(matrix, np.int32)
    call("wg_sharpyuv_convert_ex", rgb.data_ptr(), w, h, 3 * w, 3 * w * h, m.ctypes.data, int(transfer), int(bool(sharp)),
         n, Y.data_ptr(), w, h * w, U.data_ptr(), V.data_ptr(), cw, cw * ch, work.data_ptr(), _stream())
    if iterations:
        its = np.zeros(n, np.int32)
        call("wg_sharpyuv_iterations", work.data_ptr(), w, h, n, its.ctypes.data, _stream())
        return Y, U, V, its
    return Y, U, V


# ---------------- encoder macroblock RD loop (Phase A) ----------------

SQUANT_DTYPE = np.dtype([("quant", "<i4"), ("iquant", "<i4"), ("bias", "<i4"), ("zthresh", "<i4"),
                         ("dc_quant", "<i4"), ("dc_iquant", "<i4"), ("dc_bias", "<i4"), ("dc_zthresh", "<i4"),
                         ("sharpen", "<i2", (16,))])  # wg_squant
SEGMENT_DTYPE = np.dtype([("y1", SQUANT_DTYPE), ("y2", SQUANT_DTYPE), ("uv", SQUANT_DTYPE),
                          ("lambda_i4", "<i4"), ("lambda_i16", "<i4"), ("lambda_uv", "<i4"), ("lambda_mode", "<i4"),
                          ("tlambda_i4", "<i4"), ("tlambda_i16", "<i4"), ("tlambda_uv", "<i4"),
                          ("tlambda_sd", "<i4")])  # wg_segment
MB_ENC_DTYPE = np.dtype([("coeffs", "<i2", (400,)), ("modes", "u1", (16,)), ("nz_y", "u1", (16,)),
                         ("nz_uv", "u1", (8,)), ("non_zero_y", "<u4"), ("non_zero_uv", "<u4"),
                         ("mb_type", "u1"), ("i16_mode", "u1"), ("uv_mode", "u1"), ("nz_dc", "u1"),
                         ("skip", "u1"), ("segment", "u1"), ("pad", "u1", (2,)), ("score", "<u8")])  # wg_mb_enc
assert SEGMENT_DTYPE.itemsize == 224 and MB_ENC_DTYPE.itemsize == 864


def setup_segment(q, dq=(0, 0, 0, 0, 0), method=4, sns_strength=50):
    """setupSegment (encode.go:1085) on the host -> SEGMENT_DTYPE record."""
    seg = np.zeros(1, SEGMENT_DTYPE)
    d = np.asarray(dq, np.int32)
    call("wg_setup_segment", q, d.ctypes.data, method, sns_strength, seg.ctypes.data)
    return seg[0]


def encode_mbs(Y, U, V, width, height, segments, segs, proba, method=4, quality=75, recon=None, work=None,
               out=None, check=False):
    """Phase A over n frames: Y (n, 16*mbh, 16*mbw) / U, V planes (CUDA uint8),
    segments (n, mbh*mbw) uint8, segs (4,) SEGMENT_DTYPE shared by all images, or
    a (n, 4*224) uint8 CUDA tensor of per-image tables (segment_analysis), proba
    (1056,) uint8.  Returns (out uint8 tensor viewed as (n*mbw*mbh, 864)
    wg_mb_enc bytes, (RY, RU, RV))."""
    n = Y.shape[0]
    mbw, mbh = mb_dims(width, height)
    dev = Y.device
    # the kernel addresses rows at stride 16*mbw / 8*mbw (encode_rd.hip)
    assert Y.is_contiguous() and U.is_contiguous() and V.is_contiguous()
    assert tuple(Y.shape) == (n, 16 * mbh, 16 * mbw), (tuple(Y.shape), mbw, mbh)
    assert tuple(U.shape) == (n, 8 * mbh, 8 * mbw) and tuple(V.shape) == (n, 8 * mbh, 8 * mbw)
    assert segments is None or segments.numel() == n * mbw * mbh
    if recon is None:
        recon = (torch.empty_like(Y), torch.empty_like(U), torch.empty_like(V))
    if out is None:
        out = torch.empty((n * mbw * mbh, MB_ENC_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    if work is None:
        work = torch.empty(lib.wg_encode_work_bytes(mbw, mbh, n), dtype=torch.uint8, device=dev)
    if not torch.is_tensor(segs):
        segs = torch.from_numpy(np.ascontiguousarray(segs, SEGMENT_DTYPE).view(np.uint8).copy()).to(dev)
    segs_pitch = 0 if segs.numel() == 4 * SEGMENT_DTYPE.itemsize else segs[0].numel()
    assert segs_pitch == 0 or (segs.shape[0] == n and segs_pitch >= 4 * SEGMENT_DTYPE.itemsize)
    if not torch.is_tensor(proba):
        proba = torch.from_numpy(np.ascontiguousarray(proba, np.uint8)).to(dev)
    seg_ptr = None if segments is None else segments.data_ptr()
    call("wg_encode_mbs", Y.data_ptr(), U.data_ptr(), V.data_ptr(), Y[0].numel(), U[0].numel(), width, height, n,
         seg_ptr, segs.data_ptr(), segs_pitch, proba.data_ptr(), method, quality, out.data_ptr(), recon[0].data_ptr(),
         recon[1].data_ptr(), recon[2].data_ptr(), work.data_ptr(), _stream())
    if check:
        call("wg_encode_status", work.data_ptr(), mbw, n, _stream())
    return out, recon


def encode_row_order(alphas, mbw, mbh, work=None):
    """The batch's row schedule (wg_encode_row_order) from the (n, mbh*mbw) int32
    alphas, written into (and returning) the encoder work buffer."""
    n = alphas.shape[0]
    if work is None:
        work = torch.empty(lib.wg_encode_work_bytes(mbw, mbh, n), dtype=torch.uint8, device=alphas.device)
    call("wg_encode_row_order", alphas.data_ptr(), mbw, mbh, n, work.data_ptr(), _stream())
    return work


def encode_status(work, mbw, n):
    """Raises if a row-dependency wait of the last wg_encode_mbs on `work` timed out (synchronises)."""
    call("wg_encode_status", work.data_ptr(), mbw, n, _stream())


def decode_status(work, mbw, n):
    """Raises if a row-dependency wait of the last wg_decode_frames on `work` timed out (synchronises)."""
    call("wg_decode_status", work.data_ptr(), mbw, n, _stream())


def fixed_costs_i4():
    """VP8FixedCostsI4 as wg_encode_mbs uploads it: (10, 10, 10) uint16 [top][left][mode]."""
    out = np.zeros(1000, np.uint16)
    call("wg_fixed_costs_i4_host", out.ctypes.data)
    return out.reshape(10, 10, 10)


# ---------------- segment analysis (analysis() after computeAlphas) ----------------

ENC_CONFIG_DTYPE = np.dtype([("quality", "<i4"), ("method", "<i4"), ("sns_strength", "<i4"),
                             ("filter_strength", "<i4"), ("filter_sharpness", "<i4"), ("filter_type", "<i4"),
                             ("segments", "<i4"), ("preprocessing", "<i4"), ("seg_quant", "u1", (256,))])
FRAME_SEGS_DTYPE = np.dtype([("num_segments", "<i4"), ("base_quant", "<i4"), ("global_uv_alpha", "<i4"),
                             ("dq_uv_ac", "<i4"), ("dq_uv_dc", "<i4"), ("filter_level", "<i4"), ("update_map", "<i4"),
                             ("pad", "<i4"), ("quant", "<i4", (4,)), ("fstrength", "<i4", (4,)), ("alpha", "<i4", (4,)),
                             ("beta", "<i4", (4,)), ("seg_proba", "u1", (4,)), ("pad2", "<i4", (3,))])  # wg_frame_segs
assert ENC_CONFIG_DTYPE.itemsize == 288 and FRAME_SEGS_DTYPE.itemsize == 112


def encoder_config(quality=75, method=4, sns_strength=50, filter_strength=60, filter_sharpness=0, filter_type=1,
                   segments=4, preprocessing=0):
    """wg_enc_config for EncodeConfig (defaults = DefaultConfig(75), internal/lossy/encode.go:66-86)."""
    cfg = np.zeros(1, ENC_CONFIG_DTYPE)
    call("wg_encoder_config", quality, method, sns_strength, filter_strength, filter_sharpness, filter_type, segments,
         preprocessing, cfg.ctypes.data)
    return cfg


def encode_frames_devices(rgba, devices, cfg=None, has_alpha=False):
    """The multi-device batch variant (wg_encode_frames_devices): rgba (n, h, w, 4)
    uint8 HOST array, frame i encoded on devices[i % len(devices)] by the whole
    device encode path; returns host arrays in frame order: (mb_enc bytes
    (n*mbh*mbw, 864), (RY, RU, RV) planes, seg_ids (n, mbh*mbw), info (n, 112))."""
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    n, h, w, _ = rgba.shape
    mbw, mbh = mb_dims(w, h)
    cfg = encoder_config() if cfg is None else cfg
    devs = np.ascontiguousarray(devices, dtype=np.int32)
    out = np.empty((n * mbw * mbh, MB_ENC_DTYPE.itemsize), np.uint8)
    ry = np.empty((n, 16 * mbh, 16 * mbw), np.uint8)
    ru = np.empty((n, 8 * mbh, 8 * mbw), np.uint8)
    rv = np.empty_like(ru)
    seg_ids = np.empty((n, mbw * mbh), np.uint8)
    info = np.empty((n, FRAME_SEGS_DTYPE.itemsize), np.uint8)
    call("wg_encode_frames_devices", devs.ctypes.data, len(devs), rgba.ctypes.data, w, h, n, int(has_alpha),
         cfg.ctypes.data, out.ctypes.data, ry.ctypes.data, ru.ctypes.data, rv.ctypes.data, seg_ids.ctypes.data,
         info.ctypes.data)
    return out, (ry, ru, rv), seg_ids, info


def segment_analysis(cfg, alphas, uv_sum, mbw, mbh, out=None, info=True):
    """assignSegments + setSegmentParams + setSegmentProbas + setupSegment per
    image on the device: alphas (n, mbh*mbw) int32, uv_sum (n,) int32 ->
    (seg_ids (n, mbh*mbw) uint8, segs (n, 896) uint8 per-image wg_segment x 4,
    info (n, 112) uint8 wg_frame_segs bytes or None)."""
    n = alphas.shape[0]
    dev = alphas.device
    assert alphas.dtype == torch.int32 and alphas.numel() == n * mbw * mbh and uv_sum.numel() == n
    if out is None:
        seg_ids = torch.empty((n, mbw * mbh), dtype=torch.uint8, device=dev)
        segs = torch.empty((n, 4 * SEGMENT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        inf = torch.empty((n, FRAME_SEGS_DTYPE.itemsize), dtype=torch.uint8, device=dev) if info else None
    else:
        seg_ids, segs, inf = out
    call("wg_segment_analysis", cfg.ctypes.data, alphas.data_ptr(), uv_sum.data_ptr(), mbw, mbh, n, seg_ids.data_ptr(),
         segs.data_ptr(), segs[0].numel(), inf.data_ptr() if inf is not None else None, _stream())
    return seg_ids, segs, inf


def encode_frames(rgba, cfg=None, has_alpha=False, proba=None, check=True):
    """The lossy encoder's DSP path for n same-sized RGBA frames, as
    NewEncoder + EncodeFrame run it up to Phase A (internal/lossy/encode.go:452,
    :1324-1366): importImage -> computeAlphas -> analysis() segments ->
    encodeFrameParallel Phase A.  Everything stays on the device.
    Returns (mb_enc bytes (n*mbw*mbh, 864), (RY, RU, RV), seg_ids, segs, info)."""
    n, h, w, _ = rgba.shape
    mbw, mbh = mb_dims(w, h)
    cfg = encoder_config() if cfg is None else cfg
    Y, U, V = import_rgba(rgba, has_alpha=has_alpha)
    alphas, uv_sum = analysis_alphas(Y, U, V, w, h)
    seg_ids, segs, info = segment_analysis(cfg, alphas, uv_sum, mbw, mbh)
    if proba is None:
        proba = default_proba()
    work = encode_row_order(alphas, mbw, mbh)
    out, recon = encode_mbs(Y, U, V, w, h, seg_ids, segs, proba, method=int(cfg["method"][0]),
                            quality=int(cfg["quality"][0]), work=work, check=check)
    return out, recon, seg_ids, segs, info


def default_proba(device="cuda"):
    """CoeffsProba0 (internal/lossy/proba.go:45): the token probabilities Phase A
    prices with after ResetProba, from the generated table."""
    import os
    import re
    txt = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "vp8_tables.h")).read()
    body = txt[txt.index("vp8_coeffs_proba0["):]
    body = body[body.index("{") + 1:body.index("};")]
    return torch.tensor([int(x) for x in re.findall(r"\d+", body)], dtype=torch.uint8, device=device)

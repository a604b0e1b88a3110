"""TEST INFRASTRUCTURE ONLY -- the reference's encoder acceptance tests,
restated: their image generators, their PSNR, and the bitstream round trip
they measure through (EncodeFrame -> DecodeFrame), here as

    encoder MBEncInfo (wg_mb_enc) -> the decoder's MBData -> reconstruct +
    loop filter

The bitstream between the two halves carries exactly the levels, modes,
skip flags, segment ids and the frame header (quantiser indices, filter
level / sharpness / type); Phase B (token recording, the bool coder) is
lossless and stays on the CPU in the reference's design, so it
is not rebuilt.  Everything the decoder derives from the header is derived
here the way the reference's decoder derives it:

- dequantisation factors: ParseQuant (internal/lossy/decode_quant.go:27-66)
  from the header's base quantiser and the dq_uv_dc / dq_uv_ac deltas the
  encoder writes (not the encoder's own quantiser records);
- I16 DCs: inverse WHT of the dequantised Y2 levels (decode_mb.go / the
  parse in webp_amd/csrc/vp8_parse.cpp);
- skip: signalled only when some MB of the frame is skipped
  (encode_syntax.go:88-93, :371-378), and then decodeMB zeroes the MB
  (decode_mb.go:266-296);
- filter strengths per (segment, is_i4x4): decode_frame.go:220-280 (the
  restatement in vp8_parse.cpp:258-287), FInner = i4 || !skip;
- filter type: 0 when the header level is 0, else 1 simple / 2 normal
  (decode.go:399-405).

Generators and thresholds (cited per function) follow
internal/lossy/encode_color_test.go and encode_diag_test.go.
"""
import numpy as np

# --- kDcTable / kAcTable (internal/lossy/tables.go), from the generated table
# header that tests/test_tables.py re-checks against the Go source ----------
def _table(name):
    import os
    import re
    txt = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle",
                            "vp8_tables.h")).read()
    body = txt[txt.index(name + "["):]
    body = body[body.index("{") + 1:body.index("};")]
    return np.array([int(x) for x in re.findall(r"\d+", body)], np.int64)


K_DC = _table("vp8_dc_table")
K_AC = _table("vp8_ac_table")
assert K_DC.size == 128 and K_AC.size == 128


# --- generators ------------------------------------------------------------

def _nrgba(rgb):
    h, w, _ = rgb.shape
    out = np.empty((h, w, 4), np.uint8)
    out[..., :3] = rgb
    out[..., 3] = 255
    return out


def smpte_bars(w, h):
    """smpteBarImage (encode_color_test.go:15-38): 8 vertical bars."""
    bars = np.array([[255, 255, 255], [255, 255, 0], [0, 255, 255], [0, 255, 0], [255, 0, 255], [255, 0, 0],
                     [0, 0, 255], [0, 0, 0]], np.uint8)
    idx = np.minimum(np.arange(w) // (w // 8), 7)
    return _nrgba(np.broadcast_to(bars[idx][None], (h, w, 3)))


def solid_blocks(w, h):
    """solidBlockImage (encode_color_test.go:40-66): R G B / C M Y in a 3x2 grid."""
    blocks = np.array([[255, 0, 0], [0, 255, 0], [0, 0, 255], [0, 255, 255], [255, 0, 255], [255, 255, 0]],
                      np.uint8)
    col = np.minimum(np.arange(w) // (w // 3), 2)
    row = (np.arange(h) >= h // 2).astype(np.int64)
    return _nrgba(blocks[row[:, None] * 3 + col[None, :]])


def color_pattern(w, h):
    """colorPatternImage (encode_diag_test.go:14-35): red / green / blue
    gradients and a grey diagonal gradient in the four quadrants."""
    hw, hh = w // 2, h // 2
    y, x = np.mgrid[0:h, 0:w]
    rgb = np.full((h, w, 3), 30, np.int64)
    tl, tr = (x < hw) & (y < hh), (x >= hw) & (y < hh)
    bl, br = (x < hw) & (y >= hh), (x >= hw) & (y >= hh)
    rgb[..., 0] = np.where(tl, x * 255 // hw, rgb[..., 0])
    rgb[..., 1] = np.where(tr, (x - hw) * 255 // hw, rgb[..., 1])
    rgb[..., 2] = np.where(bl, (y - hh) * 255 // hh, rgb[..., 2])
    g = (x - hw + y - hh) * 255 // (hw + hh)
    for c in range(3):
        rgb[..., c] = np.where(br, g, rgb[..., c])
    return _nrgba((rgb & 0xff).astype(np.uint8))


PATTERNS = {"smpte_bars": smpte_bars, "solid_blocks": solid_blocks, "color_gradient": color_pattern}


def rich_image(w, h):
    """richTestImage (encode_test.go:1492-1508): smooth R / G / B gradients."""
    y, x = np.mgrid[0:h, 0:w]
    rgb = np.stack([x * 255 // w, y * 255 // h, (x + y) * 255 // (w + h)], -1)
    return _nrgba((rgb & 0xff).astype(np.uint8))


def gradient_image(w, h):
    """generateGradient (testc/roundtrip/roundtrip_test.go:17-30): R and G
    gradients, B = 128."""
    y, x = np.mgrid[0:h, 0:w]
    rgb = np.stack([x * 255 // w, y * 255 // h, np.full_like(x, 128)], -1)
    return _nrgba((rgb & 0xff).astype(np.uint8))


# --- source planes and PSNR (the tests' own conversion, no gamma) ----------

def rgb_to_y(r, g, b):
    """dsp.RGBToY (internal/dsp/yuv.go:151-153)."""
    return ((16839 * r + 33059 * g + 6420 * b + (1 << 15) + (16 << 16)) >> 16).astype(np.uint8)


def _clip_uv(uv, rounding):
    """dsp.VP8ClipUV (yuv.go:138-147)."""
    return np.clip((uv + rounding + (128 << 18)) >> 18, 0, 255).astype(np.uint8)


def source_yuv(rgba):
    """srcY / srcU / srcV as computeYUVPSNR builds them (encode_color_test.go:77-104):
    per-pixel RGBToY, chroma from the 2x2 sums with rounding 1<<17."""
    c = rgba[..., :3].astype(np.int64)
    h, w = c.shape[:2]
    Y = rgb_to_y(c[..., 0], c[..., 1], c[..., 2])
    s = c[:h // 2 * 2, :w // 2 * 2].reshape(h // 2, 2, w // 2, 2, 3).sum(axis=(1, 3))
    r, g, b = s[..., 0], s[..., 1], s[..., 2]
    U = _clip_uv(-9719 * r - 19081 * g + 28800 * b, 1 << 17)
    V = _clip_uv(28800 * r - 24116 * g - 4684 * b, 1 << 17)
    return Y, U, V


def go_ycbcr_rgb(Y, U, V, w, h):
    """What image.YCbCr.At(x, y).RGBA() >> 8 gives for the reference's no-alpha
    lossy Decode (webp.go:339-372 returns *image.YCbCr, 4:2:0): chroma point
    sampled at (x / 2, y / 2) and Go's color.YCbCr.RGBA() (image/color,
    ycbcr.go: 16.16 fixed point with the factors 91881, 22554, 46802,
    116130, clamped through the 0xff000000 test), as 8-bit (h, w, 3)."""
    yy = Y[:h, :w].astype(np.int64) * 0x10101
    cb = np.repeat(np.repeat(U.astype(np.int64), 2, 0), 2, 1)[:h, :w] - 128
    cr = np.repeat(np.repeat(V.astype(np.int64), 2, 0), 2, 1)[:h, :w] - 128

    def clamp16(v):
        v = v.astype(np.int64)
        inside = (v & 0xff000000) == 0       # uint32(v) & 0xff000000 == 0 (v is int32 range)
        return np.where(inside, v >> 8, np.where(v < 0, 0, 0xffff)) >> 8

    r = clamp16(yy + 91881 * cr)
    g = clamp16(yy - 22554 * cb - 46802 * cr)
    b = clamp16(yy + 116130 * cb)
    return np.stack([r, g, b], -1).astype(np.uint8)


def psnr(a, b):
    """computePSNR (encode_diag_test.go:39-53): inf for identical inputs."""
    d = a.astype(np.float64).ravel() - b.astype(np.float64).ravel()
    mse = float(np.dot(d, d)) / d.size
    return float("inf") if mse == 0 else 10 * np.log10(255 * 255 / mse)


# --- the bitstream round trip ---------------------------------------------

def decoder_quant(base_q, dq_uv_dc, dq_uv_ac):
    """ParseQuant (decode_quant.go:50-63) for one segment:
    ((y1 dc, ac), (y2 dc, ac), (uv dc, ac))."""
    clip = lambda v, m: min(max(v, 0), m)
    y1 = (K_DC[clip(base_q, 127)], K_AC[clip(base_q, 127)])
    y2ac = max((int(K_AC[clip(base_q, 127)]) * 101581) >> 16, 8)
    y2 = (K_DC[clip(base_q, 127)] * 2, y2ac)
    uv = (K_DC[clip(base_q + dq_uv_dc, 117)], K_AC[clip(base_q + dq_uv_ac, 127)])
    return tuple((int(a), int(b)) for a, b in (y1, y2, uv))


def filter_strength(level, sharpness, i4):
    """precomputeFilterStrengths (decode_frame.go:220-280) for one (segment,
    is_i4x4) with no lf deltas: (limit, ilevel, hev_thresh)."""
    lv = min(max(level, 0), 63)
    if lv == 0:
        return 0, 0, 0
    il = lv
    if sharpness > 0:
        il >>= 2 if sharpness > 4 else 1
        il = min(il, 9 - sharpness)
    il = max(il, 1)
    return 2 * lv + il, il, (2 if lv >= 40 else (1 if lv >= 15 else 0))


def _iwht(dc):
    """TransformWHT (internal/dsp/transforms.go:223-252) of (n, 16) int -> (n, 16)
    DCs in block order."""
    dc = dc.astype(np.int64)
    t = np.empty_like(dc)
    for i in range(4):
        a0 = dc[:, i] + dc[:, 12 + i]
        a1 = dc[:, 4 + i] + dc[:, 8 + i]
        a2 = dc[:, 4 + i] - dc[:, 8 + i]
        a3 = dc[:, i] - dc[:, 12 + i]
        t[:, i], t[:, 8 + i], t[:, 4 + i], t[:, 12 + i] = a0 + a1, a0 - a1, a3 + a2, a3 - a2
    out = np.empty_like(dc)
    for i in range(4):
        d = t[:, 4 * i] + 3
        a0 = d + t[:, 4 * i + 3]
        a1 = t[:, 4 * i + 1] + t[:, 4 * i + 2]
        a2 = t[:, 4 * i + 1] - t[:, 4 * i + 2]
        a3 = d - t[:, 4 * i + 3]
        out[:, 4 * i + 0] = (a0 + a1) >> 3
        out[:, 4 * i + 1] = (a3 + a2) >> 3
        out[:, 4 * i + 2] = (a0 - a1) >> 3
        out[:, 4 * i + 3] = (a3 - a2) >> 3
    return out


MB_INFO_DTYPE = np.dtype([
    ("non_zero_y", "<u4"), ("non_zero_uv", "<u4"), ("imodes", "u1", (16,)),
    ("is_i4x4", "u1"), ("uv_mode", "u1"), ("skip", "u1"), ("segment", "u1"),
    ("f_limit", "u1"), ("f_ilevel", "u1"), ("f_inner", "u1"), ("hev_thresh", "u1"),
])  # wg_mb_info (include/webpgpu.h)


def segment_filter_levels(info, filter_strength):
    """The segment header's per-segment filter values (buildSegmentHeader,
    encode_analysis.go:852-866): fDelta = (qstep_s - qstep_0) * FilterStrength
    / 100 (Go's truncating division), clamped to +-63, with qstep = kAcTable[q]
    >> 2.  The header marks them absolute (AbsoluteDelta), so the decoder
    takes fDelta itself as segment s's base level (decode_frame.go:224-231)."""
    qs = [int(K_AC[min(max(int(info["quant"][s]), 0), 127)]) >> 2 for s in range(4)]
    out = []
    for s in range(4):
        num = (qs[s] - qs[0]) * filter_strength
        d = abs(num) // 100 * (1 if num >= 0 else -1)
        out.append(min(max(d, -63), 63))
    return out


def mbdata_from_encoder(enc, info, sharpness=0, simple=False, cfg_filter_strength=None):
    """wg_mb_enc records of one frame + its wg_frame_segs header record ->
    (wg_mb_info array, int16 (n, 384) dequantised coefficients, filter_type),
    as DecodeFrame would parse them from the encoder's bitstream.  With more
    than one segment the config's FilterStrength is needed for the segment
    header's filter values (segment_filter_levels)."""
    n = len(enc)
    segs = int(info["num_segments"])
    base = int(info["base_quant"])
    dq_dc, dq_ac = int(info["dq_uv_dc"]), int(info["dq_uv_ac"])
    # header quantisers: with one segment the frame's base index; with a
    # segment header every segment's own (absolute) index
    qidx = [int(info["quant"][s]) if segs > 1 else base for s in range(4)]
    level = int(info["filter_level"])
    if segs > 1:
        assert cfg_filter_strength is not None, "the segment header's filter values need FilterStrength"
        seg_level = segment_filter_levels(info, cfg_filter_strength)
    else:
        seg_level = [level] * 4
    ftype = 0 if level == 0 else (1 if simple else 2)
    lv = enc["coeffs"].astype(np.int64)                         # (n, 400)
    seg = (enc["segment"] & 3).astype(np.int64) if segs > 1 else np.zeros(n, np.int64)
    q = np.array([decoder_quant(qidx[s], dq_dc, dq_ac) for s in range(4)], np.int64)  # (4, 3, 2)
    co = np.zeros((n, 384), np.int64)
    blk = lv[:, :384].reshape(n, 24, 16)
    cls = np.r_[np.zeros(16, np.int64), np.full(8, 2)]          # y1 / uv per block
    dcq = q[seg][:, cls, 0]                                     # (n, 24)
    acq = q[seg][:, cls, 1]
    deq = blk * acq[:, :, None]
    deq[:, :, 0] = blk[:, :, 0] * dcq
    i16 = enc["mb_type"] == 0
    if i16.any():
        y2 = lv[i16, 384:400]
        y2q = q[seg[i16], 1]                                    # (m, 2)
        y2d = y2 * y2q[:, 1:2]
        y2d[:, 0] = y2[:, 0] * y2q[:, 0]
        deq[i16, :16, 0] = _iwht(y2d)
    co[:] = deq.reshape(n, 384)
    # decodeMB: a skipped MB is all zero (skip is signalled only if some MB is)
    use_skip = bool(enc["skip"].any())
    skip = enc["skip"].astype(bool) & use_skip
    co[skip] = 0
    mb = np.zeros(n, MB_INFO_DTYPE)
    mb["is_i4x4"] = (enc["mb_type"] != 0)
    mb["imodes"] = np.where(i16[:, None], 0, enc["modes"])
    mb["imodes"][i16, 0] = enc["i16_mode"][i16]
    mb["uv_mode"] = enc["uv_mode"]
    mb["segment"] = seg
    mb["skip"] = skip
    # nz codes: 3 (full transform) for any non-zero block; the transform kinds
    # the decoder picks from finer codes are exact special cases of it
    nzb = (co.reshape(n, 24, 16) != 0).any(axis=2)
    nzy = np.zeros(n, np.int64)
    for b in range(16):
        nzy = (nzy << 2) | np.where(nzb[:, b], 3, 0)
    nzuv = np.zeros(n, np.int64)
    for ch in range(2):
        for b in range(4):
            nzuv |= np.where(nzb[:, 16 + 4 * ch + b], 3 << (2 * (3 - b) + 8 * ch), 0)
    mb["non_zero_y"], mb["non_zero_uv"] = nzy, nzuv
    if ftype > 0:
        fs = np.array([[filter_strength(seg_level[s], sharpness, i4) for i4 in (0, 1)] for s in range(4)])
        f = fs[seg, mb["is_i4x4"].astype(np.int64)]
        mb["f_limit"], mb["f_ilevel"], mb["hev_thresh"] = f[:, 0], f[:, 1], f[:, 2]
        mb["f_inner"] = mb["is_i4x4"] | ~skip
    assert np.abs(co).max(initial=0) < 32768
    return mb, co.astype(np.int16), ftype


def crop(planes, w, h):
    Y, U, V = planes
    return Y[:h, :w], U[:h // 2, :w // 2], V[:h // 2, :w // 2]


def channel_psnr(src, dec):
    return tuple(psnr(a, b) for a, b in zip(src, dec))


# --- thresholds --------------------------------------------------------------

COLOR_SIZES = [(64, 64), (256, 256), (768, 576)]          # encode_color_test.go:152-156
COLOR_QUALITIES = [(50, 38.0, 38.0), (75, 42.0, 42.0)]    # :157-160


def diag_thresholds(q):
    """TestEncodeDiag (encode_diag_test.go:112-122, :165-174): (max filter
    level, min Y PSNR, min UV PSNR)."""
    max_level = 5 if q == 100 else (15 if q <= 50 else 10)
    mn = 50.0 if q == 100 else (42.0 if q >= 75 else 38.0)
    return max_level, mn, mn


def rgb_channel_stats(src_rgb, dec_rgb):
    """TestLossyRoundtrip_PSNR's statistics (encode_test.go:1541-1600):
    per-channel PSNR (computePSNR: 99 for mse <= 0), the PSNR of the channels'
    mean MSE, and the per-channel max |delta|."""
    d = src_rgb.astype(np.int64) - dec_rgb.astype(np.int64)
    mse = [float((d[..., c] ** 2).sum()) / d[..., c].size for c in range(3)]
    p = lambda m: 99.0 if m <= 0 else 10.0 * np.log10(255.0 * 255.0 / m)
    return [p(m) for m in mse], p(sum(mse) / 3.0), [int(np.abs(d[..., c]).max()) for c in range(3)]


def rgba_psnr(a, b):
    """computePSNR of testc/roundtrip/roundtrip_test.go:33-62: all four
    channels, inf for identical images."""
    d = a.astype(np.float64).ravel() - b.astype(np.float64).ravel()
    mse = float(np.dot(d, d)) / d.size
    return float("inf") if mse == 0 else 10 * np.log10(255.0 * 255.0 / mse)


def rgb_psnr(a, b):
    """TestEncodeCompareRGB's PSNR over packed RGB (encode_compare_test.go:226-235, mse :324-331)."""
    d = a.astype(np.float64).ravel() - b.astype(np.float64).ravel()
    return 10 * np.log10(255.0 * 255.0 / (float(np.dot(d, d)) / d.size))


# {Quality: 75, Method: 4} with every other EncoderOptions field zero, as
# TestLossyRoundtrip_PSNR and TestGoEncCDecLossy pass it: encodeLossyWithAlpha
# (encode.go:478-506) keeps DefaultConfig's 4 segments (Segments 0 is not > 0)
# and takes SNSStrength 0, FilterStrength 0, FilterType 0 as given
ZERO_OPTS_Q75 = dict(quality=75, method=4, sns_strength=0, filter_strength=0, filter_sharpness=0, filter_type=0,
                     segments=4, preprocessing=0)
# webp.Encode(nil) = DefaultOptions (encode.go:196-214): the bench's configuration
DEFAULT_OPTS_Q75 = dict(quality=75, method=4, sns_strength=50, filter_strength=60, filter_sharpness=0, filter_type=1,
                        segments=4, preprocessing=0)
ROUNDTRIP_SIZES = [(32, 32), (128, 128), (768, 576)]   # roundtrip_test.go:96


def compare_thresholds(q):
    """TestEncodeCompare (encode_compare_test.go:152-158): the Go-minus-cwebp
    PSNR deltas must be >= these (Y, UV)."""
    return -2.5, (-6.0 if q <= 50 else -4.0)


def bar_regions(w):
    """TestPerColorPSNR's eight bar column ranges (encode_color_test.go:199-201)."""
    bw = w // 8
    return [(i * bw, i * bw + bw) for i in range(8)]


def per_bar_min_y(q):
    return 26.0 if q >= 75 else 22.0                      # :266-270

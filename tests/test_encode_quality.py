"""The reference's own encoder acceptance tests, run on the restatement (CPU)
and on the product's GPU encode path (-m gpu):

- TestColorFidelity (internal/lossy/encode_color_test.go:141-193)
- TestPerColorPSNR (encode_color_test.go:197-278)
- TestEncodeDiag (encode_diag_test.go:71-187)
- TestEncodeCompare (encode_compare_test.go:17-170), the cwebp side as
  committed libwebp 1.6.0 fixtures (tests/golden/cwebp_compare.npz, made by
  tests/golden/make_golden.py encode_compare)

Each encodes with DefaultConfig(q) + Segments 1 (webp.Encode's q75 method 4,
SNS 50, filter 60 defaults otherwise), decodes what the bitstream would carry
(tests/encode_quality.py: MBEncInfo -> MBData -> reconstruct + loop filter)
and asserts the reference's PSNR floors / filter-level ceilings.  These pin
the encoder's decisions (I16 / I4 / UV modes, trellis levels, the segment's
filter strength), which no reference-held golden output covers, against the
thresholds the reference's CI asserts on them.  The GPU cases also check the
whole round trip bit-exact against the restatement.
"""
import os

import numpy as np
import pytest

import encode_quality as EQ
import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cwebp_compare.npz")


def cpu_round_trip(rgba, q):
    """EncodeFrame + DecodeFrame on the restatement: (decoded Y, U, V cropped,
    frame info, mb_enc records)."""
    h, w, _ = rgba.shape
    Y, U, V = O.import_rgba(rgba, has_alpha=False)
    enc, recon, _, info = O.encode_frame(Y, U, V, w, h, O.encoder_config(quality=q, segments=1))
    mb, co, ftype = EQ.mbdata_from_encoder(enc, info)
    mbw, mbh = Y.shape[1] // 16, Y.shape[0] // 16
    # the unfiltered decode is the encoder's own reconstruction (the
    # decoder's prediction sees the same pixels the encoder's RD did)
    uy, uu, uv = O.decode_frame(mb, co, 0, mbw, mbh)
    assert (uy == recon[0]).all() and (uu == recon[1]).all() and (uv == recon[2]).all()
    dec = O.decode_frame(mb, co, ftype, mbw, mbh)
    return EQ.crop(dec, w, h), info, enc


def gpu_round_trip(rgba, q):
    """The product path: wg_import_rgba -> wg_analysis_alphas ->
    wg_segment_analysis -> wg_encode_mbs on the GPU, the MBData the bitstream
    carries, then wg_decode_frames on the GPU."""
    import torch

    from webp_amd import frames
    h, w, _ = rgba.shape
    mbw, mbh = frames.mb_dims(w, h)
    cfg = frames.encoder_config(quality=q, segments=1)
    out, recon, _, _, info = frames.encode_frames(torch.from_numpy(np.ascontiguousarray(rgba)[None]).cuda(), cfg)
    enc = out.cpu().numpy().view(frames.MB_ENC_DTYPE).reshape(-1)
    info = info.cpu().numpy().view(frames.FRAME_SEGS_DTYPE).reshape(-1)[0]
    mb, co, ftype = EQ.mbdata_from_encoder(enc, info)
    Y, U, V = frames.decode_frames(frames.mb_info_tensor(mb), torch.from_numpy(co).cuda(), ftype, mbw, mbh, 1,
                                   check=True)
    torch.cuda.synchronize()
    dec = (Y[0].cpu().numpy(), U[0].cpu().numpy(), V[0].cpu().numpy())
    return EQ.crop(dec, w, h), info, enc


def check_color_fidelity(dec, rgba, q):
    _, min_y, min_uv = next(t for t in EQ.COLOR_QUALITIES if t[0] == q)
    py, pu, pv = EQ.channel_psnr(EQ.source_yuv(rgba), dec)
    assert py >= min_y, f"Y PSNR {py:.2f} dB < {min_y}"
    assert pu >= min_uv, f"U PSNR {pu:.2f} dB < {min_uv}"
    assert pv >= min_uv, f"V PSNR {pv:.2f} dB < {min_uv}"


def check_per_color(dec, rgba, q):
    h, w, _ = rgba.shape
    sy = EQ.source_yuv(rgba)[0]
    for x0, x1 in EQ.bar_regions(w):
        p = EQ.psnr(sy[:, x0:x1], dec[0][:, x0:x1])
        assert p >= EQ.per_bar_min_y(q) or p == float("inf"), f"bar {x0}..{x1}: Y PSNR {p:.1f} dB"


def check_diag(dec, rgba, q, info):
    max_level, min_y, min_uv = EQ.diag_thresholds(q)
    assert int(info["filter_level"]) <= max_level, f"filter level {int(info['filter_level'])} > {max_level}"
    py, pu, pv = EQ.channel_psnr(EQ.source_yuv(rgba), dec)
    assert py >= min_y and pu >= min_uv and pv >= min_uv, (py, pu, pv)


def check_compare(dec, rgba, q):
    h, w, _ = rgba.shape
    f = np.load(GOLDEN)
    key = "cwebp_%dx%d_q%d" % (w, h, q)
    src = EQ.source_yuv(rgba)
    go = EQ.channel_psnr(src, dec)
    c = EQ.channel_psnr(src, (f[key + "_y"], f[key + "_u"], f[key + "_v"]))
    ty, tuv = EQ.compare_thresholds(q)
    assert go[0] - c[0] >= ty, f"Y {go[0]:.2f} dB vs cwebp {c[0]:.2f}"
    assert go[1] - c[1] >= tuv and go[2] - c[2] >= tuv, (go, c)


COLOR_CASES = [(p, w, h, q) for p in EQ.PATTERNS for (w, h) in EQ.COLOR_SIZES for (q, _, _) in EQ.COLOR_QUALITIES]
COMPARE_CASES = [(w, h, q) for (w, h) in EQ.COLOR_SIZES for q in (75, 50)]


# ---------------- CPU: the restatement against the reference's thresholds ----------------

@pytest.mark.parametrize("pattern,w,h,q", COLOR_CASES)
def test_color_fidelity_oracle(pattern, w, h, q):
    rgba = EQ.PATTERNS[pattern](w, h)
    dec, _, _ = cpu_round_trip(rgba, q)
    check_color_fidelity(dec, rgba, q)


@pytest.mark.parametrize("q", [75, 50])
def test_per_color_psnr_oracle(q):
    rgba = EQ.smpte_bars(256, 256)
    dec, _, _ = cpu_round_trip(rgba, q)
    check_per_color(dec, rgba, q)


@pytest.mark.parametrize("q", [100, 75, 50])
def test_encode_diag_oracle(q):
    rgba = EQ.color_pattern(128, 128)
    dec, info, _ = cpu_round_trip(rgba, q)
    check_diag(dec, rgba, q, info)


@pytest.mark.parametrize("w,h,q", COMPARE_CASES)
def test_encode_compare_oracle(w, h, q):
    rgba = EQ.color_pattern(w, h)
    dec, _, _ = cpu_round_trip(rgba, q)
    check_compare(dec, rgba, q)


def test_round_trip_helpers():
    """The round trip's header-derived pieces: ParseQuant equals the
    encoder's setupSegment factors at the default deltas (so the decode is
    the encoder's own reconstruction), and the WHT helper inverts a DC-only
    input to (dc + 3) >> 3 everywhere, as decodeMB's nz <= 1 path does."""
    for qi in (0, 7, 40, 90, 127):
        seg = O.setup_segment(qi)
        (y1, y2, uv) = EQ.decoder_quant(qi, 0, 0)
        assert (int(seg["y1"]["dc_quant"]), int(seg["y1"]["quant"])) == y1
        assert (int(seg["y2"]["dc_quant"]), int(seg["y2"]["quant"])) == y2, qi
        assert (int(seg["uv"]["dc_quant"]), int(seg["uv"]["quant"])) == uv
    dc = np.zeros((3, 16), np.int64)
    dc[:, 0] = [5, -700, 2047 * 8]
    out = EQ._iwht(dc)
    assert (out == ((dc[:, :1] + 3) >> 3)).all()
    assert EQ.filter_strength(0, 0, 0) == (0, 0, 0)
    assert EQ.filter_strength(20, 0, 1) == (60, 20, 1)
    assert EQ.filter_strength(40, 5, 0) == (84, 4, 2)


# ---------------- GPU: the product path, bit-exact vs the restatement + thresholds ----------------

@pytest.mark.gpu
@pytest.mark.parametrize("pattern,w,h,q", COLOR_CASES)
def test_color_fidelity_gpu(pattern, w, h, q):
    rgba = EQ.PATTERNS[pattern](w, h)
    dec, info, enc = gpu_round_trip(rgba, q)
    cdec, cinfo, cenc = cpu_round_trip(rgba, q)
    for f in ("coeffs", "modes", "mb_type", "i16_mode", "uv_mode", "skip"):
        assert (enc[f] == cenc[f]).all(), f
    assert int(info["filter_level"]) == int(cinfo["filter_level"])
    for a, b in zip(dec, cdec):
        assert (a == b).all()
    check_color_fidelity(dec, rgba, q)


@pytest.mark.gpu
@pytest.mark.parametrize("q", [75, 50])
def test_per_color_psnr_gpu(q):
    rgba = EQ.smpte_bars(256, 256)
    dec, _, _ = gpu_round_trip(rgba, q)
    check_per_color(dec, rgba, q)


@pytest.mark.gpu
@pytest.mark.parametrize("q", [100, 75, 50])
def test_encode_diag_gpu(q):
    rgba = EQ.color_pattern(128, 128)
    dec, info, _ = gpu_round_trip(rgba, q)
    cdec, _, _ = cpu_round_trip(rgba, q)
    for a, b in zip(dec, cdec):
        assert (a == b).all()
    check_diag(dec, rgba, q, info)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,q", COMPARE_CASES)
def test_encode_compare_gpu(w, h, q):
    rgba = EQ.color_pattern(w, h)
    dec, _, _ = gpu_round_trip(rgba, q)
    check_compare(dec, rgba, q)

"""CPU: the encoder MB RD restatement (oracle/lossy_rd.c, encode_parallel.go
Phase A).  There is no third-party oracle for the reference's own mode
decisions (its RD loop is not libwebp's), so the restatement is pinned by
properties: the encoder's reconstruction must equal what the VP8 decoder
(pinned bit-exact vs libwebp) reconstructs from the chosen modes and
levels; levels respect the quantiser bounds; the nz bookkeeping agrees
with the levels."""
import numpy as np
import pytest

import oracle as O
from tools import synth


def dequant_to_decoder(enc, segs):
    """MBEncInfo levels -> the decoder's MBData (dequantised coefficients,
    I16 DCs inverse-WHT'd, nz codes), like a bitstream round trip would."""
    n = len(enc)
    mb = np.zeros(n, O.MB_INFO_DTYPE)
    co = np.zeros((n, 384), np.int16)
    for i in range(n):
        e = enc[i]
        s = segs[e["segment"] & 3]
        lv = e["coeffs"].astype(np.int32)
        out = np.zeros(384, np.int32)
        for b in range(24):
            q = s["uv"] if b >= 16 else s["y1"]
            blk = lv[16 * b:16 * b + 16] * q["quant"]
            blk[0] = lv[16 * b] * q["dc_quant"]
            out[16 * b:16 * b + 16] = blk
        if e["mb_type"] == 0:
            dc = (lv[384:400] * np.r_[s["y2"]["dc_quant"], [s["y2"]["quant"]] * 15]).astype(np.int16)
            wht = np.zeros(256, np.int16)
            O.lib.or_transform_wht(O.i16(dc), O.i16(wht))
            for b in range(16):
                out[16 * b] = wht[16 * b]
            mb[i]["imodes"][0] = e["i16_mode"]
        else:
            mb[i]["imodes"] = e["modes"]
            mb[i]["is_i4x4"] = 1
        co[i] = out.astype(np.int16)
        nzy = 0
        for b in range(16):
            nzy = (nzy << 2) | (3 if np.any(co[i][16 * b:16 * b + 16]) else 0)
        nzuv = 0
        for ch in range(2):
            for b in range(4):
                if np.any(co[i][16 * (16 + 4 * ch + b):16 * (17 + 4 * ch + b)]):
                    nzuv |= 3 << (2 * (3 - b) + 8 * ch)
        mb[i]["non_zero_y"], mb[i]["non_zero_uv"] = nzy, nzuv
        mb[i]["uv_mode"] = e["uv_mode"]
    return mb, co


def frame(w, h, kind, seed=0):
    gen = {"grad": lambda: synth.gradient_rgba(w, h), "noise": lambda: synth.noise_rgba(w, h, seed=seed),
           "blobs": lambda: synth.blobs_rgba(w, h, seed=seed)}[kind]
    return O.import_rgba(gen(), has_alpha=False)


@pytest.mark.parametrize("w,h,kind,q,method", [(64, 48, "blobs", 40, 4), (37, 29, "noise", 70, 4),
                                               (80, 64, "grad", 20, 4), (48, 48, "blobs", 60, 3),
                                               (16, 16, "noise", 5, 4), (100, 20, "blobs", 100, 4)])
def test_encoder_recon_equals_decoder(w, h, kind, q, method):
    Y, U, V = frame(w, h, kind, seed=w)
    mbw, mbh = Y.shape[1] // 16, Y.shape[0] // 16
    segs = np.stack([O.setup_segment(q + 7 * k, method=method) for k in range(4)])
    seg_ids = (np.arange(mbw * mbh) % 4).astype(np.uint8)
    enc, ry, ru, rv = O.encode_frame_rd(Y, U, V, w, h, seg_ids, segs, O.default_proba(), method=method,
                                         quality=75)
    mb, co = dequant_to_decoder(enc, segs)
    dy, du, dv = O.decode_frame(mb, co, 0, mbw, mbh)
    assert (dy[:h, :w] == ry[:h, :w]).all()
    assert (du == ru).all() and (dv == rv).all()
    # bookkeeping agrees with the levels
    for e in enc:
        lv = e["coeffs"].reshape(25, 16)
        first = 1 if e["mb_type"] == 0 else 0
        for b in range(16):
            assert bool(e["non_zero_y"] >> b & 1) == bool(e["nz_y"][b] > 0) == bool(np.any(lv[b][first:]))
        for k in range(8):
            assert bool(e["non_zero_uv"] >> k & 1) == bool(np.any(lv[16 + k]))
        assert e["skip"] == (e["non_zero_y"] == 0 and e["non_zero_uv"] == 0)
        assert np.abs(lv).max() <= 2047
    if kind == "noise" and q <= 70 and mbw * mbh > 4:
        assert (enc["mb_type"] == 1).any()  # textured input at a fine quantiser picks I4 somewhere


def test_fixed_costs_i4_table():
    t = np.zeros(1000, np.uint16)
    O.lib.or_fixed_costs_i4(t.ctypes.data)
    t = t.reshape(10, 10, 10)
    assert t.min() > 0 and t.max() < 4000

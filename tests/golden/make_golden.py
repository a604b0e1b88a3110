"""Regenerates the committed golden fixtures in tests/golden/ (run in the
build container, which has the reference checkout and Pillow's libwebp):

    python tests/golden/make_golden.py

Inputs come from the reference's own test data (testdata/test.png, the
768x576 opaque RGBA used by config 1) and from synthetic generators; expected
outputs come from the third-party libwebp 1.6.0 bundled with Pillow
(tests/libwebp_ref.py), which is the normative VP8 decoder and the library the
reference's own conformance suite (testc/) compares against.  Fixtures are
plain .npz (no pickles).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import libwebp_ref as L  # noqa: E402
from tools import synth  # noqa: E402

REF_PNG = "/root/reference/testdata/test.png"


def load_test_png():
    from PIL import Image
    return np.array(Image.open(REF_PNG).convert("RGBA"))


def main():
    assert L.available, "Pillow libwebp not found"
    img = load_test_png()
    out = {}
    # --- import (RGBA -> YUV420), opaque crop, odd crop, alpha variant ---
    a = img[200:296, 300:396].copy()                       # 96x96
    b = img[17:54, 101:154].copy()                         # 37x53 (odd)
    c = img[300:340, 500:548].copy()                       # 40x48 with synthetic alpha
    yy, xx = np.mgrid[0:c.shape[0], 0:c.shape[1]]
    c[..., 3] = ((xx * yy) % 256).astype(np.uint8)         # SURVEY 8(d) alpha variant
    for name, rgba in (("imp_a", a), ("imp_b", b), ("imp_c", c)):
        Y, U, V = L.import_rgba(rgba)
        out[name + "_rgba"], out[name + "_y"], out[name + "_u"], out[name + "_v"] = rgba, Y, U, V
    # --- libwebp q75 bitstreams + normative decode (YUV planes and fancy-upsampled RGBA) ---
    for name, rgba, q in (("dec_a", img[100:164, 200:280].copy(), 75.0),   # 80x64
                          ("dec_b", img[400:437, 50:103].copy(), 60.0)):   # 53x37 odd
        data = L.encode_lossy(rgba, q)
        Y, U, V = L.decode_yuv(data)
        out[name + "_webp"] = np.frombuffer(data, np.uint8).copy()
        out[name + "_y"], out[name + "_u"], out[name + "_v"] = Y, U, V
        out[name + "_rgba"] = L.decode_rgba(data)
    # --- plane SSIM (WebPPlaneDistortion type 1, float32 result) ---
    p = img[0:120, 0:160, 1].copy()
    rng = np.random.default_rng(3)
    q = np.clip(p.astype(np.int32) + rng.integers(-12, 13, p.shape), 0, 255).astype(np.uint8)
    out["ssim_a"], out["ssim_b"] = p, q
    out["ssim_value"] = np.array([L.plane_ssim(p, q)], np.float64)
    g = synth.gradient_rgba(61, 45)[..., 0].copy()
    out["ssim_c"], out["ssim_d"] = g, q[:45, :61].copy()
    out["ssim_value2"] = np.array([L.plane_ssim(g, out["ssim_d"])], np.float64)
    np.savez_compressed(os.path.join(HERE, "libwebp_fixtures.npz"), **out)
    print("wrote", os.path.join(HERE, "libwebp_fixtures.npz"), sum(v.nbytes for v in out.values()), "bytes raw")


if __name__ == "__main__":
    main()

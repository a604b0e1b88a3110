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
    make_c1_fixture(img)
    make_bench_bitstreams()
    make_decode_fixtures(img)
    make_sharpyuv_fixtures(img)
    make_reference_testdata()
    make_c3_bitstream()
    make_encode_compare_fixtures()
    print("wrote", os.path.join(HERE, "libwebp_fixtures.npz"), sum(v.nbytes for v in out.values()), "bytes raw")


# Bitstreams covering the decoder's header / token / filter space: simple and
# normal filter, sharpness, 4 token partitions, segment maps, q0..q100,
# method 6 (I4-heavy), odd and tiny sizes.  (name, rgba, encoder config)
def decode_cases(img):
    return [
        ("v_q10", img[40:104, 10:106], dict(quality=10)),
        ("v_simple", img[200:248, 300:380], dict(quality=90, filter_type=0, filter_sharpness=3)),
        ("v_parts", img[300:372, 400:520], dict(quality=50, partitions=3, filter_sharpness=7)),
        ("v_q100", img[64:128, 64:128], dict(quality=100)),
        ("v_q0", img[500:536, 600:700], dict(quality=0, filter_strength=100)),
        ("v_seg1", img[120:195, 220:295], dict(quality=75, segments=1, filter_type=0)),
        ("v_m6", img[10:90, 700:748], dict(quality=60, method=6, filter_strength=0)),
        ("v_big", img[100:292, 200:456], dict(quality=75)),
        ("v_sharp", img[260:324, 100:164], dict(quality=40, filter_sharpness=5, partitions=1)),
        ("v_noise", synth.noise_rgba(64, 48, seed=7), dict(quality=75)),
        ("v_grad", synth.gradient_rgba(100, 36), dict(quality=30)),
        ("v_1x1", img[5:6, 5:6], dict(quality=75)),
        ("v_17x1", img[7:8, 30:47], dict(quality=75)),
        ("v_1x17", img[7:24, 30:31], dict(quality=20)),
    ]


def make_decode_fixtures(img):
    out = {}
    for name, rgba, cfg in decode_cases(img):
        data = L.encode_lossy_cfg(np.ascontiguousarray(rgba), **cfg)
        Y, U, V = L.decode_yuv(data)
        out[name + "_webp"] = np.frombuffer(data, np.uint8).copy()
        out[name + "_y"], out[name + "_u"], out[name + "_v"] = Y, U, V
    path = os.path.join(HERE, "libwebp_decode.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def make_sharpyuv_fixtures(img):
    """libsharpyuv 0.4.2 SharpYuvConvert (WebP matrix, sRGB, 8-bit) outputs:
    the C library the reference's testc/sharpyuv compares its Go code with."""
    webp_matrix = np.array([16839, 33059, 6420, 16 << 16, -9719, -19081, 28800, 128 << 16,
                            28800, -24116, -4684, 128 << 16], np.int32)
    cases = [("s_photo", img[100:196, 200:328, :3]), ("s_odd", img[300:337, 50:103, :3]),
             ("s_noise", synth.noise_rgba(61, 45, seed=11)[..., :3]), ("s_grad", synth.gradient_rgba(128, 64)[..., :3]),
             ("s_2x2", np.array([[[255, 0, 0], [0, 255, 0]], [[0, 0, 255], [255, 255, 0]]], np.uint8)),
             ("s_1x1", img[10:11, 10:11, :3]), ("s_3x5", img[20:25, 40:43, :3])]
    out = {}
    for name, rgb in cases:
        rgb = np.ascontiguousarray(rgb)
        Y, U, V = L.sharpyuv_convert(rgb, webp_matrix)
        out[name + "_rgb"], out[name + "_y"], out[name + "_u"], out[name + "_v"] = rgb, Y, U, V
    path = os.path.join(HERE, "libsharpyuv_fixtures.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def make_c1_fixture(img):
    """testdata/test.png (768x576, opaque) as decoded RGBA: the C1 frame, for
    the full-frame encode parity test (the reference checkout is not on the GPU
    box).  Data only -- no expected outputs (those come from the oracle)."""
    path = os.path.join(HERE, "test_png_rgba.npz")
    np.savez_compressed(path, rgba=img)
    print("wrote", path, os.path.getsize(path), "bytes")


def make_bench_bitstreams():
    """libwebp 1.6.0 q75 (WebPEncodeRGBA defaults) encodes of 1920x1080
    contents -- gradient, noise seed 1, photo (test_color.png tiled, seed 0;
    SURVEY 8(d) G / N / P) and blobs seed 2: the decode side of bench.py
    parses the first three with wg_vp8_parse ("real q75
    bitstreams").  Stored as raw bytes in an uncompressed .npz."""
    w, h = 1920, 1080
    out = {"grad": L.encode_lossy(synth.gradient_rgba(w, h), 75.0),
           "noise": L.encode_lossy(synth.noise_rgba(w, h, seed=1), 75.0),
           "photo": L.encode_lossy(synth.photo_rgba(w, h, seed=0), 75.0),
           "blobs": L.encode_lossy(synth.blobs_rgba(w, h, seed=2), 75.0)}
    path = os.path.join(HERE, "q75_1080p.npz")
    np.savez(path, **{k: np.frombuffer(bytes(v), np.uint8) for k, v in out.items()})
    print("wrote", path, os.path.getsize(path), "bytes")


C3_PNG = "/root/reference/testdata/test_color.png"


def c3_rgba():
    """SURVEY 8(d) C3 input "P": testdata/test_color.png (1536x1024) tiled to 4096x4096."""
    from PIL import Image
    img = np.array(Image.open(C3_PNG).convert("RGBA"))
    reps = (-(-4096 // img.shape[0]), -(-4096 // img.shape[1]), 1)
    return np.ascontiguousarray(np.tile(img, reps)[:4096, :4096])


def make_c3_bitstream():
    """C3 on real content: a libwebp 1.6.0 q75 encode (WebPEncodeRGBA) of the
    tiled test_color.png at 4096x4096, and the SHA-256 of libwebp's
    WebPDecodeRGBA / WebPDecodeYUV of it (67 MB of pixels: only the hashes are
    kept).  tests/test_gpu_c3.py decodes the stream with wg_vp8_parse ->
    wg_decode_frames -> wg_upsample_nrgba and compares with the oracle at full
    size and with these hashes (under libwebp's skip rule)."""
    import hashlib
    data = L.encode_lossy(c3_rgba(), 75.0)
    rgba = L.decode_rgba(data)
    Y, U, V = L.decode_yuv(data)
    sha = lambda a: np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)
    path = os.path.join(HERE, "c3_4096_q75.npz")
    np.savez(path, webp=np.frombuffer(bytes(data), np.uint8), rgba_sha256=sha(rgba), y_sha256=sha(Y),
             u_sha256=sha(U), v_sha256=sha(V))
    print("wrote", path, os.path.getsize(path), "bytes")


REF_TESTDATA = ["blue_16x16_lossy.webp", "red_4x4_lossy.webp", "red_4x4_lossless.webp",
                "gradient_8x8_lossless.webp", "lossless/bug-decode/input-vp8l.webp"]


def make_reference_testdata():
    """The .webp files the reference's own tests decode (testdata/, used by
    webp_test.go:135-221) as raw bytes, next to libwebp 1.6.0's
    WebPDecodeRGBA of each: they pin the VP8 decode path and, through a VP8L
    entropy decode in oracle/vp8l_dec.c, the VP8L inverse transforms.  Keys:
    <name>_webp (bytes), <name>_rgba (h, w, 4)."""
    out = {}
    for f in REF_TESTDATA:
        data = open(os.path.join("/root/reference/testdata", f), "rb").read()
        key = os.path.basename(f).replace(".webp", "").replace("-", "_")
        out[key + "_webp"] = np.frombuffer(data, np.uint8)
        out[key + "_rgba"] = L.decode_rgba(data)
    path = os.path.join(HERE, "reference_testdata.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def make_encode_compare_fixtures():
    """TestEncodeCompare's C side (internal/lossy/encode_compare_test.go:86-117):
    `cwebp -q Q -segments 1 -m 4` of colorPatternImage at 64x64 / 256x256 /
    768x576, decoded with `dwebp -yuv`.  Here: libwebp 1.6.0 WebPEncode with
    WebPConfigInit(Q) + segments 1 + method 4 (cwebp's other defaults are the
    config's), WebPDecodeYUV of the result.  Keys cwebp_<w>x<h>_q<Q>_{y,u,v}
    (decoded planes, h x w and h/2 x w/2) and _webp (the bitstream).
    TestEncodeCompareRGB's C side (:174-264, `dwebp -ppm`: fancy-upsampled
    RGB): _rgb, the RGB channels of WebPDecodeRGBA of the same bitstream
    (h x w x 3; the RGBA decode's colour channels are MODE_RGB's)."""
    import encode_quality as EQ
    out = {}
    for w, h in EQ.COLOR_SIZES:
        rgba = EQ.color_pattern(w, h)
        for q in (75, 50):
            data = L.encode_lossy_cfg(rgba, float(q), segments=1, method=4)
            Y, U, V = L.decode_yuv(data)
            key = "cwebp_%dx%d_q%d" % (w, h, q)
            out[key + "_webp"] = np.frombuffer(data, np.uint8).copy()
            out[key + "_y"], out[key + "_u"], out[key + "_v"] = Y, U[:h // 2, :w // 2], V[:h // 2, :w // 2]
            out[key + "_rgb"] = np.ascontiguousarray(L.decode_rgba(data)[..., :3])
    path = os.path.join(HERE, "cwebp_compare.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    if sys.argv[1:] == ["encode_compare"]:
        make_encode_compare_fixtures()
    elif sys.argv[1:] == ["bench_bitstreams"]:
        make_bench_bitstreams()
    else:
        main()

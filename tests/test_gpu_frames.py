"""GPU parity, frame level: the reference's row/frame seams run through the C
ABI and compared with the C restatement (bit-exact) and, where a normative
third-party answer exists, with libwebp 1.6.0 golden fixtures.

Sizes cover the reference's edge cases (edge_cases_test.go: 1x1, N x 1,
non-multiple-of-16), batches of images, and the benchmark configurations
(1920x1080; 4096x4096 decode).
"""
import os

import numpy as np
import pytest
import torch

import oracle as O
from tools import synth
from webp_amd import frames

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "libwebp_fixtures.npz"))


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


# ---------------- decoder reconstruct + loop filter ----------------

def run_decode(mbw, mbh, n_img, filter_type, seed, **kw):
    mb, co = synth.random_macroblocks(n_img * mbw * mbh, seed=seed, **kw)
    Y, U, V = frames.decode_frames(frames.mb_info_tensor(mb), dev(co), filter_type, mbw, mbh, n_img, check=True)
    Y, U, V = host(Y), host(U), host(V)
    per = mbw * mbh
    for i in range(n_img):
        ey, eu, ev = O.decode_frame(mb[i * per:(i + 1) * per], co[i * per:(i + 1) * per], filter_type, mbw, mbh)
        assert (Y[i] == ey).all(), f"Y mismatch image {i}: {np.argwhere(Y[i] != ey)[:5]}"
        assert (U[i] == eu).all(), f"U mismatch image {i}"
        assert (V[i] == ev).all(), f"V mismatch image {i}"


@pytest.mark.parametrize("filter_type", [0, 1, 2])
@pytest.mark.parametrize("mbw,mbh", [(1, 1), (1, 4), (5, 1), (2, 3), (7, 5), (17, 9)])
def test_decode_frames(cuda, mbw, mbh, filter_type):
    run_decode(mbw, mbh, 2, filter_type, seed=mbw * 100 + mbh * 10 + filter_type, levels=(0, 10, 20, 40, 63))


@pytest.mark.parametrize("sharpness", [0, 3, 6])
def test_decode_filter_strengths(cuda, sharpness):
    run_decode(9, 7, 1, 2, seed=sharpness, levels=(5, 14, 15, 39, 40, 63), sharpness=sharpness)


@pytest.mark.parametrize("p_i4", [0.0, 1.0])
def test_decode_all_i16_or_all_i4(cuda, p_i4):
    run_decode(11, 6, 1, 2, seed=int(p_i4 * 7) + 1, p_i4=p_i4)


def test_decode_full_range_coefficients(cuda):
    """Full-range int16 coefficients, nz code 3 everywhere: exercises the 64-bit
    IDCT products of transforms.go (mul1/mul2 on |tmp| > 2^17)."""
    run_decode(6, 5, 1, 2, seed=99, dense=True)


def test_decode_1080p_batch(cuda):
    """C2/C4 frame shape: 1920x1080 -> 120x68 macroblocks, 2 images."""
    run_decode(120, 68, 2, 2, seed=2024, levels=(20, 32))


@pytest.mark.parametrize("filter_type", [0, 1, 2])
def test_decode_kernel_switch(cuda, filter_type):
    """wg_decode_frames launches k_decode_split for few rows and k_decode_bands
    past twice the resident split rows (decode.hip use_split); both bit-exact,
    for every filter type (the simple filter keeps the chroma rows of a band's
    last row, the normal one hands them to the next band).  Narrow frames keep
    the oracle quick at the batch that crosses over."""
    from webp_amd import _lib
    if os.environ.get("WG_DECODE_KERNEL"):
        pytest.skip("WG_DECODE_KERNEL forces one kernel")
    mbh = 68
    assert _lib.lib.wg_decode_kernel(mbh, 1) == 1
    n = 1
    while _lib.lib.wg_decode_kernel(mbh, n) == 1:
        n *= 2
    assert _lib.lib.wg_decode_kernel(mbh, n) == 2 and n <= 1024
    run_decode(3, mbh, n, filter_type, seed=n + filter_type, levels=(0, 20, 40))


def test_decode_4096_square(cuda):
    """C3 frame shape: 4096x4096 -> 256x256 macroblocks."""
    run_decode(256, 256, 1, 2, seed=4096, levels=(20,))


# ---------------- real bitstreams: host parse -> GPU reconstruct + filter ----------------

DEC = np.load(os.path.join(os.path.dirname(__file__), "golden", "libwebp_decode.npz"))
DEC_NAMES = sorted({k[:-5] for k in DEC.files if k.endswith("_webp")})


@pytest.mark.parametrize("name", DEC_NAMES)
def test_decode_bitstreams(cuda, name):
    """libwebp-encoded streams (q0..q100, simple/normal filter, sharpness,
    partitions, segments, tiny sizes): GPU == oracle under the reference's
    rules, and GPU == libwebp WebPDecodeYUV under libwebp's skip rule
    (test_oracle.libwebp_skip_rule)."""
    from test_oracle import crop_eq, libwebp_skip_rule
    dims, mb, co = frames.vp8_parse(DEC[name + "_webp"].tobytes())
    ft, mbw, mbh = dims["filter_type"], dims["mbw"], dims["mbh"]
    for info, want in ((mb, O.decode_frame(mb, co, ft, mbw, mbh)),
                       (libwebp_skip_rule(mb), (DEC[name + "_y"], DEC[name + "_u"], DEC[name + "_v"]))):
        got = frames.decode_frames(frames.mb_info_tensor(info), dev(co), ft, mbw, mbh, 1, check=True)
        for g, w in zip(got, want):
            assert crop_eq(host(g)[0], w), name


# ---------------- RGBA -> YUV420 import ----------------

@pytest.mark.parametrize("w,h,kind,alpha", [(1, 1, "noise", False), (17, 33, "noise", True), (96, 80, "grad", False),
                                            (53, 37, "blobs", True), (200, 3, "noise", True),
                                            (1920, 1080, "grad", False), (640, 480, "blobs", True),
                                            (2050, 19, "noise", False), (1028, 16, "noise", True)])
def test_import(cuda, w, h, kind, alpha):
    gen = {"noise": lambda: synth.noise_rgba(w, h, seed=w + h, alpha=alpha),
           "grad": lambda: synth.gradient_rgba(w, h), "blobs": lambda: synth.blobs_rgba(w, h, alpha=alpha)}[kind]
    imgs = np.stack([gen(), np.ascontiguousarray(gen()[::-1])])
    Y, U, V = frames.import_rgba(dev(imgs), has_alpha=alpha)
    Y, U, V = host(Y), host(U), host(V)
    for i in range(2):
        ey, eu, ev = O.import_rgba(imgs[i], has_alpha=alpha)
        assert (Y[i] == ey).all() and (U[i] == eu).all() and (V[i] == ev).all()


@pytest.mark.parametrize("name", ["imp_a", "imp_b", "imp_c"])
def test_import_vs_libwebp_golden(cuda, name):
    rgba = GOLD[name + "_rgba"]
    h, w, _ = rgba.shape
    Y, U, V = frames.import_rgba(dev(rgba[None]), has_alpha=True)
    ey, eu, ev = GOLD[name + "_y"], GOLD[name + "_u"], GOLD[name + "_v"]
    assert (host(Y)[0][:h, :w] == ey).all()
    assert (host(U)[0][:eu.shape[0], :eu.shape[1]] == eu).all()
    assert (host(V)[0][:ev.shape[0], :ev.shape[1]] == ev).all()


# ---------------- analysis ----------------

@pytest.mark.parametrize("w,h,src", [(16, 16, "grad"), (33, 47, "noise"), (100, 60, "blobs"), (320, 240, "blobs"),
                                     (1920, 1080, "grad"), (64, 64, "random_planes")])
def test_analysis_alphas(cuda, w, h, src):
    mbw, mbh = frames.mb_dims(w, h)
    if src == "random_planes":  # arbitrary plane content (no replicated padding)
        rng = np.random.default_rng(5)
        Y = rng.integers(0, 256, (2, 16 * mbh, 16 * mbw), dtype=np.uint8)
        U = rng.integers(0, 256, (2, 8 * mbh, 8 * mbw), dtype=np.uint8)
        V = rng.integers(0, 256, (2, 8 * mbh, 8 * mbw), dtype=np.uint8)
    else:
        gen = {"grad": synth.gradient_rgba, "noise": synth.noise_rgba, "blobs": synth.blobs_rgba}[src]
        planes = [O.import_rgba(gen(w, h)), O.import_rgba(np.ascontiguousarray(gen(w, h)[:, ::-1]))]
        Y, U, V = (np.stack([p[k] for p in planes]) for k in range(3))
    alphas, uv_sum, lum, uva = frames.analysis_alphas(dev(Y), dev(U), dev(V), w, h, parts=True)
    alphas, uv_sum, lum, uva = map(host, (alphas, uv_sum, lum, uva))
    for i in range(2):
        ea, el, eu, uvavg = O.compute_alphas(Y[i], U[i], V[i], w, h)
        assert (alphas[i] == ea).all() and (lum[i] == el).all() and (uva[i] == eu).all()
        assert uv_sum[i] // (mbw * mbh) == uvavg


# ---------------- fancy upsampling ----------------

@pytest.mark.parametrize("w,h", [(1, 1), (1, 5), (2, 2), (3, 7), (8, 1), (64, 48), (53, 37), (100, 101), (1920, 1080)])
@pytest.mark.parametrize("alpha", [False, True])
def test_build_nrgba(cuda, w, h, alpha):
    rng = np.random.default_rng(w * 1000 + h)
    ys, cs = w + 5, (w + 1) // 2 + 3  # strides wider than the image
    Y = rng.integers(0, 256, (2, h, ys), dtype=np.uint8)
    U = rng.integers(0, 256, (2, (h + 1) // 2, cs), dtype=np.uint8)
    V = rng.integers(0, 256, (2, (h + 1) // 2, cs), dtype=np.uint8)
    A = rng.integers(0, 256, (2, h, w), dtype=np.uint8) if alpha else None
    out = host(frames.build_nrgba(dev(Y), dev(U), dev(V), w, h, alpha=dev(A) if alpha else None))
    for i in range(2):
        exp = O.build_nrgba(Y[i], U[i], V[i], w, h, alpha=A[i] if alpha else None)
        assert (out[i] == exp).all()


@pytest.mark.parametrize("w,h", [(16, 2), (4096, 3), (4100, 6), (8192 + 36, 5), (1936, 17)])
@pytest.mark.parametrize("alpha", [False, True])
def test_build_nrgba_aligned(cuda, w, h, alpha):
    """Aligned strides (the kernel's 16-byte luma / 8-byte chroma / 16-byte
    output paths), several 4096-column blocks per line pair."""
    rng = np.random.default_rng(w * 7 + h)
    ys, cs = (w + 15) // 16 * 16, ((w + 1) // 2 + 7) // 8 * 8
    Y = rng.integers(0, 256, (2, h, ys), dtype=np.uint8)
    U = rng.integers(0, 256, (2, (h + 1) // 2, cs), dtype=np.uint8)
    V = rng.integers(0, 256, (2, (h + 1) // 2, cs), dtype=np.uint8)
    A = rng.integers(0, 256, (2, h, w), dtype=np.uint8) if alpha else None
    out = host(frames.build_nrgba(dev(Y), dev(U), dev(V), w, h, alpha=dev(A) if alpha else None))
    for i in range(2):
        exp = O.build_nrgba(Y[i], U[i], V[i], w, h, alpha=A[i] if alpha else None)
        assert (out[i] == exp).all()


@pytest.mark.parametrize("name", ["dec_a", "dec_b"])
def test_build_nrgba_vs_libwebp_golden(cuda, name):
    Y, U, V, rgba = (GOLD[name + k] for k in ("_y", "_u", "_v", "_rgba"))
    h, w = Y.shape
    out = host(frames.build_nrgba(dev(Y[None]), dev(U[None]), dev(V[None]), w, h))
    assert (out[0] == rgba).all()


# ---------------- plane SSIM ----------------

SSIM_RTOL = 1e-6  # north_star: SSIM floats within 1e-6


@pytest.mark.parametrize("w,h", [(1, 1), (5, 9), (7, 7), (61, 45), (160, 120), (1920, 1080)])
def test_plane_ssim(cuda, w, h):
    rng = np.random.default_rng(w + 7 * h)
    a = rng.integers(0, 256, (2, h, w), dtype=np.uint8)
    b = np.clip(a.astype(np.int32) + rng.integers(-20, 21, a.shape), 0, 255).astype(np.uint8)
    b[1] = a[1]  # identity: every window SSIM is exactly 1
    got = host(frames.plane_ssim(dev(a), dev(b)))
    for i in range(2):
        exp = O.plane_ssim(a[i], b[i])
        assert abs(got[i] - exp) <= SSIM_RTOL * abs(exp)
    assert got[1] == w * h


def test_plane_ssim_vs_libwebp_golden(cuda):
    for a, b, v in (("ssim_a", "ssim_b", "ssim_value"), ("ssim_c", "ssim_d", "ssim_value2")):
        got = float(host(frames.plane_ssim(dev(GOLD[a][None]), dev(GOLD[b][None])))[0])
        want = float(GOLD[v][0])
        assert abs(got - want) <= 1e-6 * abs(want) + 1e-4  # libwebp rounds its sum to float32

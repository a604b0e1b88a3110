"""SharpYUV.

CPU: the C restatement (oracle/sharpyuv.c) against libsharpyuv 0.4.2 fixtures
(tests/golden/libsharpyuv_fixtures.npz) -- the reference's own testc accepts
+-1 against that library; the restatement matches it exactly on every
fixture, so the tests require exact equality.  The product's host gamma
tables equal the oracle's.
GPU (-m gpu): wg_sharpyuv_convert == oracle, bit-exact, on odd / tiny /
batched / 1080p / 4096-wide images."""
import os

import numpy as np
import pytest

import oracle as O
from tools import synth

FIX = np.load(os.path.join(os.path.dirname(__file__), "golden", "libsharpyuv_fixtures.npz"))
NAMES = sorted({k[:-4] for k in FIX.files if k.endswith("_rgb")})


@pytest.mark.parametrize("name", NAMES)
def test_oracle_vs_libsharpyuv(name):
    y, u, v, _ = O.sharpyuv_convert(FIX[name + "_rgb"])
    assert (y == FIX[name + "_y"]).all() and (u == FIX[name + "_u"]).all() and (v == FIX[name + "_v"]).all()


def test_gamma_tables_product_equals_oracle():
    from webp_amd._lib import call
    g, l = np.zeros(1026, np.uint32), np.zeros(514, np.uint32)  # noqa: E741
    call("wg_sharpyuv_tables_host", g.ctypes.data, l.ctypes.data)
    og, ol = O.sharpyuv_tables()
    assert (g == og).all() and (l == ol).all()
    assert g[0] == 0 and g[1024] == 65536 and l[512] == 65536 and (np.diff(g.astype(np.int64)) >= 0).all()


def rgb_cases():
    rng = np.random.default_rng(4)
    yield "1x1", rng.integers(0, 256, (1, 1, 3), dtype=np.uint8)
    yield "2x1", rng.integers(0, 256, (1, 2, 3), dtype=np.uint8)
    yield "3x5", rng.integers(0, 256, (5, 3, 3), dtype=np.uint8)
    yield "noise", rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    yield "grad", np.ascontiguousarray(synth.gradient_rgba(96, 70)[..., :3])
    yield "blobs", np.ascontiguousarray(synth.blobs_rgba(130, 66, seed=3)[..., :3])
    yield "flat", np.full((16, 16, 3), 77, np.uint8)


@pytest.mark.gpu
def test_gpu_matches_oracle(cuda):
    import torch
    from webp_amd import frames
    seen = set()
    for name, rgb in rgb_cases():
        Y, U, V, its = frames.sharpyuv_convert(torch.from_numpy(rgb[None].copy()).cuda(), iterations=True)
        ey, eu, ev, eits = O.sharpyuv_convert(rgb)
        torch.cuda.synchronize()
        assert (Y[0].cpu().numpy() == ey).all(), name
        assert (U[0].cpu().numpy() == eu).all() and (V[0].cpu().numpy() == ev).all(), name
        assert its[0] == eits, name  # the speculative pipeline stops where the reference's early exit does
        seen.add(int(eits))
    assert len(seen) >= 2, seen  # the cases reach more than one exit point


@pytest.mark.gpu
def test_gpu_fixtures_and_batch(cuda):
    import torch
    from webp_amd import frames
    for name in NAMES:
        Y, U, V = frames.sharpyuv_convert(torch.from_numpy(FIX[name + "_rgb"][None].copy()).cuda())
        assert (Y[0].cpu().numpy() == FIX[name + "_y"]).all(), name
        assert (U[0].cpu().numpy() == FIX[name + "_u"]).all() and (V[0].cpu().numpy() == FIX[name + "_v"]).all()
    imgs = np.stack([synth.noise_rgba(45, 33, seed=s)[..., :3] for s in range(3)])
    Y, U, V = frames.sharpyuv_convert(torch.from_numpy(imgs).cuda())
    for i in range(3):
        ey, eu, ev, _ = O.sharpyuv_convert(imgs[i])
        assert (Y[i].cpu().numpy() == ey).all() and (U[i].cpu().numpy() == eu).all() and (V[i].cpu().numpy() == ev).all()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(1920, 1080), (4096, 256), (4100, 40), (600, 200), (530, 131)])
def test_gpu_wide(cuda, w, h):
    """1080p, the C5 width (4096), a width past 4096, and widths whose last
    column band (k_sharp_band, 128 UV columns + a 32-column halo) is partial,
    over heights with several halo resynchronisations."""
    import torch
    from webp_amd import frames
    rgb = np.ascontiguousarray(synth.blobs_rgba(w, h, seed=w)[..., :3])
    Y, U, V = frames.sharpyuv_convert(torch.from_numpy(rgb[None].copy()).cuda())
    ey, eu, ev, _ = O.sharpyuv_convert(rgb)
    assert (Y[0].cpu().numpy() == ey).all() and (U[0].cpu().numpy() == eu).all() and (V[0].cpu().numpy() == ev).all()


@pytest.mark.gpu
def test_gpu_batch_over_several_launches(cuda):
    """A batch larger than one launch holds (k_sharp_wave runs at most as many
    images as the device keeps resident: 4 iterations x 32 bands an image at
    this width, ~14 images a launch), so the images' progress words and
    halo edge granules (per image, iteration and band) are offset per
    launch; every image bit-exact."""
    import torch
    from webp_amd import frames
    imgs = np.stack([synth.noise_rgba(2000, 20, seed=s)[..., :3] for s in range(40)])
    Y, U, V = frames.sharpyuv_convert(torch.from_numpy(imgs).cuda())
    torch.cuda.synchronize()
    for i in range(imgs.shape[0]):
        ey, eu, ev, _ = O.sharpyuv_convert(imgs[i])
        assert (Y[i].cpu().numpy() == ey).all() and (U[i].cpu().numpy() == eu).all() and (V[i].cpu().numpy() == ev).all(), i


# ---- the other transfer functions and convertStandard (sharpyuv.go:68-115, gamma.go:125-446) ----

NON_SRGB = [tf for tf in O.TRANSFER_FUNCS if tf != 13]


def product_transfer_tables(tf):
    from webp_amd import _lib
    g2l = np.zeros(1024, np.uint32)
    n = np.zeros(1, np.int32)
    _lib.call("wg_sharpyuv_transfer_tables_host", tf, g2l.ctypes.data, None, n.ctypes.data)
    l2g = np.zeros(int(n[0]), np.uint16)
    _lib.call("wg_sharpyuv_transfer_tables_host", tf, g2l.ctypes.data, l2g.ctypes.data, n.ctypes.data)
    return g2l, l2g


@pytest.mark.parametrize("tf", NON_SRGB)
def test_transfer_tables_product_equals_oracle(tf):
    """The kernels' GammaToLinear / LinearToGamma tables (host-built, product)
    equal the restatement's per-value functions over their whole domains."""
    g, l = product_transfer_tables(tf)
    eg, el = O.sharpyuv_transfer_tables(tf)
    assert (g == eg).all() and len(l) == len(el) and (l == el).all()


def test_transfer_tables_are_robust_to_the_math_library():
    """Evaluating pow / log10 / exp / log in long double instead of double
    gives the same tables for every transfer function: no entry sits close
    enough to a float32 or final rounding boundary for Go's math package and
    libm to disagree."""
    for tf in NON_SRGB:
        g, l = O.sharpyuv_transfer_tables(tf)
        O.lib.or_sharpyuv_tf_long_double(1)
        try:
            g2, l2 = O.sharpyuv_transfer_tables(tf)
        finally:
            O.lib.or_sharpyuv_tf_long_double(0)
        assert (g == g2).all() and (l == l2).all(), tf


def test_transfer_known_values():
    """Spot values from gamma.go's formulas: linear is the identity at
    bitDepth 10; every curve maps 0 -> 0 (log curves: to their floors) and
    full scale -> 65535 / 1023."""
    g, l = O.sharpyuv_transfer_tables(8)
    assert (g == np.arange(1024)).all() and (l == np.arange(1024)).all()
    for tf in (1, 4, 5, 6, 7, 11, 12, 14, 15, 16):
        g, l = O.sharpyuv_transfer_tables(tf)
        assert g[0] == 0 and g[1023] == 65535 and l[0] == 0 and l[65535] == 1023, tf
    g, _ = O.sharpyuv_transfer_tables(9)
    assert g[0] == round(0.005 * 65535)  # log100: midInterval at 0


@pytest.mark.gpu
@pytest.mark.parametrize("tf", NON_SRGB)
def test_gpu_transfer_functions(cuda, tf):
    import torch
    from webp_amd import frames
    imgs = [np.ascontiguousarray(synth.blobs_rgba(67, 41, seed=tf)[..., :3]),
            np.ascontiguousarray(synth.noise_rgba(67, 41, seed=tf)[..., :3])]
    Y, U, V, its = frames.sharpyuv_convert(torch.from_numpy(np.stack(imgs)).cuda(), transfer=tf, iterations=True)
    for i, rgb in enumerate(imgs):
        ey, eu, ev, eits = O.sharpyuv_convert(rgb, transfer=tf)
        assert (Y[i].cpu().numpy() == ey).all() and (U[i].cpu().numpy() == eu).all() and \
            (V[i].cpu().numpy() == ev).all(), (tf, i)
        assert its[i] == eits


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(1, 1), (2, 2), (3, 5), (67, 41), (1920, 1080)])
def test_gpu_convert_standard(cuda, w, h):
    """convertStandard (SharpEnabled = false): per-pixel matrix Y, 2x2 average U/V."""
    import torch
    from webp_amd import frames
    rgb = np.ascontiguousarray(synth.noise_rgba(w, h, seed=w * h)[..., :3])
    Y, U, V = frames.sharpyuv_convert(torch.from_numpy(rgb[None].copy()).cuda(), sharp=False)
    ey, eu, ev, _ = O.sharpyuv_convert(rgb, sharp=False)
    assert (Y[0].cpu().numpy() == ey).all() and (U[0].cpu().numpy() == eu).all() and (V[0].cpu().numpy() == ev).all()

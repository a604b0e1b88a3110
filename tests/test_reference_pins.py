"""The reference's own known answers for SharpYUV and the encoder's import
that the earlier suites had not harvested:

  sharpyuv/sharpyuv_test.go:48-69   GammaToLinear -> LinearToGamma round trip, +-1, bitDepth 8, sRGB / BT.709
  sharpyuv/sharpyuv_test.go:71-97   linear transfer is the identity; PQ and HLG map black to 0
  sharpyuv/sharpyuv_test.go:99-146  convertStandard of solid red (WebP matrix): uniform Y in [50, 120], uniform U / V
  sharpyuv/sharpyuv_test.go:148-183 convertStandard of grey 128 (Rec601 full): Y and U within 2 of 128
  sharpyuv/sharpyuv_test.go:185-217 the sharp path on a solid colour: every Y within 2 of Y[0]
  sharpyuv/sharpyuv_test.go:333-368 round trip of 128 within 3 for ten transfer functions
  internal/lossy/encode_test.go:120-144 importImage of a grey 16x16: Y within 2 of Y[0], U / V within 5 of 128

CPU: the oracle's restatements.  GPU: the product's kernels on the same
inputs (wg_sharpyuv_convert_ex, wg_import_rgba)."""
import numpy as np
import pytest

import oracle as O

SRGB, BT709, LINEAR, PQ, HLG = 13, 1, 8, 16, 18
ALL_TF = {"BT709": 1, "BT470M": 4, "BT470BG": 5, "BT601": 6, "SMPTE240": 7, "SRGB": 13, "BT2020_10": 14, "PQ": 16,
          "HLG": 18, "SMPTE428": 17}
REC601_FULL = np.array([19595, 38470, 7471, 0, -11058, -21710, 32768, 128 << 16, 32768, -27439, -5329, 128 << 16],
                       np.int32)  # sharpyuv/csp.go:71-75


def g2l(v, bd, tf):
    return int(O.lib.or_sharpyuv_gamma_to_linear(v, bd, tf))


def l2g(v, bd, tf):
    return int(O.lib.or_sharpyuv_linear_to_gamma(v, bd, tf))


@pytest.mark.parametrize("tf", [SRGB, BT709])
def test_gamma_round_trip_8bit(tf):
    for v in range(256):
        assert abs(l2g(g2l(v, 8, tf), 8, tf) - v) <= 1, v


def test_linear_transfer_and_black_points():
    assert g2l(128, 8, LINEAR) == 128 and l2g(128, 8, LINEAR) == 128
    assert g2l(0, 8, PQ) == 0 and g2l(0, 8, HLG) == 0


@pytest.mark.parametrize("name", sorted(ALL_TF))
def test_round_trip_128_all_transfers(name):
    tf = ALL_TF[name]
    assert abs(l2g(g2l(128, 8, tf), 8, tf) - 128) <= 3


def solid(w, h, rgb):
    return np.tile(np.array(rgb, np.uint8), (h, w, 1))


def check_solid_red(y, u, v):
    assert (y == y[0, 0]).all() and 50 <= y[0, 0] <= 120
    assert (u == u[0, 0]).all() and (v == v[0, 0]).all()


def check_gray(y, u):
    assert abs(int(y[0, 0]) - 128) <= 2 and abs(int(u[0, 0]) - 128) <= 2


def check_sharp_solid(y):
    assert (np.abs(y.astype(int) - int(y[0, 0])) <= 2).all()


def test_convert_standard_solid_red_and_gray():
    y, u, v, _ = O.sharpyuv_convert(solid(4, 4, (255, 0, 0)), sharp=False)
    check_solid_red(y, u, v)
    y, u, v, _ = O.sharpyuv_convert(solid(2, 2, (128, 128, 128)), matrix=REC601_FULL, sharp=False)
    check_gray(y, u)


def test_convert_sharp_solid_color():
    y, _, _, _ = O.sharpyuv_convert(solid(4, 4, (100, 150, 200)))
    check_sharp_solid(y)


def check_gray_import(y, u, v):
    y, u, v = y[:16, :16].astype(int), u[:8, :8].astype(int), v[:8, :8].astype(int)
    assert (np.abs(y - y[0, 0]) <= 2).all()
    assert (np.abs(u - 128) <= 5).all() and (np.abs(v - 128) <= 5).all()


def test_import_gray_solid():
    rgba = solid(16, 16, (128, 128, 128, 255))
    check_gray_import(*O.import_rgba(rgba, has_alpha=False))


@pytest.mark.gpu
def test_gpu_reference_pins(cuda):
    import torch

    from webp_amd import frames

    def conv(rgb, **kw):
        y, u, v = frames.sharpyuv_convert(torch.from_numpy(rgb[None]).cuda(), **kw)
        torch.cuda.synchronize()
        return y[0].cpu().numpy(), u[0].cpu().numpy(), v[0].cpu().numpy()
    y, u, v = conv(solid(4, 4, (255, 0, 0)), sharp=False)
    check_solid_red(y, u, v)
    y, u, _ = conv(solid(2, 2, (128, 128, 128)), matrix=REC601_FULL, sharp=False)
    check_gray(y, u)
    y, _, _ = conv(solid(4, 4, (100, 150, 200)))
    check_sharp_solid(y)
    y, u, v = frames.import_rgba(torch.from_numpy(solid(16, 16, (128, 128, 128, 255))[None]).cuda(), has_alpha=False)
    torch.cuda.synchronize()
    check_gray_import(y[0].cpu().numpy(), u[0].cpu().numpy(), v[0].cpu().numpy())

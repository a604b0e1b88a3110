"""CPU: the VP8L predictor-transform restatement (oracle/lossless.c).

Parity status: the mode choice follows the reference's own heuristic
(estimateEntropy), which no third-party library shares, so it is pinned by
restatement only; the residual / inverse pair is pinned by the round-trip
property (the inverse is the normative VP8L decoder step) on every case.
The fastSLog2 table restates Go's math.Log2 (not runnable here); it is
checked against libm within 1e-12 relative and is bit-identical between the
product (host) and the oracle."""
import math

import numpy as np
import pytest

import oracle as O
from tools import synth


def argb_of(rgba):
    rgba = np.asarray(rgba, np.uint32)
    return (rgba[..., 3] << 24) | (rgba[..., 0] << 16) | (rgba[..., 1] << 8) | rgba[..., 2]


def images():
    rng = np.random.default_rng(1)
    yield "noise", rng.integers(0, 2 ** 32, (37, 53), dtype=np.uint64).astype(np.uint32)
    yield "grad", argb_of(synth.gradient_rgba(70, 45))
    yield "blobs", argb_of(synth.blobs_rgba(64, 64, seed=2, alpha=True))
    yield "flat", np.full((20, 33), 0xff336699, np.uint32)
    yield "1x1", np.array([[0x12345678]], np.uint32)
    yield "row", rng.integers(0, 2 ** 32, (1, 40), dtype=np.uint64).astype(np.uint32)
    yield "col", rng.integers(0, 2 ** 32, (40, 1), dtype=np.uint64).astype(np.uint32)


@pytest.mark.parametrize("bits", [2, 3, 5])
@pytest.mark.parametrize("quality", [10, 30, 75])
def test_residual_inverse_round_trip(bits, quality):
    for name, img in images():
        modes, res = O.vp8l_residual_image(img, bits, quality)
        max_mode = 4 if quality < 25 else (8 if quality < 50 else 14)
        assert ((modes >> 8) & 0xff).max() < max_mode and ((modes & 0xff0000ff) == 0xff000000).all()
        assert (O.vp8l_inverse_predictor(modes, bits, res) == img).all(), name


def test_slog2_lut_vs_libm():
    lut = O.vp8l_slog2_lut()
    ref = np.array([0.0] + [i * math.log2(i) for i in range(1, 65536)])
    assert lut[0] == 0 and np.all(np.abs(lut - ref) <= 1e-12 * np.maximum(ref, 1))
    for k in range(16):  # exact powers of two take frexp's exact branch
        assert lut[1 << k] == (1 << k) * k


def test_product_lut_matches_oracle():
    from webp_amd import lossless
    assert np.array_equal(lossless.slog2_lut().view(np.uint64), O.vp8l_slog2_lut().view(np.uint64))


def test_entropy_ties_pick_first_mode():
    """A flat tile gives every predictor the same residual histogram except
    modes that see the zero border; the first minimum (strict '<') wins."""
    img = np.full((8, 8), 0xff808080, np.uint32)
    modes, _ = O.vp8l_residual_image(img, 3, 75)
    costs = [O.vp8l_estimate_entropy(img, 3, 0, 0, m) for m in range(14)]
    assert (modes[0, 0] >> 8) & 0xff == int(np.argmin(costs))


def test_subtract_green():
    px = np.array([0xff102030, 0x80ff0001], np.uint32)
    out = O.vp8l_subtract_green(px)
    g = (px >> 8) & 0xff
    assert ((out >> 16) & 0xff == ((px >> 16) - g) & 0xff).all() and (out & 0xff == (px - g) & 0xff).all()

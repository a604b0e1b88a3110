"""GPU parity: VP8L predictor transform (ResidualImage, inverse predictor,
subtract/add green) through the C ABI vs the C restatement (bit-exact:
modes, residuals, reconstructions).  Sizes: edge shapes, non-multiples of
the tile, bits 2..9 (bits 9 takes the reference's out-of-table math.Log2
path on the device), all quality bands, a batch, and C5's 4096x4096 via the
size-independent round trip."""
import numpy as np
import pytest
import torch

import oracle as O
from test_lossless_oracle import argb_of, images
from tools import synth
from webp_amd import lossless as L

pytestmark = pytest.mark.gpu


def gpu_residual(img, bits, quality):
    modes, res = L.ResidualImage(L.to_argb_tensor(img), bits, quality)
    return L.from_argb_tensor(modes)[0], L.from_argb_tensor(res)[0]


@pytest.mark.parametrize("bits", [2, 3, 4, 5])
@pytest.mark.parametrize("quality", [10, 30, 75])
def test_residual_image_matches_oracle(cuda, bits, quality):
    for name, img in images():
        em, er = O.vp8l_residual_image(img, bits, quality)
        gm, gr = gpu_residual(img, bits, quality)
        assert (gm == em).all(), (name, np.argwhere(gm != em)[:4])
        assert (gr == er).all(), name


@pytest.mark.parametrize("bits", [2, 3, 5])
def test_select_ragged_tiles(cuda, bits):
    """k_vp8l_select_q3 (bits <= 5) on ragged tiles: a 260 x 90 image leaves a
    partial tile column and row at every tile size."""
    img = argb_of(synth.blobs_rgba(260, 90, seed=11, alpha=True))
    em, er = O.vp8l_residual_image(img, bits, 75)
    gm, gr = gpu_residual(img, bits, 75)
    assert (gm == em).all() and (gr == er).all()


@pytest.mark.parametrize("bits", [6, 7, 9])
def test_large_tiles(cuda, bits):
    """Subsampled rows (tile height > 16) and, at bits 9, histogram counts
    beyond the 65536-entry table."""
    img = argb_of(synth.blobs_rgba(600, 530, seed=4, alpha=True))
    em, er = O.vp8l_residual_image(img, bits, 75)
    gm, gr = gpu_residual(img, bits, 75)
    assert (gm == em).all() and (gr == er).all()


@pytest.mark.parametrize("bits", [2, 5])
def test_inverse_matches_oracle(cuda, bits):
    for name, img in images():
        em, er = O.vp8l_residual_image(img, bits, 75)
        got = L.predictor_inverse(L.to_argb_tensor(em), bits, L.to_argb_tensor(er), check=True)
        assert (L.from_argb_tensor(got)[0] == img).all(), name


def test_inverse_random_modes_multiband(cuda):
    """Arbitrary modes (0..15, incl. the decoder's fallback) and residuals over
    several 64-row bands and images: GPU == oracle inverse."""
    rng = np.random.default_rng(9)
    h, w, bits = 200, 171, 3
    res = rng.integers(0, 2 ** 32, (3, h, w), dtype=np.uint64).astype(np.uint32)
    modes = ((rng.integers(0, 16, (3, L.subsample(h, bits), L.subsample(w, bits))) << 8) | 0xff000000).astype(np.uint32)
    got = L.from_argb_tensor(L.predictor_inverse(L.to_argb_tensor(modes), bits, L.to_argb_tensor(res), check=True))
    for i in range(3):
        assert (got[i] == O.vp8l_inverse_predictor(modes[i], bits, res[i])).all()


@pytest.mark.parametrize("shape", [(1, 200, 171, 3), (3, 300, 97, 4), (2, 130, 4100, 2), (1, 31, 64, 5)])
def test_inverse_shapes(cuda, shape):
    """Several images, partial last bands, a width past 4096, arbitrary modes."""
    n, h, w, bits = shape
    rng = np.random.default_rng(h * w + n)
    res = rng.integers(0, 2 ** 32, (n, h, w), dtype=np.uint64).astype(np.uint32)
    modes = ((rng.integers(0, 16, (n, L.subsample(h, bits), L.subsample(w, bits))) << 8) | 0xff000000).astype(np.uint32)
    got = L.from_argb_tensor(L.predictor_inverse(L.to_argb_tensor(modes), bits, L.to_argb_tensor(res), check=True))
    for i in range(n):
        assert (got[i] == O.vp8l_inverse_predictor(modes[i], bits, res[i])).all(), i


def test_batch_of_images(cuda):
    imgs = np.stack([argb_of(synth.noise_rgba(96, 80, seed=s)) for s in range(3)])
    m, r = L.ResidualImage(L.to_argb_tensor(imgs), 4, 75)
    m, r = L.from_argb_tensor(m), L.from_argb_tensor(r)
    for i in range(3):
        em, er = O.vp8l_residual_image(imgs[i], 4, 75)
        assert (m[i] == em).all() and (r[i] == er).all()


def test_c5_4096_round_trip(cuda):
    """C5 shape (4096x4096, bits 5, q75): residual -> inverse is the identity,
    subtract -> add green is the identity; modes spot-checked vs the oracle on
    a tile row band."""
    img = argb_of(synth.blobs_rgba(4096, 4096, seed=5, alpha=True))
    t = L.to_argb_tensor(img)
    g = L.SubtractGreen(t.clone())
    modes, res = L.ResidualImage(g, 5, 75)
    back = L.AddGreen(L.predictor_inverse(modes, 5, res, check=True))
    assert torch.equal(back, t.unsqueeze(0))
    band = L.from_argb_tensor(g)[:96]  # tiles rows 0..2 only depend on rows < 96
    em, _ = O.vp8l_residual_image(band, 5, 75)
    assert (L.from_argb_tensor(modes)[0][:2] == em[:2]).all()


def test_green_matches_oracle(cuda):
    rng = np.random.default_rng(3)
    px = rng.integers(0, 2 ** 32, (1, 7, 13), dtype=np.uint64).astype(np.uint32)
    got = L.from_argb_tensor(L.SubtractGreen(L.to_argb_tensor(px)))
    assert (got[0] == O.vp8l_subtract_green(px[0])).all()

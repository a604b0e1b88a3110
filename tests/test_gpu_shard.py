"""GPU parity at the C5 size (4096x4096, SURVEY.md 8(d): a noise + gradient
blend) and of the row-band kernels the multi-GPU path shards with
(webp_amd/shard.py):

  - SharpYUV (WebP matrix, sRGB) vs the oracle, bit-exact, and the refinement
    iteration count the reference's early exit gives;
  - plane SSIM vs the oracle within 1e-6 relative, and the band kernels
    (wg_plane_ssim_rows for every rank of 2-, 3- and 8-way partitions,
    reduced by wg_plane_ssim_reduce) bit-identical to wg_plane_ssim;
  - VP8L ResidualImage (bits 5, q75, 14 modes) vs the oracle, bit-exact, and
    the band kernels (wg_vp8l_residual_image_rows) assembled over the same
    partitions bit-identical to the whole-image call."""
import numpy as np
import pytest
import torch

import oracle as O
from test_lossless_oracle import argb_of
from tools import synth
from webp_amd import frames, shard
from webp_amd import lossless as L

pytestmark = pytest.mark.gpu

S = 4096


@pytest.fixture(scope="module")
def c5_rgba():
    noise = synth.noise_rgba(S, S, seed=55)
    grad = synth.gradient_rgba(S, S)
    blend = ((noise.astype(np.uint16) + 3 * grad.astype(np.uint16)) // 4).astype(np.uint8)
    blend[..., 3] = 255
    return blend


def test_sharpyuv_4096(cuda, c5_rgba):
    rgb = np.ascontiguousarray(c5_rgba[..., :3])
    Y, U, V, its = frames.sharpyuv_convert(torch.from_numpy(rgb[None]).cuda(), iterations=True)
    ey, eu, ev, eits = O.sharpyuv_convert(rgb)
    assert (Y[0].cpu().numpy() == ey).all() and (U[0].cpu().numpy() == eu).all() and (V[0].cpu().numpy() == ev).all()
    assert its[0] == eits


def test_plane_ssim_4096_and_bands(cuda, c5_rgba):
    a = np.ascontiguousarray(c5_rgba[..., 1])
    rng = np.random.default_rng(4)
    b = np.clip(a.astype(np.int16) + rng.integers(-6, 7, a.shape), 0, 255).astype(np.uint8)
    ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    whole = float(frames.plane_ssim(ta[None], tb[None])[0].item())
    want = O.plane_ssim(a, b)
    assert abs(whole - want) <= 1e-6 * abs(want)  # float64 sums in another order (tolerance of A22)
    ty = S // 16
    for world in (2, 3, 8):
        parts = [shard._device_ssim_rows(ta, tb, *shard.band_of(ty, world, r)) for r in range(world)]
        assert shard._device_ssim_reduce(torch.cat(parts)) == whole, world  # bit-identical


def test_vp8l_residual_4096_and_bands(cuda, c5_rgba):
    img = argb_of(c5_rgba)
    t = L.to_argb_tensor(img)
    modes, res = L.ResidualImage(t, 5, 75)
    em, er = O.vp8l_residual_image(img, 5, 75)
    gm, gr = L.from_argb_tensor(modes)[0], L.from_argb_tensor(res)[0]
    assert (gm == em).all() and (gr == er).all()
    ty = S >> 5
    for world in (2, 3, 8):
        bands = [shard._device_residual_rows(t, 5, 75, *shard.band_of(ty, world, r)) for r in range(world)]
        bm = torch.cat([b[0] for b in bands])
        br = torch.cat([b[1] for b in bands])
        assert torch.equal(bm, modes[0]) and torch.equal(br, res[0]), world


def test_band_reads_only_its_halo(cuda, c5_rgba):
    """A band computed from a buffer holding only its rows and the halo row
    above (everything else poisoned) equals the whole-image result: the
    kernels read nothing outside what the shard sends."""
    img = argb_of(c5_rgba[:512, :640])
    t = L.to_argb_tensor(img)
    modes, res = L.ResidualImage(t, 5, 75)
    t0, t1 = 5, 9
    poisoned = torch.full_like(t, 0x5a5a5a5a)
    y0, y1 = (t0 << 5) - 1, t1 << 5
    poisoned[y0:y1] = t[y0:y1]
    bm, br = shard._device_residual_rows(poisoned, 5, 75, t0, t1)
    assert torch.equal(bm, modes[0][t0:t1]) and torch.equal(br, res[0][t0 << 5:t1 << 5])
    a = torch.from_numpy(np.ascontiguousarray(c5_rgba[:512, :640, 0])).cuda()
    b = torch.from_numpy(np.ascontiguousarray(c5_rgba[:512, :640, 2])).cuda()
    full = shard._device_ssim_rows(a, b, 0, 32)
    pa, pb = torch.full_like(a, 17), torch.full_like(b, 200)
    r0, r1 = 16 * 11 - 3, 16 * 20 + 3
    pa[r0:r1], pb[r0:r1] = a[r0:r1], b[r0:r1]
    part = shard._device_ssim_rows(pa, pb, 11, 20)
    tx = shard.ssim_row_partials(640)
    assert torch.equal(part, full[11 * tx:20 * tx])

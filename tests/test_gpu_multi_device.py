"""GPU: the multi-device batch entry point (wg_encode_frames_devices, SURVEY.md
8(b) last bullet / 8(e) C4) -- frames owned round-robin by the listed devices,
each running the whole device encode path, outputs gathered to host memory in
frame order -- against the single-device path (frames.encode_frames, itself
parity-tested against the oracle) and, for one frame, the oracle directly.
The box has one GPU: a device list may name a device more than once (each
entry its own stream and buffers), so lists like [0, 0, 0] exercise the
round-robin split, the row bands with their halos and the in-order gather
on it."""
import numpy as np
import pytest
import torch

import oracle as O
from tools import synth
from webp_amd import frames

pytestmark = pytest.mark.gpu


def test_multi_device_equals_single_device(cuda):
    w, h = 160, 96
    rgba = np.stack([synth.noise_rgba(w, h, seed=1), synth.gradient_rgba(w, h), synth.blobs_rgba(w, h, seed=2),
                     synth.noise_rgba(w, h, seed=4)])
    out, (ry, ru, rv), seg_ids, info = frames.encode_frames_devices(rgba, [0, 0, 0])
    ref_out, (RY, RU, RV), ref_ids, _, ref_info = frames.encode_frames(torch.from_numpy(rgba).cuda())
    assert (out == ref_out.cpu().numpy()).all()
    assert (ry == RY.cpu().numpy()).all() and (ru == RU.cpu().numpy()).all() and (rv == RV.cpu().numpy()).all()
    assert (seg_ids == ref_ids.cpu().numpy()).all() and (info == ref_info.cpu().numpy()).all()


def test_multi_device_frame_matches_oracle(cuda):
    w, h = 128, 80
    rgba = synth.blobs_rgba(w, h, seed=7)
    out, (ry, ru, rv), seg_ids, info = frames.encode_frames_devices(rgba[None], [0])
    y, u, v = O.import_rgba(rgba, has_alpha=False)
    enc, (ey, eu, ev), e_ids, e_info = O.encode_frame(y, u, v, w, h, O.encoder_config())
    got = out.view(frames.MB_ENC_DTYPE).reshape(-1)
    for f in ("coeffs", "modes", "nz_y", "nz_uv", "non_zero_y", "non_zero_uv", "mb_type", "i16_mode", "uv_mode", "nz_dc",
              "skip", "segment", "score"):
        assert (got[f] == enc[f]).all(), f
    assert (ry[0][:h, :w] == ey[:h, :w]).all() and (ru[0] == eu).all() and (rv[0] == ev).all()
    assert (seg_ids[0] == e_ids).all() and info[0].tobytes() == e_info.tobytes()


def test_multi_device_rejects_bad_device_lists(cuda):
    from webp_amd._lib import WebpGpuError
    rgba = synth.gradient_rgba(64, 64)[None]
    with pytest.raises(WebpGpuError, match="invalid argument"):
        frames.encode_frames_devices(rgba, [torch.cuda.device_count()])
    with pytest.raises(WebpGpuError, match="mbh >= 4"):
        frames.encode_frames_devices(synth.gradient_rgba(64, 48)[None], [0])


@pytest.mark.parametrize("w,h,bits,n_bands", [(4096, 4096, 5, 8), (333, 517, 3, 3), (333, 517, 3, 1), (64, 20, 3, 5)])
def test_residual_image_devices_equals_one_device(cuda, w, h, bits, n_bands):
    """C5 VP8L ResidualImage by tile-row bands from one host process == the one-device kernel."""
    from webp_amd import lossless
    rng = np.random.default_rng(w)
    argb = (rng.integers(0, 2**32, size=(h, w), dtype=np.uint64) | 0xff000000).astype(np.uint32)
    argb[: h // 2] = (argb[: h // 2] & 0xff0f0f0f)  # smoother upper half: other modes win there
    modes, res = lossless.ResidualImage_devices(argb, bits, 75, [0] * n_bands)
    m1, r1 = lossless.ResidualImage(torch.from_numpy(argb.view(np.int32)).cuda(), bits, 75)
    assert (modes.view(np.int32) == m1[0].cpu().numpy()).all()
    assert (res.view(np.int32) == r1[0].cpu().numpy()).all()


@pytest.mark.parametrize("w,h,n_bands", [(4096, 4096, 8), (301, 77, 3), (301, 77, 1), (40, 20, 4)])
def test_plane_ssim_devices_equals_one_device(cuda, w, h, n_bands):
    """C5 plane SSIM by 16-row bands from one host process == wg_plane_ssim, bit for bit."""
    rng = np.random.default_rng(h)
    a = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    b = np.clip(a.astype(np.int32) + rng.integers(-9, 10, size=(h, w)), 0, 255).astype(np.uint8)
    got = frames.plane_ssim_devices(a, b, [0] * n_bands)
    ref = frames.plane_ssim(torch.from_numpy(a[None]).cuda(), torch.from_numpy(b[None]).cuda())[0].item()
    assert got == ref

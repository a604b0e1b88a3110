"""GPU: the multi-device batch entry point (wg_encode_frames_devices, SURVEY.md
8(b) last bullet / 8(e) C4) -- frames owned round-robin by the listed devices,
each running the whole device encode path, outputs gathered to host memory in
frame order -- against the single-device path (frames.encode_frames, itself
parity-tested against the oracle) and, for one frame, the oracle directly.
The box has one GPU, so the device list is [0]; the round-robin split and
the in-order gather over several devices are covered by the CPU test of the
ownership map (tests/test_shard.py) and by the argument checks below."""
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
    out, (ry, ru, rv), seg_ids, info = frames.encode_frames_devices(rgba, [0])
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
        frames.encode_frames_devices(rgba, [0, 0])  # a device listed twice
    with pytest.raises(WebpGpuError, match="invalid argument"):
        frames.encode_frames_devices(rgba, [torch.cuda.device_count()])
    with pytest.raises(WebpGpuError, match="mbh >= 4"):
        frames.encode_frames_devices(synth.gradient_rgba(64, 48)[None], [0])

"""GPU parity: the encoder macroblock RD loop (Phase A, methods 4 and 3) through the
C ABI vs the C restatement (oracle/lossy_rd.c): every MBEncInfo field
(modes, levels, nz bookkeeping, skip, score) and the reconstruction,
bit-exact.  Frames cover image edges (non-multiple-of-16 sizes), all four
segments with different quantisers, fine / coarse quantisers (I4-heavy and
I16-heavy), SNS on / off, quality < 50 (2 I4 RD candidates), a batch, and
the 1920x1080 C2 frame; method 3 (plain quantisation instead of the trellis in
the I4 RD and the final I16 residuals, encode_parallel.go:793, :1202, TLambdaSD
0) on the same cases.  Frames have mbh >= 4: smaller ones take the
reference's serial encodeFrame (encode.go:1356), which wg_encode_mbs refuses.

test_encode_pipeline_* run the whole device encode path of frames.encode_frames
(import -> analysis -> segment analysis -> Phase A) against oracle.encode_frame
on the C1 frame (testdata/test.png) and 1080p frames of each content type."""
import os

import numpy as np
import pytest
import torch

import oracle as O
from tools import synth
from webp_amd import frames

pytestmark = pytest.mark.gpu

FIELDS = ("coeffs", "modes", "nz_y", "nz_uv", "non_zero_y", "non_zero_uv", "mb_type", "i16_mode", "uv_mode", "nz_dc",
          "skip", "segment", "score")


def planes(w, h, kind, seed):
    gen = {"grad": lambda: synth.gradient_rgba(w, h), "noise": lambda: synth.noise_rgba(w, h, seed=seed),
           "blobs": lambda: synth.blobs_rgba(w, h, seed=seed)}[kind]
    return O.import_rgba(gen(), has_alpha=False)


def run(imgs, w, h, qs, sns=50, quality=75, method=4):
    n = len(imgs)
    mbw, mbh = frames.mb_dims(w, h)
    segs = np.stack([O.setup_segment(q, method=method, sns_strength=sns) for q in qs])
    seg_ids = np.stack([((np.arange(mbw * mbh) * 7 + i) % 4).astype(np.uint8) for i in range(n)])
    proba = O.default_proba()
    Y = torch.from_numpy(np.stack([p[0] for p in imgs])).cuda()
    U = torch.from_numpy(np.stack([p[1] for p in imgs])).cuda()
    V = torch.from_numpy(np.stack([p[2] for p in imgs])).cuda()
    out, (RY, RU, RV) = frames.encode_mbs(Y, U, V, w, h, torch.from_numpy(seg_ids).cuda(), segs.view(frames.SEGMENT_DTYPE),
                                          proba, method=method, quality=quality, check=True)
    got = out.cpu().numpy().view(frames.MB_ENC_DTYPE).reshape(n, mbw * mbh)
    RY, RU, RV = RY.cpu().numpy(), RU.cpu().numpy(), RV.cpu().numpy()
    for i, (y, u, v) in enumerate(imgs):
        enc, ry, ru, rv = O.encode_frame_rd(y, u, v, w, h, seg_ids[i], segs, proba, method=method, quality=quality)
        for f in FIELDS:
            bad = np.argwhere(np.asarray(got[i][f] != enc[f]).reshape(len(enc), -1).any(axis=1))
            assert len(bad) == 0, f"image {i} field {f}: MBs {bad[:5].ravel()} (of {len(enc)})"
        assert (RY[i][:h, :w] == ry[:h, :w]).all() and (RU[i] == ru).all() and (RV[i] == rv).all()


@pytest.mark.parametrize("w,h,kind,qs", [(16, 64, "noise", (20, 30, 40, 50)), (48, 64, "blobs", (10, 20, 30, 40)),
                                         (37, 61, "noise", (30, 30, 30, 30)), (80, 64, "grad", (60, 70, 80, 90)),
                                         (100, 64, "blobs", (5, 15, 100, 127))])
@pytest.mark.parametrize("method", [4, 3])
def test_encode_matches_oracle(cuda, w, h, kind, qs, method):
    run([planes(w, h, kind, seed=w)], w, h, qs, method=method)


@pytest.mark.parametrize("method", [4, 3])
def test_encode_low_quality_and_no_sns(cuda, method):
    run([planes(64, 64, "noise", 3)], 64, 64, (25, 35, 45, 55), sns=0, quality=30, method=method)


@pytest.mark.parametrize("method", [4, 3])
def test_encode_batch(cuda, method):
    run([planes(96, 80, k, s) for s, k in enumerate(("noise", "blobs", "grad"))], 96, 80, (20, 40, 60, 80), method=method)


@pytest.mark.parametrize("method", [4, 3])
def test_encode_1080p(cuda, method):
    run([planes(1920, 1080, "blobs", 7)], 1920, 1080, (30, 35, 40, 45), method=method)


def test_methods_below_3_refused(cuda):
    """Methods 0-2 take the serial encodeFrame with non-RD mode choice (encode.go:1356)."""
    from webp_amd._lib import WebpGpuError
    with pytest.raises(WebpGpuError, match="methods 3-6"):
        run([planes(64, 64, "noise", 3)], 64, 64, (25, 35, 45, 55), method=2)


def test_small_frames_refused(cuda):
    """mbh < 4: EncodeFrame uses the serial encodeFrame (encode.go:1356)."""
    from webp_amd._lib import WebpGpuError
    with pytest.raises(WebpGpuError, match="mbh >= 4"):
        run([planes(64, 48, "noise", 3)], 64, 48, (25, 35, 45, 55))


def pipeline(rgbas, w, h, **cfg):
    out, (RY, RU, RV), seg_ids, segs, info = frames.encode_frames(torch.from_numpy(np.stack(rgbas)).cuda(),
                                                                  frames.encoder_config(**cfg))
    n = len(rgbas)
    mbw, mbh = frames.mb_dims(w, h)
    got = out.cpu().numpy().view(frames.MB_ENC_DTYPE).reshape(n, mbw * mbh)
    RY, RU, RV, seg_ids = RY.cpu().numpy(), RU.cpu().numpy(), RV.cpu().numpy(), seg_ids.cpu().numpy()
    info = info.cpu().numpy().view(frames.FRAME_SEGS_DTYPE).reshape(n)
    for i, rgba in enumerate(rgbas):
        y, u, v = O.import_rgba(rgba, has_alpha=False)
        enc, (ry, ru, rv), e_ids, e_info = O.encode_frame(y, u, v, w, h, O.encoder_config(**cfg))
        assert (seg_ids[i] == e_ids).all() and info[i].tobytes() == e_info.tobytes(), f"image {i}: segments"
        for f in FIELDS:
            bad = np.argwhere(np.asarray(got[i][f] != enc[f]).reshape(len(enc), -1).any(axis=1))
            assert len(bad) == 0, f"image {i} field {f}: MBs {bad[:5].ravel()} (of {len(enc)})"
        assert (RY[i][:h, :w] == ry[:h, :w]).all() and (RU[i] == ru).all() and (RV[i] == rv).all()
    return info


def test_encode_pipeline_c1_test_png(cuda):
    """C1: testdata/test.png (768x576), webp.Encode defaults (q75, method 4)."""
    rgba = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "test_png_rgba.npz"))["rgba"]
    info = pipeline([rgba], 768, 576)
    assert info[0]["base_quant"] > 0


def test_encode_pipeline_1080p_contents(cuda):
    """C2 frames of each content at the reference's q75 defaults, one batch."""
    w, h = 1920, 1080
    pipeline([synth.gradient_rgba(w, h), synth.noise_rgba(w, h, seed=1), synth.blobs_rgba(w, h, seed=2)], w, h)


def test_encode_pipeline_presets(cuda):
    """Non-default analysis knobs feeding Phase A: smoothing, 2 segments, low quality."""
    w, h = 320, 240
    imgs = [synth.blobs_rgba(w, h, seed=5), synth.noise_rgba(w, h, seed=6)]
    pipeline(imgs, w, h, quality=30, sns_strength=80, filter_strength=35, filter_sharpness=4, preprocessing=1)
    pipeline(imgs, w, h, quality=90, sns_strength=0, segments=2)


def test_encode_pipeline_method3(cuda):
    """webp.Encode with Method 3 (the parallel Phase A without the trellis) on the C1 frame and noise."""
    rgba = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "test_png_rgba.npz"))["rgba"]
    pipeline([rgba], 768, 576, method=3)
    pipeline([synth.noise_rgba(320, 240, seed=9), synth.gradient_rgba(320, 240)], 320, 240, method=3, quality=40)


@pytest.mark.parametrize("schedule", ["0", "1"])
@pytest.mark.parametrize("method", [4, 3])
def test_encode_row_schedules(cuda, monkeypatch, schedule, method):
    """Both row schedules of k_encode_rows on the same frames: one wave a row
    (the batch schedule) and a wave pair a row (I4 RD beside the I16 / chroma
    work, the schedule of launches whose rows fit the wave slots twice);
    WG_ENCODE_PAIR forces either."""
    monkeypatch.setenv("WG_ENCODE_PAIR", schedule)
    run([planes(160, 96, k, s) for s, k in enumerate(("noise", "blobs", "grad"))], 160, 96, (20, 40, 60, 80), method=method)
    run([planes(64, 64, "noise", 3)], 64, 64, (25, 35, 45, 55), sns=0, quality=30, method=method)


@pytest.mark.parametrize("schedule", ["0", "1"])
def test_row_schedule_keeps_outputs(cuda, monkeypatch, schedule):
    """wg_encode_row_order only reorders the row dequeue (textured frames' rows
    first): the outputs equal the (row, frame)-order launch and the oracle."""
    monkeypatch.setenv("WG_ENCODE_PAIR", schedule)
    w, h = 320, 240
    rgba = np.stack([[synth.gradient_rgba, synth.noise_rgba, synth.blobs_rgba][i % 3](w, h, **({} if i % 3 == 0 else
                     {"seed": i})) for i in range(9)])
    t = torch.from_numpy(rgba).cuda()
    mbw, mbh = frames.mb_dims(w, h)
    Y, U, V = frames.import_rgba(t, has_alpha=False)
    alphas, uv_sum = frames.analysis_alphas(Y, U, V, w, h)
    seg_ids, segs, _ = frames.segment_analysis(frames.encoder_config(), alphas, uv_sum, mbw, mbh)
    proba = frames.default_proba()
    plain, rec0 = frames.encode_mbs(Y, U, V, w, h, seg_ids, segs, proba, check=True)
    work = frames.encode_row_order(alphas, mbw, mbh)
    ordered, rec1 = frames.encode_mbs(Y, U, V, w, h, seg_ids, segs, proba, work=work, check=True)
    again, _ = frames.encode_mbs(Y, U, V, w, h, seg_ids, segs, proba, work=work, check=True)  # the schedule persists
    assert torch.equal(plain, ordered) and torch.equal(plain, again)
    assert all(torch.equal(a, b) for a, b in zip(rec0, rec1))
    got = ordered.cpu().numpy().view(frames.MB_ENC_DTYPE).reshape(9, mbw * mbh)
    for i in (1, 2):
        y, u, v = O.import_rgba(rgba[i], has_alpha=False)
        enc, _, _, _ = O.encode_frame(y, u, v, w, h, O.encoder_config())
        for f in FIELDS:
            assert (got[i][f] == enc[f]).all(), (i, f)


def test_row_schedule_table(cuda):
    """k_row_slack / k_row_order build exactly the order the key (y - slack_i, y, i)
    sorts to, slack_i = (2 mbh / 5) (1 - (m_i / 242)^4), m_i = min(mean alpha_i,
    242) (integers), and every frame's rows appear in row order (the kernel's
    waits stay on running waves)."""
    w, h = 320, 240
    rgba = np.stack([[synth.gradient_rgba, synth.noise_rgba, synth.blobs_rgba][i % 3](w, h, **({} if i % 3 == 0 else
                     {"seed": i})) for i in range(7)])
    t = torch.from_numpy(rgba).cuda()
    mbw, mbh = frames.mb_dims(w, h)
    Y, U, V = frames.import_rgba(t, has_alpha=False)
    alphas, _ = frames.analysis_alphas(Y, U, V, w, h)
    n, rows = 7, 7 * mbh
    work = frames.encode_row_order(alphas, mbw, mbh).cpu().numpy()
    base = n * mbw * 128 // 4 + 4  # int32 index of the tag: records | ctl[4] | tag
    words = work.view(np.int32)
    order, slack = words[base + 4:base + 4 + rows], words[base + 4 + rows:base + 4 + rows + n]
    a = np.clip(alphas.cpu().numpy().astype(np.int64), 0, 255)
    mean = a.sum(axis=1) // a.shape[1]
    m4 = np.minimum(mean, 242) ** 4
    f4 = 242 ** 4
    assert (slack == (2 * mbh // 5) * (f4 - m4) // f4).all()
    keys = sorted(((y - slack[i], y, i) for y in range(mbh) for i in range(n)))
    assert order.tolist() == [y * n + i for (_, y, i) in keys]
    assert slack[1] > slack[0] and slack[1] > slack[2]  # the noise frame goes ahead

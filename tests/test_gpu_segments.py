"""GPU parity: the segment analysis kernel (k_segments, wg_segment_analysis)
against the restatement (oracle/segments.c) -- segment ids, the per-image
wg_frame_segs record and the four setupSegment quantiser records, bit-exact.
Cases: the hand-derived ones of tests/test_segments.py, every config knob the
analysis reads (segments 1-4, SNS 0/50/100, filter strength 0/60/100,
sharpness, smoothing), tiny and large frames, and the alphas of real frames."""
import numpy as np
import pytest
import torch

import oracle as O
from tools import synth
from webp_amd import frames

pytestmark = pytest.mark.gpu


def check(alpha_list, mbw, mbh, uv_sums, **kw):
    n = len(alpha_list)
    cfg_p = frames.encoder_config(**kw)
    cfg_o = O.encoder_config(**kw)
    A = torch.from_numpy(np.stack([np.asarray(a, np.int32).reshape(-1) for a in alpha_list])).cuda()
    S = torch.tensor(uv_sums, dtype=torch.int32).cuda()
    ids, segs, info = frames.segment_analysis(cfg_p, A, S, mbw, mbh)
    ids, segs = ids.cpu().numpy(), segs.cpu().numpy()
    info = info.cpu().numpy().view(frames.FRAME_SEGS_DTYPE).reshape(n)
    for i in range(n):
        e_ids, e_info, e_segs = O.segment_analysis(alpha_list[i], mbw, mbh, uv_sums[i], cfg_o)
        assert (ids[i] == e_ids).all(), f"image {i}: segment ids"
        assert info[i].tobytes() == e_info.tobytes(), (i, info[i], e_info)
        assert segs[i].tobytes() == e_segs.tobytes(), f"image {i}: quantiser records"
    return ids, info


def test_hand_cases(cuda):
    check([np.array([20] * 10 + [200] * 10)], 5, 4, [0], sns_strength=100, filter_strength=0)
    ids, info = check([np.array([0] * 8150 + [100] * 5 + [255] * 5)], 120, 68, [0], sns_strength=100,
                      filter_strength=0, segments=3)
    assert not ids.any() and info[0]["update_map"] == 0
    a = np.full((6, 6), 30)
    a[:, 3:] = 220
    a[2, 1] = 220
    check([a], 6, 6, [0], sns_strength=100, filter_strength=0, preprocessing=1)


@pytest.mark.parametrize("segments,sns,fs,sharp,pre,quality", [
    (4, 50, 60, 0, 0, 75), (4, 0, 60, 0, 0, 75), (4, 100, 100, 7, 1, 90), (3, 80, 35, 4, 1, 40),
    (2, 25, 10, 6, 0, 10), (1, 50, 60, 0, 0, 75), (4, 50, 0, 0, 3, 0), (4, 50, 60, 3, 0, 100)])
def test_configs_random_alphas(cuda, segments, sns, fs, sharp, pre, quality):
    rng = np.random.default_rng(segments * 1000 + sns + fs)
    mbw, mbh = 23, 17
    alist = []
    for k in range(6):
        mode = k % 3
        if mode == 0:
            a = rng.integers(0, 256, mbw * mbh)
        elif mode == 1:
            a = np.clip(rng.normal(rng.integers(30, 220), 15, mbw * mbh), 0, 255)
        else:  # two clusters
            a = np.where(rng.random(mbw * mbh) < 0.3, rng.integers(0, 40, mbw * mbh), rng.integers(180, 256, mbw * mbh))
        alist.append(a.astype(np.int32))
    uv = [int(x) * mbw * mbh for x in rng.integers(0, 200, 6)]
    check(alist, mbw, mbh, uv, segments=segments, sns_strength=sns, filter_strength=fs, filter_sharpness=sharp,
          preprocessing=pre, quality=quality)


@pytest.mark.parametrize("mbw,mbh", [(1, 1), (2, 1), (1, 5), (3, 3), (256, 256)])
def test_sizes(cuda, mbw, mbh):
    rng = np.random.default_rng(mbw * 7 + mbh)
    alist = [rng.integers(0, 256, mbw * mbh).astype(np.int32) for _ in range(2)] + [np.full(mbw * mbh, 77, np.int32)]
    check(alist, mbw, mbh, [5 * mbw * mbh, 90 * mbw * mbh, 0], preprocessing=1)


def test_real_frame_alphas(cuda):
    """alphas and uv sums from k_analysis on the three synthetic contents and
    the C1 frame, then the segment analysis of the same alphas."""
    w, h = 768, 576
    c1 = np.load(frames_golden("test_png_rgba.npz"))["rgba"]
    imgs = [c1, synth.gradient_rgba(w, h), synth.noise_rgba(w, h, seed=3), synth.blobs_rgba(w, h, seed=4)]
    Y, U, V = frames.import_rgba(torch.from_numpy(np.stack(imgs)).cuda(), has_alpha=False)
    alphas, uv_sum = frames.analysis_alphas(Y, U, V, w, h)
    mbw, mbh = frames.mb_dims(w, h)
    check(list(alphas.cpu().numpy()), mbw, mbh, [int(x) for x in uv_sum.cpu().numpy()])


def frames_golden(name):
    import os
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name)
